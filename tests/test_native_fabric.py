"""xGMI link state as a placement input in the native daemon (`-smi_xgmi`):
the native engine's watcher reaches the same degraded pairs as
health/fabric.py on the same readings. The daemon re-weights
GetPreferredAllocation when a link goes down and again when it comes back,
and the devices stay Healthy.

Readings are fake amd-smi snapshots shaped like the MI355X one: 8 link slots
per GPU, 7 up (one to each peer) and 1 disabled. The engine reads them from a
JSON file (`xgmi_file` / `$MI355X_SMI_XGMI_FILE`)."""
import asyncio
import json
import subprocess
import urllib.request

import pytest

from rocm_k8s_device_plugin_amd.allocator import group_key
from rocm_k8s_device_plugin_amd.health.fabric import FabricWatcher
from rocm_k8s_device_plugin_amd.ops.native import core
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.topology import discover

from test_fabric import FakeLinks
from test_native_health import EXE, _stop
from test_native_metrics import _free_port, _series


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)


class FileLinks(FakeLinks):
    """FakeLinks whose reading is written to a file the native side reads."""

    def __init__(self, path, bdfs, name_peers=True):
        super().__init__(bdfs, name_peers)
        self.path = path

    def publish(self):
        tmp = self.path.with_suffix(".tmp")
        tmp.write_text(json.dumps(self()))
        tmp.replace(self.path)


@pytest.mark.parametrize("name_peers", [True, False])
def test_engine_degraded_pairs_equal_the_python_watcher(tmp_path, name_peers):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    src = FileLinks(tmp_path / "xgmi.json", fi.bdfs, name_peers)
    src.publish()
    py = FabricWatcher(inv, src)
    eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev), "smi_xgmi": True,
                                              "xgmi_file": str(src.path)})
    try:
        def step():
            src.publish()
            py.check()
            eng.sweep()
            assert sorted(tuple(p) for p in eng.degraded_links()) == sorted(py.degraded)
            assert eng.links_down() == py.links_down
            return eng.fabric_version()

        assert step() == 0                                  # baseline
        src.cut.add(frozenset((fi.bdfs[0], fi.bdfs[3])))
        assert step() == 1 and eng.degraded_links()
        src.cut.add(frozenset((fi.bdfs[2], fi.bdfs[5])))
        assert step() == 2
        assert step() == 2                                  # unchanged: no new version
        src.cut.clear()
        assert step() == 3 and eng.degraded_links() == []
        src.ok = False                                      # amd-smi going away is not a fabric change
        assert step() == 3
        assert all(ok for ok, _ in eng.snapshot().values())  # a placement input, never a verdict
    finally:
        eng.close()


def test_daemon_reweights_preferred_allocation_on_link_down(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    src = FileLinks(tmp_path / "xgmi.json", fi.bdfs)
    src.publish()
    kdir = str(tmp_path / "dp")
    port = _free_port()
    key = {d.id: group_key(d) for d in inv.devices}

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        import os
        p = subprocess.Popen([EXE, "-kubelet_dir", kdir, "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                              "-exporter_socket", "", "-pulse", "1", "-smi_xgmi", "-metrics_port", str(port)],
                             stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                             env=dict(os.environ, MI355X_SMI_XGMI_FILE=str(src.path)))
        try:
            await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            adm = await k.admit("amd.com/gpu", 2)
            before = set(adm.device_ids)
            k.release("amd.com/gpu", adm.device_ids)
            a, b = sorted(before)
            src.cut.add(frozenset((a, b)))
            src.publish()
            for _ in range(100):
                adm = await k.admit("amd.com/gpu", 2)
                k.release("amd.com/gpu", adm.device_ids)
                if set(adm.device_ids) != before:
                    break
                await asyncio.sleep(0.1)
            assert set(adm.device_ids) != before
            st = k.resources["amd.com/gpu"]
            assert all(h == "Healthy" for h in st.devices.values())
            with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
                s = _series(r.read().decode())
            assert s["mi355x_dp_xgmi_links_down"] == 2 and s["mi355x_dp_fabric_reweights_total"] >= 1
            # the link is back: the original pair is preferred again
            src.cut.clear()
            src.publish()
            for _ in range(100):
                adm = await k.admit("amd.com/gpu", 2)
                k.release("amd.com/gpu", adm.device_ids)
                if set(adm.device_ids) == before:
                    break
                await asyncio.sleep(0.1)
            assert set(adm.device_ids) == before
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        pair = sorted((key[a], key[b]))
        assert f"xGMI link between GPUs {pair[0]} and {pair[1]} is down" in err
        assert "is back up" in err

    asyncio.run(asyncio.wait_for(go(), 60))
