"""Topology reload in the native daemon (`mi355x-device-plugin -topology_watch`):
the node's GPUs are re-partitioned while it runs, as with
``amd-smi set --compute-partition CPX``, and it re-discovers and re-advertises.
These are the scenarios tests/test_reload.py runs against the Python plugin.
The reference keeps advertising the devices it found at start-up."""
import asyncio
import os
import urllib.request

import pytest

from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.topology import discover

from test_native_health import EXE, _stop
from test_native_metrics import _free_port, _series
from test_reload import repartition


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)


def _daemon(kdir, fi, *extra):
    import subprocess
    return subprocess.Popen([EXE, "-kubelet_dir", kdir, "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                             "-exporter_socket", "", "-topology_watch", "0.1", *extra],
                            stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)


def _run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


def test_single_strategy_spx_to_cpx(tmp_path):
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    kdir = str(tmp_path / "dp")
    port = _free_port()

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = _daemon(kdir, fi, "-metrics_port", str(port))
        try:
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            before = st.updates
            repartition(root, compute_partition="cpx", generation=2)
            st = await k.wait_for_update("amd.com/gpu", before, timeout=10)
            while len(st.devices) != 64:
                st = await k.wait_for_update("amd.com/gpu", st.updates, timeout=10)
            assert any(d.startswith("amdgpu_xcp_") for d in st.devices)
            # the allocator was re-initialised on the partitions: 8 of one GPU
            adm = await k.admit("amd.com/gpu", 8)
            inv = discover(str(fi.sysfs))
            assert len({inv.by_id[d].unique_id for d in adm.device_ids}) == 1
            with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
                s = _series(r.read().decode())
            assert s["mi355x_dp_topology_reloads_total"] == 1
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        assert "GPU topology changed: 8 -> 64 devices; resources [gpu] -> [gpu]" in err

    _run(go())


def test_mixed_strategy_resource_switch(tmp_path):
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = _daemon(kdir, fi, "-resource_naming_strategy", "mixed")
        try:
            await k.wait_for_resource("amd.com/spx_nps1", 8, timeout=20)
            repartition(root, compute_partition="cpx", memory_partition="nps2", generation=2)
            st = await k.wait_for_resource("amd.com/cpx_nps2", 64, timeout=10)
            assert all(h == "Healthy" for h in st.devices.values())
            for _ in range(100):   # the old resource's server stops and removes its socket
                if not os.path.exists(os.path.join(kdir, "amd.com_spx_nps1")):
                    break
                await asyncio.sleep(0.05)
            assert not os.path.exists(os.path.join(kdir, "amd.com_spx_nps1"))
            assert os.path.exists(os.path.join(kdir, "amd.com_cpx_nps2"))
            adm = await k.admit("amd.com/cpx_nps2", 3)
            assert len(adm.device_ids) == 3
            # and back: the old resource name returns in its old slot
            old = k.resources["amd.com/spx_nps1"]
            repartition(root, generation=3)
            for _ in range(200):   # registered again: a new ListAndWatch with the 8 GPUs
                st = k.resources["amd.com/spx_nps1"]
                if st is not old and len(st.devices) == 8:
                    break
                await asyncio.sleep(0.05)
            assert st is not old and len(st.devices) == 8
            adm = await k.admit("amd.com/spx_nps1", 2)
            assert len(adm.device_ids) == 2
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        assert "resource spx_nps1 no longer exists" in err and "new resource cpx_nps2 (64 devices)" in err

    _run(go())


def test_single_strategy_turning_heterogeneous_advertises_nothing(tmp_path):
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = _daemon(kdir, fi)
        try:
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            repartition(root, per_gpu_compute=["spx"] * 4 + ["cpx"] * 4, generation=2)
            st = await k.wait_for_update("amd.com/gpu", st.updates, timeout=10)
            # mixed partition modes under "single" are refused, as at start-up: nothing to allocate
            assert st.devices == {}
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        assert "Advertising no devices until then" in err

    _run(go())


def test_same_devices_new_generation_is_a_no_op(tmp_path):
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = _daemon(kdir, fi)
        try:
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            (fi.sysfs / "class/kfd/kfd/topology/generation_id").write_text("7\n")
            await asyncio.sleep(0.6)
            assert k.resources["amd.com/gpu"].updates == st.updates
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0 and "GPU topology changed" not in err, err[-3000:]

    _run(go())
