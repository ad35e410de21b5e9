"""CDI device lists in the native daemon (`-device_list_strategy`,
`-cdi_spec_dir`): spec files byte-equal to the Python CLI's
(rocm_k8s_device_plugin_amd/cdi.py), Allocate answers equal to the Python
plugin's for every strategy combination, and specs follow a partition switch.
The reference returns DeviceSpecs only (internal/pkg/amdgpu/amdgpu.go:255-297)."""
import asyncio
import os
import random
import subprocess

import pytest

from rocm_k8s_device_plugin_amd import cdi
from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
from rocm_k8s_device_plugin_amd.plugin.base import new_context
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node

from test_native_health import EXE, _stop
from test_reload import repartition


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)


def _daemon(kdir, fi, *extra):
    return subprocess.Popen([EXE, "-kubelet_dir", kdir, "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                             "-exporter_socket", "", *extra], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                            text=True)


@pytest.mark.parametrize("partition,naming,resource,lists", [
    ("spx", "single", "gpu", "cdi-cri"),
    ("spx", "single", "gpu", "device-specs,cdi-cri,cdi-annotations"),
    ("cpx", "single", "gpu", "cdi-annotations"),
    ("cpx", "mixed", "cpx_nps1", "device-specs,cdi-cri"),
])
def test_specs_and_answers_equal_the_python_plugin(tmp_path, partition, naming, resource, lists):
    fi = make_mi355x_node(tmp_path / "n", compute_partition=partition)
    py_dir, nat_dir = tmp_path / "cdi-py", tmp_path / "cdi-native"
    impl = ContainerImpl(naming, str(fi.sysfs), HealthConfig(exporter_socket=None),
                         device_list_strategy=cdi.parse_strategies(lists), cdi_spec_dir=str(py_dir))
    ctx = new_context(resource)
    impl.start(ctx)
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = _daemon(kdir, fi, "-resource_naming_strategy", naming, "-device_list_strategy", lists,
                    "-cdi_spec_dir", str(nat_dir))
        try:
            st = await k.wait_for_resource(f"amd.com/{resource}", len(impl.devices(resource)), timeout=20)
            rng = random.Random(5)
            ids = sorted(st.devices)
            for _ in range(15):
                chosen = sorted(rng.sample(ids, rng.randint(1, min(8, len(ids)))))
                areq = pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(devices_ids=chosen),
                                                              pb.ContainerAllocateRequest(devices_ids=[])])
                got = await k._call(st, "Allocate", areq, pb.AllocateResponse)
                assert got == impl.allocate(ctx, areq)
                car = got.container_responses[0]
                if "cdi-cri" in lists:
                    assert [c.name for c in car.cdi_devices] == [f"amd.com/{resource}={i}" for i in chosen]
                assert bool(car.devices) == ("device-specs" in lists)
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        assert "CDI specs written" in err

    asyncio.run(asyncio.wait_for(go(), 60))
    name = cdi.spec_filename(resource)
    assert sorted(os.listdir(nat_dir)) == [name]          # no temp file left behind
    assert (nat_dir / name).read_bytes() == (py_dir / name).read_bytes()
    assert oct((nat_dir / name).stat().st_mode & 0o777) == "0o644"


def test_specs_follow_a_partition_switch(tmp_path):
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    kdir, spec_dir = str(tmp_path / "dp"), tmp_path / "cdi"

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = _daemon(kdir, fi, "-resource_naming_strategy", "mixed", "-device_list_strategy", "cdi-cri",
                    "-cdi_spec_dir", str(spec_dir), "-topology_watch", "0.1")
        try:
            await k.wait_for_resource("amd.com/spx_nps1", 8, timeout=20)
            assert sorted(os.listdir(spec_dir)) == ["amd.com-spx_nps1.json"]
            repartition(root, compute_partition="cpx", memory_partition="nps2", generation=2)
            st = await k.wait_for_resource("amd.com/cpx_nps2", 64, timeout=10)
            assert sorted(os.listdir(spec_dir)) == ["amd.com-cpx_nps2.json"]
            adm = await k.admit("amd.com/cpx_nps2", 2)
            assert len(adm.device_ids) == 2
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]

    asyncio.run(asyncio.wait_for(go(), 60))
    py_dir = tmp_path / "cdi-py"
    cdi.write_specs(str(py_dir), {"cpx_nps2": ContainerImpl("mixed", str(fi.sysfs),
                                                            HealthConfig(exporter_socket=None)).devices("cpx_nps2")})
    assert (spec_dir / "amd.com-cpx_nps2.json").read_bytes() == (py_dir / "amd.com-cpx_nps2.json").read_bytes()


def test_bad_strategy_and_unwritable_dir(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    p = subprocess.run([EXE, "-device_list_strategy", "cdi-bogus"], capture_output=True, text=True, timeout=20)
    assert p.returncode == 1 and "invalid device_list_strategy 'cdi-bogus'" in p.stderr
    blocker = tmp_path / "file"
    blocker.write_text("x")
    p = _daemon(str(tmp_path / "dp"), fi, "-device_list_strategy", "cdi-cri", "-cdi_spec_dir", str(blocker / "cdi"))
    rc, err = _stop(p) if p.wait(timeout=20) is not None else (None, "")
    assert rc == 1 and "cannot write CDI specs to" in err
