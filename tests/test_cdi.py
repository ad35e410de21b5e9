"""CDI device lists (-device_list_strategy): spec files for the advertised
devices and CDI names in Allocate. The reference returns DeviceSpecs only
(internal/pkg/amdgpu/amdgpu.go:255-297); that stays the default."""
import asyncio
import json
import os
from contextlib import asynccontextmanager

import pytest

from rocm_k8s_device_plugin_amd import cdi
from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.plugin.manager import ManagerConfig, PluginManager
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node

from test_reload import repartition


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


@asynccontextmanager
async def plugin_env(tmp_path, impl):
    pdir = str(tmp_path / "dp")
    k = FakeKubelet(pdir)
    await k.start()
    mgr = PluginManager(impl, ManagerConfig(pulse_s=0, plugin_dir=pdir, handle_signals=False, retry_wait_s=0.05,
                                            watch_interval_s=0.05, topology_watch_s=0))
    task = asyncio.create_task(mgr.run())
    try:
        yield k, mgr
    finally:
        mgr.request_stop()
        await asyncio.wait_for(task, 20)
        await k.stop()


def impl_for(fi, tmp_path, strategies, naming="single"):
    return ContainerImpl(naming, str(fi.sysfs), HealthConfig(exporter_socket=None),
                         device_list_strategy=strategies, cdi_spec_dir=str(tmp_path / "cdi"))


def test_strategy_parsing():
    assert cdi.parse_strategies("") == ["device-specs"]
    assert cdi.parse_strategies("cdi-cri, device-specs,cdi-cri") == ["cdi-cri", "device-specs"]
    with pytest.raises(ValueError):
        cdi.parse_strategies("volume-mounts")
    assert cdi.qualified_name("gpu", "0000:23:00.0") == "amd.com/gpu=0000:23:00.0"
    assert cdi.qualified_name("cpx_nps2", "amdgpu_xcp_9") == "amd.com/cpx_nps2=amdgpu_xcp_9"
    for bad in ("", "-x", "a b", "x/y", "0000:23:00.0:"):
        with pytest.raises(ValueError):
            cdi.qualified_name("gpu", bad)


def test_default_writes_no_spec(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    impl_for(fi, tmp_path, ["device-specs"])
    assert not (tmp_path / "cdi").exists()


def test_spec_file_matches_advertised_devices(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    impl = impl_for(fi, tmp_path, ["cdi-cri"])
    path = tmp_path / "cdi" / "amd.com-gpu.json"
    spec = json.loads(path.read_text())
    assert spec["cdiVersion"] == cdi.CDI_VERSION and spec["kind"] == "amd.com/gpu"
    assert spec["containerEdits"]["deviceNodes"] == [{"path": "/dev/kfd", "hostPath": "/dev/kfd", "permissions": "rw"}]
    assert sorted(d["name"] for d in spec["devices"]) == sorted(fi.bdfs)
    for d in spec["devices"]:
        g = impl.inv.by_id[d["name"]]
        assert [n["path"] for n in d["containerEdits"]["deviceNodes"]] == g.dev_paths()
        assert all(n["permissions"] == "rw" and n["hostPath"] == n["path"] for n in d["containerEdits"]["deviceNodes"])
    # written atomically: nothing but the spec in the directory
    assert os.listdir(tmp_path / "cdi") == ["amd.com-gpu.json"]
    assert oct(path.stat().st_mode & 0o777) == "0o644"


@pytest.mark.parametrize("strategies", [["cdi-cri"], ["device-specs", "cdi-cri"], ["cdi-annotations"]])
def test_allocate_returns_cdi_names(tmp_path, strategies):
    fi = make_mi355x_node(tmp_path / "n")
    impl = impl_for(fi, tmp_path, strategies)

    async def go():
        async with plugin_env(tmp_path, impl) as (k, mgr):
            await k.wait_for_resource("amd.com/gpu", 8)
            adm = await k.admit("amd.com/gpu", 2)
            car = adm.response.container_responses[0]
            names = [f"amd.com/gpu={i}" for i in adm.device_ids]
            if "cdi-cri" in strategies:
                assert [c.name for c in car.cdi_devices] == names
            else:
                assert not car.cdi_devices
            if "cdi-annotations" in strategies:
                assert dict(car.annotations) == {"cdi.k8s.io/amd.com_gpu": ",".join(names)}
            else:
                assert not car.annotations
            specs = [d.host_path for d in car.devices]
            if "device-specs" in strategies:
                assert specs[0] == "/dev/kfd" and len(specs) == 1 + 2 * 2
            else:
                assert specs == []
            # every name resolves in the written spec
            spec = json.loads((tmp_path / "cdi" / "amd.com-gpu.json").read_text())
            known = {f"{spec['kind']}={d['name']}" for d in spec["devices"]}
            assert set(names) <= known

    run(go())


def test_cpx_partitions_are_cdi_devices(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", compute_partition="cpx", memory_partition="nps2")
    impl = impl_for(fi, tmp_path, ["cdi-cri"], naming="mixed")
    spec = json.loads((tmp_path / "cdi" / "amd.com-cpx_nps2.json").read_text())
    assert spec["kind"] == "amd.com/cpx_nps2"
    names = {d["name"] for d in spec["devices"]}
    assert len(names) == 64 and names == {d.id for d in impl.inv.devices}
    assert sum(n.startswith("amdgpu_xcp_") for n in names) == 56


def test_topology_reload_rewrites_specs(tmp_path):
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    impl = impl_for(fi, tmp_path, ["cdi-cri"], naming="mixed")
    assert os.listdir(tmp_path / "cdi") == ["amd.com-spx_nps1.json"]

    async def go():
        repartition(root, compute_partition="cpx", memory_partition="nps2", generation=2)
        change = await impl.reload_topology()
        assert change and change["resources_changed"]
        await impl.close()

    run(go())
    # the old resource's spec is gone, the new one lists the 64 partitions
    assert os.listdir(tmp_path / "cdi") == ["amd.com-cpx_nps2.json"]
    spec = json.loads((tmp_path / "cdi" / "amd.com-cpx_nps2.json").read_text())
    assert len(spec["devices"]) == 64


def test_cli_rejects_unknown_strategy():
    from rocm_k8s_device_plugin_amd.cli import device_plugin as cli
    assert cli.main(["-device_list_strategy=volume-mounts"]) == 1


def test_cli_dry_run_with_cdi(tmp_path, capsys):
    fi = make_mi355x_node(tmp_path / "n")
    from rocm_k8s_device_plugin_amd.cli import device_plugin as cli
    rc = cli.main(["-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-exporter_socket=",
                   "-device_list_strategy=cdi-cri", "-cdi_spec_dir", str(tmp_path / "cdi"),
                   "-kubelet_dir", str(tmp_path / "dp")])
    assert rc == 0
    assert (tmp_path / "cdi" / "amd.com-gpu.json").exists()


def test_unwritable_spec_dir_is_an_init_error(tmp_path):
    from rocm_k8s_device_plugin_amd.plugin.base import DeviceImplError
    fi = make_mi355x_node(tmp_path / "n")
    blocker = tmp_path / "file"
    blocker.write_text("")
    with pytest.raises(DeviceImplError, match="CDI specs"):
        ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None), device_list_strategy=["cdi-cri"],
                      cdi_spec_dir=str(blocker / "cdi"))
