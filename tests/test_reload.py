"""Topology reload: the node's GPUs are re-partitioned while the plugin runs
(e.g. ``amd-smi set --compute-partition CPX``). The reference keeps
advertising the devices it found at start-up; here the plugin re-discovers
and re-advertises (CPU, fixtures + fake kubelet)."""
import asyncio
import os
import shutil
from contextlib import asynccontextmanager

from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.plugin.manager import ManagerConfig, PluginManager
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


@asynccontextmanager
async def plugin_env(tmp_path, impl, **mcfg):
    pdir = str(tmp_path / "dp")
    k = FakeKubelet(pdir)
    await k.start()
    cfg = ManagerConfig(pulse_s=0, plugin_dir=pdir, handle_signals=False, retry_wait_s=0.05,
                        watch_interval_s=0.05, **mcfg)
    mgr = PluginManager(impl, cfg)
    task = asyncio.create_task(mgr.run())
    try:
        yield k, mgr
    finally:
        mgr.request_stop()
        await asyncio.wait_for(task, 20)
        await k.stop()


def repartition(root, **spec):
    """Swap in a freshly generated tree for the node (what the driver shows
    after a partition switch), replacing the old one in two renames."""
    new = root.parent / (root.name + ".new")
    shutil.rmtree(new, ignore_errors=True)
    make_mi355x_node(new, **spec)
    old = root.parent / (root.name + ".old")
    os.rename(root / "sys", old)
    os.rename(new / "sys", root / "sys")
    shutil.rmtree(old)
    shutil.rmtree(new)


def test_signature_and_no_op_reload(tmp_path):
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None))

    async def go():
        assert await impl.reload_topology() is None                 # nothing changed
        (fi.sysfs / "class/kfd/kfd/topology/generation_id").write_text("7\n")
        v = impl.health_version()
        assert await impl.reload_topology() is None                 # generation moved, same devices
        assert impl.health_version() == v
        await impl.close()

    run(go())


def test_single_strategy_spx_to_cpx(tmp_path):
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None))

    async def go():
        async with plugin_env(tmp_path, impl, topology_watch_s=0) as (k, mgr):
            st = await k.wait_for_resource("amd.com/gpu", 8)
            before = st.updates
            repartition(root, compute_partition="cpx", generation=2)
            change = await impl.reload_topology()
            assert change and not change["resources_changed"]
            assert len(change["added"]) == 56 and change["removed"] == []
            await mgr._apply_topology_change(change)
            st = await k.wait_for_update("amd.com/gpu", before)
            assert len(st.devices) == 64 and any(d.startswith("amdgpu_xcp_") for d in st.devices)
            # the allocator was re-initialised on the partitions: 8 of one GPU
            adm = await k.admit("amd.com/gpu", 8)
            assert len({impl.inv.by_id[d].unique_id for d in adm.device_ids}) == 1
            assert mgr.topology_reloads == 1

    run(go())


def test_mixed_strategy_resource_switch(tmp_path):
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    impl = ContainerImpl("mixed", str(fi.sysfs), HealthConfig(exporter_socket=None))

    async def go():
        async with plugin_env(tmp_path, impl, topology_watch_s=0.05) as (k, mgr):
            await k.wait_for_resource("amd.com/spx_nps1", 8)
            repartition(root, compute_partition="cpx", memory_partition="nps2", generation=2)
            # the watch loop notices by itself: new resource registered, old one gone
            st = await k.wait_for_resource("amd.com/cpx_nps2", 64, timeout=10)
            assert all(h == "Healthy" for h in st.devices.values())
            assert set(mgr.plugins) == {"cpx_nps2"}
            assert not os.path.exists(tmp_path / "dp" / "amd.com_spx_nps1")
            assert os.path.exists(tmp_path / "dp" / "amd.com_cpx_nps2")
            adm = await k.admit("amd.com/cpx_nps2", 3)
            assert len(adm.device_ids) == 3

    run(go())


def test_single_strategy_turning_heterogeneous_advertises_nothing(tmp_path):
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None))

    async def go():
        async with plugin_env(tmp_path, impl, topology_watch_s=0) as (k, mgr):
            st = await k.wait_for_resource("amd.com/gpu", 8)
            before = st.updates
            repartition(root, per_gpu_compute=["spx"] * 4 + ["cpx"] * 4, generation=2)
            change = await impl.reload_topology()
            await mgr._apply_topology_change(change)
            st = await k.wait_for_update("amd.com/gpu", before)
            # mixed partition modes under "single" are refused, as at start-up: nothing to allocate
            assert st.devices == {}

    run(go())


def test_topology_watch_waits_for_a_fingerprint_to_hold(tmp_path):
    """A fingerprint seen once (a switch half done) does not trigger a
    re-discovery; one that holds for a second poll does."""
    fi = make_mi355x_node(tmp_path / "n")
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None))
    seq = ["A", "A", "B", "A", "A", "C", "C"]
    polls, reloads = [], []

    def fingerprint():
        v = seq[min(len(polls), len(seq) - 1)]
        polls.append(v)
        return v

    async def reload_topology():
        reloads.append(polls[-1])
        return None

    impl.topology_fingerprint = fingerprint
    impl.reload_topology = reload_topology
    mgr = PluginManager(impl, ManagerConfig(pulse_s=0, plugin_dir=str(tmp_path / "dp"), handle_signals=False,
                                            topology_watch_s=0.01))

    async def go():
        mgr._impl_lock = asyncio.Lock()   # run() creates it on its loop
        task = asyncio.create_task(mgr._topology_loop())
        while len(polls) < len(seq):
            await asyncio.sleep(0.005)
        mgr.stopped.set()
        await asyncio.wait_for(task, 5)

    run(go())
    # first sighting of each value skips (A, B, A again, C); stable repeats re-discover
    assert reloads[:3] == ["A", "A", "C"], reloads
