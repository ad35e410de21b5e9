"""The real plugin on the reference's captured kfd topologies (CPU).

BASELINE config 1 is "ListAndWatch against fake-kubelet on
testdata/topology-parsing sysfs fixture". The reference's captures hold only
``class/kfd/kfd/topology`` and its GetAMDGPUs hard-codes ``/sys``
(amdgpu.go:448-568), so the reference itself cannot run on them;
``wrap_kfd_topology`` adds the PCI / drm / dev entries discovery joins the
nodes with, and the whole plugin (registration, ListAndWatch, preferred
allocation, Allocate) runs over UDS against the fake kubelet. Timings land in
the test log (``-s``); ``tools/bench_alloc.py`` has the allocator numbers.
"""
import asyncio
import time
from contextlib import asynccontextmanager

import pytest

from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.plugin.manager import ManagerConfig, PluginManager
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import wrap_kfd_topology

CAPTURES = {
    # name: (topology dir under testdata, GPU nodes, physical GPUs)
    "topology-parsing": ("topology-parsing/topology", 2, 2),
    "mi308-cpx": ("topology-parsing-mi308/topology", 32, 8),
    "mi300x-cpx": ("topo-mi300-cpx/topology", 63, 8),
    "mi210-2hives": ("topo-mi210-xgmi-pcie", 8, 8),
}


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


@pytest.mark.parametrize("name", sorted(CAPTURES))
def test_plugin_on_reference_capture(tmp_path, ref_testdata, name):
    sub, n_nodes, n_gpus = CAPTURES[name]
    fi = wrap_kfd_topology(ref_testdata / sub, tmp_path / "n")
    assert len(fi.bdfs) == n_nodes
    t0 = time.perf_counter()
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None))
    assert len(impl.inv) == n_nodes
    groups = {}
    for d in impl.inv.devices:
        groups.setdefault(d.unique_id or d.bdf, []).append(d.id)
    assert len(groups) == n_gpus

    async def go():
        async with plugin_env(tmp_path, impl) as (k, mgr):
            st = await k.wait_for_resource("amd.com/gpu", n_nodes)
            t_law = (time.perf_counter() - t0) * 1e3
            assert sorted(st.devices) == sorted(fi.bdfs)
            assert all(h == "Healthy" for h in st.devices.values())
            lat = []
            for size in sorted({1, 2, min(4, n_nodes), min(8, n_nodes)}):
                adm = await k.admit("amd.com/gpu", size)
                lat.append(adm.total_ms)
                assert adm.preferred_used and len(set(adm.device_ids)) == size
                car = adm.response.container_responses[0]
                paths = [d.host_path for d in car.devices]
                assert paths[0] == "/dev/kfd" and len(paths) == 1 + 2 * size
                for i in adm.device_ids:
                    g = impl.inv.by_id[i]
                    assert f"/dev/dri/renderD{g.render_minor}" in paths
                picked = {impl.inv.by_id[i].unique_id or i for i in adm.device_ids}
                if (name == "mi308-cpx" and size <= 4) or (name == "mi300x-cpx" and size <= 8):
                    assert len(picked) == 1, (size, adm.device_ids)   # partitions of one GPU
                if name == "mi210-2hives" and size == 4:
                    hives = {impl.inv.by_id[i].hive_id for i in adm.device_ids}
                    assert len(hives) == 1, adm.device_ids          # one xGMI hive, never split
                k.release("amd.com/gpu", adm.device_ids)
            print(f"{name}: {n_nodes} devices listed {t_law:.1f} ms after plugin init; "
                  f"admission p50 {sorted(lat)[len(lat) // 2]:.2f} ms")

    run(go())
