"""Concurrent admissions under health flips and a partition switch (CPU,
fixtures + fake kubelet + fake exporter).

The reference serves RPCs on goroutines that share mutable Device objects
with the health updater and was never exercised
concurrently. Here many kubelet-side clients hammer GetPreferredAllocation +
Allocate on separate channels while the exporter flips verdicts every pulse
and the node is re-partitioned mid-run; every response must be internally
consistent with one device snapshot (old or new), never a mix.
"""
import asyncio
import random

import grpc

from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.plugin.manager import ManagerConfig, PluginManager
from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
from rocm_k8s_device_plugin_amd.testing.fake_exporter import FakeExporter
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.topology import discover

from test_reload import repartition


def run(coro, timeout=120):
    return asyncio.run(asyncio.wait_for(coro, timeout))


def _specs_by_id(inv):
    return {d.id: set(["/dev/kfd"] + d.dev_paths()) for d in inv.devices}


def test_concurrent_admissions_health_flips_and_repartition(tmp_path):
    root = tmp_path / "n"
    fi = make_mi355x_node(root, compute_partition="cpx")          # 64 devices
    sock = str(tmp_path / "exp" / "exporter.sock")
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=sock))
    old_specs = _specs_by_id(impl.inv)
    rng = random.Random(1234)
    stats = {"ok": 0, "stale": 0, "pref_err": 0}

    async def client(stub, n_iter, ids_fn):
        for _ in range(n_iter):
            ids = ids_fn()
            avail = rng.sample(ids, rng.randint(1, len(ids)))
            size = rng.randint(1, len(avail))
            must = rng.sample(avail, rng.randint(0, min(2, size)))
            req = pb.PreferredAllocationRequest()
            req.container_requests.add(available_deviceIDs=avail, must_include_deviceIDs=must, allocation_size=size)
            try:
                pref = await stub.GetPreferredAllocation(req, timeout=10)
            except grpc.aio.AioRpcError as e:
                # only an ID the plugin no longer advertises (after the switch) may fail
                assert e.code() == grpc.StatusCode.UNKNOWN, e
                stats["pref_err"] += 1
                continue
            got = list(pref.container_responses[0].deviceIDs)
            assert len(got) == size and len(set(got)) == size, (got, size)
            assert set(must) <= set(got) <= set(avail)
            areq = pb.AllocateRequest()
            areq.container_requests.add(devices_ids=got)
            try:
                resp = await stub.Allocate(areq, timeout=10)
            except grpc.aio.AioRpcError as e:
                assert e.code() == grpc.StatusCode.INVALID_ARGUMENT, e
                stats["stale"] += 1
                continue
            paths = {d.host_path for d in resp.container_responses[0].devices}
            # one snapshot: the union of the chosen devices' nodes in the old or the new inventory
            cur = _specs_by_id(impl.inv)
            for snap in (old_specs, cur):
                if all(i in snap for i in got) and paths == set().union(*(snap[i] for i in got)):
                    break
            else:
                raise AssertionError(f"Allocate specs {sorted(paths)} match no snapshot for {got}")
            assert sum(d.host_path == "/dev/kfd" for d in resp.container_responses[0].devices) == 1
            stats["ok"] += 1
            await asyncio.sleep(0)

    async def go():
        exp = FakeExporter(sock, {b: "healthy" for b in fi.bdfs})
        await exp.start()
        pdir = str(tmp_path / "dp")
        k = FakeKubelet(pdir)
        await k.start()
        mgr = PluginManager(impl, ManagerConfig(pulse_s=0.02, plugin_dir=pdir, handle_signals=False,
                                                retry_wait_s=0.05, watch_interval_s=0.05, topology_watch_s=0.05))
        task = asyncio.create_task(mgr.run())
        chans = []
        try:
            st = await k.wait_for_resource("amd.com/gpu", 64)
            sock_path = f"unix://{pdir}/amd.com_gpu"
            stubs = []
            for _ in range(8):
                ch = grpc.aio.insecure_channel(sock_path)
                chans.append(ch)
                stubs.append(pb.DevicePluginStub(ch))

            async def flipper():
                for i in range(40):
                    for b in fi.bdfs:
                        exp.states[b] = "unhealthy" if rng.random() < 0.3 else "healthy"
                    await asyncio.sleep(0.01)
                for b in fi.bdfs:
                    exp.states[b] = "healthy"

            async def switcher():
                await asyncio.sleep(0.15)
                repartition(root, compute_partition="spx", generation=2)

            ids_now = lambda: [d.id for d in impl.inv.devices]   # noqa: E731
            await asyncio.gather(flipper(), switcher(), *(client(s, 40, ids_now) for s in stubs))
            # the switch was picked up: 8 whole GPUs advertised, all healthy once the flips stop
            st = await k.wait_for_resource("amd.com/gpu", 1)
            for _ in range(200):
                if len(st.devices) == 8 and all(h == "Healthy" for h in st.devices.values()):
                    break
                await asyncio.sleep(0.02)
            assert sorted(st.devices) == sorted(fi.bdfs), sorted(st.devices)
            assert all(h == "Healthy" for h in st.devices.values())
            assert mgr.topology_reloads == 1
            # the re-initialised allocator packs whole GPUs again
            adm = await k.admit("amd.com/gpu", 2)
            assert len(adm.device_ids) == 2
        finally:
            for ch in chans:
                await ch.close()
            mgr.request_stop()
            await asyncio.wait_for(task, 20)
            await k.stop()
            await exp.stop()

    run(go())
    print("stress", stats)  # e.g. {ok: 312, stale: 5, pref_err: 3}: the switch lands mid-run
    assert stats["ok"] >= 100, stats
    assert len(discover(str(fi.sysfs)).devices) == 8
