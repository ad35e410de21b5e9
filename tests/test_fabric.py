"""xGMI link state as a placement input (-smi_xgmi, health/fabric.py), CPU:
a fake amd-smi source shaped like the MI355X reading (8 link slots: 7 up, one
to each peer, 1 disabled; gpurun_out/xgmi_links_box.json)."""
import asyncio

from rocm_k8s_device_plugin_amd.allocator import BestEffortPolicy, group_key
from rocm_k8s_device_plugin_amd.health.fabric import FabricWatcher
from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig, HealthMonitor
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.plugin.manager import ManagerConfig, PluginManager
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.topology import discover


class FakeLinks:
    """amd-smi xGMI reading for a fully connected hive; links can be cut."""

    def __init__(self, bdfs, name_peers=True):
        self.bdfs = list(bdfs)
        self.cut = set()          # frozenset({a, b})
        self.name_peers = name_peers
        self.ok = True

    def __call__(self):
        if not self.ok:
            return {"ok": False, "error": "amdsmi_init failed", "gpus": []}
        gpus = []
        for b in self.bdfs:
            peers = [p for p in self.bdfs if p != b]
            up = [p for p in peers if frozenset((b, p)) not in self.cut]
            gpus.append({"bdf": b, "status_ok": True, "status": [2] + [1] * len(up) + [0] * (len(peers) - len(up)),
                         "metrics_ok": self.name_peers,
                         "peers": [{"peer_bdf": "ffffffffffff:ff:1f.7", "link_type": 2, "bit_rate_gbps": 38}] +
                                  [{"peer_bdf": p, "link_type": 2, "bit_rate_gbps": 38, "max_bandwidth_gbps": 608}
                                   for p in up],
                         "error": ""})
        return {"ok": True, "error": "", "gpus": gpus}


def test_watcher_names_the_pair_and_clears_it(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    src = FakeLinks(fi.bdfs)
    w = FabricWatcher(inv, src)
    assert not w.check() and w.degraded == frozenset()          # baseline
    assert not w.check()
    key = {d.bdf: group_key(d) for d in inv.devices}
    src.cut.add(frozenset((fi.bdfs[0], fi.bdfs[3])))
    assert w.check()
    assert w.degraded == {tuple(sorted((key[fi.bdfs[0]], key[fi.bdfs[3]])))}
    assert w.links_down == {fi.bdfs[0]: 1, fi.bdfs[3]: 1}
    assert not w.check()                                         # unchanged: no new version
    v = w.version
    src.cut.clear()
    assert w.check() and w.degraded == frozenset() and w.version == v + 1
    # amd-smi going away is not a fabric change
    src.ok = False
    assert not w.check() and w.error


def test_watcher_without_peer_names_degrades_every_pair_of_the_gpu(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    src = FakeLinks(fi.bdfs, name_peers=False)
    w = FabricWatcher(inv, src)
    w.check()
    src.cut.add(frozenset((fi.bdfs[2], fi.bdfs[5])))
    assert w.check()
    key = {d.bdf: group_key(d) for d in inv.devices}
    g2 = key[fi.bdfs[2]]
    assert {p for p in w.degraded if g2 in p} == {tuple(sorted((g2, key[b]))) for b in fi.bdfs if b != fi.bdfs[2]}


def test_allocator_avoids_a_degraded_pair(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ids = [d.id for d in inv.devices]
    pol = BestEffortPolicy()
    pol.init(inv.devices, inv.topology)
    first = pol.allocate(ids, [], 2)
    a, b = (inv.by_id[i] for i in first)
    pol.init(inv.devices, inv.topology, degraded_links=[(group_key(a), group_key(b))])
    second = pol.allocate(ids, [], 2)
    assert set(second) != set(first)
    # a request that must include one end avoids the other end
    third = pol.allocate(ids, [first[0]], 2)
    assert first[0] in third and first[1] not in third
    # 8 of 8 still works (short-circuit: every GPU)
    assert sorted(pol.allocate(ids, [], 8)) == sorted(ids)


def test_plugin_reweights_on_link_down(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    src = FakeLinks(fi.bdfs)
    cfg = HealthConfig(exporter_socket=None, smi_xgmi=True)
    impl = ContainerImpl("single", str(fi.sysfs), cfg, inventory=inv,
                         monitor=HealthMonitor(inv, cfg, fabric_source=src))

    async def go():
        pdir = str(tmp_path / "dp")
        k = FakeKubelet(pdir)
        await k.start()
        mgr = PluginManager(impl, ManagerConfig(pulse_s=0.05, plugin_dir=pdir, handle_signals=False,
                                                topology_watch_s=0))
        task = asyncio.create_task(mgr.run())
        try:
            await k.wait_for_resource("amd.com/gpu", 8)
            adm = await k.admit("amd.com/gpu", 2)
            before = set(adm.device_ids)
            k.release("amd.com/gpu", adm.device_ids)
            a, b = sorted(before)
            src.cut.add(frozenset((a, b)))
            for _ in range(100):
                if impl.monitor.fabric_version:
                    break
                await asyncio.sleep(0.02)
            await asyncio.sleep(0.1)       # the manager re-inits allocators after the sweep
            assert impl.monitor.degraded_links()
            adm = await k.admit("amd.com/gpu", 2)
            assert set(adm.device_ids) != before
            st = k.resources["amd.com/gpu"]
            assert all(h == "Healthy" for h in st.devices.values())   # placement input, not a verdict
            # link back: the original pair is preferred again
            k.release("amd.com/gpu", adm.device_ids)
            src.cut.clear()
            for _ in range(100):
                if not impl.monitor.degraded_links():
                    break
                await asyncio.sleep(0.02)
            await asyncio.sleep(0.1)
            adm = await k.admit("amd.com/gpu", 2)
            assert set(adm.device_ids) == before
        finally:
            mgr.request_stop()
            await asyncio.wait_for(task, 20)
            await k.stop()

    asyncio.run(asyncio.wait_for(go(), 60))
