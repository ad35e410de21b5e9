"""Device plugin end to end over real gRPC/UDS against the fake kubelet.

Covers what the reference never tested: registration,
ListAndWatch streaming, Allocate / GetPreferredAllocation responses, kubelet
restart re-registration, late kubelet start, shutdown cleanup, health flips
from the exporter, liveness fault injection, kfd node loss, the mixed
strategy on heterogeneous nodes and passthrough modes.
"""
import asyncio
import json
import os
import sys
from contextlib import asynccontextmanager

import grpc
import pytest

from rocm_k8s_device_plugin_amd import constants as C
from rocm_k8s_device_plugin_amd.health.liveness import LivenessProber
from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig, HealthMonitor
from rocm_k8s_device_plugin_amd.plugin.base import DeviceImplError
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.plugin.manager import ManagerConfig, PluginManager
from rocm_k8s_device_plugin_amd.plugin.passthrough import PfImpl, VfImpl
from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
from rocm_k8s_device_plugin_amd.testing.fake_exporter import FakeExporter
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.topology import discover

STUB = os.path.join(os.path.dirname(__file__), "..", "rocm_k8s_device_plugin_amd", "testing", "stub_probe.py")


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


@asynccontextmanager
async def plugin_env(tmp_path, impl, pulse=0.0, start_kubelet=True, **mcfg):
    pdir = str(tmp_path / "dp")
    k = FakeKubelet(pdir)
    if start_kubelet:
        await k.start()
    cfg = ManagerConfig(**{"pulse_s": pulse, "plugin_dir": pdir, "handle_signals": False, "retry_wait_s": 0.05,
                           "watch_interval_s": 0.05, **mcfg})
    mgr = PluginManager(impl, cfg)
    task = asyncio.create_task(mgr.run())
    try:
        yield k, mgr
    finally:
        mgr.request_stop()
        await asyncio.wait_for(task, 20)
        await k.stop()


def container(fi, strategy="single", **hc):
    hc.setdefault("exporter_socket", None)
    return ContainerImpl(strategy, str(fi.sysfs), HealthConfig(**hc))


# ------------------------------------------------------------------ basics

def test_register_list_allocate(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    impl = container(fi)

    async def go():
        async with plugin_env(tmp_path, impl) as (k, mgr):
            st = await k.wait_for_resource("amd.com/gpu", 8)
            reg = k.registrations[0]
            assert reg.version == "v1beta1" and reg.endpoint == "amd.com_gpu"
            assert reg.resource_name == "amd.com/gpu"
            assert reg.options.get_preferred_allocation_available and not reg.options.pre_start_required
            assert set(st.devices) == set(fi.bdfs)
            assert all(h == "Healthy" for h in st.devices.values())
            assert st.numa["0000:05:00.0"] == [0] and st.numa["0000:f5:00.0"] == [1]
            adm = await k.admit("amd.com/gpu", 2)
            specs = [(d.container_path, d.host_path, d.permissions) for d in adm.response.container_responses[0].devices]
            assert specs[0] == ("/dev/kfd", "/dev/kfd", "rw")
            for dev in adm.device_ids:
                g = impl.inv.by_id[dev]
                assert (f"/dev/dri/card{g.card}", f"/dev/dri/card{g.card}", "rw") in specs
                assert (f"/dev/dri/renderD{g.render_minor}", f"/dev/dri/renderD{g.render_minor}", "rw") in specs
            assert len(specs) == 1 + 2 * 2
            assert not adm.response.container_responses[0].envs
            # PreStartContainer is a no-op
            r = await st.stub.PreStartContainer(pb.PreStartContainerRequest(devices_ids=adm.device_ids))
            assert r == pb.PreStartContainerResponse()
            # unknown device -> INVALID_ARGUMENT, not a silent empty spec list
            req = pb.AllocateRequest()
            req.container_requests.add(devices_ids=["0000:ff:00.0"])
            with pytest.raises(grpc.aio.AioRpcError) as e:
                await st.stub.Allocate(req)
            assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
            # multi-container pod: one /dev/kfd per container
            req = pb.AllocateRequest()
            req.container_requests.add(devices_ids=[fi.bdfs[0]])
            req.container_requests.add(devices_ids=[fi.bdfs[1]])
            resp = await st.stub.Allocate(req)
            assert [sum(d.host_path == "/dev/kfd" for d in c.devices) for c in resp.container_responses] == [1, 1]
        assert not os.path.exists(tmp_path / "dp" / "amd.com_gpu"), "socket not cleaned up"

    run(go())


def test_preferred_allocation_packs_one_hive(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", hive_size=4)   # two xGMI hives of 4 GPUs
    impl = container(fi)
    hive = {d.id: d.hive_id for d in impl.inv.devices}

    async def go():
        async with plugin_env(tmp_path, impl) as (k, mgr):
            await k.wait_for_resource("amd.com/gpu", 8)
            for n in (2, 3, 4):
                adm = await k.admit("amd.com/gpu", n)
                assert adm.preferred_used
                assert len({hive[d] for d in adm.device_ids}) == 1, adm.device_ids
                k.release("amd.com/gpu", adm.device_ids)
            # fragment hive A: 2 free there, 4 free in B -> a 3-GPU pod goes to B
            first = await k.admit("amd.com/gpu", 2, available=fi.bdfs[:4])
            adm = await k.admit("amd.com/gpu", 3)
            assert {hive[d] for d in adm.device_ids} == {hive[fi.bdfs[4]]}
            # must_include is honoured
            k.release("amd.com/gpu", adm.device_ids + first.device_ids)
            adm = await k.admit("amd.com/gpu", 2, must_include=[fi.bdfs[6]])
            assert fi.bdfs[6] in adm.device_ids and len({hive[d] for d in adm.device_ids}) == 1
            # an impossible request surfaces the allocator's error string
            st = k.resources["amd.com/gpu"]
            req = pb.PreferredAllocationRequest()
            req.container_requests.add(available_deviceIDs=fi.bdfs[:2], must_include_deviceIDs=[],
                                       allocation_size=3)
            with pytest.raises(grpc.aio.AioRpcError) as e:
                await st.stub.GetPreferredAllocation(req)
            assert "available devices count less than allocation size" in e.value.details()

    run(go())


def test_cpx_partitions_prefer_same_gpu(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", compute_partition="cpx")
    impl = container(fi)
    uid = {d.id: d.unique_id for d in impl.inv.devices}

    async def go():
        async with plugin_env(tmp_path, impl) as (k, mgr):
            st = await k.wait_for_resource("amd.com/gpu", 64)
            assert any(d.startswith("amdgpu_xcp_") for d in st.devices)
            adm = await k.admit("amd.com/gpu", 4)
            assert len({uid[d] for d in adm.device_ids}) == 1
            adm2 = await k.admit("amd.com/gpu", 4)
            # anti-fragmentation: the second 4 fills the same, already-opened GPU
            assert {uid[d] for d in adm2.device_ids} == {uid[d] for d in adm.device_ids}

    run(go())


# ------------------------------------------------------------ strategies

def test_mixed_strategy_heterogeneous(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", per_gpu_compute=["spx"] * 4 + ["cpx"] * 4)
    with pytest.raises(DeviceImplError, match="not supported with single strategy"):
        container(fi, "single")
    impl = container(fi, "mixed")
    assert impl.resource_names() == ["cpx_nps1", "spx_nps1"]

    async def go():
        async with plugin_env(tmp_path, impl, pulse=0.1, send_every_pulse=True) as (k, mgr):
            a = await k.wait_for_resource("amd.com/spx_nps1", 4)
            b = await k.wait_for_resource("amd.com/cpx_nps1", 32)
            assert len(a.devices) == 4 and len(b.devices) == 32
            ua, ub = a.updates, b.updates
            # every pulse reaches EVERY resource's stream (reference Appendix B #1)
            await k.wait_for_update("amd.com/spx_nps1", ua + 2, timeout=10)
            await k.wait_for_update("amd.com/cpx_nps1", ub + 2, timeout=10)
            adm = await k.admit("amd.com/cpx_nps1", 3)
            assert all(impl.inv.by_id[d].partition_type == "cpx_nps1" for d in adm.device_ids)

    run(go())


def test_mixed_strategy_homogeneous_partition_name(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", compute_partition="dpx", memory_partition="nps2")
    assert container(fi, "mixed").resource_names() == ["dpx_nps2"]
    assert container(fi, "single").resource_names() == ["gpu"]
    fi2 = make_mi355x_node(tmp_path / "m", partition_support=False)
    assert container(fi2, "mixed").resource_names() == ["gpu"]


def test_device_count_limit(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", compute_partition="qpx")
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None), device_count_limit=2)
    assert len(impl.devices("gpu")) == 8  # 2 physical GPUs x 4 partitions
    assert len({d.unique_id for d in impl.devices("gpu")}) == 2


def test_no_kfd_is_an_init_error(tmp_path):
    with pytest.raises(DeviceImplError, match="No amd gpu driver loaded"):
        ContainerImpl("single", str(tmp_path), HealthConfig(exporter_socket=None))


# ----------------------------------------------------------- lifecycle

def test_kubelet_restart_reregisters(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    impl = container(fi)

    async def go():
        async with plugin_env(tmp_path, impl) as (k, mgr):
            await k.wait_for_resource("amd.com/gpu", 8)
            assert len(k.registrations) == 1
            await k.restart(downtime_s=0.2)
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=10)
            assert len(k.registrations) == 2
            adm = await k.admit("amd.com/gpu", 1)
            assert len(adm.device_ids) == 1
            # quick delete+recreate (inode reuse) is also detected
            await k.restart()
            await k.wait_for_resource("amd.com/gpu", 8, timeout=10)
            assert len(k.registrations) == 3
            assert mgr.plugins["gpu"].registrations == 3

    run(go())


def test_late_kubelet(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    impl = container(fi)

    async def go():
        async with plugin_env(tmp_path, impl, start_kubelet=False, start_retries=2) as (k, mgr):
            await asyncio.wait_for(mgr.ready.wait(), 10)
            assert not mgr.plugins["gpu"].running          # registration failed, retries exhausted
            await k.start()                                  # kubelet comes up later
            await k.wait_for_resource("amd.com/gpu", 8, timeout=10)
            assert mgr.plugins["gpu"].running

    run(go())


def test_no_impl_idles(tmp_path):
    async def go():
        async with plugin_env(tmp_path, None) as (k, mgr):
            await asyncio.wait_for(mgr.ready.wait(), 5)
            assert mgr.resources() == []
            await asyncio.sleep(0.2)
            assert k.registrations == []

    run(go())


# -------------------------------------------------------------- health

def test_exporter_health_flip_reaches_partitions(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", compute_partition="dpx")
    sock = str(tmp_path / "exp" / "exporter.sock")
    impl = container(fi, exporter_socket=sock)
    bad_bdf = fi.bdfs[3]

    async def go():
        exp = FakeExporter(sock, {b: "healthy" for b in fi.bdfs})
        await exp.start()
        try:
            async with plugin_env(tmp_path, impl, pulse=0.1) as (k, mgr):
                st = await k.wait_for_resource("amd.com/gpu", 16)
                u = st.updates
                exp.states[bad_bdf] = "unhealthy"
                st = await k.wait_for_update("amd.com/gpu", u, timeout=10)
                bad = sorted(d for d, h in st.devices.items() if h == "Unhealthy")
                # the BDF verdict applies to the GPU's xcp partition too (reference Appendix B #4)
                want = sorted(d.id for d in impl.inv.devices if d.bdf == bad_bdf)
                assert bad == want and len(want) == 2
                # kubelet must not hand out unhealthy devices
                assert not set(bad) & set(k.healthy_free("amd.com/gpu"))
                u = st.updates
                exp.states[bad_bdf] = "healthy"
                st = await k.wait_for_update("amd.com/gpu", u, timeout=10)
                assert all(h == "Healthy" for h in st.devices.values())
                assert exp.calls >= 2
        finally:
            await exp.stop()

    run(go())


def _stub_prober(tmp_path, control, timeout=2.0):
    ctl = tmp_path / "probe_ctl.json"
    ctl.write_text(json.dumps(control))
    return ctl, LivenessProber(exe=STUB, argv_prefix=[sys.executable], timeout_s=timeout,
                               extra_env={"MI355X_STUB_PROBE_CONTROL": str(ctl)})


def test_liveness_fault_injection_hysteresis(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ords = {d.id: i for i, d in enumerate(inv.devices)}
    ctl, prober = _stub_prober(tmp_path, {"2": "fail", "5": "hang", "6": "stale", "7": "garbage"}, timeout=1.5)
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, fail_threshold=2,
                                          recover_threshold=1), prober=prober, ordinal_map=ords)

    async def go():
        changed = await mon.check_once()          # 1st failure: below threshold
        assert not changed and all(v.health == "Healthy" for v in mon.snapshot().values())
        changed = await mon.check_once()          # 2nd consecutive failure
        assert changed
        snap = mon.snapshot()
        bad = {d for d, v in snap.items() if v.health == "Unhealthy"}
        assert bad == {fi.bdfs[2], fi.bdfs[5], fi.bdfs[6], fi.bdfs[7]}
        assert "differ" in snap[fi.bdfs[2]].reasons[0]
        assert "deadline" in snap[fi.bdfs[5]].reasons[0]
        assert "stale" in snap[fi.bdfs[6]].reasons[0]
        assert "unparseable" in snap[fi.bdfs[7]].reasons[0]
        ctl.write_text("{}")                        # everything recovers
        assert await mon.check_once()
        assert all(v.health == "Healthy" for v in mon.snapshot().values())

    run(go(), timeout=60)


def test_liveness_through_listandwatch(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    ctl, prober = _stub_prober(tmp_path, {})
    inv = discover(str(fi.sysfs))
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, fail_threshold=1), prober=prober,
                        ordinal_map={d.id: i for i, d in enumerate(inv.devices)})
    impl = ContainerImpl("single", str(fi.sysfs), inventory=inv, monitor=mon)

    async def go():
        async with plugin_env(tmp_path, impl, pulse=0.1) as (k, mgr):
            st = await k.wait_for_resource("amd.com/gpu", 8)
            u = st.updates
            ctl.write_text(json.dumps({"4": "fail"}))
            st = await k.wait_for_update("amd.com/gpu", u, timeout=15)
            assert st.devices[fi.bdfs[4]] == "Unhealthy"
            assert sum(h == "Unhealthy" for h in st.devices.values()) == 1

    run(go())


def test_first_listandwatch_already_carries_health(tmp_path):
    """With a pulse, one sweep runs before registration: a dead GPU is never advertised Healthy."""
    fi = make_mi355x_node(tmp_path / "n")
    ctl, prober = _stub_prober(tmp_path, {"3": "fail"})
    inv = discover(str(fi.sysfs))
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, fail_threshold=1), prober=prober,
                        ordinal_map={d.id: i for i, d in enumerate(inv.devices)})
    impl = ContainerImpl("single", str(fi.sysfs), inventory=inv, monitor=mon)

    async def go():
        async with plugin_env(tmp_path, impl, pulse=30) as (k, mgr):
            st = await k.wait_for_resource("amd.com/gpu", 8)
            assert st.updates == 1                                  # the initial list, no pulse yet
            assert {d for d, h in st.devices.items() if h == "Unhealthy"} == {fi.bdfs[3]}

    run(go())


def test_kfd_node_loss_marks_device_unhealthy(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    impl = container(fi)
    victim = impl.inv.by_id[fi.bdfs[1]]

    async def go():
        async with plugin_env(tmp_path, impl, pulse=0.1) as (k, mgr):
            st = await k.wait_for_resource("amd.com/gpu", 8)
            u = st.updates
            os.remove(fi.sysfs / "class/kfd/kfd/topology/nodes" / str(victim.node_id) / "properties")
            st = await k.wait_for_update("amd.com/gpu", u, timeout=10)
            assert st.devices[victim.id] == "Unhealthy"
            assert sum(h == "Unhealthy" for h in st.devices.values()) == 1

    run(go())


# ---------------------------------------------------------- passthrough

def test_vf_passthrough(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", mode="vf", vfs_per_gpu=2)
    sock = str(tmp_path / "exp.sock")
    impl = VfImpl("mixed", str(fi.sysfs), exporter_socket=sock)
    assert impl.resource_names() == ["gpu_vf"]
    assert VfImpl("single", str(fi.sysfs)).resource_names() == ["gpu"]

    async def go():
        exp = FakeExporter(sock, {b: "healthy" for b in fi.bdfs})
        await exp.start()
        try:
            async with plugin_env(tmp_path, impl, pulse=0.1) as (k, mgr):
                st = await k.wait_for_resource("amd.com/gpu_vf", 16)
                assert not k.registrations[0].options.get_preferred_allocation_available
                groups = sorted(st.devices, key=int)[:3]
                adm = await k.admit("amd.com/gpu_vf", 3, available=groups)
                car = adm.response.container_responses[0]
                paths = [d.host_path for d in car.devices]
                assert [d.permissions for d in car.devices] == ["mrw"] * len(paths)
                assert paths.count("/dev/vfio/vfio") == 1           # once per container (Appendix B #9)
                for g in groups:
                    assert f"/dev/vfio/{g}" in paths
                env = car.envs["PCI_RESOURCE_AMD_COM_GPU_VF"].split(",")
                assert len(env) == 3                               # all groups, not only the last
                # PF unhealthy -> its VF groups unhealthy
                u = st.updates
                exp.states[fi.bdfs[0]] = "unhealthy"
                st = await k.wait_for_update("amd.com/gpu_vf", u, timeout=10)
                bad = sorted((d for d, h in st.devices.items() if h == "Unhealthy"), key=int)
                assert bad == ["100", "101"]
        finally:
            await exp.stop()

    run(go())


def test_vf_driver_removed(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", mode="vf")
    impl = VfImpl("single", str(fi.sysfs), exporter_socket=None)
    os.rmdir(fi.sysfs / "bus/pci/drivers/gim")
    assert run(impl.refresh_health())
    assert all(d.health == "Unhealthy" for d in impl.enumerate(None))


def test_pf_passthrough(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", mode="pf")
    impl = PfImpl("mixed", str(fi.sysfs))
    assert impl.resource_names() == ["gpu_pf"]
    devs = impl.enumerate(None)
    assert [d.ID for d in devs] == [str(10 + i) for i in range(8)]
    from rocm_k8s_device_plugin_amd.plugin.base import PluginContext
    req = pb.AllocateRequest()
    req.container_requests.add(devices_ids=["10", "13"])
    resp = impl.allocate(PluginContext("gpu_pf"), req)
    assert resp.container_responses[0].envs["PCI_RESOURCE_AMD_COM_GPU_PF"] == f"{fi.bdfs[0]},{fi.bdfs[3]}"
    with pytest.raises(DeviceImplError, match="not found"):
        bad = pb.AllocateRequest()
        bad.container_requests.add(devices_ids=["99"])
        impl.allocate(PluginContext("gpu_pf"), bad)
    os.rmdir(fi.sysfs / "bus/pci/drivers/vfio-pci")
    assert run(impl.refresh_health())
    assert all(d.health == "Unhealthy" for d in impl.enumerate(None))
    with pytest.raises(DeviceImplError, match="vfio-pci"):
        PfImpl("single", str(fi.sysfs))


# ----------------------------------------------------------------- CLI

def test_cli_validation(tmp_path):
    from rocm_k8s_device_plugin_amd.cli import device_plugin as cli
    assert cli.main(["-pulse=-1"]) == 1
    assert cli.main(["-driver_type", "bogus"]) == 1
    assert cli.main(["--resource_naming_strategy=weird"]) == 1
    assert cli.main(["-liveness_mode=sometimes"]) == 1
    with pytest.raises(SystemExit) as e:
        cli.main(["-driver_type=container", "-sysfs_root", str(tmp_path)])
    assert e.value.code == 1


def test_cli_flag_spellings():
    from rocm_k8s_device_plugin_amd.cli import device_plugin as cli
    ns = cli.build_parser().parse_args(["-logtostderr=true", "-stderrthreshold=INFO", "-v=5", "-pulse=2",
                                        "--resource_naming_strategy", "mixed", "-liveness"])
    assert ns.pulse == 2 and ns.v == 5 and ns.logtostderr is True and ns.liveness is True
    assert ns.resource_naming_strategy == "mixed"
    assert ns.liveness_mode == "persistent"
    assert cli.build_parser().parse_args(["-liveness_mode=spawn"]).liveness_mode == "spawn"


def test_cli_autoselect_order(tmp_path):
    from rocm_k8s_device_plugin_amd.cli import device_plugin as cli
    from rocm_k8s_device_plugin_amd.utils import log
    lg = log.setup(0)
    p = cli.build_parser()
    fi = make_mi355x_node(tmp_path / "vf", mode="vf")
    ns = p.parse_args(["-sysfs_root", str(fi.sysfs), "-exporter_socket", ""])
    impl = cli.select_impl(ns, None, lg)
    assert impl.name == C.VF_PASSTHROUGH           # no kfd -> container fails -> VF
    fi2 = make_mi355x_node(tmp_path / "c")
    ns = p.parse_args(["-sysfs_root", str(fi2.sysfs), "-exporter_socket", ""])
    assert cli.select_impl(ns, None, lg).name == C.CONTAINER
    ns = p.parse_args(["-sysfs_root", str(tmp_path / "empty")])
    assert cli.select_impl(ns, None, lg) is None


def test_cli_config_file_device_count(tmp_path, monkeypatch):
    from rocm_k8s_device_plugin_amd.cli import device_plugin as cli
    cfgf = tmp_path / "config.yaml"
    cfgf.write_text("gpu:\n  device_count: 3\n")
    assert cli.load_config(str(cfgf))["gpu"]["device_count"] == 3
    from rocm_k8s_device_plugin_amd.topology import device_count_limit_from_env
    assert device_count_limit_from_env({"AMD_GPU_DEVICE_COUNT": "2"}) == 2
    assert device_count_limit_from_env({"AMD_GPU_DEVICE_COUNT": "x"}) is None
    assert device_count_limit_from_env({}) is None


def test_trace_spans(tmp_path):
    from rocm_k8s_device_plugin_amd.utils.trace import TRACER
    fi = make_mi355x_node(tmp_path / "n")
    impl = container(fi)
    TRACER.configure(str(tmp_path / "trace.json"))
    try:
        async def go():
            async with plugin_env(tmp_path, impl) as (k, mgr):
                await k.wait_for_resource("amd.com/gpu", 8)
                await k.admit("amd.com/gpu", 3)
        run(go())
        TRACER.flush()
        doc = json.loads((tmp_path / "trace.json").read_text())
        names = {e["name"] for e in doc["traceEvents"]}
        assert {"GetPreferredAllocation", "Allocate", "allocator.allocate"} <= names
    finally:
        TRACER.configure(None)


def test_liveness_persistent_server_reused(tmp_path):
    """Healthy sweeps go through ONE long-lived probe server, no per-device spawns."""
    log_path = tmp_path / "starts.log"
    ctl, prober = _stub_prober(tmp_path, {"3": "fail"})
    prober.extra_env["MI355X_STUB_PROBE_LOG"] = str(log_path)
    ords = {f"dev{i}": i for i in range(8)}

    async def go():
        for _ in range(3):
            res = await prober.probe(ords)
            assert {d for d, r in res.items() if not r.ok} == {"dev3"}
            assert "differ" in res["dev3"].reason and "(server: " in res["dev3"].reason
        assert prober.server_starts == 1 and prober.fallbacks == 0 and prober._server.requests == 3
        await prober.close()
        assert prober._server is None

    run(go())
    # each sweep's failure is confirmed by a fresh process for that device only
    assert log_path.read_text().split() == ["serve+keep", "3", "3", "3"]


def test_liveness_stale_server_failure_is_not_reported(tmp_path):
    """A device the server fails but a fresh process finds healthy is Healthy, and the server is restarted."""
    log_path = tmp_path / "starts.log"
    ctl, prober = _stub_prober(tmp_path, {"4": "server_fail"})
    prober.extra_env["MI355X_STUB_PROBE_LOG"] = str(log_path)
    ords = {f"dev{i}": i for i in range(8)}

    async def go():
        res = await prober.probe(ords)
        assert all(r.ok for r in res.values()), {d: r.reason for d, r in res.items() if not r.ok}
        assert prober.server_restarts == 1 and prober._server is None
        ctl.write_text("{}")                       # the fresh server is fine
        res = await prober.probe(ords)
        assert all(r.ok for r in res.values())
        assert prober.server_starts == 2 and prober.server_restarts == 1
        await prober.close()

    run(go())
    assert log_path.read_text().split() == ["serve+keep", "4", "serve+keep"]


def test_liveness_keep_queues_flag_reaches_server(tmp_path):
    """-liveness_keep_queues (default on) starts the server as `--serve --keep` (resources kept between sweeps)."""
    from rocm_k8s_device_plugin_amd.cli import device_plugin as cli
    assert cli.build_parser().parse_args([]).liveness_keep_queues is True
    assert cli.build_parser().parse_args(["-liveness_keep_queues=false"]).liveness_keep_queues is False
    log_path = tmp_path / "starts.log"
    ctl, prober = _stub_prober(tmp_path, {})
    prober.keep_queues = True
    prober.extra_env["MI355X_STUB_PROBE_LOG"] = str(log_path)

    async def go():
        for _ in range(2):
            res = await prober.probe({"dev0": 0, "dev1": 1})
            assert all(r.ok for r in res.values())
        await prober.close()

    run(go())
    assert log_path.read_text().split() == ["serve+keep"]


def test_liveness_server_failure_isolates_per_device(tmp_path):
    """A hanging server is killed and the sweep re-run one process per device."""
    log_path = tmp_path / "starts.log"
    ctl, prober = _stub_prober(tmp_path, {"5": "hang"}, timeout=1.0)
    prober.extra_env["MI355X_STUB_PROBE_LOG"] = str(log_path)
    ords = {f"dev{i}": i for i in range(8)}

    async def go():
        res = await prober.probe(ords)
        assert {d for d, r in res.items() if not r.ok} == {"dev5"}
        assert "deadline" in res["dev5"].reason
        assert prober.fallbacks == 1 and prober._server is None
        # backoff: the next sweeps stay in spawn mode, then the server is retried
        ctl.write_text("{}")
        for _ in range(LivenessProber.SERVER_BACKOFF_SWEEPS):
            assert all(r.ok for r in (await prober.probe(ords)).values())
            assert prober._server is None
        assert all(r.ok for r in (await prober.probe(ords)).values())
        assert prober._server is not None and prober.server_starts == 2
        await prober.close()

    run(go(), timeout=60)
    starts = log_path.read_text().split()
    assert starts[0] == "serve+keep" and sorted(starts[1:9]) == [str(i) for i in range(8)] and starts[-1] == "serve+keep"


def test_liveness_server_start_failure_falls_back(tmp_path):
    ctl, prober = _stub_prober(tmp_path, {"serve": "broken", "1": "stale"})
    ords = {f"dev{i}": i for i in range(4)}

    async def go():
        res = await prober.probe(ords)
        assert prober.fallbacks == 1
        assert {d for d, r in res.items() if not r.ok} == {"dev1"} and "stale" in res["dev1"].reason

    run(go())


def test_liveness_spawn_mode_never_starts_server(tmp_path):
    ctl = tmp_path / "probe_ctl.json"
    ctl.write_text("{}")
    prober = LivenessProber(exe=STUB, argv_prefix=[sys.executable], timeout_s=2.0, mode="spawn",
                            extra_env={"MI355X_STUB_PROBE_CONTROL": str(ctl)})

    async def go():
        assert all(r.ok for r in (await prober.probe({"a": 0, "b": 1})).values())
        assert prober.server_starts == 0

    run(go())
    with pytest.raises(ValueError):
        LivenessProber(mode="bogus")


class _FakeEvents:
    def __init__(self):
        self.queue, self.mask, self.running, self.stopped = [], None, False, False

    def start(self, mask):
        self.mask, self.running = mask, True
        return ""

    def poll(self, timeout_ms=0):
        out, self.queue = self.queue, []
        return out

    def stop(self):
        self.stopped, self.running = True, False


def test_smi_events_reset_window_marks_device_unhealthy(tmp_path):
    from rocm_k8s_device_plugin_amd.utils.metrics import REGISTRY
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ev = _FakeEvents()
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, smi_events=True), event_source=ev)
    victim = inv.by_id[fi.bdfs[3]]

    async def go():
        assert not await mon.check_once()
        assert ev.mask == (1 << 0) | (1 << 1) | (1 << 2) | (1 << 3) | (1 << 8)
        ev.queue = [{"bdf": victim.bdf, "type": 3, "name": "gpu_pre_reset", "message": "RAS"},
                    {"bdf": fi.bdfs[5], "type": 1, "name": "vmfault", "message": "pasid 7"}]
        assert await mon.check_once()
        snap = mon.snapshot()
        assert {d for d, v in snap.items() if v.health == "Unhealthy"} == {victim.id}
        assert "reset in progress" in snap[victim.id].reasons[0]
        assert not await mon.check_once()          # still resetting, nothing new
        ev.queue = [{"bdf": victim.bdf, "type": 4, "name": "gpu_post_reset", "message": ""}]
        assert await mon.check_once()
        assert all(v.health == "Healthy" for v in mon.snapshot().values())
        assert mon.event_counts[(fi.bdfs[5], "vmfault")] == 1
        await mon.close()
        assert ev.stopped

    run(go())
    assert 'mi355x_dp_gpu_events_total{bdf="%s",event="vmfault"}' % fi.bdfs[5] in REGISTRY.render()


def test_smi_events_unavailable_is_not_fatal(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, smi_events=True))   # real watcher, no GPU here

    async def go():
        await mon.check_once()
        await mon.check_once()
        assert all(v.health == "Healthy" for v in mon.snapshot().values())
        await mon.close()

    run(go())


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="CPU-only: exercises the failure path of the real probe")
def test_real_probe_binary_without_gpu_reports_unhealthy():
    """The real mi355x-liveness-probe (server and one-shot) on a machine without a
    GPU: the server refuses to start, the prober falls back per device, and the
    verdict carries the runtime error instead of hanging or crashing."""
    from rocm_k8s_device_plugin_amd.ops.native import probe_executable
    prober = LivenessProber(exe=str(probe_executable("hsa")), timeout_s=20)

    async def go():
        res = await prober.probe({"a": 0})
        assert not res["a"].ok and "runtime init failed" in res["a"].reason
        assert prober.fallbacks == 1 and prober._server is None

    run(go())


def test_chip_sweep_ignores_the_probe_servers_own_queues(tmp_path):
    """A kept-queue probe server has a queue on every GPU; those must not make the GPUs look busy."""
    from rocm_k8s_device_plugin_amd.topology import kfd_busy_gpu_ids
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    proc = fi.sysfs / "class/kfd/kfd/proc"
    gids = [inv.topology.node(d.node_id).gpu_id for d in inv.devices]
    busy_dev = inv.by_id[fi.bdfs[5]]
    q = proc / "777/queues/0"          # a pod's process on GPU 5
    q.mkdir(parents=True)
    (q / "gpuid").write_text(f"{gids[5]}\n")
    ctl, prober = _stub_prober(tmp_path, {})
    prober.kfd_proc_dir = str(proc)
    prober.extra_env.update({"MI355X_STUB_KFD_PROC": str(proc),
                             "MI355X_STUB_KFD_GPUIDS": ",".join(str(g) for g in gids)})
    kinds = []
    orig = prober.probe

    async def spy(ordinals, kind="probe", busy=()):
        kinds.append((kind, sorted(ordinals)))
        return await orig(ordinals, kind, busy)

    prober.probe = spy
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, chip_sweep_every=2), prober=prober,
                        ordinal_map={d.id: i for i, d in enumerate(inv.devices)})

    async def go():
        for _ in range(3):
            await mon.check_once()
        own = prober.own_kfd_entries
        assert own == {str(prober._server.proc.pid)}
        assert kfd_busy_gpu_ids(str(fi.sysfs)) == set(gids)                 # everyone, counting the server
        assert kfd_busy_gpu_ids(str(fi.sysfs), exclude=own) == {gids[5]}    # only the pod's GPU
        await mon.close()
        assert prober.own_kfd_entries == frozenset()

    run(go())
    everyone = sorted(d.id for d in inv.devices)
    idle = sorted(set(everyone) - {busy_dev.id})
    # pulse 2 runs while the server holds queues on all 8 GPUs: still swept as idle
    assert kinds == [("sweep", idle), ("probe", [busy_dev.id]), ("probe", everyone),
                     ("sweep", idle), ("probe", [busy_dev.id])]
    assert mon.chip_sweeps == 2


def test_chip_sweep_runs_on_idle_gpus_only(tmp_path):
    """Every N-th pulse, GPUs without user queues get the full-chip sweep; a GPU
    with another process' queues keeps the one-wave probe."""
    from rocm_k8s_device_plugin_amd.topology import kfd_busy_gpu_ids
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    busy_dev = inv.by_id[fi.bdfs[2]]
    busy_gid = inv.topology.node(busy_dev.node_id).gpu_id
    q = fi.sysfs / "class/kfd/kfd/proc/4242/queues/0"
    q.mkdir(parents=True)
    (q / "gpuid").write_text(f"{busy_gid}\n")
    assert kfd_busy_gpu_ids(str(fi.sysfs)) == {busy_gid}
    ctl, prober = _stub_prober(tmp_path, {})
    kinds = []
    orig = prober.probe

    async def spy(ordinals, kind="probe", busy=()):
        kinds.append((kind, sorted(ordinals)))
        return await orig(ordinals, kind, busy)

    prober.probe = spy
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, chip_sweep_every=2), prober=prober,
                        ordinal_map={d.id: i for i, d in enumerate(inv.devices)})

    async def go():
        for _ in range(3):
            await mon.check_once()
        assert all(v.health == "Healthy" for v in mon.snapshot().values())
        await mon.close()

    run(go())
    everyone = sorted(d.id for d in inv.devices)
    idle = sorted(set(everyone) - {busy_dev.id})
    assert kinds == [("sweep", idle), ("probe", [busy_dev.id]), ("probe", everyone),
                     ("sweep", idle), ("probe", [busy_dev.id])]
    assert mon.chip_sweeps == 2


def test_cli_dry_run_reports_node(tmp_path):
    """-dry_run: implementation, resources, devices and preferred allocations as JSON, no registration."""
    import subprocess
    fi = make_mi355x_node(tmp_path / "n", hive_size=4)
    env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    p = subprocess.run([sys.executable, "-m", "rocm_k8s_device_plugin_amd.cli.device_plugin", "-dry_run",
                        "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-exporter_socket", "",
                        "-kubelet_dir", str(tmp_path / "dp")], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    doc = json.loads(p.stdout)
    assert doc["implementation"] == "container" and list(doc["resources"]) == ["amd.com/gpu"]
    r = doc["resources"]["amd.com/gpu"]
    assert [d["id"] for d in r["devices"]] == fi.bdfs and r["preferred_allocation"]
    four = r["allocations"]["4"]
    assert four["one_hive"] and four["allreduce_bound_gbs"] > 0     # a whole hive of 4
    assert not r["allocations"]["8"]["one_hive"]                    # 8 spans both hives
    assert not os.path.exists(tmp_path / "dp" / "amd.com_gpu")      # nothing served


def test_chip_sweep_skipped_when_kfd_queues_unreadable(tmp_path, monkeypatch):
    """Without permission to read another process' kfd queues the plugin cannot
    tell idle GPUs from busy ones: no device is treated as idle."""
    from rocm_k8s_device_plugin_amd import topology as T
    fi = make_mi355x_node(tmp_path / "n")
    proc = fi.sysfs / "class/kfd/kfd/proc/4242/queues"
    proc.mkdir(parents=True)
    real_listdir = os.listdir

    def listdir(p):
        if str(p).endswith("4242/queues"):
            raise PermissionError(13, "Permission denied")
        return real_listdir(p)

    monkeypatch.setattr(T.os, "listdir", listdir)
    with pytest.raises(T.KfdBusyUnknown):
        T.kfd_busy_gpu_ids(str(fi.sysfs))
    inv = discover(str(fi.sysfs))
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None))
    assert mon._idle_devices([d.id for d in inv.devices]) == set()


def test_health_metrics_per_device(tmp_path):
    """After a sweep every device has a health gauge (and a probe latency with liveness)."""
    from rocm_k8s_device_plugin_amd.utils.metrics import REGISTRY
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ctl, prober = _stub_prober(tmp_path, {"2": "fail"})
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, fail_threshold=1), prober=prober,
                        ordinal_map={d.id: i for i, d in enumerate(inv.devices)})

    async def go():
        try:
            await mon.check_once()
        finally:
            await mon.close()

    run(go())
    text = REGISTRY.render()
    bad = inv.devices[2].id
    assert f'mi355x_dp_device_healthy{{device="{bad}"}} 0' in text
    assert f'mi355x_dp_device_healthy{{device="{inv.devices[0].id}"}} 1' in text
    assert f'mi355x_dp_liveness_probe_ms{{device="{bad}"}}' in text


def _busy_gpu(fi, inv, dev_id, pid="777"):
    """A foreign process with a queue on dev_id's GPU (kfd proc entry)."""
    node = inv.topology.node(inv.by_id[dev_id].node_id)
    q = fi.sysfs / "class/kfd/kfd/proc" / pid / "queues" / "0"
    q.mkdir(parents=True, exist_ok=True)
    (q / "gpuid").write_text(f"{node.gpu_id}\n")


@pytest.mark.parametrize("busy,grace,unhealthy_after", [(True, 300.0, None), (True, 0.0, 2), (False, 300.0, 2)])
def test_liveness_pending_behind_tenant(tmp_path, busy, grace, unhealthy_after):
    """A probe whose dispatch stays queued behind a tenant's kernel (measured on
    MI355X: 390 ms waits behind 441 ms GEMMs, profiles/archive/measurements_r1_r3.md) is
    inconclusive on a GPU that runs other processes' queues, for up to
    -liveness_busy_grace; on an idle GPU, or after the grace, it is a failure
    (confirmed in a fresh process first)."""
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    dev = inv.devices[3].id
    if busy:
        _busy_gpu(fi, inv, dev)
    log_path = tmp_path / "starts.log"
    ctl, prober = _stub_prober(tmp_path, {"3": "pending"})
    prober.extra_env["MI355X_STUB_PROBE_LOG"] = str(log_path)
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, fail_threshold=2,
                                          liveness_busy_grace_s=grace),
                        prober=prober, ordinal_map={d.id: i for i, d in enumerate(inv.devices)})

    async def go():
        healthy = []
        try:
            for _ in range(3):
                await mon.check_once()
                healthy.append(mon.health(dev) == "Healthy")
        finally:
            await mon.close()
        return healthy

    healthy = run(go())
    spawned = [x for x in log_path.read_text().split() if x == "3"]
    if unhealthy_after is None:
        assert healthy == [True, True, True]
        assert spawned == []                       # no fresh-process re-probe of a busy GPU
    else:
        assert healthy[:unhealthy_after - 1] == [True] * (unhealthy_after - 1) and not healthy[-1]
        if not busy:
            assert spawned                          # idle GPU: confirmed in a fresh process
    assert all(mon.health(d.id) == "Healthy" for d in inv.devices if d.id != dev)


def test_server_without_kept_queues_restarts_after_a_timeout(tmp_path):
    """Without kept queues the server cannot free a timed-out dispatch's queue
    (181 MB save area on MI355X): the prober restarts it to reclaim the memory."""
    ctl, prober = _stub_prober(tmp_path, {"1": "timeout"})
    prober.keep_queues = False
    ords = {f"dev{i}": i for i in range(4)}

    async def go():
        res = await prober.probe(ords)
        assert not res["dev1"].ok and all(res[f"dev{i}"].ok for i in (0, 2, 3))
        assert prober._server is None            # killed after the sweep
        ctl.write_text("{}")
        assert all(r.ok for r in (await prober.probe(ords)).values())
        assert prober.server_starts == 2
        await prober.close()

    run(go())


def test_server_kfd_entry_ambiguity_resolved_by_queue_coverage(tmp_path):
    """Another GPU process starting in the same instant as the probe server
    leaves two candidate kfd entries; the server's is the one with a queue on
    every probed GPU (a pod's process only queues on its own GPUs)."""
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    proc = fi.sysfs / "class/kfd/kfd/proc"
    gids = [inv.topology.node(d.node_id).gpu_id for d in inv.devices]

    def entry(pid, gpu_ids):
        for i, g in enumerate(gpu_ids):
            q = proc / pid / "queues" / str(i)
            q.mkdir(parents=True, exist_ok=True)
            (q / "gpuid").write_text(f"{g}\n")

    entry("1001", gids)            # the server: one kept queue per GPU
    entry("1002", gids[2:4])       # a pod that started at the same moment, 2 GPUs
    ctl, prober = _stub_prober(tmp_path, {})
    prober.kfd_proc_dir = str(proc)
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True), prober=prober,
                        ordinal_map={d.id: i for i, d in enumerate(inv.devices)})

    async def go():
        try:
            await prober.probe({"dev0": 0})          # server up
            prober._own_kfd = frozenset({"1001", "1002"})
            assert prober.own_kfd_entries == frozenset()          # ambiguous on its own
            assert mon._own_entries() == frozenset({"1001"})     # resolved by coverage
            # the pod's two GPUs are busy, the rest are idle
            busy = mon._busy_devices([d.id for d in inv.devices])
            assert busy == {inv.devices[2].id, inv.devices[3].id}
        finally:
            await prober.close()

    run(go())


def test_chip_sweep_leaves_a_pending_probe_slot_alone(tmp_path):
    """A probe left pending behind a tenant, then a chip sweep of that GPU (its
    own queue), then the next probe: the late verdict still carries the first
    probe's nonce and is accepted -- no stale-result failure, no fresh-process
    re-probe, no server restart."""
    log_path = tmp_path / "starts.log"
    ctl, prober = _stub_prober(tmp_path, {"3": "pending"})
    prober.extra_env["MI355X_STUB_PROBE_LOG"] = str(log_path)
    ords = {f"dev{i}": i for i in range(4)}

    async def go():
        try:
            r1 = await prober.probe(ords, busy={3})
            assert r1["dev3"].pending and not r1["dev3"].ok
            ctl.write_text("{}")                      # the tenant finished
            assert all(r.ok for r in (await prober.sweep(ords)).values())
            r3 = await prober.probe(ords)
            assert r3["dev3"].ok and r3["dev3"].detail.get("late") == 1, r3["dev3"]
            assert prober.server_restarts == 0 and prober.server_starts == 1
        finally:
            await prober.close()

    run(go())
    assert [x for x in log_path.read_text().split() if x == "3"] == []


def test_kfd_proc_list_unreadable_is_busy_unknown(tmp_path, monkeypatch):
    """An unreadable kfd process list itself (not just one process' queues)
    means busy state unknown, never 'every GPU idle'; a missing list is idle."""
    from rocm_k8s_device_plugin_amd import topology as T
    fi = make_mi355x_node(tmp_path / "n")
    root = fi.sysfs / "class/kfd/kfd/proc"
    root.mkdir(parents=True, exist_ok=True)
    real_listdir = os.listdir

    def listdir(p):
        if str(p).endswith("kfd/kfd/proc"):
            raise PermissionError(13, "Permission denied")
        return real_listdir(p)

    monkeypatch.setattr(T.os, "listdir", listdir)
    with pytest.raises(T.KfdBusyUnknown):
        T.kfd_busy_gpu_ids(str(fi.sysfs))
    monkeypatch.setattr(T.os, "listdir", real_listdir)
    assert T.kfd_busy_gpu_ids(str(tmp_path / "nothing")) == set()


def test_busy_unknown_uses_the_short_grace(tmp_path, monkeypatch):
    """When busy GPUs cannot be identified every GPU counts as busy (no chip
    sweep), but a pending probe only gets -liveness_unknown_busy_grace, not
    the full busy grace: a GPU wedged while idle is still reported."""
    from rocm_k8s_device_plugin_amd.health import monitor as M
    from rocm_k8s_device_plugin_amd.utils.metrics import REGISTRY
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    dev = inv.devices[3].id

    def unknown(*a, **k):
        raise M.KfdBusyUnknown("proc: Permission denied")

    monkeypatch.setattr(M, "kfd_busy_gpu_ids", unknown)
    ctl, prober = _stub_prober(tmp_path, {"3": "pending"})
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, fail_threshold=2,
                                          liveness_busy_grace_s=300.0, liveness_unknown_busy_grace_s=0.0),
                        prober=prober, ordinal_map={d.id: i for i, d in enumerate(inv.devices)})

    async def go():
        try:
            for _ in range(2):
                await mon.check_once()
        finally:
            await mon.close()

    run(go())
    assert not mon.busy_state_known
    assert mon.health(dev) == "Unhealthy"
    assert all(mon.health(d.id) == "Healthy" for d in inv.devices if d.id != dev)
    assert "mi355x_dp_busy_state_known 0" in REGISTRY.render()


def test_spawn_mode_deadline_on_busy_gpu_is_inconclusive(tmp_path):
    """Without kept queues (spawn mode) a deadline miss on a GPU that runs a
    tenant's kernels is inconclusive under the busy grace, like a pending
    kept-queue probe; on an idle GPU it is a failure."""
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    busy_dev, idle_dev = inv.devices[3].id, inv.devices[5].id
    _busy_gpu(fi, inv, busy_dev)
    ctl = tmp_path / "probe_ctl.json"
    ctl.write_text(json.dumps({"3": "hang", "5": "hang"}))
    prober = LivenessProber(exe=STUB, argv_prefix=[sys.executable], timeout_s=1.0, mode="spawn",
                            extra_env={"MI355X_STUB_PROBE_CONTROL": str(ctl)},
                            kfd_proc_dir=str(fi.sysfs / "class/kfd/kfd/proc"))
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, fail_threshold=1,
                                          liveness_mode="spawn"),
                        prober=prober, ordinal_map={d.id: i for i, d in enumerate(inv.devices)})

    async def go():
        try:
            await mon.check_once()
        finally:
            await mon.close()

    run(go(), timeout=60)
    assert mon.health(busy_dev) == "Healthy"
    assert mon.health(idle_dev) == "Unhealthy"


def _bus_id(d):
    loc = d.location_id
    return f"{d.domain:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"


@pytest.mark.parametrize("mode", ["single", "cpx"])
def test_probe_identity_rekeys_verdicts(tmp_path, mode):
    """The positional ordinal map is wrong (ROCr enumerated the agents in
    another order): every reply names its agent (kfd node, location_id with
    the partition index in the function bits), so the failing agent's verdict
    lands on its own kubelet ID and the ordinal map is rebuilt from the replies."""
    fi = make_mi355x_node(tmp_path / "n", **({"compute_partition": "CPX"} if mode == "cpx" else {}))
    inv = discover(str(fi.sysfs))
    n = len(inv.devices)
    truth = {d.id: i for i, d in enumerate(inv.devices)}               # what ROCr really enumerates
    wrong = {d.id: n - 1 - i for i, d in enumerate(inv.devices)}        # what the plugin assumed
    ident = {str(i): {"kfd_node_id": d.node_id, "pci_bus_id": _bus_id(d)} for i, d in enumerate(inv.devices)}
    ctl, prober = _stub_prober(tmp_path, {"3": "fail"})
    prober.extra_env["MI355X_STUB_PROBE_IDENTITY"] = json.dumps(ident)
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, fail_threshold=1),
                        prober=prober, ordinal_map=wrong)

    async def go():
        try:
            await mon.check_once()
            await mon.check_once()
        finally:
            await mon.close()

    run(go(), timeout=60)
    bad = inv.devices[3].id
    assert mon.health(bad) == "Unhealthy"
    assert all(mon.health(d.id) == "Healthy" for d in inv.devices if d.id != bad)
    assert mon.ordinals() == truth
    assert mon.identity_remaps == 1                   # second sweep already used the rebuilt map


def test_probe_identity_unmatched_device_loses_its_ordinal(tmp_path):
    """A reply from an agent no advertised device corresponds to: the device
    the verdict was meant for is reported without a HIP device, not Healthy."""
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ident = {str(i): {"kfd_node_id": d.node_id, "pci_bus_id": _bus_id(d)} for i, d in enumerate(inv.devices)}
    ident["5"] = {"kfd_node_id": 999, "pci_bus_id": "0000:ff:00.0"}
    ctl, prober = _stub_prober(tmp_path, {})
    prober.extra_env["MI355X_STUB_PROBE_IDENTITY"] = json.dumps(ident)
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True),
                        prober=prober, ordinal_map={d.id: i for i, d in enumerate(inv.devices)})

    async def go():
        try:
            await mon.check_once()
        finally:
            await mon.close()

    run(go(), timeout=60)
    victim = inv.devices[5].id
    assert mon.health(victim) == "Unhealthy"
    assert any("no HIP device" in r for r in mon.snapshot()[victim].reasons)
    assert sum(mon.health(d.id) == "Healthy" for d in inv.devices) == len(inv.devices) - 1


@pytest.mark.parametrize("activity,unhealthy", [(0, True), (87, False), (None, False)])
def test_busy_grace_needs_gfx_activity(tmp_path, activity, unhealthy):
    """A pending probe on a GPU that runs another process's queues is
    inconclusive only while the GPU is executing: amd-smi reporting 0% GFX
    activity on consecutive sweeps (a wedged queue, not a long tenant kernel)
    ends the 300 s grace; with activity, or without amd-smi, the grace holds."""
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    dev = inv.devices[3]
    _busy_gpu(fi, inv, dev.id)
    ctl, prober = _stub_prober(tmp_path, {"3": "pending"})
    src = (lambda: {}) if activity is None else (lambda: {d.bdf: (activity if d.id == dev.id else 50)
                                                          for d in inv.devices})
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, fail_threshold=2,
                                          liveness_busy_grace_s=300.0), prober=prober,
                        ordinal_map={d.id: i for i, d in enumerate(inv.devices)}, activity_source=src)

    async def go():
        try:
            for _ in range(4):
                await mon.check_once()
        finally:
            await mon.close()

    run(go())
    assert (mon.health(dev.id) == "Unhealthy") == unhealthy
    if unhealthy:
        assert any("0% GFX activity" in r for r in mon.snapshot()[dev.id].reasons)
    assert all(mon.health(d.id) == "Healthy" for d in inv.devices if d.id != dev.id)


def test_crowded_gpu_gets_no_probe_server_queue(tmp_path):
    """7 other processes with queues on one GPU (an oversubscribed HWS
    runlist): the probe server is restarted without that GPU (ROCr never opens
    it: no queue, no runlist slot) and its probe is skipped while the GPU is
    computing; at 0% GFX activity it is probed from a fresh process instead.
    Uncrowded again, the GPU returns to the server after the release window."""
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    dev = inv.devices[3]
    for pid in range(800, 807):
        _busy_gpu(fi, inv, dev.id, pid=str(pid))
    log_path = tmp_path / "starts.log"
    ctl, prober = _stub_prober(tmp_path, {"3": "fail"})
    prober.extra_env["MI355X_STUB_PROBE_LOG"] = str(log_path)
    prober.kfd_proc_dir = str(fi.sysfs / "class/kfd/kfd/proc")
    activity = {"v": 60}
    mon = HealthMonitor(inv, HealthConfig(exporter_socket=None, liveness=True, fail_threshold=2,
                                          liveness_crowded_release_sweeps=2), prober=prober,
                        ordinal_map={d.id: i for i, d in enumerate(inv.devices)},
                        activity_source=lambda: {d.bdf: (activity["v"] if d.id == dev.id else 40)
                                                 for d in inv.devices})

    async def go():
        try:
            for _ in range(3):
                await mon.check_once()
            assert mon.health(dev.id) == "Healthy" and mon.crowded_skips == 3
            assert prober._server_visible == (0, 1, 2, 4, 5, 6, 7)
            activity["v"] = 0                     # crowded but idle: a fresh process probes it
            for _ in range(2):
                await mon.check_once()
            assert mon.health(dev.id) == "Unhealthy"
            ctl.write_text("{}")
            import shutil
            for pid in range(800, 807):
                shutil.rmtree(fi.sysfs / "class/kfd/kfd/proc" / str(pid))
            for _ in range(4):
                await mon.check_once()
            assert prober._server_visible is None and mon.health(dev.id) == "Healthy"
        finally:
            await mon.close()

    run(go(), timeout=120)
    log = log_path.read_text().split()
    assert "visible=0,1,2,4,5,6,7" in log
    assert log.count("3") >= 2                   # the fresh-process probes of the idle crowded GPU
    assert all(mon.health(d.id) == "Healthy" for d in inv.devices if d.id != dev.id)


def test_kubelet_restart_seen_by_inotify_not_the_poll(tmp_path):
    """With a 30 s poll interval, a kubelet restart still re-registers within
    a second: the manager waits on an inotify watch of the plugin directory
    (the reference's dpm uses fsnotify)."""
    import time as _t
    fi = make_mi355x_node(tmp_path / "n")
    impl = container(fi)

    async def go():
        async with plugin_env(tmp_path, impl, watch_interval_s=30.0) as (k, mgr):
            await k.wait_for_resource("amd.com/gpu", 8)
            t0 = _t.monotonic()
            await k.restart()
            await k.wait_for_resource("amd.com/gpu", 8, timeout=10)
            return _t.monotonic() - t0, len(k.registrations)

    dt, regs = run(go())
    assert regs == 2 and dt < 1.5, dt


def test_histograms_keep_a_bounded_window():
    """A long-running daemon keeps bucket totals for every observation but only a
    recent window of raw samples (found by the 15-minute MI355X soak)."""
    from rocm_k8s_device_plugin_amd.utils.metrics import Histogram
    h = Histogram("x", "")
    for i in range(20000):
        h.observe(float(i))
    assert h.n == 20000 and sum(h.counts) == 20000 and len(h.samples) == 4096
    assert h.quantile(0.0) == 20000 - 4096
