"""The native health engine (native/src/health/health_engine.cpp) — what the
interpreter-free daemon `mi355x-device-plugin` runs each pulse — under the
same stub-probe fault injection as the Python monitor's tests
(tests/test_plugin.py): hysteresis, deadlines, stale nonces, garbage output,
persistent server reuse and restart, server start failure, spawn mode, busy
grace with amd-smi corroboration, crowded step-off, probe identity re-keying.
Then end to end through the daemon: verdicts reach kubelet's ListAndWatch,
a hung metrics exporter blocks neither re-registration nor shutdown, and the
transport watchdog exits when kubelet never lists.

Reference behaviour replaced: internal/pkg/amdgpu/amdgpu.go:322-345,865-974
(node-global kfd verdict + exporter per BDF)."""
import asyncio
import json
import os
import shutil
import signal
import subprocess
import sys
import time

import pytest

from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR, core
from rocm_k8s_device_plugin_amd.testing import gopeer as gp
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.topology import discover

STUB = os.path.join(os.path.dirname(__file__), "..", "rocm_k8s_device_plugin_amd", "testing", "stub_probe.py")
EXE = os.environ.get("MI355X_NATIVE_DAEMON_EXE") or os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)


def _busy_gpu(fi, inv, dev_id, pid="777"):
    """A foreign process with a queue on dev_id's GPU (kfd proc entry)."""
    node = inv.topology.node(inv.by_id[dev_id].node_id)
    q = fi.sysfs / "class/kfd/kfd/proc" / pid / "queues" / "0"
    q.mkdir(parents=True, exist_ok=True)
    (q / "gpuid").write_text(f"{node.gpu_id}\n")


def _engine(fi, tmp_path, control, timeout=2.0, env=None, **opts):
    ctl = tmp_path / "probe_ctl.json"
    ctl.write_text(json.dumps(control))
    extra = {"MI355X_STUB_PROBE_CONTROL": str(ctl), **(env or {})}
    o = dict(dev_root=str(fi.dev), liveness=True, probe_exe=STUB, argv_prefix=[sys.executable],
             probe_timeout_s=timeout, extra_env=extra, fail_threshold=2)
    o.update(opts)
    return ctl, core().HealthEngine(str(fi.sysfs), o)


def _by_ordinal(eng):
    return {o: d for d, o in eng.ordinals().items()}


def _unhealthy(eng):
    return {d for d, (ok, _) in eng.snapshot().items() if not ok}


def test_fault_injection_hysteresis(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    ctl, eng = _engine(fi, tmp_path, {"2": "fail", "5": "hang", "6": "stale", "7": "garbage"}, timeout=1.5)
    dev = _by_ordinal(eng)
    assert sorted(dev) == list(range(8))
    try:
        assert not eng.sweep() and not _unhealthy(eng)         # 1st failure: below the threshold
        assert eng.sweep()                                      # 2nd consecutive failure
        snap = eng.snapshot()
        assert _unhealthy(eng) == {dev[2], dev[5], dev[6], dev[7]}
        assert "differ" in snap[dev[2]][1][0]
        assert "deadline" in snap[dev[5]][1][0]
        assert "stale" in snap[dev[6]][1][0]
        assert "unparseable" in snap[dev[7]][1][0]
        assert eng.stats()["fallbacks"] >= 1                   # the hung server was isolated per device
        ctl.write_text("{}")                                    # everything recovers
        assert eng.sweep() and not _unhealthy(eng)
    finally:
        eng.close()


def test_persistent_server_reused_and_failures_confirmed_fresh(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    log = tmp_path / "starts.log"
    ctl, eng = _engine(fi, tmp_path, {"3": "fail"}, env={"MI355X_STUB_PROBE_LOG": str(log)})
    try:
        for _ in range(3):
            eng.sweep()
        assert _unhealthy(eng) == {_by_ordinal(eng)[3]}
        st = eng.stats()
        assert st["server_starts"] == 1 and st["server_running"]
        lines = log.read_text().split()
        assert lines.count("serve+keep") == 1 and lines.count("3") == 3   # one fresh confirmation per sweep
    finally:
        eng.close()
    assert not eng.stats()["server_running"]


def test_stale_server_failure_is_not_reported(tmp_path):
    """The server fails a device a fresh process finds healthy (stale runtime):
    the device stays Healthy and the server is restarted."""
    fi = make_mi355x_node(tmp_path / "n")
    ctl, eng = _engine(fi, tmp_path, {"4": "server_fail"})
    try:
        for _ in range(3):
            eng.sweep()
        assert not _unhealthy(eng)
        st = eng.stats()
        assert st["server_restarts"] >= 2 and st["server_starts"] >= 3
    finally:
        eng.close()


def test_server_without_kept_queues_and_spawn_mode(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    log = tmp_path / "starts.log"
    ctl, eng = _engine(fi, tmp_path, {}, env={"MI355X_STUB_PROBE_LOG": str(log)}, keep_queues=False)
    try:
        eng.sweep()
        assert "serve" in log.read_text().split() and "serve+keep" not in log.read_text().split()
    finally:
        eng.close()
    log.write_text("")
    ctl, eng = _engine(fi, tmp_path, {"1": "fail"}, env={"MI355X_STUB_PROBE_LOG": str(log)}, persistent=False,
                       fail_threshold=1)
    try:
        eng.sweep()
        assert _unhealthy(eng) == {_by_ordinal(eng)[1]}
        assert not any(x.startswith("serve") for x in log.read_text().split())
        assert sorted(log.read_text().split()) == [str(i) for i in range(8)]
    finally:
        eng.close()


def test_server_start_failure_falls_back_per_device(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    ctl, eng = _engine(fi, tmp_path, {"serve": "broken", "1": "stale"})
    try:
        eng.sweep()
        eng.sweep()
        assert _unhealthy(eng) == {_by_ordinal(eng)[1]}
        assert eng.stats()["fallbacks"] >= 1
    finally:
        eng.close()


@pytest.mark.parametrize("busy,grace,unhealthy_after", [(True, 300.0, None), (True, 0.0, 2), (False, 300.0, 2)])
def test_pending_behind_tenant(tmp_path, busy, grace, unhealthy_after):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    log = tmp_path / "starts.log"
    ctl, eng = _engine(fi, tmp_path, {"3": "pending"}, env={"MI355X_STUB_PROBE_LOG": str(log)}, busy_grace_s=grace)
    dev = _by_ordinal(eng)[3]
    if busy:
        _busy_gpu(fi, inv, dev)
    eng.set_activity({})   # amd-smi unavailable: no corroboration, the grace decides
    healthy = []
    try:
        for _ in range(3):
            eng.sweep()
            healthy.append(dev not in _unhealthy(eng))
    finally:
        eng.close()
    spawned = [x for x in log.read_text().split() if x == "3"]
    if unhealthy_after is None:
        assert healthy == [True, True, True] and spawned == []   # no fresh-process re-probe of a busy GPU
    else:
        assert healthy[:unhealthy_after - 1] == [True] * (unhealthy_after - 1) and not healthy[-1]
        if not busy:
            assert spawned
    assert _unhealthy(eng) <= {dev}


@pytest.mark.parametrize("activity,unhealthy", [(0, True), (87, False), (None, False)])
def test_busy_grace_needs_gfx_activity(tmp_path, activity, unhealthy):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ctl, eng = _engine(fi, tmp_path, {"3": "pending"}, busy_grace_s=300.0)
    dev = _by_ordinal(eng)[3]
    _busy_gpu(fi, inv, dev)
    eng.set_activity({} if activity is None else {d.bdf: (activity if d.id == dev else 50) for d in inv.devices})
    try:
        for _ in range(4):
            eng.sweep()
    finally:
        eng.close()
    assert (dev in _unhealthy(eng)) == unhealthy
    if unhealthy:
        assert any("0% GFX activity" in r for r in eng.snapshot()[dev][1])
    assert _unhealthy(eng) <= {dev}


def test_kfd_proc_list_unreadable_means_busy_unknown(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    proc = fi.sysfs / "class/kfd/kfd/proc"
    (proc / "999" / "queues").mkdir(parents=True)
    ctl, eng = _engine(fi, tmp_path, {"3": "pending"}, busy_grace_s=300.0, unknown_busy_grace_s=0.0)
    eng.set_activity({})
    os.chmod(proc / "999" / "queues", 0)
    try:
        if os.access(proc / "999" / "queues", os.R_OK):
            pytest.skip("running as root: permissions are not enforced")
        for _ in range(2):
            eng.sweep()
        assert not eng.stats()["busy_state_known"]
        assert _unhealthy(eng) == {_by_ordinal(eng)[3]}      # the short grace (0 s) applied
    finally:
        os.chmod(proc / "999" / "queues", 0o755)
        eng.close()


def test_crowded_gpu_gets_no_probe_server_queue(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    log = tmp_path / "starts.log"
    ctl, eng = _engine(fi, tmp_path, {"3": "fail"}, env={"MI355X_STUB_PROBE_LOG": str(log)},
                       crowded_release_sweeps=2)
    dev = _by_ordinal(eng)[3]
    for pid in range(800, 807):
        _busy_gpu(fi, inv, dev, pid=str(pid))
    act = {d.bdf: (60 if d.id == dev else 40) for d in inv.devices}
    eng.set_activity(act)
    try:
        for _ in range(3):
            eng.sweep()
        assert dev not in _unhealthy(eng) and eng.stats()["crowded_skips"] == 3
        act[inv.by_id[dev].bdf] = 0          # crowded but idle: a fresh process probes it
        eng.set_activity(act)
        for _ in range(2):
            eng.sweep()
        assert dev in _unhealthy(eng)
        ctl.write_text("{}")
        for pid in range(800, 807):
            shutil.rmtree(fi.sysfs / "class/kfd/kfd/proc" / str(pid))
        for _ in range(4):
            eng.sweep()
        assert not _unhealthy(eng)
    finally:
        eng.close()
    words = log.read_text().split()
    assert "visible=0,1,2,4,5,6,7" in words and words.count("3") >= 2


def test_own_kfd_entry_told_apart_from_a_pod_started_with_the_server(tmp_path):
    """A pod's GPU process that appears in the same instant as the probe server
    leaves two new kfd entries; the server's own is the one with a queue on
    every probed GPU. Only the pod's GPUs then count as busy: a pending probe
    there waits out the busy grace, one on an idle GPU is a fault."""
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    proc = fi.sysfs / "class/kfd/kfd/proc"
    proc.mkdir(parents=True, exist_ok=True)
    gid = lambda d: inv.topology.node(inv.by_id[d].node_id).gpu_id   # noqa: E731
    everyone = ",".join(str(gid(d.id)) for d in inv.devices)
    ctl, eng = _engine(fi, tmp_path, {}, busy_grace_s=300.0, unknown_busy_grace_s=300.0, keep_queues=True,
                       env={"MI355X_STUB_KFD_PROC": str(proc), "MI355X_STUB_KFD_GPUIDS": everyone})
    by_ord = _by_ordinal(eng)
    pod = [by_ord[2], by_ord[3]]
    eng.close()
    ctl, eng = _engine(fi, tmp_path, {"2": "pending", "5": "pending"}, busy_grace_s=300.0,
                       unknown_busy_grace_s=300.0, keep_queues=True,
                       env={"MI355X_STUB_KFD_PROC": str(proc), "MI355X_STUB_KFD_GPUIDS": everyone,
                            "MI355X_STUB_KFD_ALSO": "424242:" + ",".join(str(gid(d)) for d in pod)})
    eng.set_activity({})
    try:
        for _ in range(3):
            eng.sweep()
        assert eng.stats()["busy_state_known"]              # the server's entry was resolved
        assert _unhealthy(eng) == {by_ord[5]}                # idle GPU: pending is a fault
    finally:
        eng.close()


def _bus_id(d):
    loc = d.location_id
    return f"{d.domain:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"


@pytest.mark.parametrize("mode", ["single", "cpx"])
def test_probe_identity_rekeys_verdicts(tmp_path, mode):
    """ROCr enumerated the agents in another order than the positional map
    assumes: every reply names its agent, so the failing agent's verdict lands
    on its own kubelet ID and the ordinal map is rebuilt from the replies."""
    fi = make_mi355x_node(tmp_path / "n", **({"compute_partition": "CPX"} if mode == "cpx" else {}))
    inv = discover(str(fi.sysfs))
    probe_env = {}
    ctl, eng = _engine(fi, tmp_path, {"3": "fail"}, fail_threshold=1)
    pos = eng.ordinals()
    n = len(pos)
    order = sorted(pos, key=pos.get)
    # the agent at ordinal i is really device order[n-1-i]
    ident = {str(i): {"kfd_node_id": inv.by_id[order[n - 1 - i]].node_id,
                      "pci_bus_id": _bus_id(inv.by_id[order[n - 1 - i]])} for i in range(n)}
    eng.close()
    probe_env["MI355X_STUB_PROBE_IDENTITY"] = json.dumps(ident)
    ctl, eng = _engine(fi, tmp_path, {"3": "fail"}, env=probe_env, fail_threshold=1)
    try:
        eng.sweep()
        eng.sweep()
        assert _unhealthy(eng) == {order[n - 1 - 3]}
        assert eng.ordinals() == {order[n - 1 - i]: i for i in range(n)}
        assert eng.stats()["identity_remaps"] == 1        # the second sweep already used the rebuilt map
    finally:
        eng.close()


def test_probe_identity_unmatched_device_loses_its_ordinal(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ctl, eng = _engine(fi, tmp_path, {})
    pos = eng.ordinals()
    eng.close()
    ident = {str(o): {"kfd_node_id": inv.by_id[d].node_id, "pci_bus_id": _bus_id(inv.by_id[d])} for d, o in pos.items()}
    ident["5"] = {"kfd_node_id": 999, "pci_bus_id": "0000:ff:00.0"}
    ctl, eng = _engine(fi, tmp_path, {}, env={"MI355X_STUB_PROBE_IDENTITY": json.dumps(ident)})
    try:
        eng.sweep()
    finally:
        eng.close()
    victim = {o: d for d, o in pos.items()}[5]
    assert _unhealthy(eng) == {victim}
    assert any("no HIP device" in r for r in eng.snapshot()[victim][1])


def test_kfd_node_loss_and_exporter_reach_partitions(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", compute_partition="CPX")
    inv = discover(str(fi.sysfs))
    eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
    victim = inv.devices[1]
    bdf = inv.devices[9].bdf
    eng.set_exporter({bdf: False})
    try:
        (fi.sysfs / "class/kfd/kfd/topology/nodes" / str(victim.node_id) / "properties").unlink()
        assert eng.sweep()
        bad = _unhealthy(eng)
        assert victim.id in bad and "missing" in eng.snapshot()[victim.id][1][0]
        # the exporter's BDF verdict lands on every partition of that GPU (reference: BDF only)
        assert {d.id for d in inv.devices if d.bdf == bdf} <= bad
    finally:
        eng.close()


def test_exporter_list_through_a_grpc_go_exporter(tmp_path):
    """metricssvc.MetricsService/List against a grpc-go-shaped exporter."""
    from rocm_k8s_device_plugin_amd.proto import metricssvc as ms
    resp = ms.GPUStateResponse()
    resp.GPUState.add(ID="0", Health="healthy", Device="0000:05:00.0")
    resp.GPUState.add(ID="1", Health="UNHEALTHY", Device="0000:15:00.0")
    path = str(tmp_path / "exp.sock")
    with gp.GoServer(path, {"/metricssvc.MetricsService/List": lambda m: (0, "", resp.SerializeToString())},
                     gp.GoServerConfig(continuation_chunk=4)):
        h, err = core().exporter_list(path, 5.0)
    assert err == "" and h == {"0000:05:00.0": True, "0000:15:00.0": False}
    # no verdict from an exporter that answers nonsense or an error, or is not there
    for answer, want in (((0, "", b"\x0a\x05ab"), "malformed GPUStateResponse from the metrics exporter"),
                         ((14, "exporter restarting", b""), "exporter restarting")):
        with gp.GoServer(path, {"/metricssvc.MetricsService/List": lambda m, a=answer: a}):
            h, err = core().exporter_list(path, 5.0)
        assert h == {} and err == want
    assert core().exporter_list(str(tmp_path / "absent.sock"), 5.0) == ({}, "")


# ------------------------------------------------------------------ the daemon end to end

def _daemon(kdir, fi, *extra, env=None):
    return subprocess.Popen([EXE, "-kubelet_dir", kdir, "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                             *extra], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                            env=dict(os.environ, **(env or {})))


def _stop(p, timeout=20):
    if p.poll() is None:
        p.send_signal(signal.SIGTERM)
    try:
        _, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        _, err = p.communicate()
        return None, err
    return p.returncode, err


def test_daemon_liveness_verdicts_reach_listandwatch(tmp_path):
    """-liveness with the stub probe: the first list already carries the
    failing device, a later fault arrives as an update, recovery too."""
    fi = make_mi355x_node(tmp_path / "n")
    ctl = tmp_path / "ctl.json"
    ctl.write_text(json.dumps({"3": "fail"}))
    log = tmp_path / "starts.log"
    kdir = str(tmp_path / "dp")
    eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
    dev = {o: d for d, o in eng.ordinals().items()}
    eng.close()

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = _daemon(kdir, fi, "-pulse", "1", "-liveness", "-liveness_probe", STUB, "-liveness_fail_threshold", "1",
                    "-liveness_timeout", "3", "-exporter_socket", "",
                    env={"MI355X_STUB_PROBE_CONTROL": str(ctl), "MI355X_STUB_PROBE_LOG": str(log)})
        try:
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            assert {d for d, h in st.devices.items() if h == "Unhealthy"} == {dev[3]}   # before any pulse
            u = st.updates
            ctl.write_text(json.dumps({"5": "fail"}))
            st = await k.wait_for_update("amd.com/gpu", u, timeout=20)
            assert {d for d, h in st.devices.items() if h == "Unhealthy"} == {dev[5]}
            ctl.write_text("{}")
            st = await k.wait_for_update("amd.com/gpu", st.updates, timeout=20)
            assert all(h == "Healthy" for h in st.devices.values())
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        assert "liveness probe: " in err and "device " + dev[3] in err
        # one persistent kept-queue server for the daemon's lifetime, killed at shutdown
        assert log.read_text().split().count("serve+keep") == 1

    asyncio.run(asyncio.wait_for(go(), 90))


def test_prestart_liveness_gate(tmp_path):
    """-prestart_liveness: the options ask kubelet for PreStartContainer, which
    probes the container's GPUs through the probe server right before the start
    and fails it (FAILED_PRECONDITION, naming the device) on a definite fault.
    The check runs off the RPC thread: a slow one holds back no other call."""
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    from rocm_k8s_device_plugin_amd.testing.fake_kubelet import NativeRpcError
    fi = make_mi355x_node(tmp_path / "n")
    ctl = tmp_path / "ctl.json"
    ctl.write_text("{}")
    kdir = str(tmp_path / "dp")
    eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
    dev = {o: d for d, o in eng.ordinals().items()}
    eng.close()
    bad = subprocess.run([EXE, "-dry_run", "-sysfs_root", str(fi.sysfs), "-prestart_liveness"],
                         capture_output=True, text=True, timeout=30)
    assert bad.returncode == 1 and "prestart_liveness needs -liveness" in bad.stderr

    async def go():
        k = FakeKubelet(kdir, rpc_client="native")
        await k.start()
        p = _daemon(kdir, fi, "-pulse", "3600", "-liveness", "-liveness_probe", STUB, "-prestart_liveness",
                    "-liveness_timeout", "5", "-exporter_socket", "", env={"MI355X_STUB_PROBE_CONTROL": str(ctl)})
        try:
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            assert st.options.pre_start_required and st.options.get_preferred_allocation_available
            adm = await k.admit("amd.com/gpu", 2)          # kubelet's sequence, the check included
            assert adm.prestart_ms > 0 and len(adm.device_ids) == 2
            k.release("amd.com/gpu", adm.device_ids)

            async def prestart(ids):
                return await k._call(st, "PreStartContainer", pb.PreStartContainerRequest(devices_ids=ids),
                                     pb.PreStartContainerResponse, timeout=30.0)
            ctl.write_text(json.dumps({"3": "fail"}))         # the GPU broke after the last sweep
            with pytest.raises(NativeRpcError) as e:
                await prestart([dev[2], dev[3]])
            assert e.value.status == 9 and dev[3] in e.value.message and dev[2] not in e.value.message
            assert "MFMA liveness check failed" in e.value.message
            await prestart([dev[2]])
            # a slow check (1.5 s) on one connection; Allocate on another is answered meanwhile
            ctl.write_text(json.dumps({"4": "slow", "slow_s": 1.5}))
            slow = asyncio.create_task(asyncio.to_thread(
                lambda: _unary_fresh(kdir, "PreStartContainer", pb.PreStartContainerRequest(devices_ids=[dev[4]]))))
            await asyncio.sleep(0.3)
            t0 = time.monotonic()
            areq = pb.AllocateRequest()
            areq.container_requests.add(devices_ids=[dev[6]])
            await asyncio.to_thread(lambda: _unary_fresh(kdir, "Allocate", areq))
            assert time.monotonic() - t0 < 1.0
            status, msg, took = await slow
            assert status == 0 and took >= 1.2, (status, msg, took)
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        assert "PreStartContainer: MFMA liveness check failed (" + dev[3] in err

    asyncio.run(asyncio.wait_for(go(), 90))


def test_prestart_gate_on_cpx_partitions(tmp_path):
    """CPX: each partition is its own ROCr agent. A container given three
    partitions of one GPU is checked on exactly those three agents; a fault on
    one of them names that partition only."""
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    fi = make_mi355x_node(tmp_path / "n", compute_partition="cpx")
    ctl = tmp_path / "ctl.json"
    ctl.write_text("{}")
    log = tmp_path / "starts.log"
    kdir = str(tmp_path / "dp")
    os.makedirs(kdir)
    eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
    ords = eng.ordinals()
    eng.close()
    inv = discover(str(fi.sysfs))
    gpu0 = sorted((d for d in inv.devices if d.bdf == fi.bdfs[0]), key=lambda d: ords[d.id])
    picked = [d.id for d in gpu0[:3]]
    kub = gp.GoServer(os.path.join(kdir, "kubelet.sock"), {"/v1beta1.Registration/Register": lambda m: (0, "", b"")})
    p = _daemon(kdir, fi, "-pulse", "3600", "-liveness", "-liveness_probe", STUB, "-prestart_liveness",
                "-liveness_timeout", "5", "-exporter_socket", "", "-grpc_watchdog", "0",
                env={"MI355X_STUB_PROBE_CONTROL": str(ctl)})
    try:
        deadline = time.monotonic() + 30
        while not os.path.exists(os.path.join(kdir, "amd.com_gpu")) and time.monotonic() < deadline:
            time.sleep(0.05)
        time.sleep(0.3)
        req = pb.PreStartContainerRequest(devices_ids=picked)
        assert _unary_fresh(kdir, "PreStartContainer", req)[0] == 0
        ctl.write_text(json.dumps({str(ords[picked[1]]): "fail"}))
        status, msg, _ = _unary_fresh(kdir, "PreStartContainer", req)
        assert status == 9 and picked[1] in msg and picked[0] not in msg and picked[2] not in msg, msg
        # a container on other partitions of the same GPU is not held back
        other = pb.PreStartContainerRequest(devices_ids=[d.id for d in gpu0[3:5]])
        assert _unary_fresh(kdir, "PreStartContainer", other)[0] == 0
    finally:
        rc, err = _stop(p)
        kub.close()
    assert rc == 0, err[-2000:]


def test_prestart_gate_pending_behind_a_tenant_is_no_fault(tmp_path):
    """A dispatch still queued behind another process' kernels (its queues are on
    that GPU) is pending: the start goes ahead at once, with no fresh probe
    process the container would then wait for. On an idle GPU the same silence
    is confirmed by a fresh process and fails the start."""
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ctl = tmp_path / "ctl.json"
    ctl.write_text("{}")
    log = tmp_path / "starts.log"
    kdir = str(tmp_path / "dp")
    os.makedirs(kdir)
    eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
    dev = {o: d for d, o in eng.ordinals().items()}
    eng.close()
    kub = gp.GoServer(os.path.join(kdir, "kubelet.sock"), {"/v1beta1.Registration/Register": lambda m: (0, "", b"")})
    p = _daemon(kdir, fi, "-pulse", "3600", "-liveness", "-liveness_probe", STUB, "-prestart_liveness",
                "-liveness_timeout", "5", "-exporter_socket", "", "-grpc_watchdog", "0",
                env={"MI355X_STUB_PROBE_CONTROL": str(ctl), "MI355X_STUB_PROBE_LOG": str(log)})
    try:
        deadline = time.monotonic() + 30
        while not os.path.exists(os.path.join(kdir, "amd.com_gpu")) and time.monotonic() < deadline:
            time.sleep(0.05)
        time.sleep(0.3)
        _busy_gpu(fi, inv, dev[3])
        ctl.write_text(json.dumps({"3": "pending", "5": "pending"}))
        status, msg, took = _unary_fresh(kdir, "PreStartContainer", pb.PreStartContainerRequest(devices_ids=[dev[3]]))
        assert status == 0 and took < 2.0, (status, msg, took)
        assert "3" not in log.read_text().split()                # no fresh process on the busy GPU
        status, msg, _ = _unary_fresh(kdir, "PreStartContainer", pb.PreStartContainerRequest(devices_ids=[dev[5]]))
        assert status == 9 and dev[5] in msg, (status, msg)
        assert "5" in log.read_text().split()                    # confirmed by a fresh process
    finally:
        rc, err = _stop(p)
        kub.close()
    assert rc == 0, err[-2000:]


def test_prestart_gate_leaves_crowded_gpus_alone(tmp_path):
    """A GPU crowded with tenant processes has no probe-server queue (the sweep
    steps off it); a container start there is not checked either, rather than
    restarting the server onto that GPU."""
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ctl = tmp_path / "ctl.json"
    ctl.write_text(json.dumps({"3": "fail"}))
    log = tmp_path / "starts.log"
    kdir = str(tmp_path / "dp")
    os.makedirs(kdir)
    eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
    dev = {o: d for d, o in eng.ordinals().items()}
    eng.close()
    for pid in range(800, 807):
        _busy_gpu(fi, inv, dev[3], pid=str(pid))
    kub = gp.GoServer(os.path.join(kdir, "kubelet.sock"), {"/v1beta1.Registration/Register": lambda m: (0, "", b"")})
    p = _daemon(kdir, fi, "-pulse", "3600", "-liveness", "-liveness_probe", STUB, "-prestart_liveness",
                "-liveness_timeout", "5", "-exporter_socket", "", "-grpc_watchdog", "0",
                env={"MI355X_STUB_PROBE_CONTROL": str(ctl), "MI355X_STUB_PROBE_LOG": str(log)})
    try:
        deadline = time.monotonic() + 30
        while not os.path.exists(os.path.join(kdir, "amd.com_gpu")) and time.monotonic() < deadline:
            time.sleep(0.05)
        time.sleep(0.3)
        starts = log.read_text().split().count("serve+keep")
        status, msg, _ = _unary_fresh(kdir, "PreStartContainer", pb.PreStartContainerRequest(devices_ids=[dev[3]]))
        assert status == 0, msg
        status, msg, _ = _unary_fresh(kdir, "PreStartContainer", pb.PreStartContainerRequest(devices_ids=[dev[2]]))
        assert status == 0, msg
        words = log.read_text().split()
        assert words.count("serve+keep") == starts == 1 and "visible=0,1,2,4,5,6,7" in words
    finally:
        rc, err = _stop(p)
        kub.close()
    assert rc == 0, err[-2000:]


def test_prestart_gate_does_not_wait_for_a_hung_exporter(tmp_path):
    """A sweep stuck in the metrics exporter (10 s deadline) holds the engine's
    prober only for its liveness pass: a PreStartContainer check meanwhile is
    answered at once."""
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    fi = make_mi355x_node(tmp_path / "n")
    ctl = tmp_path / "ctl.json"
    ctl.write_text("{}")
    kdir = str(tmp_path / "dp")
    os.makedirs(kdir)
    eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
    dev = {o: d for d, o in eng.ordinals().items()}
    eng.close()
    exp = gp.GoServer(str(tmp_path / "exp.sock"), {}, gp.GoServerConfig(never_answer=True))
    kub = gp.GoServer(os.path.join(kdir, "kubelet.sock"), {"/v1beta1.Registration/Register": lambda m: (0, "", b"")})
    p = _daemon(kdir, fi, "-pulse", "1", "-liveness", "-liveness_probe", STUB, "-prestart_liveness",
                "-liveness_timeout", "5", "-exporter_socket", str(tmp_path / "exp.sock"), "-grpc_watchdog", "0",
                env={"MI355X_STUB_PROBE_CONTROL": str(ctl)})
    try:
        deadline = time.monotonic() + 40       # the first sweep waits out the exporter's 10 s
        while not os.path.exists(os.path.join(kdir, "amd.com_gpu")) and time.monotonic() < deadline:
            time.sleep(0.05)
        n = len(exp.calls)
        while len(exp.calls) == n and time.monotonic() < deadline:   # the next sweep is now in the exporter
            time.sleep(0.05)
        assert len(exp.calls) > n, "no second exporter call"
        time.sleep(0.5)
        status, msg, took = _unary_fresh(kdir, "PreStartContainer", pb.PreStartContainerRequest(devices_ids=[dev[1]]))
        assert status == 0 and took < 3.0, (status, msg, took)
    finally:
        rc, err = _stop(p)
        kub.close()
        exp.close()
    assert rc == 0, err[-2000:]


def _unary_fresh(kdir, method, req):
    """One call on a connection of its own: (status, message, seconds)."""
    c = core().GrpcClient()
    assert c.connect(os.path.join(kdir, "amd.com_gpu"), 5.0) == ""
    try:
        t0 = time.monotonic()
        status, msg, _ = c.unary(f"/v1beta1.DevicePlugin/{method}", req.SerializeToString(), 30.0)
        return status, msg, time.monotonic() - t0
    finally:
        c.close()


def test_prestart_pending_at_shutdown_is_answered(tmp_path):
    """SIGTERM while a PreStartContainer check is running: the check is cut
    short, which is no fault (OK), or the server stops first (UNAVAILABLE);
    either way the call is answered at once, not after the 30 s check, and the
    daemon exits promptly."""
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    fi = make_mi355x_node(tmp_path / "n")
    ctl = tmp_path / "ctl.json"
    ctl.write_text("{}")
    kdir = str(tmp_path / "dp")
    os.makedirs(kdir)
    kub = gp.GoServer(os.path.join(kdir, "kubelet.sock"), {"/v1beta1.Registration/Register": lambda m: (0, "", b"")})
    p = _daemon(kdir, fi, "-pulse", "3600", "-liveness", "-liveness_probe", STUB, "-prestart_liveness",
                "-liveness_timeout", "20", "-exporter_socket", "", "-grpc_watchdog", "0",
                env={"MI355X_STUB_PROBE_CONTROL": str(ctl)})
    try:
        deadline = time.monotonic() + 30
        while not os.path.exists(os.path.join(kdir, "amd.com_gpu")) and time.monotonic() < deadline:
            time.sleep(0.05)
        time.sleep(0.3)
        eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
        d0 = {o: d for d, o in eng.ordinals().items()}[0]
        eng.close()
        ctl.write_text(json.dumps({"0": "slow", "slow_s": 30}))
        import concurrent.futures
        with concurrent.futures.ThreadPoolExecutor(1) as ex:
            fut = ex.submit(_unary_fresh, kdir, "PreStartContainer", pb.PreStartContainerRequest(devices_ids=[d0]))
            time.sleep(0.5)
            t0 = time.monotonic()
            rc, err = _stop(p)
            status, msg, took = fut.result(timeout=20)
        assert rc == 0 and time.monotonic() - t0 < 10, err[-2000:]
        assert status in (0, 14) and took < 10, (status, msg, took)
    finally:
        if p.poll() is None:
            p.kill()
        kub.close()


def test_daemon_hung_exporter_blocks_neither_registration_nor_shutdown(tmp_path):
    """An exporter that accepts and never answers (10 s deadline per call): a
    kubelet restart is re-registered within a second, RPCs are answered at
    once, and SIGTERM during the stuck call ends the daemon promptly."""
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")
    os.makedirs(kdir)
    exp = gp.GoServer(str(tmp_path / "exp.sock"), {}, gp.GoServerConfig(never_answer=True))
    regs = []

    def kubelet():
        return gp.GoServer(os.path.join(kdir, "kubelet.sock"),
                           {"/v1beta1.Registration/Register": lambda m: (regs.append(time.monotonic()), (0, "", b""))[1]})

    kub = kubelet()
    p = _daemon(kdir, fi, "-pulse", "1", "-exporter_socket", str(tmp_path / "exp.sock"), "-grpc_watchdog", "0")
    try:
        deadline = time.monotonic() + 30
        while not regs and time.monotonic() < deadline:
            time.sleep(0.02)
        assert regs, "never registered"
        time.sleep(1.5)   # a pulse is now stuck in the exporter call
        assert exp.calls, "the exporter was not asked"
        kub.close()
        kub = kubelet()
        t0 = time.monotonic()
        while len(regs) < 2 and time.monotonic() - t0 < 5:
            time.sleep(0.01)
        # the exporter call hangs for its 10 s deadline: anything well under that did not wait for it
        # (bounds loose enough for a loaded CI host)
        assert len(regs) >= 2 and regs[-1] - t0 < 3.0, "re-registration waited for the exporter"
        c = gp.GoClientConn(os.path.join(kdir, "amd.com_gpu"))
        try:
            t1 = time.monotonic()
            assert c.unary("/v1beta1.DevicePlugin/GetDevicePluginOptions", b"", 5.0)[0] == 0
            assert time.monotonic() - t1 < 2.0
        finally:
            c.close()
        t2 = time.monotonic()
        rc, err = _stop(p)
        assert rc == 0 and time.monotonic() - t2 < 5.0, err[-2000:]
    finally:
        if p.poll() is None:
            p.kill()
        kub.close()
        exp.close()


def test_daemon_watchdog_exits_when_kubelet_never_lists(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")
    os.makedirs(kdir)
    kub = gp.GoServer(os.path.join(kdir, "kubelet.sock"), {"/v1beta1.Registration/Register": lambda m: (0, "", b"")})
    t0 = time.monotonic()
    p = _daemon(kdir, fi, "-grpc_watchdog", "1", "-exporter_socket", "")
    try:
        rc, err = _stop(p, timeout=20) if p.wait(timeout=15) is not None else (None, "")
    finally:
        kub.close()
    assert rc == 3 and "no ListAndWatch stream within 1s" in err and time.monotonic() - t0 < 10
    assert not os.path.exists(os.path.join(kdir, "amd.com_gpu"))      # sockets removed on the way out


def test_daemon_refuses_unknown_flags_and_bad_liveness(tmp_path):
    # -grpc_server was the Python CLI's transport switch; the daemon is the only
    # plugin entrypoint, so it is an undefined flag like any other: Go's flag
    # package prints the error and the usage and exits 2; validation errors
    # (validateFlags, main.go:59-75) are logged and exit 1
    for args, want, rc in ((["-grpc_server", "aio"], "flag provided but not defined: -grpc_server", 2),
                           (["-liveness"], "-pulse > 0", 1),
                           (["-liveness_mode", "bogus"], "liveness_mode", 1),
                           (["-vmodule", "nolevel"], "vmodule", 1)):
        p = subprocess.run([EXE, *args], capture_output=True, text=True, timeout=20)
        assert p.returncode == rc and want in p.stderr, (args, p.stderr)
    p = subprocess.run([EXE, "-grpc_server", "aio"], capture_output=True, text=True, timeout=20)
    assert "usage:" in p.stderr.lower() and not p.stdout
