"""The shipped native health engine on the real MI355X (all marked ``gpu``).

These drive `health_engine.cpp` / `liveness_prober.cpp` — through the
`core().HealthEngine` binding or the `mi355x-device-plugin` daemon itself —
on the behaviours tests/test_gpu.py once checked only through the Python
monitor (health/monitor.py, health/liveness.py):

  identity      every reply names its device; no re-keying on a real box
  tenant        the kept-queue server's own kfd entry is not a tenant
  replacement   a SIGKILLed probe server is replaced by the next sweep
  throughput    the throughput check in the sweep's cadence on an idle GPU
  xGMI          amd-smi link state read each sweep, first reading = baseline
  admission     the health DaemonSet's sources (liveness + amd-smi ECC,
                events, xGMI) through the daemon: per-source readings in
                /metrics, Healthy in ListAndWatch, a container started on the
                allocated GPU becomes ready

Reference behaviour replaced: a node-global kfd verdict plus the exporter
(internal/pkg/amdgpu/amdgpu.go:322-345,865-974).
"""
import asyncio
import json
import os
import signal
import socket
import time
import urllib.request

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def inv():
    from rocm_k8s_device_plugin_amd.topology import discover
    return discover("/sys")


@pytest.fixture(scope="module")
def ordinals(inv):
    from rocm_k8s_device_plugin_amd.topology import hip_ordinals
    return hip_ordinals(inv, "/dev")


def _probe_exe():
    from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
    return os.path.join(str(PKG_DIR), "bin", "mi355x-liveness-probe")


def _present_kfd_entries():
    """kfd proc entries now. They are named by host PID, which a container's PID
    namespace (the gpurun box) does not show as os.getpid(): this pytest
    process, which may hold HIP queues from earlier GPU tests, is among them."""
    root = "/sys/class/kfd/kfd/proc"
    return sorted(os.listdir(root)) if os.path.isdir(root) else []


def _engine(ordinals, **opts):
    """The engine on the accessible GPUs. The processes already on the GPU
    (this pytest process among them) are never counted as tenants, as a
    process embedding the engine would not be (Config::kfd_exclude)."""
    from rocm_k8s_device_plugin_amd.ops.native import core
    o = dict(dev_root="/dev", liveness=True, probe_exe=_probe_exe(), probe_timeout_s=60.0,
             device_ids=sorted(ordinals), kfd_exclude=_present_kfd_entries())
    o.update(opts)
    return core().HealthEngine("/sys", o)


def _location(pci_bus_id):
    d, b, df = pci_bus_id.split(":")
    dev, fn = df.split(".")
    return int(d, 16), (int(b, 16) << 8) | (int(dev, 16) << 3) | int(fn, 16)


def test_native_engine_live_devices_keep_their_identity(inv, ordinals):
    """The native engine's ordinal map equals the kfd-derived one, every real
    reply names the device its verdict is written to (the check path reports
    it), and three sweeps re-key nothing: every accessible device Healthy."""
    eng = _engine(ordinals)
    try:
        assert eng.ordinals() == dict(ordinals)
        for _ in range(3):
            eng.sweep()
        snap = eng.snapshot()
        assert snap and all(ok for ok, _ in snap.values()), snap
        st = eng.stats()
        assert st["identity_remaps"] == 0 and st["server_starts"] == 1 and st["fallbacks"] == 0, st
        res = eng.check(sorted(ordinals), 10.0)              # PreStartContainer's path, same server
        assert set(res) == set(ordinals) and all(r["ok"] for r in res.values()), res
        assert eng.stats()["server_starts"] == 1
    finally:
        eng.close()
    assert not eng.stats()["server_running"]


def test_native_kept_queue_server_is_not_a_tenant(inv, ordinals):
    """The kept-queue server's own kfd entry is found and excluded: its queue on
    the GPU does not make the GPU look busy to the engine."""
    from rocm_k8s_device_plugin_amd.topology import kfd_busy_gpu_ids
    dev_id = min(ordinals, key=ordinals.get)
    gid = inv.topology.node(inv.by_id[dev_id].node_id).gpu_id
    initial = set(_present_kfd_entries())          # this test process among them
    eng = _engine({dev_id: ordinals[dev_id]})
    try:
        eng.sweep()
        assert eng.snapshot()[dev_id][0], eng.snapshot()
        own = eng.own_kfd_entries({gid})
        for _ in range(100):                       # another GPU process started with the server: wait it out
            if own:
                break
            time.sleep(0.1)
            own = eng.own_kfd_entries({gid})
        if not own:
            pytest.skip("another GPU process started with the probe server and is still running")
        # kfd names its proc entries by host PID, which differs from the server's PID
        # inside a container's PID namespace (as on the gpurun box): one entry, with our queue
        assert len(own) == 1 and eng.stats()["server_pid"] > 0, (own, eng.stats())
        qdir = os.path.join("/sys/class/kfd/kfd/proc", next(iter(own)), "queues")
        gids = {int(open(os.path.join(qdir, q, "gpuid")).read()) for q in os.listdir(qdir)}
        assert gid in gids                                       # the server's kept queue ...
        assert gid in kfd_busy_gpu_ids("/sys", exclude=initial)   # ... makes the GPU look busy to a naive reader
        eng.sweep()
        assert eng.stats()["busy_state_known"]
        # ... but not to the engine (other processes of the shared host may come and go: same view)
        assert (gid in eng.gpu_load()) == (gid in kfd_busy_gpu_ids("/sys", exclude=initial | own))
    finally:
        eng.close()


def test_native_probe_server_killed_is_replaced(inv, ordinals):
    """SIGKILL of the real probe server between sweeps (OOM killer, operator):
    the next sweep starts a new one, the device stays Healthy."""
    eng = _engine(ordinals)
    try:
        eng.sweep()
        pid = eng.stats()["server_pid"]
        assert pid > 0
        os.kill(pid, signal.SIGKILL)
        time.sleep(0.5)
        eng.sweep()
        st = eng.stats()
        assert st["server_starts"] == 2 and st["server_pid"] not in (-1, pid), st
        assert all(ok for ok, _ in eng.snapshot().values()), eng.snapshot()
        # a check after a kill: no server until the sweep restarts it -> a fresh process.
        # Until the dead server's kfd process is torn down its queue still counts as
        # another process' (the GPU is busy): such a check is inconclusive, not failed.
        gids = {inv.topology.node(inv.by_id[d].node_id).gpu_id for d in ordinals}
        own = eng.own_kfd_entries(gids)
        os.kill(st["server_pid"], signal.SIGKILL)
        res = eng.check(sorted(ordinals), 10.0)
        assert all(r["ok"] or r["pending"] for r in res.values()), res
        deadline = time.monotonic() + 30
        while own & set(_present_kfd_entries()) and time.monotonic() < deadline:
            time.sleep(0.1)
        res = eng.check(sorted(ordinals), 10.0)
        assert all(r["ok"] for r in res.values()), res
        assert eng.stats()["check_fresh"] >= len(ordinals)
    finally:
        eng.close()


def test_native_throughput_check_on_idle_gpu(ordinals):
    """The sweep's cadence with -perf_check_every 1: liveness, then the throughput
    check on the idle GPU in the same sweep; a healthy MI355X clears every floor."""
    eng = _engine(ordinals, perf_check_every=1, perf_mib=1024, perf_iters=16384, perf_action="unhealthy")
    try:
        eng.sweep()
        assert eng.stats()["perf_checks"] == 1, eng.stats()
        verdicts = eng.perf_verdicts()
        assert verdicts and all(state == "ok" for state, _ in verdicts.values()), verdicts
        assert all(ok for ok, _ in eng.snapshot().values()), eng.snapshot()
    finally:
        eng.close()
    from rocm_k8s_device_plugin_amd.ops.native import core
    m = core().metrics_render()
    tf = [float(ln.rsplit(" ", 1)[1]) for ln in m.splitlines() if ln.startswith("mi355x_dp_perf_mfma_tflops{")]
    assert tf and all(x > 700 for x in tf), tf


def test_native_xgmi_link_state(inv, ordinals):
    """-smi_xgmi on the real node: amd-smi's link state is read every sweep, the
    first reading is the baseline, and a healthy node degrades no pair."""
    from rocm_k8s_device_plugin_amd.ops.native import core
    snap = core().smi_xgmi_links()
    if not snap["ok"]:
        pytest.skip(f"amd-smi xGMI link state unavailable: {snap.get('error')}")
    eng = _engine(ordinals, liveness=False, smi_xgmi=True)
    try:
        eng.sweep()
        eng.sweep()
        st = eng.stats()
        assert st["xgmi_readings"] == 2 and st["xgmi_error"] == "", st
        assert eng.degraded_links() == [] and eng.links_down() == {}
        assert eng.fabric_version() == 0
    finally:
        eng.close()


def test_native_daemon_admission_with_smi_sources(inv, ordinals, tmp_path):
    """The health DaemonSet's configuration through the daemon: -liveness with
    amd-smi ECC, events and xGMI link state. Every source reads ok each pulse
    (/metrics), ListAndWatch shows the GPUs Healthy, a container given the
    allocated DeviceSpecs runs its MFMA probe on exactly that GPU, and /healthz
    and /readyz answer 200."""
    from rocm_k8s_device_plugin_amd.container_runtime import render_minors_from_specs, start_container
    from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
    from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet

    exe = os.environ.get("MI355X_NATIVE_DAEMON_EXE") or os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")
    kdir = str(tmp_path / "dp")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]

    def metrics():
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
            return {k: float(v) for k, v in (ln.rsplit(" ", 1) for ln in r.read().decode().splitlines()
                                             if ln and not ln.startswith("#"))}

    def reading(m, source, result):
        return sum(v for k, v in m.items() if k.startswith("mi355x_dp_health_source_readings_total{")
                   and f'source="{source}"' in k and f'result="{result}"' in k)

    async def go():
        k = FakeKubelet(kdir, rpc_client="native")
        await k.start()
        proc = await asyncio.create_subprocess_exec(
            exe, "-kubelet_dir", kdir, "-exporter_socket", "", "-pulse", "1", "-liveness", "-liveness_probe",
            _probe_exe(), "-liveness_timeout", "30", "-smi_ecc", "-smi_events", "-smi_xgmi", "-prestart_liveness",
            "-device_ids", ",".join(sorted(ordinals)), "-metrics_port", str(port),
            stdout=asyncio.subprocess.DEVNULL, stderr=asyncio.subprocess.PIPE)
        try:
            st = await k.wait_for_resource("amd.com/gpu", len(ordinals), timeout=60)
            assert all(h == "Healthy" for h in st.devices.values()), st.devices
            await asyncio.sleep(2.5)                              # two more pulses
            m = await asyncio.to_thread(metrics)
            for source in ("kfd", "liveness", "smi_ecc", "smi_events", "smi_xgmi"):
                assert reading(m, source, "ok") >= 2 and reading(m, source, "error") == 0, (source, {
                    k: v for k, v in m.items() if "source_readings" in k})
            adm = await k.admit("amd.com/gpu", 1)                 # PreStartContainer included
            car = adm.response.container_responses[0]
            minors = render_minors_from_specs(car)
            m2o = {inv.by_id[i].render_minor: o for i, o in ordinals.items()}
            r = await asyncio.to_thread(start_container, [m2o[x] for x in minors],
                                        device_paths=[ds.host_path for ds in car.devices])
            assert r.ok, r.error
            assert r.doc["hip_device_count"] == 1
            assert r.doc["devices"][0]["pci_bus_id"].lower() == adm.device_ids[0].lower()
            st = k.resources["amd.com/gpu"]
            assert all(h == "Healthy" for h in st.devices.values()), st.devices
            m = await asyncio.to_thread(metrics)
            assert m['mi355x_dp_prestart_checks_total{result="ok"}'] >= 1
            assert m.get("mi355x_dp_xgmi_links_down", 0.0) == 0.0
            # what the chart's probes read (dp.metricsPort): the loop runs, the resource is registered
            for path in ("/healthz", "/readyz"):
                with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=5) as r:
                    assert (r.status, r.read()) == (200, b"ok\n"), path
        finally:
            if proc.returncode is None:
                proc.send_signal(signal.SIGTERM)
            _, err = await asyncio.wait_for(proc.communicate(), 60)
            print(err.decode(errors="replace")[-3000:])
            await k.stop()
        assert proc.returncode == 0
        return err.decode(errors="replace")

    err = asyncio.run(asyncio.wait_for(go(), 240))
    assert "amd-smi event notification unavailable" not in err, err[-2000:]
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/native_daemon_smi_sources.log", "w") as f:
        f.write(err[-20000:])


_TENANT = r"""
import sys, time, torch
n, seconds = int(sys.argv[1]), float(sys.argv[2])
a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
torch.matmul(a, b, out=c)
torch.cuda.synchronize()
print("READY", flush=True)
t_end = time.perf_counter() + seconds
while time.perf_counter() < t_end:
    torch.matmul(a, b, out=c)
    torch.cuda.synchronize()
print("DONE", flush=True)
"""


def test_native_prestart_beside_a_long_kernel_tenant(ordinals, tmp_path):
    """A tenant's long bf16 GEMMs (n = 49152, ~180 ms each, every CU held) on the
    GPU: PreStartContainer through the daemon is answered within the 50 ms busy
    deadline plus overhead, never failed, while 1 s sweeps go on (round 5: the
    gate waited for the running GEMM, up to the 9.5 s deadline;
    tools/prestart_tenant.py is the longer measurement)."""
    import subprocess
    import sys
    from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet, NativeRpcError

    dev_id = min(ordinals, key=ordinals.get)
    exe = os.environ.get("MI355X_NATIVE_DAEMON_EXE") or os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")
    kdir = str(tmp_path / "dp")
    out = {}

    async def go():
        k = FakeKubelet(kdir, rpc_client="native")
        await k.start()
        proc = await asyncio.create_subprocess_exec(
            exe, "-kubelet_dir", kdir, "-exporter_socket", "", "-pulse", "1", "-liveness", "-liveness_probe",
            _probe_exe(), "-prestart_liveness", "-device_ids", dev_id, stdout=asyncio.subprocess.DEVNULL,
            stderr=asyncio.subprocess.PIPE)
        tenant = None
        try:
            st = await k.wait_for_resource("amd.com/gpu", 1, timeout=60)
            req = pb.PreStartContainerRequest(devices_ids=[dev_id])
            tenant = subprocess.Popen([sys.executable, "-c", _TENANT, "49152", "6"], stdout=subprocess.PIPE, text=True)
            line = await asyncio.to_thread(tenant.stdout.readline)
            assert line.strip() == "READY", line
            lat, statuses = [], []
            for _ in range(16):
                t0 = time.perf_counter()
                try:
                    await k._call(st, "PreStartContainer", req, pb.PreStartContainerResponse, timeout=30.0)
                    statuses.append(0)
                except NativeRpcError as e:
                    statuses.append(e.status)
                lat.append((time.perf_counter() - t0) * 1e3)
                await asyncio.sleep(0.25)
            out["prestart_ms"] = sorted(lat)
            out["statuses"] = statuses
            await asyncio.to_thread(tenant.wait, 60)
            tenant = None
        finally:
            if tenant is not None:
                tenant.kill()
            if proc.returncode is None:
                proc.send_signal(signal.SIGTERM)
            _, err = await asyncio.wait_for(proc.communicate(), 60)
            await k.stop()
        assert proc.returncode == 0, err.decode(errors="replace")[-3000:]

    asyncio.run(asyncio.wait_for(go(), 240))
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/prestart_beside_tenant.json", "w") as f:
        json.dump(out, f)
    assert out["statuses"] == [0] * 16, out
    assert out["prestart_ms"][-1] < 150, out      # busy deadline 50 ms + the check's own overhead
