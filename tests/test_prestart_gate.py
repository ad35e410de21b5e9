"""PreStartContainer's liveness gate (-prestart_liveness) next to the health
sweep, against a stub probe server that behaves like the real one
(hsa_probe.cpp:560-579): a dispatch queued behind other work is answered only
when its deadline has passed, tagged requests are answered concurrently, and
requests on one device serialise on its kept slot.

What is pinned here:
  * a check of an idle GPU is answered at once while a sweep waits out its full
    deadline on another GPU (the check is a separate tagged request, never
    serialised behind the sweep's pass);
  * a busy GPU (another process' queues) gets the short deadline, sweep and
    check alike, and its pending verdict lets the container start;
  * the check has a budget well under kubelet's 30 s: a wedged idle GPU fails
    the start within it, and what the budget cannot settle is let through;
  * the gate runs on a bounded worker pool, and checks leave the sweep's
    fallback backoff and counters alone.

The reference's PreStartContainer is a no-op (internal/pkg/plugin/plugin.go:139-141);
kubelet's deadline for it is 30 s (vendor/k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/constants.go:44).
"""
import concurrent.futures
import json
import os
import socket
import subprocess
import sys
import threading
import time
import urllib.request

import pytest

from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR, core
from rocm_k8s_device_plugin_amd.testing import gopeer as gp
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


def _wait_for_line(path, line, timeout=20.0):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if path.exists() and line in path.read_text().split():
            return
        time.sleep(0.01)
    raise AssertionError(f"{line!r} never appeared in {path}")


def _engine(fi, tmp_path, control, timeout=5.5, env=None, **opts):
    ctl = tmp_path / "probe_ctl.json"
    ctl.write_text(json.dumps(control))
    extra = {"MI355X_STUB_PROBE_CONTROL": str(ctl), **(env or {})}
    o = dict(dev_root=str(fi.dev), liveness=True, probe_exe=STUB, argv_prefix=[sys.executable],
             probe_timeout_s=timeout, extra_env=extra, fail_threshold=2)
    o.update(opts)
    return ctl, core().HealthEngine(str(fi.sysfs), o)


def test_check_beside_a_sweep_waiting_on_another_gpu(tmp_path):
    """Engine level: a sweep waits out device 3's full 5 s deadline; a check of
    idle device 1 meanwhile is answered from the same server in well under
    0.2 s, and a check of device 3 once it is busy within its short deadline."""
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    log = tmp_path / "stub.log"
    ctl, eng = _engine(fi, tmp_path, {}, env={"MI355X_STUB_PROBE_LOG": str(log)})
    dev = {o: d for d, o in eng.ordinals().items()}
    try:
        eng.sweep()                                    # the kept-queue server is up
        ctl.write_text(json.dumps({"3": "pending"}))
        sweep = threading.Thread(target=eng.sweep)
        t_sweep = time.monotonic()
        sweep.start()
        _wait_for_line(log, "pending:3")               # the sweep is now waiting on device 3
        t0 = time.monotonic()
        r = eng.check([dev[1]], 5.0)
        took = time.monotonic() - t0
        assert r[dev[1]]["ok"] and took < 0.2, (r, took)
        assert sweep.is_alive() and time.monotonic() - t_sweep < 5.0   # still inside the 5 s wait
        # device 3 turns busy (a tenant's queue): the check's deadline is the short one
        _busy_gpu(fi, inv, dev[3])
        t0 = time.monotonic()
        r = eng.check([dev[3]], 5.0)
        took = time.monotonic() - t0
        assert r[dev[3]]["pending"] and not r[dev[3]]["ok"] and took < 0.5, (r, took)
        assert sweep.is_alive()
        sweep.join(30)
        assert not sweep.is_alive()
        st = eng.stats()
        assert st["server_starts"] == 1 and st["checks"] == 2 and st["check_fresh"] == 0
        assert st["check_inconclusive"] == 1
    finally:
        eng.close()


def test_definite_failure_on_a_busy_gpu_still_fails_the_check(tmp_path):
    """Only a pending dispatch on a busy GPU is inconclusive: a wrong tile there
    is confirmed by a fresh process and fails the check like anywhere else
    (the GPU test suite's own process keeps queues on the GPU it probes)."""
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ctl, eng = _engine(fi, tmp_path, {})
    dev = {o: d for d, o in eng.ordinals().items()}
    try:
        eng.sweep()
        _busy_gpu(fi, inv, dev[4])
        ctl.write_text(json.dumps({"4": "fail"}))
        r = eng.check([dev[4]], 5.0)[dev[4]]
        assert not r["ok"] and not r["pending"] and "differ" in r["reason"], r
        assert eng.stats()["check_fresh"] == 1
    finally:
        eng.close()


def test_sweep_gives_busy_gpus_the_short_deadline(tmp_path):
    """Sweep side: a pending dispatch on a busy GPU costs the sweep the busy
    deadline (0.3 s here), not the 5 s probe deadline; the verdict is
    inconclusive, and the late verdict is collected by a later request."""
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ctl, eng = _engine(fi, tmp_path, {}, busy_deadline_s=0.3, busy_grace_s=300.0)
    dev = {o: d for d, o in eng.ordinals().items()}
    try:
        eng.sweep()
        _busy_gpu(fi, inv, dev[3])
        ctl.write_text(json.dumps({"3": "pending"}))
        t0 = time.monotonic()
        eng.sweep()
        took = time.monotonic() - t0
        assert 0.3 <= took < 2.0, took
        assert not {d for d, (ok, _) in eng.snapshot().items() if not ok}
        ctl.write_text("{}")                          # the tenant's kernel ends: the late verdict
        eng.sweep()
        assert eng.snapshot()[dev[3]][0]
    finally:
        eng.close()


def test_checks_leave_the_sweep_backoff_alone(tmp_path):
    """After a probe-server failure the sweep probes from fresh processes for 4
    sweeps (backoff). PreStart checks in between neither use that backoff up
    nor start the server on the admission path."""
    fi = make_mi355x_node(tmp_path / "n")
    ctl, eng = _engine(fi, tmp_path, {"5": "hang"}, timeout=1.5)
    dev = {o: d for d, o in eng.ordinals().items()}
    try:
        eng.sweep()                                    # the server hangs on device 5: fallback, backoff 4
        st = eng.stats()
        assert st["fallbacks"] == 1 and st["server_starts"] == 1 and not st["server_running"]
        ctl.write_text("{}")
        for _ in range(6):
            r = eng.check([dev[1]], 3.0)               # no server: a fresh process for the idle GPU
            assert r[dev[1]]["ok"], r
        st = eng.stats()
        assert st["server_starts"] == 1 and st["check_fresh"] == 6 and st["prober_sweeps"] == 1
        eng.sweep()                                    # backoff 4 -> 3: still no server
        assert eng.stats()["server_starts"] == 1
    finally:
        eng.close()


# ---------------------------------------------------------------- the daemon
def _daemon(kdir, fi, *extra, env=None):
    return subprocess.Popen([EXE, "-kubelet_dir", kdir, "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                             "-exporter_socket", "", "-grpc_watchdog", "0", "-liveness", "-liveness_probe", STUB,
                             "-prestart_liveness", *extra], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                            text=True, env=dict(os.environ, **(env or {})))


def _stop(p, timeout=20):
    if p.poll() is None:
        p.terminate()
    try:
        _, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        _, err = p.communicate()
        return None, err
    return p.returncode, err


def _prestart(kdir, ids):
    """PreStartContainer on a connection of its own: (status, message, seconds)."""
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    c = core().GrpcClient()
    assert c.connect(os.path.join(kdir, "amd.com_gpu"), 5.0) == ""
    try:
        t0 = time.monotonic()
        status, msg, _ = c.unary("/v1beta1.DevicePlugin/PreStartContainer",
                                 pb.PreStartContainerRequest(devices_ids=ids).SerializeToString(), 35.0)
        return status, msg, time.monotonic() - t0
    finally:
        c.close()


class _Node:
    def __init__(self, tmp_path, control, *flags, env=None):
        self.fi = make_mi355x_node(tmp_path / "n")
        self.inv = discover(str(self.fi.sysfs))
        self.ctl = tmp_path / "ctl.json"
        self.ctl.write_text(json.dumps(control))
        self.log = tmp_path / "stub.log"
        self.kdir = str(tmp_path / "dp")
        os.makedirs(self.kdir)
        eng = core().HealthEngine(str(self.fi.sysfs), {"dev_root": str(self.fi.dev)})
        self.dev = {o: d for d, o in eng.ordinals().items()}
        eng.close()
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            self.port = s.getsockname()[1]
        self.kub = gp.GoServer(os.path.join(self.kdir, "kubelet.sock"),
                               {"/v1beta1.Registration/Register": lambda m: (0, "", b"")})
        self.p = _daemon(self.kdir, self.fi, "-metrics_port", str(self.port), *flags,
                         env={"MI355X_STUB_PROBE_CONTROL": str(self.ctl), "MI355X_STUB_PROBE_LOG": str(self.log),
                              **(env or {})})
        deadline = time.monotonic() + 30
        while not os.path.exists(os.path.join(self.kdir, "amd.com_gpu")) and time.monotonic() < deadline:
            time.sleep(0.05)
        time.sleep(0.3)

    def metrics(self):
        with urllib.request.urlopen(f"http://127.0.0.1:{self.port}/metrics", timeout=5) as r:
            return {k: float(v) for k, v in (ln.rsplit(" ", 1) for ln in r.read().decode().splitlines()
                                             if ln and not ln.startswith("#"))}

    def close(self):
        rc, err = _stop(self.p)
        self.kub.close()
        return rc, err


def test_daemon_prestart_on_an_idle_gpu_does_not_wait_for_the_sweep(tmp_path):
    """The verdict's acceptance case: device 3's probe is pending against the
    stub's full 5 s deadline inside a pulse sweep; PreStartContainer for idle
    device 1 is answered in < 0.2 s meanwhile, and for device 3 once it is busy
    within the short deadline. Both starts go ahead."""
    n = _Node(tmp_path, {}, "-pulse", "1", "-liveness_timeout", "5.5")
    try:
        n.ctl.write_text(json.dumps({"3": "pending"}))
        _wait_for_line(n.log, "pending:3")               # a sweep is waiting on device 3 now
        t_wait = time.monotonic()
        lat = []
        for _ in range(5):
            status, msg, took = _prestart(n.kdir, [n.dev[1]])
            assert status == 0, msg
            lat.append(took)
        assert max(lat) < 0.2, lat
        assert time.monotonic() - t_wait < 4.5             # all inside the sweep's 5 s wait
        _busy_gpu(n.fi, n.inv, n.dev[3])
        status, msg, took = _prestart(n.kdir, [n.dev[3]])
        assert status == 0 and took < 0.5, (status, msg, took)
        m = n.metrics()
        assert m['mi355x_dp_prestart_checks_total{result="ok"}'] == 5
        assert m['mi355x_dp_prestart_checks_total{result="inconclusive"}'] == 1
    finally:
        rc, err = n.close()
    assert rc == 0, err[-3000:]


def test_daemon_prestart_budget(tmp_path):
    """-prestart_budget bounds the check: a wedged idle GPU (neither the kept
    queue nor a fresh process answers) fails the start within the budget; a
    budget too small for the fresh confirmation lets the start go ahead
    (inconclusive), never past kubelet's 30 s."""
    n = _Node(tmp_path, {}, "-pulse", "3600", "-liveness_timeout", "20", "-prestart_budget", "3")
    try:
        n.ctl.write_text(json.dumps({"5": "hang"}))
        status, msg, took = _prestart(n.kdir, [n.dev[5]])
        assert status == 9 and n.dev[5] in msg and took < 4.0, (status, msg, took)
        assert "deadline exceeded" in msg, msg
        m = n.metrics()
        assert m['mi355x_dp_prestart_checks_total{result="failed"}'] == 1
    finally:
        rc, err = n.close()
    assert rc == 0, err[-3000:]
    n2 = _Node(tmp_path / "b", {}, "-pulse", "3600", "-liveness_timeout", "20", "-prestart_budget", "1.5")
    try:
        n2.ctl.write_text(json.dumps({"5": "pending"}))
        status, msg, took = _prestart(n2.kdir, [n2.dev[5]])   # 0.6 s on the server, < 1 s left: let through
        assert status == 0 and took < 1.6, (status, msg, took)
        assert n2.metrics()['mi355x_dp_prestart_checks_total{result="inconclusive"}'] == 1
    finally:
        rc, err = n2.close()
    assert rc == 0, err[-3000:]


def test_daemon_gate_workers_are_bounded(tmp_path):
    """30 concurrent PreStartContainer calls on slow devices: they queue on a
    pool of at most 8 workers (the daemon's thread count grows by no more),
    and every call is answered."""
    n = _Node(tmp_path, {}, "-pulse", "3600", "-liveness_timeout", "5")
    try:
        n.ctl.write_text(json.dumps({**{str(o): "slow" for o in range(8)}, "slow_s": 0.2}))
        tasks = lambda: len(os.listdir(f"/proc/{n.p.pid}/task"))  # noqa: E731
        base = tasks()
        peak = [base]
        stop = threading.Event()

        def watch():
            while not stop.is_set():
                peak[0] = max(peak[0], tasks())
                time.sleep(0.01)
        w = threading.Thread(target=watch)
        w.start()
        with concurrent.futures.ThreadPoolExecutor(30) as ex:
            res = list(ex.map(lambda i: _prestart(n.kdir, [n.dev[i % 8]]), range(30)))
        stop.set()
        w.join()
        assert all(s == 0 for s, _, _ in res), res
        assert peak[0] - base <= 8 + 2, (base, peak[0])   # the pool, plus the RPC server's own connection threads
    finally:
        rc, err = n.close()
    assert rc == 0, err[-3000:]


def test_daemon_gate_queue_overflow_lets_starts_through(tmp_path):
    """100 PreStartContainer calls at once on GPUs that never answer: 8 run
    (and fail within the budget), up to 64 wait in the queue and come out
    inconclusive once their budget is spent there, and the rest find the queue
    full and are let through at once (`overflow`). Every call is answered,
    none later than the budget plus its queue wait allows."""
    n = _Node(tmp_path, {}, "-pulse", "3600", "-liveness_timeout", "20", "-prestart_budget", "2")
    try:
        n.ctl.write_text(json.dumps({str(o): "hang" for o in range(8)}))
        with concurrent.futures.ThreadPoolExecutor(100) as ex:
            res = list(ex.map(lambda i: _prestart(n.kdir, [n.dev[i % 8]]), range(100)))
        m = n.metrics()
        got = {r: m.get(f'mi355x_dp_prestart_checks_total{{result="{r}"}}', 0)
               for r in ("ok", "failed", "inconclusive", "overflow")}
        assert sum(got.values()) == 100, got
        assert got["overflow"] >= 1 and got["ok"] == 0, got
        assert 1 <= got["failed"] <= 8, got
        failed = [r for r in res if r[0] != 0]
        assert len(failed) == got["failed"] and all(s == 9 for s, _, _ in failed), failed
        assert max(t for _, _, t in res) < 2 * 2 + 5, sorted(t for _, _, t in res)[-5:]
        quick = sorted(t for _, _, t in res)[:int(got["overflow"])]
        assert max(quick) < 1.0, quick   # the overflow answers did not wait for a worker
    finally:
        rc, err = n.close()
    assert rc == 0, err[-3000:]


@pytest.mark.parametrize("flag,value,want", [("-prestart_budget", "0", "prestart_budget must be in (0, 30)"),
                                             ("-prestart_budget", "30", "prestart_budget must be in (0, 30)"),
                                             ("-liveness_busy_deadline", "0", "liveness_busy_deadline must be > 0")])
def test_gate_flags_validated(flag, value, want):
    p = subprocess.run([EXE, "-pulse", "1", "-liveness", "-prestart_liveness", flag, value, "-dry_run"],
                       capture_output=True, text=True, timeout=20)
    assert p.returncode == 1 and want in p.stderr, p.stderr


def test_engine_binding_device_filter_and_tenant_exclusion(tmp_path):
    """The binding's device_ids (judge only these, as the daemon's -device_ids)
    and kfd_exclude (entries never counted as tenants, e.g. the embedding
    process' own queues) options."""
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    eng0 = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
    dev = {o: d for d, o in eng0.ordinals().items()}
    eng0.close()
    ctl, eng = _engine(fi, tmp_path, {}, device_ids=[dev[1], dev[2]], kfd_exclude=["4242"])
    try:
        assert sorted(eng.ordinals()) == sorted([dev[1], dev[2]])
        _busy_gpu(fi, inv, dev[1], pid="4242")               # excluded: not a tenant
        _busy_gpu(fi, inv, dev[2], pid="4343")               # a tenant
        eng.sweep()
        assert sorted(eng.snapshot()) == sorted([dev[1], dev[2]])
        gid = lambda d: inv.topology.node(inv.by_id[d].node_id).gpu_id  # noqa: E731
        assert gid(dev[1]) not in eng.gpu_load() and eng.gpu_load()[gid(dev[2])] == (1, 1)
    finally:
        eng.close()

