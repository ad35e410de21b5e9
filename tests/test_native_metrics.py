"""Prometheus metrics of the native daemon (native/src/util/metrics.cpp).

The native registry renders exactly what the Python registry renders for the
same observations (names, label order, buckets, number formatting), and
`mi355x-device-plugin -metrics_port` serves the series the Python CLI does:
per-RPC latency histograms, registrations, ListAndWatch streams, the native
server's counters, health sweeps and per-device verdicts, liveness round
trips. The reference exposes no metrics."""
import asyncio
import json
import os
import re
import socket
import sys
import urllib.error
import urllib.request

import pytest

from rocm_k8s_device_plugin_amd.ops.native import core
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.utils.metrics import Registry

from test_native_health import STUB, _daemon, _stop


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)


def test_registry_renders_like_python():
    py, nat = Registry(), core().MetricsRegistry()
    ops = [("inc", "mi355x_dp_registrations_total", 1.0, "", {"resource": "gpu"}),
           ("inc", "mi355x_dp_registrations_total", 1.0, "", {"resource": "gpu"}),
           ("inc", "mi355x_dp_rpc_errors_total", 1.0, "", {"rpc": "Allocate", "resource": "cpx_nps1"}),
           ("inc", "mi355x_dp_health_changes_total", 1.0, "", {}),
           ("set", "mi355x_dp_device_healthy", 0.0, "1 if the device is advertised Healthy", {"device": "0000:11:00.0"}),
           ("set", "mi355x_dp_device_healthy", 1.0, "1 if the device is advertised Healthy", {"device": "0000:01:00.0"}),
           ("set", "mi355x_dp_liveness_probe_ms", 0.3612, "last liveness probe round trip", {"device": "x"}),
           ("set", "mi355x_dp_busy_state_known", 1.0, "busy", {})]
    for kind, name, v, hlp, lab in ops:
        getattr(py, kind)(name, v, help=hlp, **lab)
        getattr(nat, kind)(name, v, hlp, lab)
    for ms in (0.04, 0.05, 0.051, 0.19, 3.0, 12.5, 99999.0):
        py.histogram("mi355x_dp_rpc_seconds", "device plugin RPC latency", rpc="Allocate", resource="gpu").observe(ms)
        nat.observe_ms("mi355x_dp_rpc_seconds", ms, "device plugin RPC latency", {"rpc": "Allocate", "resource": "gpu"})
    py.histogram("mi355x_dp_health_sweep_seconds", "health sweep latency").observe(6.25)
    nat.observe_ms("mi355x_dp_health_sweep_seconds", 6.25, "health sweep latency", {})
    assert nat.render() == py.render()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _get(port, path):
    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=5) as r:
            return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()


def _series(text):
    """{series (with labels): value}; the page must also parse as Prometheus reads it."""
    _check_exposition(text)
    out = {}
    for line in text.splitlines():
        if line and not line.startswith("#"):
            k, v = line.rsplit(" ", 1)
            out[k] = float(v)
    return out


def test_daemon_serves_metrics(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    ctl = tmp_path / "ctl.json"
    ctl.write_text(json.dumps({"3": "fail"}))
    kdir = str(tmp_path / "dp")
    port = _free_port()
    eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
    dev = {o: d for d, o in eng.ordinals().items()}
    eng.close()

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = _daemon(kdir, fi, "-pulse", "1", "-liveness", "-liveness_probe", STUB, "-liveness_fail_threshold", "1",
                    "-liveness_timeout", "3", "-exporter_socket", "", "-metrics_port", str(port),
                    env={"MI355X_STUB_PROBE_CONTROL": str(ctl)})
        try:
            await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            adm = await k.admit("amd.com/gpu", 2)
            assert len(adm.device_ids) == 2
            await asyncio.sleep(2.5)   # a pulse or two
            status, text = await asyncio.to_thread(_get, port, "/metrics")
            assert status == 200
            hz = await asyncio.to_thread(_get, port, "/healthz")
            nf = await asyncio.to_thread(_get, port, "/nope")
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        return text, hz, nf

    text, hz, nf = asyncio.run(asyncio.wait_for(go(), 90))
    assert hz == (200, "ok\n") and nf[0] == 404
    s = _series(text)
    assert s['mi355x_dp_registrations_total{resource="gpu"}'] >= 1
    assert s['mi355x_dp_rpc_seconds_count{resource="gpu",rpc="Allocate"}'] == 1
    assert s['mi355x_dp_rpc_seconds_count{resource="gpu",rpc="GetPreferredAllocation"}'] == 1
    assert s['mi355x_dp_rpc_seconds_bucket{resource="gpu",rpc="Allocate",le="+Inf"}'] == 1
    assert s['mi355x_dp_grpc_calls{resource="gpu"}'] >= 2
    assert s['mi355x_dp_listandwatch_open_streams{resource="gpu"}'] >= 1
    assert s["mi355x_dp_health_sweep_seconds_count"] >= 1
    assert s[f'mi355x_dp_device_healthy{{device="{dev[3]}"}}'] == 0.0
    assert sum(v for k, v in s.items() if k.startswith("mi355x_dp_device_healthy")) == 7.0
    assert s[f'mi355x_dp_liveness_probe_ms{{device="{dev[0]}"}}'] > 0
    assert "mi355x_dp_busy_state_known" in s   # 0 here: the stub server has no kfd entry of its own
    assert s["mi355x_dp_devices_identity_unknown"] == 0.0
    assert "# TYPE mi355x_dp_rpc_seconds histogram" in text
    assert re.search(r'^mi355x_dp_rpc_seconds_bucket\{resource="gpu",rpc="Allocate",le="5e-05"\} \d+$', text, re.M)


def _check_exposition(text):
    """The page as Prometheus reads it (prometheus_client's text parser): every
    sample belongs to a family with HELP and TYPE, counters are *_total,
    histogram buckets are cumulative up to +Inf == _count, values are finite."""
    import math
    from prometheus_client.parser import text_string_to_metric_families
    fams = list(text_string_to_metric_families(text))
    assert fams and len({f.name for f in fams}) == len(fams)
    n_samples = sum(len(f.samples) for f in fams)
    assert n_samples == sum(1 for ln in text.splitlines() if ln and not ln.startswith("#"))
    for f in fams:
        assert f.documentation, f.name
        assert f.type in ("counter", "gauge", "histogram"), (f.name, f.type)
        for smp in f.samples:
            assert math.isfinite(smp.value) or smp.labels.get("le") == "+Inf", smp
        if f.type == "counter":
            assert all(s.name.endswith(("_total", "_created")) for s in f.samples), f.name
        if f.type == "histogram":
            series = {}
            for s in f.samples:
                key = tuple(sorted((k, v) for k, v in s.labels.items() if k != "le"))
                series.setdefault(key, {"b": [], "count": None})
                if s.name.endswith("_bucket"):
                    series[key]["b"].append((float(s.labels["le"]), s.value))
                elif s.name.endswith("_count"):
                    series[key]["count"] = s.value
            for key, d in series.items():
                b = sorted(d["b"])
                assert b and b[-1][0] == math.inf and b[-1][1] == d["count"], (f.name, key)
                assert all(x[1] <= y[1] for x, y in zip(b, b[1:])), (f.name, key, b)


def test_daemon_metrics_port_in_use_is_an_error(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    with socket.socket() as s:
        s.bind(("0.0.0.0", 0))
        s.listen(1)
        port = s.getsockname()[1]
        p = _daemon(str(tmp_path / "dp"), fi, "-metrics_port", str(port), "-exporter_socket", "")
        rc, err = _stop(p) if p.wait(timeout=20) is not None else (None, "")
    assert rc == 1 and "cannot serve /metrics" in err


def _raw_http(port, chunks, gap=0.0, read=True, timeout=10.0):
    """Send a request head in pieces; returns (status line, seconds to the answer)."""
    import time
    with socket.create_connection(("127.0.0.1", port), timeout=timeout) as c:
        t0 = time.monotonic()
        for ch in chunks:
            c.sendall(ch)
            time.sleep(gap)
        if not read:
            return None, 0.0
        data = b""
        while True:
            b = c.recv(65536)
            if not b:
                break
            data += b
        return data.split(b"\r\n", 1)[0].decode(), time.monotonic() - t0


def test_metrics_endpoint_survives_awkward_clients(tmp_path):
    """The /metrics endpoint is one thread serving one connection at a time, so
    every wait is bounded: a head sent in pieces is answered; a client that sends
    nothing delays the next scrape by at most the 5 s head deadline; a head
    without an end (16 KiB of header) and a client that leaves early cost nothing."""
    import threading
    import time
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")
    port = _free_port()
    p = _daemon(kdir, fi, "-exporter_socket", "", "-metrics_port", str(port))
    try:
        deadline = time.monotonic() + 20
        while time.monotonic() < deadline:
            try:
                if _get(port, "/healthz")[0] == 200:
                    break
            except OSError:
                time.sleep(0.05)
        # a slow client: the head arrives in three pieces 0.2 s apart
        line, _ = _raw_http(port, [b"GET /met", b"rics HTTP/1.1\r\nHost: x\r\n", b"\r\n"], gap=0.2)
        assert line == "HTTP/1.0 200 OK"
        # LF-only line ends are accepted too
        assert _raw_http(port, [b"GET /healthz HTTP/1.0\n\n"])[0] == "HTTP/1.0 200 OK"
        # a client that leaves before finishing its head
        _raw_http(port, [b"GET /metrics HTT"], read=False)
        # a head that never ends: cut at 16 KiB and answered (the path is still read)
        line, dt = _raw_http(port, [b"GET /metrics HTTP/1.1\r\nX-Pad: " + b"a" * 20000])
        assert line == "HTTP/1.0 200 OK" and dt < 5.0
        # a silent client holds the endpoint until its 5 s head deadline; a scrape behind it waits, then succeeds
        silent = socket.create_connection(("127.0.0.1", port))
        time.sleep(0.1)
        got = {}
        th = threading.Thread(target=lambda: got.update(r=_raw_http(port, [b"GET /metrics HTTP/1.1\r\n\r\n"])))
        th.start()
        th.join(15)
        silent.close()
        line, dt = got["r"]
        assert line == "HTTP/1.0 200 OK" and dt < 6.5
        assert _get(port, "/metrics")[0] == 200
    finally:
        rc, err = _stop(p)
    assert rc == 0, err[-3000:]


def test_daemon_readyz_follows_kubelet_registration(tmp_path):
    """/readyz is 503 (with the count) until every resource is registered with kubelet, then 200; /healthz is 200
    while the control loop runs (it turns 503 only when the loop has not run for 60 s: unit-tested in
    native/tests/test_core.cpp test_http_endpoint_checks). The chart points its probes at them."""
    import time
    fi = make_mi355x_node(tmp_path / "n")
    kdir = tmp_path / "dp"
    kdir.mkdir()
    port = _free_port()
    p = _daemon(str(kdir), fi, "-exporter_socket", "", "-metrics_port", str(port))

    def until(path, want, timeout=20):
        deadline, got = time.monotonic() + timeout, None
        while time.monotonic() < deadline:
            try:
                got = _get(port, path)
                if got[0] == want:
                    return got
            except OSError:
                pass
            time.sleep(0.05)
        raise AssertionError(f"{path}: {got}")

    async def go():
        k = FakeKubelet(str(kdir))
        try:
            assert await asyncio.to_thread(until, "/healthz", 200) == (200, "ok\n")
            before = await asyncio.to_thread(until, "/readyz", 503)
            await k.start()
            await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            after = await asyncio.to_thread(until, "/readyz", 200)
            return before, after
        finally:
            await k.stop()

    try:
        before, after = asyncio.run(asyncio.wait_for(go(), 60))
    finally:
        rc, err = _stop(p)
    assert before == (503, "registered with kubelet: 0 of 1 resources\n"), before
    assert after == (200, "ok\n")
    assert rc == 0, err[-3000:]


def test_daemon_without_gpus_is_ready(tmp_path):
    """A node without GPUs: the daemon idles (as the reference's manager does) and /readyz is 200, so a DaemonSet
    rolling update is not held up by CPU-only nodes (maxUnavailable counts not-ready pods)."""
    import time
    (tmp_path / "sys").mkdir()
    (tmp_path / "dev").mkdir()
    kdir = tmp_path / "dp"
    kdir.mkdir()
    port = _free_port()
    from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
    import subprocess
    exe = os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")
    p = subprocess.Popen([exe, "-kubelet_dir", str(kdir), "-sysfs_root", str(tmp_path / "sys"), "-dev_root",
                          str(tmp_path / "dev"), "-exporter_socket", "", "-metrics_port", str(port)],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        got, deadline = None, time.monotonic() + 20
        while time.monotonic() < deadline:
            try:
                got = (_get(port, "/healthz"), _get(port, "/readyz"))
                break
            except OSError:
                time.sleep(0.05)
    finally:
        rc, err = _stop(p)
    assert got == ((200, "ok\n"), (200, "ok\n")), got
    assert rc == 0, err[-3000:]
