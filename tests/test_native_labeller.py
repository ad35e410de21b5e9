"""The native labeller (`mi355x-node-labeller`, native/src/daemon/node_labeller_main.cpp):
the node labeller as one C++ process. Its labels must equal the Python
labeller's (labeller/labels.py, the reference schema of
cmd/k8s-node-labeller/main.go:123-505) on every generated node layout, and
its apiserver loop follows the Python controller: merge PATCH, GET + PUT when
RBAC denies patch, a watch that restores stripped labels, rotated tokens,
TLS with the cluster CA, SIGTERM."""
import json
import os
import signal
import subprocess
import sys
import time

import pytest

from rocm_k8s_device_plugin_amd import constants as C
from rocm_k8s_device_plugin_amd.labeller import labels as L
from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
from rocm_k8s_device_plugin_amd.testing.fake_apiserver import FakeApiServer
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node

# MI355X_NATIVE_LABELLER_EXE: run against another build (e.g. the sanitizer builds)
EXE = os.environ.get("MI355X_NATIVE_LABELLER_EXE") or os.path.join(str(PKG_DIR), "bin", "mi355x-node-labeller")
KINDS = C.SUPPORTED_LABELS + L.EXTRA_LABELS


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} was not built")


def _dry_run(fi, kinds, driver_type=""):
    argv = [EXE, "-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev)] + [f"-{k}" for k in kinds]
    if driver_type:
        argv += ["-driver_type", driver_type]
    p = subprocess.run(argv, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    return p.stdout


def _python(fi, kinds, driver_type=""):
    return L.generate_labels({k: k in kinds for k in KINDS}, driver_type, str(fi.sysfs), str(fi.dev))


LAYOUTS = {
    "spx": dict(),
    "cpx": dict(compute_partition="cpx"),
    "qpx_nps2": dict(compute_partition="qpx", memory_partition="nps2"),
    "dpx": dict(compute_partition="dpx"),
    "two_hives": dict(hive_size=4),
    "mixed_partitions": dict(per_gpu_compute=["spx"] * 4 + ["cpx"] * 4),
    "no_partition_support": dict(partition_support=False),
    "vf": dict(mode="vf", vfs_per_gpu=2),
    "pf": dict(mode="pf"),
}


@pytest.mark.parametrize("layout", sorted(LAYOUTS))
def test_labels_equal_the_python_labeller(tmp_path, layout):
    fi = make_mi355x_node(tmp_path, **LAYOUTS[layout])
    for kinds in (KINDS, ["vram", "cu-count", "simd-count", "device-id", "family"], ["mode"], []):
        for dt in ("", "container", "vf-passthrough", "pf-passthrough"):
            out = _dry_run(fi, kinds, dt)
            want = _python(fi, kinds, dt)
            assert json.loads(out) == want, (layout, kinds, dt)
            # byte-identical to the Python CLI's json.dumps(indent=1, sort_keys=True)
            assert out == json.dumps(want, indent=1, sort_keys=True) + "\n"


def test_label_values_are_sanitised_like_the_python_labeller(tmp_path):
    fi = make_mi355x_node(tmp_path)
    card = fi.sysfs / "class/drm/card1/device"
    (card / "product_name").write_text("  AMD Instinct MI355X (OAM) / rev:A?" + "x" * 80 + "\n")
    mod = card / "driver/module"
    (mod / "version").write_text("6.12.12+build/meta\n")
    out = json.loads(_dry_run(fi, KINDS))
    assert out == _python(fi, KINDS)
    assert all(len(v) <= 63 for v in out.values())
    # a value that goes into a key ("<prefix>.<product name>" counters) must not make the
    # key invalid: the apiserver would reject the whole patch; such labels are dropped
    assert all(L.valid_label_key(k) and L.sanitize_label_value(v) == v for k, v in out.items())
    assert not [k for k in out if "OAM" in k]                # card1's counter key is dropped
    assert out["amd.com/gpu.product-name.AMD_Instinct_MI355X"] == "7"   # the other GPUs' is kept
    assert out["amd.com/gpu.vram.288G"] == "8"     # and the rest of the node's labels


def test_driver_version_fallbacks_equal_the_python_labeller(tmp_path):
    """No driver/module/version on the cards (amdgpu built in, the MI355X test
    host): /sys/module/amdgpu/version, then amd-smi (absent here), then the
    reference's empty value."""
    fi = make_mi355x_node(tmp_path)
    kinds = ["driver-version", "driver-src-version"]
    os.unlink(fi.sysfs / "bus/pci/drivers/amdgpu/module")
    out = json.loads(_dry_run(fi, kinds))
    assert out == _python(fi, kinds) and out["amd.com/gpu.driver-version"] == "6.12.12"
    (fi.sysfs / "module/amdgpu/version").unlink()
    out = json.loads(_dry_run(fi, kinds))
    assert out == _python(fi, kinds) and out["amd.com/gpu.driver-version"] == ""


@pytest.mark.parametrize("key,ok", [
    ("amd.com/gpu.vram", True), ("beta.amd.com/gpu.firmware.SMC.fw.12", True), ("gpu", True),
    ("amd.com/" + "x" * 63, True), ("amd.com/" + "x" * 64, False), ("amd.com/gpu.product-name.a/b", False),
    ("Amd.com/gpu", False), ("amd.com/", False), ("/gpu", False), ("amd..com/gpu", False),
    ("amd.com/gpu.name.A?", False), ("amd.com/-gpu", False), ("a" * 254 + "/x", False)])
def test_label_key_validation(key, ok):
    assert L.valid_label_key(key) is ok


def test_flags_follow_go_syntax(tmp_path):
    fi = make_mi355x_node(tmp_path)
    base = [EXE, "-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev)]
    p = subprocess.run(base + ["--vram=true", "-cu-count=false", "-v=5", "-logtostderr"], capture_output=True,
                       text=True, timeout=30)
    assert p.returncode == 0 and set(json.loads(p.stdout)) == {"amd.com/gpu.vram", "amd.com/gpu.vram.288G",
                                                               "beta.amd.com/gpu.vram", "beta.amd.com/gpu.vram.288G"}
    # the flag package's own errors exit 2 (with the usage); the labeller's validation exits 1
    for bad, rc in ((["-nope"], 2), (["-driver_type", "gim"], 1), (["-vram=maybe"], 2), (["-resync", "x"], 2),
                    (["-watch_timeout", "x"], 2), (["---vram"], 2), (["-resync"], 2)):
        p = subprocess.run(base + bad, capture_output=True, text=True, timeout=30)
        assert p.returncode == rc, (bad, p.returncode, p.stderr)
    # parsing stops at the first non-flag argument and after "--", as Go's does
    for tail in (["extra", "-nope"], ["--", "-nope"]):
        p = subprocess.run(base + ["-vram"] + tail, capture_output=True, text=True, timeout=30)
        assert p.returncode == 0 and "amd.com/gpu.vram" in json.loads(p.stdout), (tail, p.stderr)
    p = subprocess.run([EXE, "-h"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 0 and "-compute-memory-partition" in p.stdout
    # an unreadable kubeconfig, no cluster env -> clear errors
    env = {k: v for k, v in os.environ.items() if k not in ("KUBERNETES_SERVICE_HOST", "DS_NODE_NAME", "KUBECONFIG")}
    p = subprocess.run([EXE, "-node_name", "n", "-kubeconfig", "/x"], capture_output=True, text=True, timeout=30,
                       env=env)
    assert p.returncode == 1 and "kubeconfig" in p.stderr
    p = subprocess.run([EXE, "-node_name", "n", "-sa_dir", str(tmp_path)], capture_output=True, text=True, timeout=30,
                       env=env)
    assert p.returncode == 1 and "KUBERNETES_SERVICE_HOST" in p.stderr
    p = subprocess.run([EXE], capture_output=True, text=True, timeout=30, env=env)
    assert p.returncode == 1 and "node name" in p.stderr


def _wait(pred, timeout=30.0):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(0.02)
    return pred()


def _start(fi, srv, tmp_path, *extra, token="tok", node="node-n", stderr=subprocess.PIPE):
    tok = tmp_path / "token"
    tok.write_text(token + "\n")
    argv = [EXE, "-node_name", node, "-apiserver", srv.url, "-token_file", str(tok), "-sysfs_root", str(fi.sysfs),
            "-dev_root", str(fi.dev), "-vram", "-cu-count", "-mode", "-device-id", "-compute-memory-partition",
            *extra]
    return subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=stderr, text=True), tok


def _stop(p):
    if p.poll() is None:
        p.send_signal(signal.SIGTERM)
    out, err = p.communicate(timeout=20)
    return p.returncode, err


def test_once_applies_and_exits(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", compute_partition="cpx")
    srv = FakeApiServer(token="tok").start()
    try:
        srv.add_node("node-n", {"amd.com/gpu.vram": "1G", "beta.amd.com/gpu.vram": "1G",
                                "beta.amd.com/gpu.vram.1G": "8", "keep": "me"})
        p, _ = _start(fi, srv, tmp_path, "-once")
        assert p.wait(30) == 0, p.stderr.read()
        want = L.generate_labels({k: k in ("vram", "cu-count", "mode", "device-id", "compute-memory-partition")
                                  for k in KINDS}, "", str(fi.sysfs), str(fi.dev))
        got = srv.labels("node-n")
        assert got == {**want, "keep": "me"}
        assert [m for m, *_ in srv.requests] == ["GET", "PATCH"]
        assert srv.requests[1][2]["metadata"]["labels"]["beta.amd.com/gpu.vram.1G"] is None
    finally:
        srv.stop()


def test_resync_zero_is_the_reference_controller(tmp_path):
    """-resync 0 behaves like the reference's controller (main.go:553-586):
    labels at start, keeps running, relabels a re-created Node (ADDED), and does
    not re-assert on other edits (its predicate drops Update events)."""
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok").start()
    try:
        srv.add_node("node-n")
        p, _ = _start(fi, srv, tmp_path, "-resync", "0")
        assert _wait(lambda: srv.labels("node-n").get("amd.com/gpu.mode") == "container", 10), p.stderr
        assert _wait(lambda: srv.watch_starts >= 1, 30.0)
        srv.set_labels("node-n", {"other": "x"})            # an edit strips them: not re-asserted
        time.sleep(1.5)
        assert "amd.com/gpu.mode" not in srv.labels("node-n") and p.poll() is None
        srv.delete_node("node-n")
        srv.add_node("node-n")                              # the node object is re-created: relabelled
        assert _wait(lambda: srv.labels("node-n").get("amd.com/gpu.mode") == "container", 30.0)
        rc, err = _stop(p)
        assert rc == 0, err
    finally:
        srv.stop()


def test_watch_restores_stripped_labels_and_survives_expiry(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok").start()
    p = None
    try:
        srv.add_node("node-n")
        p, _ = _start(fi, srv, tmp_path, "-resync", "300", "-topology_watch", "0")
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-n"))
        assert _wait(lambda: srv.watch_starts >= 1)
        t0 = time.monotonic()
        srv.set_labels("node-n", {"other": "x"})               # someone strips ours
        # from the watch event, not the 300 s resync (bounded loosely: a loaded CI host)
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-n"), 60.0)
        assert time.monotonic() - t0 < 60.0 and srv.labels("node-n")["other"] == "x"
        srv.expire_watches()                                     # server ends the stream: reconnect
        assert _wait(lambda: srv.watch_starts >= 2, 30.0)
        srv.delete_node("node-n")
        srv.add_node("node-n")                                   # re-created node
        assert _wait(lambda: "amd.com/gpu.cu-count" in srv.labels("node-n"), 30.0)
        # no reconnect spin when the server cuts every watch at once
        srv.watch_max_s = 0.0
        srv.expire_watches()
        n0 = srv.watch_starts
        time.sleep(1.5)
        assert srv.watch_starts - n0 <= 10, srv.watch_starts - n0
        rc, err = _stop(p)
        assert rc == 0 and "shutting down" in err
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        srv.stop()


def test_watch_from_a_compacted_resource_version_relists(tmp_path):
    """A watch resumed from a compacted resourceVersion gets a 410 ERROR event:
    the labeller re-lists (a reconcile: GET of the node) and watches again
    without a resourceVersion, so later edits are still seen."""
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok").start()
    p = None
    try:
        srv.add_node("node-n")
        p, _ = _start(fi, srv, tmp_path, "-resync", "300", "-topology_watch", "0", "-watch_backoff_max", "0.2")
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-n"))
        assert _wait(lambda: srv.watch_starts >= 1)

        def gets():
            return sum(1 for m, path, _ in list(srv.requests) if m == "GET")

        gets0, starts = gets(), srv.watch_starts
        srv.min_rv = 10 ** 6
        srv.expire_watches()                       # reconnects from its last resourceVersion: 410
        assert _wait(lambda: srv.watch_starts >= starts + 2, 30.0)
        srv.min_rv = 0
        watches = [path for m, path, _ in list(srv.requests) if m == "WATCH"][starts:]
        assert "resourceVersion=" in watches[0]    # the resumed watch
        assert _wait(lambda: gets() > gets0, 3.0)  # the re-list
        assert any("resourceVersion=" not in w for w in watches[1:]), watches
        srv.set_labels("node-n", {"other": "x"})   # the fresh watch still restores stripped labels
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-n"), 30.0)
        rc, err = _stop(p)
        assert rc == 0, err
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        srv.stop()


def test_update_fallback_when_patch_is_forbidden(tmp_path):
    """The upstream ClusterRole grants update, not patch: GET + PUT (controller.go:23-58)."""
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok").start()
    try:
        srv.add_node("node-n", {"amd.com/gpu.family": "AI", "keep": "me"})
        srv.forbid = {"PATCH"}
        p, _ = _start(fi, srv, tmp_path, "-once")
        assert p.wait(30) == 0, p.stderr.read()
        got = srv.labels("node-n")
        assert got["amd.com/gpu.vram"] == "288G" and got["keep"] == "me" and "amd.com/gpu.family" not in got
        assert [m for m, *_ in srv.requests] == ["GET", "PATCH", "GET", "PUT"]
    finally:
        srv.stop()


def test_rotated_token_is_picked_up(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok").start()
    p = None
    try:
        srv.add_node("node-n")
        p, tok = _start(fi, srv, tmp_path, "-resync", "0.5", "-watch=false", "-topology_watch", "0")
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-n"))
        srv.token = "tok-2"                       # the server moves on; the file follows
        tok.write_text("tok-2\n")
        os.utime(tok, ns=(time.time_ns(), time.time_ns() + 10**9))
        srv.set_labels("node-n", {})
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-n"), 30.0)
        rc, err = _stop(p)
        assert rc == 0 and "HTTP 401" not in err
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        srv.stop()


def test_topology_change_relabels(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok").start()
    p = None
    try:
        srv.add_node("node-n")
        p, _ = _start(fi, srv, tmp_path, "-resync", "300", "-watch=false", "-topology_watch", "0.2")
        assert _wait(lambda: srv.labels("node-n").get("amd.com/gpu.compute-memory-partition") == "spx_nps1")
        # a partition switch: every GPU's mode file changes (the generated tree keeps the kfd side)
        drv = fi.sysfs / "module/amdgpu/drivers/pci:amdgpu"
        for b in sorted(x for x in os.listdir(drv) if ":" in x):
            (drv / b / "current_memory_partition").write_text("NPS2\n")
        assert _wait(lambda: srv.labels("node-n").get("amd.com/gpu.compute-memory-partition") == "spx_nps2", 30.0)
        rc, err = _stop(p)
        assert rc == 0 and "topology_changes=1" in err
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        srv.stop()


def test_in_cluster_over_ipv6(tmp_path):
    """An IPv6 cluster: KUBERNETES_SERVICE_HOST=::1 becomes https://[::1]:port
    (net.JoinHostPort, as client-go builds it) and the certificate is checked
    against the IP; -apiserver takes a bracketed URL too."""
    import socket
    try:
        socket.socket(socket.AF_INET6).bind(("::1", 0))
    except OSError:
        pytest.skip("no IPv6 loopback")
    from rocm_k8s_device_plugin_amd.testing.fake_apiserver import tls_material as _tls_material
    crt, key, ca = _tls_material(tmp_path)
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="sa-token", tls=(crt, key), host="::1").start()
    plain = FakeApiServer(token=None, host="::1").start()
    try:
        srv.add_node("worker-6")
        plain.add_node("worker-6")
        sa = tmp_path / "sa"
        sa.mkdir()
        (sa / "token").write_text("sa-token\n")
        (sa / "ca.crt").write_text(open(ca).read())
        env = dict(os.environ, KUBERNETES_SERVICE_HOST="::1", KUBERNETES_SERVICE_PORT=str(srv.port),
                   DS_NODE_NAME="worker-6")
        base = [EXE, "-once", "-mode", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev)]
        p = subprocess.run(base + ["-sa_dir", str(sa)], capture_output=True, text=True, timeout=60, env=env)
        assert p.returncode == 0, p.stderr
        assert srv.labels("worker-6")["amd.com/gpu.mode"] == "container"
        assert plain.url.startswith("http://[::1]:")
        p = subprocess.run(base + ["-node_name", "worker-6", "-apiserver", plain.url, "-token_file", os.devnull],
                           capture_output=True, text=True, timeout=60,
                           env={k: v for k, v in os.environ.items() if not k.startswith("KUBERNETES_")})
        assert p.returncode == 0, p.stderr
        assert plain.labels("worker-6")["amd.com/gpu.mode"] == "container"
    finally:
        srv.stop()
        plain.stop()


def test_in_cluster_https_with_the_cluster_ca(tmp_path, monkeypatch):
    from rocm_k8s_device_plugin_amd.testing.fake_apiserver import tls_material as _tls_material
    crt, key, ca = _tls_material(tmp_path)
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="sa-token", tls=(crt, key)).start()
    try:
        srv.add_node("worker-9")
        sa = tmp_path / "sa"
        sa.mkdir()
        (sa / "token").write_text("sa-token\n")
        (sa / "ca.crt").write_text(open(ca).read())
        env = dict(os.environ, KUBERNETES_SERVICE_HOST="127.0.0.1", KUBERNETES_SERVICE_PORT=str(srv.port),
                   DS_NODE_NAME="worker-9")
        argv = [EXE, "-sa_dir", str(sa), "-once", "-mode", "-cu-count", "-sysfs_root", str(fi.sysfs),
                "-dev_root", str(fi.dev)]
        p = subprocess.run(argv, capture_output=True, text=True, timeout=60, env=env)
        assert p.returncode == 0, p.stderr
        got = srv.labels("worker-9")
        assert got["amd.com/gpu.mode"] == "container" and got["amd.com/gpu.cu-count"] == "256"
        # a CA that did not sign the server certificate is refused (retried, never applied)
        other = tmp_path / "other"
        other.mkdir()
        _, _, bad_ca = _tls_material(other)
        (sa / "ca.crt").write_text(open(bad_ca).read())
        srv.set_labels("worker-9", {})
        p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
        time.sleep(1.0)
        rc, err = _stop(p)
        assert rc == 0 and "certificate verify failed" in err and srv.labels("worker-9") == {}
    finally:
        srv.stop()


@pytest.mark.gpu
def test_real_node_labels_equal_the_python_labeller():
    """On the MI355X box's own /sys and /dev (libdrm family/firmware, amd-smi
    driver version and xGMI links, kfd-denied GPUs): the same labels as the
    Python labeller, and the process cost of one labelling pass."""
    t0 = time.monotonic()
    p = subprocess.Popen([EXE, "-dry_run", *[f"-{k}" for k in KINDS]], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    out, err = p.communicate(timeout=120)
    wall_ms = (time.monotonic() - t0) * 1e3
    assert p.returncode == 0, err
    assert "ERROR: AddressSanitizer" not in err and "runtime error:" not in err, err[-3000:]
    got = json.loads(out)
    want = L.generate_labels({k: True for k in KINDS}, "")
    assert got == want
    assert got["amd.com/gpu.family"] == "AI" and got["amd.com/gpu.gfx-target"] == "gfx950"
    # counts against the raw sysfs, not only the twin: every amdgpu PCI function is
    # counted in device-id, and in vram / cu-count / simd-count too (kfd-denied
    # GPUs from PCI sysfs); the readable kfd GPU nodes are a subset
    pci = [b for b in os.listdir("/sys/module/amdgpu/drivers/pci:amdgpu") if b.count(":") == 2]
    readable = []
    for n in os.listdir("/sys/class/kfd/kfd/topology/nodes"):
        try:
            with open(f"/sys/class/kfd/kfd/topology/nodes/{n}/properties") as f:
                props = dict(ln.split() for ln in f if len(ln.split()) == 2)
        except OSError:
            continue
        if props.get("cpu_cores_count") == "0" and int(props.get("gfx_target_version", "0")) > 0:
            readable.append(n)
    spx = got.get("amd.com/gpu.compute-memory-partition", "").startswith("spx")
    if spx:
        dev_key = next(k for k in got if k.startswith("amd.com/gpu.device-id."))
        assert int(got[dev_key]) == len(pci), (got[dev_key], pci)
        for kind in ("vram", "cu-count", "simd-count"):
            counts = [int(v) for k, v in got.items() if k.startswith(f"amd.com/gpu.{kind}.")]
            assert sum(counts) == len(pci), (kind, counts, len(pci))
    assert 1 <= len(readable) <= len(pci), (readable, pci)
    # the Python CLI's cost for the same pass, for the footprint comparison
    t1 = time.monotonic()
    py = subprocess.run([sys.executable, "-m", "rocm_k8s_device_plugin_amd.cli.node_labeller", "-dry_run",
                         *[f"-{k}" for k in KINDS]], capture_output=True, text=True, timeout=120)
    py_ms = (time.monotonic() - t1) * 1e3
    assert py.returncode == 0 and json.loads(py.stdout) == got
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/native_labeller_box.json", "w") as f:
        json.dump({"labels": got, "pci_amdgpu_functions": len(pci), "readable_kfd_gpu_nodes": len(readable),
                   "native_dry_run_wall_ms": round(wall_ms, 1),
                   "python_cli_dry_run_wall_ms": round(py_ms, 1)}, f, indent=1)


def test_malformed_watch_events_are_survived(tmp_path):
    """Garbage, truncated and hostile JSON on the watch stream (random bytes,
    deep nesting, huge numbers, bad escapes) neither crashes nor wedges the
    labeller: a later real event still relabels the node."""
    import random
    rng = random.Random(7)
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok").start()
    p = None
    try:
        srv.add_node("node-n")
        p, _ = _start(fi, srv, tmp_path, "-resync", "300", "-topology_watch", "0")
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-n"))
        assert _wait(lambda: srv.watch_starts >= 1)
        good = json.dumps({"type": "MODIFIED", "object": {"metadata": {"name": "node-n", "labels": {}}}})
        samples = [b"{", b"}", b"[]", b"null", b"\"x\"", b"{\"type\":", b"{\"type\": \"MODIFIED\", \"object\": 7}",
                   b"{\"type\": \"ERROR\", \"object\": {\"code\": \"x\"}}", b"[" * 5000, b"{\"a\": 1e999999}",
                   b"{\"a\": \"\\ud800\\u\"}", b"{\"a\": \"\\q\"}", b"\xff\xfe\x00garbage"]
        for _ in range(60):
            cut = rng.randrange(1, len(good))
            samples.append(good[:cut].encode())
            samples.append(bytes(rng.randrange(256) for _ in range(rng.randrange(1, 200))))
        for s in samples:
            srv.send_raw_event("node-n", s.replace(b"\n", b" ") + b"\n")
        time.sleep(0.5)
        assert p.poll() is None
        srv.set_labels("node-n", {})
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-n"), 30.0)
        rc, err = _stop(p)
        assert rc == 0, err
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        srv.stop()


def test_no_leaks_under_connection_churn(tmp_path):
    """Hundreds of TLS connections (resync every 0.1 s, watches cut every
    0.1 s, labels stripped every 0.2 s): open fds and RSS stay flat (and the
    ASan build's leak check at exit stays clean)."""
    from rocm_k8s_device_plugin_amd.testing.fake_apiserver import tls_material as _tls_material
    crt, key, ca = _tls_material(tmp_path)
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok", tls=(crt, key)).start()
    p = None
    try:
        srv.add_node("node-n")
        p, _ = _start(fi, srv, tmp_path, "-resync", "0.1", "-topology_watch", "0.1", "-ca_file", ca,
                      "-watch_backoff_max", "0.1")
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-n"), 30.0)

        def sample():
            """(fds, RSS KiB), each the least of a few readings once the labels are back:
            a connection in flight at one reading is not a leak, a leaked one stays"""
            _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-n"), 30.0)
            rows = []
            for _ in range(5):
                with open(f"/proc/{p.pid}/status") as f:
                    rss = next(int(x.split()[1]) for x in f if x.startswith("VmRSS"))
                rows.append((len(os.listdir(f"/proc/{p.pid}/fd")), rss))
                time.sleep(0.05)
            return min(r[0] for r in rows), min(r[1] for r in rows)

        def churn(requests, cap_s=120.0):
            """Strip the labels and cut the watch until the labeller has made `requests`
            more API requests: a fixed amount of reconnecting, however loaded the machine"""
            target = len(srv.requests) + requests
            end = time.monotonic() + cap_s
            while len(srv.requests) < target:
                assert time.monotonic() < end, f"{len(srv.requests)} of {target} requests after {cap_s} s"
                srv.set_labels("node-n", {})
                time.sleep(0.1)
                srv.expire_watches()
                time.sleep(0.1)

        churn(40)
        fds0, rss0 = sample()
        churn(150)
        fds1, rss1 = sample()
        assert fds1 <= fds0 + 1, (fds0, fds1)
        if "MI355X_NATIVE_LABELLER_EXE" not in os.environ:   # ASan's quarantine holds freed memory by design
            assert rss1 - rss0 < 2048, (rss0, rss1)           # KiB
        rc, err = _stop(p)
        assert rc == 0, err[-2000:]
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        srv.stop()


def test_resync_patches_only_changes_and_survives_apiserver_errors(tmp_path):
    """The reconcile contract (reference controller.go:23-58, as the resync runs
    it): stale kinds removed and ours set in one PATCH, nothing written while the
    node already carries the labels, a deleted label re-asserted at the next
    resync, a 500 from the apiserver retried rather than fatal."""
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok").start()
    p = None
    try:
        srv.add_node("node-n", {"amd.com/gpu.family": "stale", "beta.amd.com/gpu.family": "stale",
                                "beta.amd.com/gpu.family.stale": "8", "kubernetes.io/hostname": "node-n"})
        p, _ = _start(fi, srv, tmp_path, "-resync", "0.2", "-watch=false", "-topology_watch", "0")
        assert _wait(lambda: srv.labels("node-n").get("amd.com/gpu.vram") == "288G")
        got = srv.labels("node-n")
        assert got["kubernetes.io/hostname"] == "node-n"
        assert "amd.com/gpu.family" not in got and "beta.amd.com/gpu.family.stale" not in got
        patches = lambda: sum(1 for r in srv.requests if r[0] == "PATCH")   # noqa: E731
        gets = lambda: sum(1 for r in srv.requests if r[0] == "GET")         # noqa: E731
        assert patches() == 1
        g0 = gets()
        assert _wait(lambda: gets() >= g0 + 3)            # three more resyncs: reads, no writes
        assert patches() == 1
        srv.nodes["node-n"]["metadata"]["labels"].pop("amd.com/gpu.vram")
        assert _wait(lambda: srv.labels("node-n").get("amd.com/gpu.vram") == "288G")
        assert patches() == 2
        srv.fail_next = 2                                  # the next resyncs get 500s
        g1 = gets()
        assert _wait(lambda: gets() >= g1 + 3)
        srv.nodes["node-n"]["metadata"]["labels"].pop("amd.com/gpu.mode")
        assert _wait(lambda: srv.labels("node-n").get("amd.com/gpu.mode") == "container")
        assert p.poll() is None
        rc, err = _stop(p)
        assert rc == 0, err[-2000:]
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        srv.stop()


def test_unauthorized_token_and_missing_node_are_retried(tmp_path):
    """401 (a wrong or expired token) and 404 (the node object not created yet)
    are not fatal: the labeller keeps trying and labels the node once the
    token is right and the node exists."""
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok").start()
    p = None
    try:
        log = tmp_path / "labeller.log"
        p, tok = _start(fi, srv, tmp_path, "-resync", "0.2", "-watch=false", "-topology_watch", "0", token="bad",
                        stderr=open(log, "w"))
        assert _wait(lambda: len(srv.requests) >= 2)       # refused, and tried again
        assert p.poll() is None and not srv.nodes
        n401 = len(srv.requests)
        tok.write_text("tok\n")                            # a rotated, now valid token
        assert _wait(lambda: len(srv.requests) > n401)     # the next try is let in: 404, no node yet
        assert _wait(lambda: "not found" in open(log).read() or "404" in open(log).read())
        assert p.poll() is None                            # still running
        srv.add_node("node-n")
        assert _wait(lambda: srv.labels("node-n").get("amd.com/gpu.vram") == "288G")
        rc, _ = _stop(p)
        err = open(log).read()
        assert rc == 0, err[-2000:]
        assert "401" in err or "Unauthorized" in err, err[-2000:]
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        srv.stop()


def test_kubeconfig_with_embedded_ca_and_token_over_https(tmp_path):
    """-kubeconfig as kubectl writes it: https server, certificate-authority-data,
    a token user, current-context; the labeller verifies the server with that CA."""
    import base64
    from rocm_k8s_device_plugin_amd.testing.fake_apiserver import tls_material as _tls_material
    crt, key, ca = _tls_material(tmp_path)
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="abc", tls=(crt, key)).start()
    p = None
    try:
        srv.add_node("node-k")
        ca_data = base64.b64encode(open(ca, "rb").read()).decode()
        kc = tmp_path / "kubeconfig"
        kc.write_text(f"""apiVersion: v1
kind: Config
current-context: c1
clusters:
- name: k1
  cluster: {{server: "{srv.url}/", certificate-authority-data: "{ca_data}"}}
- name: other
  cluster: {{server: "https://10.9.9.9:6443"}}
contexts:
- name: c0
  context: {{cluster: other, user: u1}}
- name: c1
  context: {{cluster: k1, user: u1}}
users:
- name: u1
  user: {{token: abc}}
""")
        p = subprocess.Popen([EXE, "-node_name", "node-k", "-kubeconfig", str(kc), "-once", "-vram", "-mode",
                              "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev)],
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        assert p.wait(60) == 0, p.stderr.read()[-2000:]
        got = srv.labels("node-k")
        assert got["amd.com/gpu.vram"] == "288G" and got["amd.com/gpu.mode"] == "container"
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        srv.stop()


def test_metrics_port_health_and_readiness(tmp_path):
    """-metrics_port (an addition; the reference's labeller serves nothing): /readyz is 503 while the node cannot
    be labelled (it does not exist yet) and 200 once a reconcile succeeded; /healthz is 200 while the controller
    loop runs; /metrics counts the reconciles by result and the patches."""
    import socket
    import urllib.error
    import urllib.request

    def get(port, path):
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=5) as r:
                return r.status, r.read().decode()
        except urllib.error.HTTPError as e:
            return e.code, e.read().decode()
        except OSError:
            return 0, ""

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok").start()
    p = None
    try:
        log = tmp_path / "labeller.log"
        p, _ = _start(fi, srv, tmp_path, "-resync", "0.5", "-watch=false", "-topology_watch", "0",
                      "-metrics_port", str(port), stderr=open(log, "w"))
        assert _wait(lambda: get(port, "/healthz")[0] == 200)
        assert _wait(lambda: len(srv.requests) >= 1)                 # a reconcile ran: 404, no node yet
        assert get(port, "/readyz") == (503, "node labels not reconciled yet (see the log)\n")
        srv.add_node("node-n")
        assert _wait(lambda: get(port, "/readyz")[0] == 200)
        assert srv.labels("node-n").get("amd.com/gpu.vram") == "288G"
        status, text = get(port, "/metrics")
        assert status == 200
        series = {ln.rsplit(" ", 1)[0]: float(ln.rsplit(" ", 1)[1]) for ln in text.splitlines()
                  if ln and not ln.startswith("#")}
        assert series['mi355x_labeller_reconciles_total{result="error"}'] >= 1
        assert series['mi355x_labeller_reconciles_total{result="ok"}'] >= 1
        assert series["mi355x_labeller_patches_total"] == 1
        rc, _ = _stop(p)
        assert rc == 0, open(log).read()[-2000:]
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        srv.stop()


def test_metrics_port_flag_syntax(tmp_path):
    p = subprocess.run([EXE, "-metrics_port", "x"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 2 and 'invalid value "x" for flag -metrics_port' in p.stderr


def test_metrics_port_in_use_is_an_error(tmp_path):
    """A -metrics_port that cannot be bound is a start-up error (exit 1), as in the device plugin."""
    import socket
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="tok").start()
    try:
        srv.add_node("node-n")
        with socket.socket() as s:
            s.bind(("0.0.0.0", 0))
            s.listen(1)
            p, _ = _start(fi, srv, tmp_path, "-metrics_port", str(s.getsockname()[1]))
            rc = p.wait(30)
            err = p.stderr.read()
        assert rc == 1 and "cannot serve /metrics" in err, err[-2000:]
    finally:
        if p.poll() is None:
            p.kill()
        srv.stop()
