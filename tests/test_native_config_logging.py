"""glog behaviour and kubeconfig handling of the native binaries.

glog (vendor/github.com/golang/glog/glog_flags.go:388-397, glog_file.go): the
reference binaries honour -v, -vmodule, -logtostderr=false + -log_dir (one
file per severity, <program>.<SEV> symlinks), -stderrthreshold and
-alsologtostderr; a DaemonSet that sets them must not lose its logs when it
switches to mi355x-device-plugin / mi355x-node-labeller.

kubeconfig (vendor/sigs.k8s.io/controller-runtime/pkg/client/config/
config.go:32-58,116-156): -kubeconfig, else in-cluster unless $KUBECONFIG is
set, else $KUBECONFIG; token, tokenFile (relative to the file) and
client-certificate auth, CA from a file or inline data, block or flow YAML.
"""
import base64
import os
import signal
import socket
import subprocess
import threading
import time

import pytest

from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
from rocm_k8s_device_plugin_amd.testing import gopeer as gp
from rocm_k8s_device_plugin_amd.testing.fake_apiserver import FakeApiServer
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node

DP = os.environ.get("MI355X_NATIVE_DAEMON_EXE") or os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")
LBL = os.environ.get("MI355X_NATIVE_LABELLER_EXE") or os.path.join(str(PKG_DIR), "bin", "mi355x-node-labeller")


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("KUBERNETES_SERVICE_HOST", "KUBERNETES_SERVICE_PORT", "KUBECONFIG", "DS_NODE_NAME")
           and k.lower() not in ("https_proxy", "http_proxy", "no_proxy")}
    env.update(kw)
    return env


def _wait(pred, timeout=10.0):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(0.02)
    return pred()


def _term(p, timeout=20):
    if p.poll() is None:
        p.send_signal(signal.SIGTERM)
    _, err = p.communicate(timeout=timeout)
    return p.returncode, err


# ------------------------------------------------------------------ glog

def test_device_plugin_log_files_per_severity(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    logs = tmp_path / "logs"
    kdir = tmp_path / "dp"
    kdir.mkdir()
    kub = gp.GoServer(str(kdir / "kubelet.sock"), {"/v1beta1.Registration/Register": lambda m: (0, "", b"")})
    p = subprocess.Popen([DP, "-kubelet_dir", str(kdir), "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                          "-exporter_socket", "", "-logtostderr=false", f"-log_dir={logs}", "-vmodule",
                          "daemon=2", "-grpc_watchdog", "0", f"-log_link={tmp_path}",
                          "-logbuflevel=-1"],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        assert _wait(lambda: (logs / "k8s-device-plugin.INFO").exists() and
                     "Registration for endpoint" in (logs / "k8s-device-plugin.INFO").read_text())
        c = gp.GoClientConn(str(kdir / "amd.com_gpu"))
        try:
            assert c.unary("/v1beta1.DevicePlugin/GetDevicePluginOptions", b"", 3.0)[0] == 0
            a = c.unary("/v1beta1.DevicePlugin/Allocate", b"\x0a\x00", 3.0)    # one empty container request
            assert a[0] == 0
        finally:
            c.close()
        # -vmodule=daemon=2: per-RPC lines without -v
        assert _wait(lambda: "rpc rpc=GetDevicePluginOptions resource=gpu latency_ms="
                     in (logs / "k8s-device-plugin.INFO").read_text())
    finally:
        rc, err = _term(p)
        kub.close()
    assert rc == 0
    info = (logs / "k8s-device-plugin.INFO").read_text()
    target = os.readlink(logs / "k8s-device-plugin.INFO")
    assert target.startswith("k8s-device-plugin.") and ".log.INFO." in target and target.endswith(f".{p.pid}")
    assert info.startswith("Log file created at:") and "Log line format: [IWEF]mmdd" in info
    # -log_link: a second link, to the full path (glog_file.go:133-137); -logbuflevel accepted
    assert os.readlink(tmp_path / "k8s-device-plugin.INFO") == str(logs / target)
    assert "Found 8 AMDGPUs" in info and "Received signal, shutting down." in info
    assert "Found 8 AMDGPUs" not in err                     # INFO stays out of stderr (-stderrthreshold=ERROR)
    assert not (logs / "k8s-device-plugin.ERROR").exists()  # created on first use only


def test_labeller_log_files_threshold_and_alsologtostderr(tmp_path):
    logs = tmp_path / "logs"
    base = [LBL, "-node_name", "n", "-apiserver", "http://127.0.0.1:9", "-token_file", os.devnull, "-mode",
            "-logtostderr=false", f"-log_dir={logs}", "-sysfs_root", str(tmp_path)]
    p = subprocess.Popen(base + ["-once"], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, env=_env())
    assert _wait(lambda: (logs / "k8s-node-labeller.ERROR").exists())
    rc, err = _term(p)
    assert rc == 0
    errs = (logs / "k8s-node-labeller.ERROR").read_text()
    info = (logs / "k8s-node-labeller.INFO").read_text()
    assert "reconcile of node n failed" in errs and "reconcile of node n failed" in info
    assert "AMD GPU Node Labeller" in info and "AMD GPU Node Labeller" not in errs
    assert "reconcile of node n failed" in err and "AMD GPU Node Labeller" not in err
    # -alsologtostderr: INFO on stderr too; -stderrthreshold=INFO without files: same
    p = subprocess.Popen(base + ["-once", "-alsologtostderr", f"-log_dir={tmp_path / 'l2'}"],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, env=_env())
    time.sleep(0.5)
    rc, err = _term(p)
    assert "AMD GPU Node Labeller" in err and (tmp_path / "l2" / "k8s-node-labeller.INFO").exists()
    # a malformed -vmodule is refused, like glog
    p = subprocess.run([LBL, "-dry_run", "-vmodule", "nolevel"], capture_output=True, text=True, timeout=20)
    assert p.returncode == 1 and "vmodule" in p.stderr


def test_stderrthreshold_names_numbers_and_backtrace_at(tmp_path):
    """glog's severity flag takes a name in any case or a number
    (vendor/github.com/golang/glog/glog.go severity.Set); -log_backtrace_at=FILE:N
    appends a stack trace to the record logged at that line."""
    fi = make_mi355x_node(tmp_path / "n")
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "native", "src", "daemon",
                       "resources.cpp")
    with open(src) as f:
        line = next(i + 1 for i, s in enumerate(f) if '"Found %zu AMDGPUs"' in s)
    base = [DP, "-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-exporter_socket="]
    # a number is a logsink.Severity (int8): 256 wraps to INFO, 259 to FATAL (glog_flags.go:341-356)
    for thr, info_on_stderr in (("warning", False), ("0", True), ("INFO", True), ("Error", False), ("2", False),
                                ("+1", False), ("256", True), ("259", False)):
        logs = tmp_path / f"logs-{thr}"
        p = subprocess.run(base + ["-logtostderr=false", f"-log_dir={logs}", f"-stderrthreshold={thr}"],
                           capture_output=True, text=True, timeout=30)
        assert p.returncode == 0, p.stderr
        assert ("Found 8 AMDGPUs" in p.stderr) == info_on_stderr, thr
        assert "Found 8 AMDGPUs" in (logs / "k8s-device-plugin.INFO").read_text()
    bad = subprocess.run(base + ["-stderrthreshold=loud"], capture_output=True, text=True, timeout=30)
    assert bad.returncode == 2 and 'invalid value "loud" for flag -stderrthreshold' in bad.stderr
    # numbers outside INFO..FATAL are refused, as golang/glog refuses them
    for thr in ("-1", "7", "4", "255"):
        bad = subprocess.run(base + [f"-stderrthreshold={thr}"], capture_output=True, text=True, timeout=30)
        assert bad.returncode == 2 and f"Severity {thr} out of range (min 0, max 3)." in bad.stderr, (thr, bad.stderr)
    # -v is strconv.Atoi (64-bit) stored as an int32: 2^32+2 is level 2
    p = subprocess.run(base + ["-v", str(2 ** 32 + 2)], capture_output=True, text=True, timeout=30)
    assert p.returncode == 0, p.stderr
    p = subprocess.run(base + ["-v", str(2 ** 63)], capture_output=True, text=True, timeout=30)
    assert p.returncode == 2 and "for flag -v" in p.stderr
    # the stack follows exactly the record logged at resources.cpp:<line>, nowhere else
    p = subprocess.run(base + [f"-log_backtrace_at=resources.cpp:{line}"], capture_output=True, text=True,
                       timeout=30)
    assert p.returncode == 0, p.stderr
    out = p.stderr.splitlines()
    at = next(i for i, s in enumerate(out) if s.endswith(f"resources.cpp:{line}] Found 8 AMDGPUs"))
    assert out[at + 1].startswith("    ") and out[at + 2].startswith("    ")
    assert sum(1 for s in out if s.startswith("    ")) == sum(1 for s in out[at + 1:] if s.startswith("    "))
    for spec in ("nocolon", "resources.cpp:0", "resources.cpp:x"):
        q = subprocess.run(base + [f"-log_backtrace_at={spec}"], capture_output=True, text=True, timeout=30)
        assert q.returncode != 0 and "log_backtrace_at" in q.stderr, (spec, q.returncode, q.stderr[-300:])


def test_json_log_format_in_both_binaries(tmp_path):
    """-log_format=json: one JSON object per record with the Python CLIs' keys
    (utils/log.py JsonFormatter) and structured fields as keys."""
    import json
    fi = make_mi355x_node(tmp_path / "n")
    kdir = tmp_path / "dp"
    kdir.mkdir()
    kub = gp.GoServer(str(kdir / "kubelet.sock"), {"/v1beta1.Registration/Register": lambda m: (0, "", b"")})
    p = subprocess.Popen([DP, "-kubelet_dir", str(kdir), "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                          "-exporter_socket", "", "-log_format=json", "-v", "2", "-grpc_watchdog", "0"],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        assert _wait(lambda: os.path.exists(kdir / "amd.com_gpu"))
        time.sleep(0.3)
        c = gp.GoClientConn(str(kdir / "amd.com_gpu"))
        try:
            assert c.unary("/v1beta1.DevicePlugin/GetDevicePluginOptions", b"", 3.0)[0] == 0
        finally:
            c.close()
        time.sleep(0.3)
    finally:
        rc, err = _term(p)
        kub.close()
    assert rc == 0
    recs = [json.loads(line) for line in err.splitlines() if line.strip()]
    assert recs and all(set(r) >= {"ts", "level", "src", "msg"} for r in recs)
    assert any(r["msg"] == "Found 8 AMDGPUs" and r["level"] == "INFO" and r["src"].startswith("resources.cpp:")
               for r in recs)
    rpc = [r for r in recs if r["msg"] == "rpc" and r.get("rpc") == "GetDevicePluginOptions"]
    assert rpc and rpc[0]["resource"] == "gpu" and float(rpc[0]["latency_ms"]) >= 0
    # the labeller: same format; a bad value is refused by both
    q = subprocess.Popen([LBL, "-node_name", "n", "-apiserver", "http://127.0.0.1:9", "-token_file", os.devnull,
                          "-mode", "-once", "-log_format", "json", "-sysfs_root", str(tmp_path)],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, env=_env())
    time.sleep(1.0)   # the apiserver is unreachable: -once keeps retrying
    _, lerr = _term(q)
    lrecs = [json.loads(line) for line in lerr.splitlines() if line.strip()]
    assert any("reconcile of node n failed" in r["msg"] and r["level"] == "ERROR" for r in lrecs)
    for exe in (DP, LBL):
        bad = subprocess.run([exe, "-log_format", "xml"], capture_output=True, text=True, timeout=20)
        # an unparsable flag value is the flag package's error: usage, exit 2
        assert bad.returncode == 2 and "log_format" in bad.stderr


# ------------------------------------------------------------------ kubeconfig

def _tls_material(d, client=False):
    import shutil
    if not shutil.which("openssl"):
        pytest.skip("openssl not installed")

    def run(*a):
        subprocess.run(["openssl", *a], check=True, capture_output=True, timeout=60)
    run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(d / "ca.key"), "-out", str(d / "ca.crt"),
        "-days", "2", "-subj", "/CN=test-ca")
    run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", str(d / "srv.key"), "-out", str(d / "srv.csr"),
        "-subj", "/CN=kubernetes")
    (d / "ext.cnf").write_text("subjectAltName=IP:127.0.0.1,DNS:kubernetes.default.svc\n")
    run("x509", "-req", "-in", str(d / "srv.csr"), "-CA", str(d / "ca.crt"), "-CAkey", str(d / "ca.key"),
        "-CAcreateserial", "-out", str(d / "srv.crt"), "-days", "2", "-extfile", str(d / "ext.cnf"))
    if client:
        run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", str(d / "cli.key"), "-out", str(d / "cli.csr"),
            "-subj", "/CN=system:node:worker/O=system:nodes")
        run("x509", "-req", "-in", str(d / "cli.csr"), "-CA", str(d / "ca.crt"), "-CAkey", str(d / "ca.key"),
            "-CAcreateserial", "-out", str(d / "cli.crt"), "-days", "2")


def _label_once(kc, fi, env=None, extra=()):
    argv = [LBL, "-node_name", "worker", "-once", "-mode", "-vram", "-sysfs_root", str(fi.sysfs), "-dev_root",
            str(fi.dev), *extra]
    if kc is not None:
        argv += ["-kubeconfig", str(kc)]
    return subprocess.run(argv, capture_output=True, text=True, timeout=60, env=env or _env())


def test_kubeconfig_token_file_relative_block_yaml(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="kc-token").start()
    try:
        srv.add_node("worker")
        d = tmp_path / "cfg"
        d.mkdir()
        (d / "tok").write_text("kc-token\n")
        kc = d / "config"
        kc.write_text(f"""# a kubeconfig as kubectl writes it
apiVersion: v1
kind: Config
clusters:
- cluster:
    server: "{srv.url}/"
  name: other
- name: lab
  cluster:
    server: {srv.url}
contexts:
- context:
    cluster: lab
    user: robot   # the labeller's identity
  name: lab-ctx
current-context: lab-ctx
preferences: {{}}
users:
- name: robot
  user:
    tokenFile: tok
""")
        p = _label_once(kc, fi)
        assert p.returncode == 0, p.stderr
        got = srv.labels("worker")
        assert got["amd.com/gpu.mode"] == "container" and got["amd.com/gpu.vram"] == "288G"
    finally:
        srv.stop()


def test_kubeconfig_flow_yaml_static_token_and_env_order(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="t0").start()
    try:
        srv.add_node("worker")
        kc = tmp_path / "kc"
        kc.write_text(f"clusters: [{{name: a, cluster: {{server: '{srv.url}'}}}}]\n"
                      "contexts: [{name: a, context: {cluster: a, user: a}}]\ncurrent-context: a\n"
                      "users: [{name: a, user: {token: t0}}]\n")
        assert _label_once(kc, fi).returncode == 0
        assert srv.labels("worker")["amd.com/gpu.mode"] == "container"
        # no flag, no in-cluster env: $KUBECONFIG (missing entries of the list skipped)
        srv.set_labels("worker", {})
        p = _label_once(None, fi, env=_env(KUBECONFIG=f"{tmp_path}/missing:{kc}"))
        assert p.returncode == 0, p.stderr and srv.labels("worker")["amd.com/gpu.mode"] == "container"
        # a JSON kubeconfig is YAML too
        kj = tmp_path / "kc.json"
        kj.write_text('{"clusters": [{"name": "a", "cluster": {"server": "%s"}}], "users": [{"name": "a", "user": '
                      '{"token": "t0"}}], "contexts": [{"name": "a", "context": {"cluster": "a", "user": "a"}}], '
                      '"current-context": "a"}' % srv.url)
        assert _label_once(kj, fi).returncode == 0
        # a wrong token: a clear error, retried (as the reference's controller retries)
        kc.write_text(kc.read_text().replace("token: t0", "token: nope"))
        p = subprocess.Popen([LBL, "-node_name", "worker", "-once", "-mode", "-sysfs_root", str(fi.sysfs),
                              "-kubeconfig", str(kc)], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                             env=_env())
        time.sleep(0.8)
        rc, err = _term(p)
        assert rc == 0 and "HTTP 401" in err
    finally:
        srv.stop()


@pytest.mark.parametrize("inline", [True, False])
def test_kubeconfig_client_certificate_over_tls(tmp_path, inline):
    """Client-certificate auth against an apiserver that requires it, the CA
    from certificate-authority-data (or a relative certificate-authority path)."""
    d = tmp_path / "pki"
    d.mkdir()
    _tls_material(d, client=True)
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token=None, tls=(str(d / "srv.crt"), str(d / "srv.key")), client_ca=str(d / "ca.crt")).start()
    try:
        srv.add_node("worker")
        b64 = lambda f: base64.b64encode((d / f).read_bytes()).decode()   # noqa: E731
        if inline:
            cluster = f"certificate-authority-data: {b64('ca.crt')}"
            user = f"client-certificate-data: {b64('cli.crt')}\n    client-key-data: {b64('cli.key')}"
        else:
            cluster = "certificate-authority: pki/ca.crt"
            user = "client-certificate: pki/cli.crt\n    client-key: pki/cli.key"
        kc = tmp_path / "kubeconfig"
        kc.write_text(f"""clusters:
- name: c
  cluster:
    server: {srv.url}
    {cluster}
contexts:
- name: x
  context: {{cluster: c, user: u}}
current-context: x
users:
- name: u
  user:
    {user}
""")
        p = _label_once(kc, fi)
        assert p.returncode == 0, p.stderr
        assert srv.labels("worker")["amd.com/gpu.vram"] == "288G"
        # without the client certificate the handshake is refused
        kc.write_text("\n".join(line for line in kc.read_text().splitlines() if "client-" not in line) + "\n")
        p = subprocess.Popen([LBL, "-node_name", "worker", "-once", "-mode", "-sysfs_root", str(fi.sysfs),
                              "-kubeconfig", str(kc)], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                             env=_env())
        time.sleep(1.0)
        rc, err = _term(p)
        assert "reconcile of node worker failed" in err
    finally:
        srv.stop()


_KC = """clusters:
- name: c
  cluster: {{server: "http://127.0.0.1:9"}}
contexts:
- name: x
  context: {{cluster: {cluster}, user: {user}}}
current-context: {ctx}
users:
- name: u
  user: {{{cred}}}
"""


def test_kubeconfig_list_is_merged_like_clientcmd(tmp_path):
    """$KUBECONFIG=a:b: current-context from the first file that sets it, each named
    entry from the first file naming it, relative paths against that entry's file."""
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="t0").start()
    try:
        srv.add_node("worker")
        (tmp_path / "a").mkdir()
        (tmp_path / "b").mkdir()
        (tmp_path / "a" / "tok").write_text("t0\n")
        ka, kb = tmp_path / "a" / "config", tmp_path / "b" / "config"
        ka.write_text("current-context: x\ncontexts: [{name: x, context: {cluster: c, user: u}}]\n"
                      "users: [{name: u, user: {tokenFile: tok}}]\n")
        kb.write_text(f"current-context: other\nclusters: [{{name: c, cluster: {{server: '{srv.url}'}}}}]\n"
                      "contexts: [{name: other, context: {cluster: c, user: v}}]\n"
                      "users: [{name: u, user: {token: nope}}, {name: v, user: {token: nope}}]\n")
        p = _label_once(None, fi, env=_env(KUBECONFIG=f"{ka}:{tmp_path}/missing:{kb}"))
        assert p.returncode == 0, p.stderr
        assert srv.labels("worker")["amd.com/gpu.mode"] == "container"
        # the other order: b's context and user win, whose token the apiserver refuses
        srv.set_labels("worker", {})
        proc = subprocess.Popen([LBL, "-node_name", "worker", "-once", "-mode", "-sysfs_root", str(fi.sysfs)],
                                stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                                env=_env(KUBECONFIG=f"{kb}:{ka}"))
        time.sleep(0.8)
        rc, err = _term(proc)
        assert "HTTP 401" in err and "amd.com/gpu.mode" not in srv.labels("worker")
    finally:
        srv.stop()


def test_kubeconfig_tls_server_name(tmp_path):
    """tls-server-name replaces the server's host for SNI and the certificate check:
    the server's certificate names kubernetes.default.svc and 127.0.0.1."""
    d = tmp_path / "pki"
    d.mkdir()
    _tls_material(d)
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="t0", tls=(str(d / "srv.crt"), str(d / "srv.key"))).start()
    try:
        srv.add_node("worker")
        kc = tmp_path / "kc"
        for name, ok in (("kubernetes.default.svc", True), ("other.example", False), ("", True)):
            line = f"    tls-server-name: {name}\n" if name else ""
            kc.write_text(f"clusters:\n- name: c\n  cluster:\n    server: {srv.url}\n    certificate-authority: pki/ca.crt\n"
                          f"{line}contexts: [{{name: x, context: {{cluster: c, user: u}}}}]\ncurrent-context: x\n"
                          "users: [{name: u, user: {token: t0}}]\n")
            srv.set_labels("worker", {})
            if ok:
                p = _label_once(kc, fi)
                assert p.returncode == 0, (name, p.stderr)
                assert srv.labels("worker")["amd.com/gpu.mode"] == "container"
                continue
            proc = subprocess.Popen([LBL, "-node_name", "worker", "-once", "-mode", "-sysfs_root", str(fi.sysfs),
                                     "-kubeconfig", str(kc)], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                    text=True, env=_env())
            time.sleep(1.0)
            rc, err = _term(proc)
            assert "certificate verify failed" in err, err
            assert "amd.com/gpu.mode" not in srv.labels("worker")
    finally:
        srv.stop()


@pytest.mark.parametrize("trailing", ["", "/"])
def test_server_url_path_prefix_and_host_header(tmp_path, trailing):
    """A server URL with a path (an apiserver behind a proxy at /k8s/clusters/<id>, as
    client-go takes it) prefixes every request, watches included; the Host header
    carries the URL's host:port, as Go's net/http sends it."""
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="t0", prefix="/k8s/clusters/c-1").start()
    try:
        srv.add_node("worker")
        kc = tmp_path / "kc"
        kc.write_text(f"clusters: [{{name: c, cluster: {{server: '{srv.url}{trailing}'}}}}]\n"
                      "contexts: [{name: x, context: {cluster: c, user: u}}]\ncurrent-context: x\n"
                      "users: [{name: u, user: {token: t0}}]\n")
        p = _label_once(kc, fi)
        assert p.returncode == 0, p.stderr
        assert srv.labels("worker")["amd.com/gpu.mode"] == "container"
        assert srv.requests and all(r[1].startswith("/api/v1/nodes") for r in srv.requests), srv.requests
        assert set(srv.host_headers) == {f"127.0.0.1:{srv.port}"}, srv.host_headers
        # the watch goes below the prefix too
        proc = subprocess.Popen([LBL, "-node_name", "worker", "-mode", "-sysfs_root", str(fi.sysfs),
                                 "-kubeconfig", str(kc)], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                text=True, env=_env())
        deadline = time.monotonic() + 10
        while srv.watch_starts == 0 and time.monotonic() < deadline:
            time.sleep(0.05)
        rc, err = _term(proc)
        assert srv.watch_starts >= 1, err
    finally:
        srv.stop()


class _Proxy:
    """An HTTP proxy that sends every connection to 127.0.0.1:<upstream>: CONNECT
    tunnels (https servers) and absolute-form requests rewritten to origin form."""

    def __init__(self, upstream: int):
        self.upstream = upstream
        self.lines, self.auth = [], []
        self.sock = socket.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(16)
        self.port = self.sock.getsockname()[1]
        threading.Thread(target=self._accept, daemon=True).start()

    def _accept(self):
        while True:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    @staticmethod
    def _pipe(a, b):
        try:
            while (d := a.recv(65536)):
                b.sendall(d)
        except OSError:
            pass
        finally:
            for x in (a, b):
                try:
                    x.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass

    def _serve(self, c):
        head = b""
        while b"\r\n\r\n" not in head:
            d = c.recv(1)
            if not d:
                return c.close()
            head += d
        lines = head.decode().split("\r\n")
        self.lines.append(lines[0])
        self.auth += [ln.split(":", 1)[1].strip() for ln in lines if ln.lower().startswith("proxy-authorization:")]
        up = socket.create_connection(("127.0.0.1", self.upstream))
        method, target, ver = lines[0].split(" ")
        if method == "CONNECT":
            c.sendall(b"HTTP/1.1 200 Connection established\r\n\r\n")
        else:  # http://host:port/path -> /path, the other header lines as they came
            path = "/" + target.split("://", 1)[1].split("/", 1)[1]
            up.sendall((" ".join((method, path, ver)) + "\r\n" + "\r\n".join(
                ln for ln in lines[1:] if not ln.lower().startswith("proxy-authorization:"))).encode())
        threading.Thread(target=self._pipe, args=(up, c), daemon=True).start()
        self._pipe(c, up)

    def close(self):
        self.sock.close()


def test_apiserver_through_an_http_proxy(tmp_path):
    """$HTTPS_PROXY (with credentials) tunnels an https apiserver through CONNECT by
    name, $NO_PROXY bypasses it, $HTTP_PROXY carries an http one in absolute form and
    a kubeconfig proxy-url applies without any environment, as client-go does."""
    d = tmp_path / "pki"
    d.mkdir()
    _tls_material(d)
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="t0", tls=(str(d / "srv.crt"), str(d / "srv.key"))).start()
    proxy = _Proxy(srv.port)
    try:
        srv.add_node("worker")
        kc = tmp_path / "kc"

        def write(server, extra=""):
            kc.write_text(f"clusters:\n- name: c\n  cluster:\n    server: {server}\n    certificate-authority: pki/ca.crt\n"
                          f"{extra}contexts: [{{name: x, context: {{cluster: c, user: u}}}}]\ncurrent-context: x\n"
                          "users: [{name: u, user: {token: t0}}]\n")

        # the certificate names kubernetes.default.svc, which only the proxy can reach
        write(f"https://kubernetes.default.svc:{srv.port}")
        p = _label_once(kc, fi, env=_env(HTTPS_PROXY=f"http://robot:p%40ss@127.0.0.1:{proxy.port}"))
        assert p.returncode == 0, p.stderr
        assert srv.labels("worker")["amd.com/gpu.mode"] == "container"
        assert proxy.lines and set(proxy.lines) == {f"CONNECT kubernetes.default.svc:{srv.port} HTTP/1.1"}
        assert set(proxy.auth) == {"Basic " + base64.b64encode(b"robot:p@ss").decode()}
        # NO_PROXY: straight to kubernetes.default.svc, which does not resolve here
        n = len(proxy.lines)
        srv.set_labels("worker", {})
        proc = subprocess.Popen([LBL, "-node_name", "worker", "-once", "-mode", "-sysfs_root", str(fi.sysfs),
                                 "-kubeconfig", str(kc)], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                                env=_env(HTTPS_PROXY=f"127.0.0.1:{proxy.port}", NO_PROXY="10.0.0.0/8, .svc"))
        time.sleep(1.0)
        rc, err = _term(proc)
        assert "resolve kubernetes.default.svc" in err and len(proxy.lines) == n
        assert "amd.com/gpu.mode" not in srv.labels("worker")
        # proxy-url in the kubeconfig, no environment
        write(f"https://kubernetes.default.svc:{srv.port}", f"    proxy-url: http://127.0.0.1:{proxy.port}\n")
        p = _label_once(kc, fi)
        assert p.returncode == 0, p.stderr
        assert srv.labels("worker")["amd.com/gpu.mode"] == "container" and len(proxy.lines) > n
    finally:
        proxy.close()
        srv.stop()
    # an http apiserver through $HTTP_PROXY: absolute-form requests
    srv = FakeApiServer(token="t0").start()
    proxy = _Proxy(srv.port)
    try:
        srv.add_node("worker")
        kc.write_text(f"clusters: [{{name: c, cluster: {{server: 'http://apiserver.test:{srv.port}'}}}}]\n"
                      "contexts: [{name: x, context: {cluster: c, user: u}}]\ncurrent-context: x\n"
                      "users: [{name: u, user: {token: t0}}]\n")
        p = _label_once(kc, fi, env=_env(HTTP_PROXY=f"http://127.0.0.1:{proxy.port}"))
        assert p.returncode == 0, p.stderr
        assert srv.labels("worker")["amd.com/gpu.mode"] == "container"
        assert proxy.lines and all(ln.split(" ")[1].startswith(f"http://apiserver.test:{srv.port}/api/v1/nodes")
                                   for ln in proxy.lines), proxy.lines
        assert set(srv.host_headers) == {f"apiserver.test:{srv.port}"}
    finally:
        proxy.close()
        srv.stop()


def test_kubeconfig_errors_are_reported(tmp_path):
    for text, want in (("clusters: [", "kubeconfig"), ("users: []\n", "no cluster server"),
                       ("clusters:\n- name: a\n  cluster:\n    server: http://x\n    certificate-authority-data: '%%%'\n",
                        "base64"),
                       # a dangling current-context / cluster / user name is not replaced by the first entry
                       (_KC.format(ctx="y", cluster="c", user="u", cred="token: t"), 'context "y" not found'),
                       (_KC.format(ctx="x", cluster="c2", user="u", cred="token: t"), 'cluster "c2" of context "x"'),
                       (_KC.format(ctx="x", cluster="c", user="u2", cred="token: t"), 'user "u2" of context "x"'),
                       # credential plugins are refused, not skipped into unauthenticated requests
                       (_KC.format(ctx="x", cluster="c", user="u", cred="exec: {command: aws}"), "authenticates with exec"),
                       (_KC.format(ctx="x", cluster="c", user="u", cred="auth-provider: {name: gcp}"),
                        "authenticates with auth-provider"),
                       (_KC.format(ctx="x", cluster="c", user="u", cred="username: admin"), "authenticates with username"),
                       # a CA and insecure-skip-tls-verify together, as client-go's transport refuses them
                       (_KC.format(ctx="x", cluster="c", user="u", cred="token: t").replace(
                           'server: "http://127.0.0.1:9"', 'server: "https://127.0.0.1:9", certificate-authority-data: QUJD, '
                           'insecure-skip-tls-verify: true'), "root certificates file with the insecure flag")):
        kc = tmp_path / "kc"
        kc.write_text(text)
        p = subprocess.run([LBL, "-node_name", "n", "-kubeconfig", str(kc)], capture_output=True, text=True,
                           timeout=20, env=_env())
        assert p.returncode == 1 and want in p.stderr, (text, p.stderr)
