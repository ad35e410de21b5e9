"""Interop of the native HTTP/2 transport with grpc-go, the kubelet's stack.

No Go toolchain exists here, so grpc-go's transport is replayed frame by frame
from the vendored sources (rocm_k8s_device_plugin_amd/testing/gopeer.py):

* GoClientConn (a kubelet's client connection) against the plugin socket of
  the native daemon: preface, empty SETTINGS, x/net HPACK with dynamic-table
  inserts and evictions, ``user-agent`` / ``te`` / ``grpc-timeout``, BDP pings
  interleaved with DATA, a mid-connection SETTINGS{INITIAL_WINDOW_SIZE} after
  a BDP update, concurrent streams, RST_STREAM(CANCEL) of ListAndWatch and a
  re-open, header blocks split by CONTINUATION;
* GoServer (the kubelet's Registration server, the metrics exporter) against
  the native client: its SETTINGS, response header blocks split into
  CONTINUATION frames, server PINGs, SETTINGS changes mid-call, small windows
  for large requests, GOAWAY ENHANCE_YOUR_CALM ``too_many_pings``, graceful
  GOAWAY, RST_STREAM(REFUSED_STREAM), non-gRPC HTTP status, a server that
  never answers (deadline, abort fd); and what other HTTP/2 servers may send
  (padding, HEADERS priority, PRIORITY / unknown frames, other RST_STREAM
  codes, GOAWAY before the call) or break (oversized frames, interrupted or
  orphan header blocks).

Reference: vendor/google.golang.org/grpc/internal/transport/{http2_client,
http2_server,controlbuf,flowcontrol,bdp_estimator}.go, vendor/golang.org/x/net/
http2/hpack/{encode,tables,static_table}.go.
"""
import os
import re
import signal
import socket
import struct
import subprocess
import threading
import time

import pytest

from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR, core
from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
from rocm_k8s_device_plugin_amd.testing import go_kubelet
from rocm_k8s_device_plugin_amd.testing import gopeer as gp
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node

EXE = os.environ.get("MI355X_NATIVE_DAEMON_EXE") or os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")
XNET = "/root/reference/vendor/golang.org/x/net/http2/hpack"
DP = "/v1beta1.DevicePlugin/"
REGISTER = "/v1beta1.Registration/Register"


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} was not built")


def _wait(cond, timeout=10.0, step=0.02):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if cond():
            return True
        time.sleep(step)
    return cond()


# ------------------------------------------------------------------ the peers' own HPACK

def _xnet(name):
    path = os.path.join(XNET, name)
    if not os.path.exists(path):
        pytest.skip("vendored x/net sources not available")
    with open(path) as f:
        return f.read()


def test_huffman_code_equals_xnet_tables():
    """The peers' canonical code (from RFC 7541 code lengths) is x/net's table."""
    src = _xnet("tables.go")
    codes = src[src.index("var huffmanCodes"):src.index("var huffmanCodeLen")]
    lens = src[src.index("var huffmanCodeLen"):]
    codes = [int(x, 16) for x in re.findall(r"0x[0-9a-f]+", codes)]
    lens = [int(x) for x in re.findall(r"\b\d+\b", lens[lens.index("{"):lens.index("}")])]
    assert len(codes) == 256 and len(lens) == 256
    assert gp.HUFF_CODE[:256] == codes and list(gp.HUFF_LEN[:256]) == lens


def test_static_table_and_name_index_equal_xnet():
    src = _xnet("static_table.go")
    ents = re.findall(r'\{Name: "([^"]*)", Value: "([^"]*)", Sensitive: false\}', src)
    assert tuple(ents) == gp.STATIC_TABLE
    by_name = dict(re.findall(r'^\s*"([^"]+)":\s+(\d+),$', src[:src.index("byNameValue")], re.M))
    assert {k: int(v) for k, v in by_name.items()} == gp._STATIC_NAME


def test_go_encoder_rfc7541_c4_request():
    """RFC 7541 C.4.1-C.4.3: x/net's encoder indexes :authority and custom
    headers, Huffman-codes them, and refers to the dynamic table on repeats."""
    enc = gp.GoHpackEncoder()
    first = enc.encode([(":method", "GET"), (":scheme", "http"), (":path", "/"), (":authority", "www.example.com")])
    assert first.hex() == "828684418cf1e3c2e5f23a6ba0ab90f4ff"
    second = enc.encode([(":method", "GET"), (":scheme", "http"), (":path", "/"), (":authority", "www.example.com"),
                         ("cache-control", "no-cache")])
    assert second.hex() == "828684be5886a8eb10649cbf"
    third = enc.encode([(":method", "GET"), (":scheme", "https"), (":path", "/index.html"),
                        (":authority", "www.example.com"), ("custom-key", "custom-value")])
    assert third.hex() == "828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf"


def test_go_encoder_streams_decode_with_evictions_natively_and_in_python():
    """A long grpc-go header sequence (a new grpc-timeout value on every call
    fills and evicts the dynamic table): the independent Python decoder and
    the native decoder (one block at a time, fresh table) read the same fields
    where the block is self-contained."""
    enc, dec = gp.GoHpackEncoder(), gp.HpackDecoder()
    conn = gp.GoClientConn.__new__(gp.GoClientConn)
    conn.user_agent, conn.authority = gp.GRPC_GO_USER_AGENT, "localhost"
    for i in range(400):
        fields = conn.request_fields(DP + ("Allocate" if i % 2 else "GetPreferredAllocation"), 9.9 - i * 1e-4)
        block = enc.encode(fields)
        assert dec.decode(block) == fields
    assert enc.evictions > 0 and enc.inserts > 400
    # a first block decodes natively too (only static / new-name literals)
    fresh = gp.GoHpackEncoder()
    f0 = conn.request_fields(DP + "Allocate", 10.0)
    assert [(k.decode(), v.decode()) for k, v in core().hpack_decode_block(fresh.encode(f0))] == f0


def test_encode_duration_matches_grpcutil():
    assert gp.encode_duration(10.0) == "10000000u"
    assert gp.encode_duration(0.0999999) == "99999900n"
    assert gp.encode_duration(3600 * 100) == "360000S" and gp.encode_duration(200e6) == "3333334M" and gp.encode_duration(0) == "0n"


# ------------------------------------------------------------------ grpc-go client -> native server

def GoKubelet(kdir, config=None, **kw):
    """kubelet's Registration server as grpc-go runs it, on <dir>/kubelet.sock;
    by default it connects back and opens ListAndWatch inside its Register
    handler, as kubelet does (testing/go_kubelet.py)."""
    return go_kubelet.GoKubelet(kdir, config=config, **kw)


def _daemon(kdir, fi, *extra):
    return subprocess.Popen([EXE, "-kubelet_dir", kdir, "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                             "-exporter_socket", "", *extra], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                            text=True)


def _stop(p):
    if p.poll() is None:
        p.send_signal(signal.SIGTERM)
    try:
        _, err = p.communicate(timeout=20)
    except subprocess.TimeoutExpired:
        p.kill()
        _, err = p.communicate()
    return p.returncode, err


@pytest.fixture
def daemon_node(tmp_path, request):
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")
    kub = GoKubelet(kdir)
    p = _daemon(kdir, fi, *getattr(request, "param", ()))
    try:
        assert _wait(lambda: kub.registrations and kub.updates(), 20), "the daemon never registered / listed"
        yield kdir, kub, p
    finally:
        rc, err = _stop(p)
        kub.close()
        assert rc == 0, err[-2000:]


@pytest.mark.parametrize("cfg", [
    gp.GoServerConfig(continuation_chunk=2),
    gp.GoServerConfig(ping_before_response=True, settings_after_headers=[(gp.S_INITIAL_WINDOW_SIZE, 1 << 20)]),
    gp.GoServerConfig(graceful_goaway=True),
    gp.GoServerConfig(refuse_calls=2),          # REFUSED_STREAM: the daemon retries (100 ms, doubling)
    gp.GoServerConfig(max_concurrent_streams=1, initial_window=16384),
], ids=["continuation", "ping+settings", "graceful-goaway", "refused-twice", "tight-limits"])
def test_daemon_registers_through_grpc_go_server_variants(tmp_path, cfg):
    """The daemon's native client (Register) against what a grpc-go
    Registration server may send; runs under ASan/TSan in CI with
    MI355X_NATIVE_DAEMON_EXE pointing at the sanitizer builds."""
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")
    kub = GoKubelet(kdir, cfg)
    p = _daemon(kdir, fi)
    try:
        assert _wait(lambda: kub.registrations, 20), "never registered"
        assert kub.srv.violations == []
        # and the plugin socket then serves a grpc-go client
        c = gp.GoClientConn(os.path.join(kdir, "amd.com_gpu"))
        try:
            assert c.unary(DP + "GetDevicePluginOptions", b"", 3.0)[0] == 0
        finally:
            c.close()
    finally:
        rc, err = _stop(p)
        kub.close()
    assert rc == 0, err[-2000:]
    if cfg.refuse_calls:
        assert kub.srv.refused == 2 and "REFUSED_STREAM" in err


def _pref_req(ids, size):
    r = pb.PreferredAllocationRequest()
    r.container_requests.add(available_deviceIDs=ids, allocation_size=size)
    return r.SerializeToString()


def test_native_client_registers_like_grpc_go_expects(daemon_node):
    """Register through the native client against a grpc-go server: request
    headers, one message, SETTINGS exchange, no protocol violations."""
    kdir, kub, _ = daemon_node
    reg = kub.registrations[0]
    assert reg.version == "v1beta1" and reg.resource_name == "amd.com/gpu" and reg.endpoint == "amd.com_gpu"
    hdr = dict(kub.srv.calls[0].headers)
    assert hdr[":method"] == "POST" and hdr[":path"] == REGISTER and hdr["te"] == "trailers"
    assert hdr["content-type"] == "application/grpc"
    assert kub.srv.violations == []
    # the client acknowledged the server preface SETTINGS and sent its own first (the ack may
    # follow the call's last frame: the server thread records it when it gets to it)
    deadline = time.monotonic() + 30
    while ("SETTINGS", 1, 0) not in kub.srv.frames and time.monotonic() < deadline:
        time.sleep(0.01)
    assert ("SETTINGS", 1, 0) in kub.srv.frames and kub.srv.frames[0][0] == "SETTINGS"


def test_grpc_go_client_session_against_the_daemon(daemon_node):
    kdir, kub, _ = daemon_node
    c = gp.GoClientConn(os.path.join(kdir, "amd.com_gpu"))
    try:
        # server preface acknowledged; options with a deadline (grpc-timeout)
        code, _, body = c.unary(DP + "GetDevicePluginOptions", b"", timeout_s=10.0)
        assert code == 0 and pb.DevicePluginOptions.FromString(body).get_preferred_allocation_available
        # ListAndWatch: no deadline (kubelet's stream context)
        lw = c.start_call(DP + "ListAndWatch", b"")
        first = pb.ListAndWatchResponse.FromString(c.next_message(lw))
        ids = sorted(d.ID for d in first.devices)
        assert len(ids) == 8
        # the first DATA of a sample triggers grpc-go's BDP ping, after a connection WINDOW_UPDATE
        assert c.wait(lambda: gp.BDP_PING in c.ping_acks, 5)
        sent = [n for n, _, _ in c.sent]
        assert sent.index("PING") > 0 and "WINDOW_UPDATE" in sent[:sent.index("PING")]
        # hundreds of admission RPCs on one connection: the dynamic table fills and evicts
        for i in range(300):
            size = 1 + i % 8
            code, msg, body = c.unary(DP + "GetPreferredAllocation", _pref_req(ids, size), timeout_s=10.0 - i * 1e-3)
            assert code == 0, msg
            got = list(pb.PreferredAllocationResponse.FromString(body).container_responses[0].deviceIDs)
            assert len(got) == size
            a = pb.AllocateRequest()
            a.container_requests.add(devices_ids=got)
            code, msg, body = c.unary(DP + "Allocate", a.SerializeToString(), timeout_s=10.0)
            assert code == 0, msg
            assert pb.AllocateResponse.FromString(body).container_responses[0].devices
        assert c.enc.evictions > 0
        # BDP growth: connection WINDOW_UPDATE + SETTINGS{INITIAL_WINDOW_SIZE} mid-connection
        acks = c.settings_acks
        c.update_flow_control(1 << 20)
        assert c.wait(lambda: c.settings_acks > acks, 5), "SETTINGS change not acknowledged"
        code, _, _ = c.unary(DP + "GetDevicePluginOptions", b"")
        assert code == 0
        # concurrent streams, answered in any order
        sids = [c.start_call(DP + "GetPreferredAllocation", _pref_req(ids, k % 4 + 1), 5.0) for k in range(16)]
        assert c.wait(lambda: all(c.streams[s].ended for s in sids), 10)
        assert all(c.streams[s].status()[0] == 0 for s in sids)
        # a client PING mid-session
        c.ping(b"12345678")
        assert c.wait(lambda: b"12345678" in c.ping_acks, 5)
        # metadata large enough for HEADERS + CONTINUATION
        big = [(f"x-md-{k}", "v" * 900) for k in range(30)]
        sid = c.start_call(DP + "GetDevicePluginOptions", b"", 5.0, metadata=big)
        assert "CONTINUATION" in [n for n, _, s in c.sent if s == sid]
        assert c.wait(lambda: c.streams[sid].ended, 5) and c.streams[sid].status()[0] == 0
        # kubelet drops ListAndWatch (context cancel) and opens it again on the same connection
        c.cancel(lw)
        lw2 = c.start_call(DP + "ListAndWatch", b"")
        again = pb.ListAndWatchResponse.FromString(c.next_message(lw2))
        assert sorted(d.ID for d in again.devices) == ids
        # nothing the server objected to
        assert c.goaway is None and all(c.streams[s].rst_code is None for s in c.streams if s != lw)
    finally:
        c.close()


def test_two_grpc_go_connections_and_a_restart_of_the_list_stream(daemon_node):
    """kubelet re-dials after its own restart: a fresh connection (fresh HPACK
    state) next to a stale one; both answered."""
    kdir, _, _ = daemon_node
    a = gp.GoClientConn(os.path.join(kdir, "amd.com_gpu"))
    b = gp.GoClientConn(os.path.join(kdir, "amd.com_gpu"))
    try:
        for c in (a, b, a, b):
            code, _, body = c.unary(DP + "GetDevicePluginOptions", b"", 3.0)
            assert code == 0
        la = a.start_call(DP + "ListAndWatch", b"")
        lb = b.start_call(DP + "ListAndWatch", b"")
        assert a.next_message(la) and b.next_message(lb)
    finally:
        a.close()
        b.close()


# ------------------------------------------------------------------ native client -> grpc-go server

ECHO = "/test.Echo/Call"


def _echo(msg):
    return 0, "", msg


def _client(path, timeout=5.0):
    c = core().GrpcClient()
    assert c.connect(path, timeout) == ""
    return c


@pytest.mark.parametrize("cfg,nbytes", [
    (gp.GoServerConfig(), 10),
    (gp.GoServerConfig(continuation_chunk=3), 10),                  # every header block in 3-byte fragments
    (gp.GoServerConfig(ping_before_response=True), 10),
    (gp.GoServerConfig(settings_after_headers=[(gp.S_INITIAL_WINDOW_SIZE, 1 << 20),
                                               (gp.S_MAX_FRAME_SIZE, 1 << 20)]), 10),
    (gp.GoServerConfig(graceful_goaway=True), 10),
    (gp.GoServerConfig(max_concurrent_streams=1), 10),
    (gp.GoServerConfig(), 300_000),                                 # larger than the default windows
    (gp.GoServerConfig(initial_window=16384), 100_000),             # RFC-legal window below grpc-go's minimum
    (gp.GoServerConfig(continuation_chunk=1, initial_window=16384), 70_000),
], ids=["plain", "continuation", "server-ping", "settings-mid-call", "graceful-goaway", "one-stream",
        "large-request", "small-window", "continuation+small-window"])
def test_native_client_against_grpc_go_server(tmp_path, cfg, nbytes):
    path = str(tmp_path / "go.sock")
    with gp.GoServer(path, {ECHO: _echo}, cfg) as srv:
        c = _client(path)
        payload = bytes(range(256)) * (nbytes // 256) + b"x" * (nbytes % 256)
        status, msg, body = c.unary(ECHO, payload, 10.0)
        assert (status, msg) == (0, ""), msg
        assert body == payload
        if cfg.graceful_goaway:
            # answered, then the connection is draining: a new call needs a new connection
            assert c.going_away
            assert c.unary(ECHO, b"again", 2.0)[0] == -1
            c = _client(path)
        for k in range(5):   # the connection (and both HPACK tables) stay in step
            if c.going_away:  # this server drains after every call
                c = _client(path)
            assert c.unary(ECHO, b"m%d" % k, 5.0) == (0, "", b"m%d" % k)
        assert srv.violations == []
        c.close()


def test_native_client_too_many_pings_goaway(tmp_path):
    path = str(tmp_path / "go.sock")
    with gp.GoServer(path, {ECHO: _echo}, gp.GoServerConfig(too_many_pings=True)):
        c = _client(path)
        t0 = time.monotonic()
        status, msg, _ = c.unary(ECHO, b"x", 60.0)
        assert status == -1 and "ENHANCE_YOUR_CALM" in msg and "too_many_pings" in msg, msg
        # the GOAWAY ends the call: far sooner than its deadline, however loaded the machine
        assert time.monotonic() - t0 < 30.0 and not c.connected


def test_native_client_refused_stream_keeps_the_connection(tmp_path):
    path = str(tmp_path / "go.sock")
    with gp.GoServer(path, {ECHO: _echo}, gp.GoServerConfig(refuse_calls=1)) as srv:
        c = _client(path)
        status, msg, _ = c.unary(ECHO, b"x", 5.0)
        assert status == 14 and "REFUSED_STREAM" in msg        # UNAVAILABLE, retryable
        assert c.connected and c.unary(ECHO, b"y", 5.0) == (0, "", b"y")
        assert srv.connections == 1


def test_native_client_http_error_status(tmp_path):
    path = str(tmp_path / "go.sock")
    with gp.GoServer(path, {ECHO: _echo}, gp.GoServerConfig(http_status=503)):
        status, msg, _ = _client(path).unary(ECHO, b"x", 5.0)
        assert status == 14 and "503" in msg


@pytest.mark.parametrize("http,status", [(400, 13), (401, 16), (403, 7), (404, 12), (418, 2)])
def test_native_client_http_status_mapping(tmp_path, http, status):
    """A non-gRPC HTTP answer (a proxy in front of the exporter) maps as grpc-go's HTTPStatusConvTab."""
    path = str(tmp_path / "go.sock")
    with gp.GoServer(path, {ECHO: _echo}, gp.GoServerConfig(http_status=http)):
        got, msg, _ = _client(path).unary(ECHO, b"x", 5.0)
        assert got == status and str(http) in msg


@pytest.mark.parametrize("cfg", [
    gp.GoServerConfig(pad=0),
    gp.GoServerConfig(pad=7),
    gp.GoServerConfig(pad=255),
    gp.GoServerConfig(priority_in_headers=True),
    gp.GoServerConfig(pad=3, priority_in_headers=True, continuation_chunk=4),
    gp.GoServerConfig(noise_frames=True),
], ids=["pad0", "pad7", "pad255", "priority", "pad+priority+continuation", "priority-and-unknown-frames"])
def test_native_client_accepts_what_other_http2_servers_send(tmp_path, cfg):
    """Padding, HEADERS priority fields, PRIORITY and unknown extension frames
    are legal HTTP/2 (RFC 7540 6.1, 6.2, 6.3, 4.1) that grpc-go never sends: the
    answer is read past them, padding included, and the connection stays usable."""
    path = str(tmp_path / "go.sock")
    with gp.GoServer(path, {ECHO: _echo}, cfg) as srv:
        c = _client(path)
        for payload in (b"", b"hello", bytes(range(256)) * 300):   # 76.8 kB: several DATA frames and credits
            assert c.unary(ECHO, payload, 10.0) == (0, "", payload)
        assert c.connected and srv.violations == []


@pytest.mark.parametrize("code,status", [(gp.CANCEL, 1), (gp.ENHANCE_YOUR_CALM, 8), (12, 7), (2, 13)])
def test_native_client_rst_stream_codes(tmp_path, code, status):
    """RST_STREAM codes map as grpc-go's http2ErrConvTab; the connection survives a reset stream."""
    path = str(tmp_path / "go.sock")
    with gp.GoServer(path, {ECHO: _echo}, gp.GoServerConfig(rst_code=code)):
        c = _client(path)
        got, msg, _ = c.unary(ECHO, b"x", 5.0)
        assert got == status and "RST_STREAM" in msg
        assert c.connected


def test_native_client_goaway_before_the_call(tmp_path):
    """GOAWAY with a last-stream-id below ours: the call was never processed; the
    error names the code and the debug text, and the connection is closed."""
    path = str(tmp_path / "go.sock")
    with gp.GoServer(path, {ECHO: _echo}, gp.GoServerConfig(goaway_first=gp.NO_ERROR)):
        c = _client(path)
        status, msg, _ = c.unary(ECHO, b"x", 5.0)
        assert status == -1 and "before the call" in msg and "shutting down" in msg
        assert not c.connected and c.unary(ECHO, b"y", 1.0)[0] == -1


@pytest.mark.parametrize("cfg,text", [
    (gp.GoServerConfig(oversized_data=True), "frame larger than 16384"),
    (gp.GoServerConfig(interrupted_headers=True), "CONTINUATION expected"),
    (gp.GoServerConfig(orphan_continuation=True), "CONTINUATION without HEADERS"),
], ids=["oversized-frame", "interrupted-header-block", "orphan-continuation"])
def test_native_client_protocol_violations_end_the_call_cleanly(tmp_path, cfg, text):
    """A peer that breaks the framing rules: the call fails at once with the
    reason, the connection is dropped, and a fresh one works."""
    path = str(tmp_path / "go.sock")
    with gp.GoServer(path, {ECHO: _echo}, cfg):
        c = _client(path)
        t0 = time.monotonic()
        status, msg, _ = c.unary(ECHO, b"x", 60.0)
        assert status == -1 and text in msg, msg
        # at once, not at the deadline (bounded loosely: a loaded CI host)
        assert time.monotonic() - t0 < 30.0 and not c.connected


def test_native_client_unknown_method_and_grpc_error(tmp_path):
    path = str(tmp_path / "go.sock")
    with gp.GoServer(path, {ECHO: lambda m: (9, "precondition: ünïcode", b"")}):
        c = _client(path)
        assert c.unary("/nope/Nope", b"", 5.0)[0] == 12
        status, msg, _ = c.unary(ECHO, b"", 5.0)
        # sent percent-encoded as grpc-go does (encodeGrpcMessage), decoded by the client
        assert status == 9 and msg == "precondition: ünïcode"


def test_native_client_deadline_and_abort_against_a_silent_server(tmp_path):
    """An exporter that accepts and never answers: the call ends at its
    deadline, or at once when the abort fd (a daemon's signal pipe) fires."""
    path = str(tmp_path / "go.sock")
    with gp.GoServer(path, {ECHO: _echo}, gp.GoServerConfig(never_answer=True)):
        c = _client(path)
        t0 = time.monotonic()
        status, msg, _ = c.unary(ECHO, b"x", 0.3)
        dt = time.monotonic() - t0
        assert status == -1 and "deadline" in msg and 0.25 < dt < 10.0
        r, w = os.pipe()
        try:
            c = _client(path)
            c.set_abort_fd(r)
            threading.Timer(0.2, lambda: os.write(w, b"x")).start()
            t0 = time.monotonic()
            status, msg, _ = c.unary(ECHO, b"x", 120.0)
            assert status == -1 and msg == "interrupted" and time.monotonic() - t0 < 60.0
        finally:
            os.close(r)
            os.close(w)


def test_native_client_survives_signals_during_a_call(tmp_path):
    """EINTR in the wait (a signal handler without SA_RESTART) re-polls with
    the time left instead of falling into a blocking read."""
    path = str(tmp_path / "go.sock")
    old = signal.signal(signal.SIGUSR1, lambda *a: None)
    try:
        with gp.GoServer(path, {ECHO: _echo}, gp.GoServerConfig(never_answer=True)):
            c = _client(path)
            tid = threading.get_ident()
            stop = threading.Event()

            def pester():
                while not stop.wait(0.02):
                    signal.pthread_kill(tid, signal.SIGUSR1)

            t = threading.Thread(target=pester)
            t.start()
            t0 = time.monotonic()
            try:
                status, msg, _ = c.unary(ECHO, b"x", 0.5)
            finally:
                stop.set()
                t.join()
            # EINTR every 20 ms must not restart the 0.5 s deadline (which would never end)
            assert status == -1 and "deadline" in msg and time.monotonic() - t0 < 15.0
    finally:
        signal.signal(signal.SIGUSR1, old)


# ------------------------------------------------------------------ native server conformance (RFC 7540)

def _raw(path, first_settings=True):
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.connect(path)
    s.sendall(gp.PREFACE + (gp.frame(gp.SETTINGS, 0, 0) if first_settings else b""))
    return s, gp.FrameReader(s)


def _goaway_code(rd, timeout=5.0):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        try:
            f = rd.read(0.2)
        except EOFError:
            return None
        if f and f[0] == gp.GOAWAY:
            return struct.unpack(">I", f[3][4:8])[0]
    return None


def _open_lw(s, sid=1):
    enc = gp.GoHpackEncoder()
    block = enc.encode([(":method", "POST"), (":scheme", "http"), (":path", DP + "ListAndWatch"),
                        (":authority", "localhost"), ("content-type", "application/grpc"), ("te", "trailers")])
    s.sendall(gp.frame(gp.HEADERS, gp.END_HEADERS, sid, block) +
              gp.frame(gp.DATA, gp.END_STREAM, sid, gp.grpc_message(b"")))


@pytest.mark.parametrize("case,want", [
    ("no-settings-first", gp.PROTOCOL_ERROR),
    ("rst-idle", gp.PROTOCOL_ERROR),
    ("window-update-idle", gp.PROTOCOL_ERROR),
    ("continuation-after-complete-headers", gp.PROTOCOL_ERROR),
    ("settings-window-overflow", gp.FLOW_CONTROL_ERROR),
    ("enable-push-2", gp.PROTOCOL_ERROR),
])
def test_native_server_connection_errors(daemon_node, case, want):
    kdir, _, _ = daemon_node
    path = os.path.join(kdir, "amd.com_gpu")
    s, rd = _raw(path, first_settings=case != "no-settings-first")
    try:
        if case == "no-settings-first":
            s.sendall(gp.frame(gp.PING, 0, 0, b"\0" * 8))
        elif case == "rst-idle":
            s.sendall(gp.frame(gp.RST_STREAM, 0, 7, struct.pack(">I", gp.CANCEL)))
        elif case == "window-update-idle":
            s.sendall(gp.frame(gp.WINDOW_UPDATE, 0, 9, struct.pack(">I", 100)))
        elif case == "continuation-after-complete-headers":
            _open_lw(s)
            s.sendall(gp.frame(gp.CONTINUATION, gp.END_HEADERS, 1, b"\x82"))
        elif case == "settings-window-overflow":
            _open_lw(s)
            s.sendall(gp.frame(gp.WINDOW_UPDATE, 0, 1, struct.pack(">I", gp.MAX_WINDOW - 65535)) +
                      gp.frame(gp.SETTINGS, 0, 0, gp.settings_payload([(gp.S_INITIAL_WINDOW_SIZE, 70000)])))
        elif case == "enable-push-2":
            s.sendall(gp.frame(gp.SETTINGS, 0, 0, gp.settings_payload([(gp.S_ENABLE_PUSH, 2)])))
        assert _goaway_code(rd) == want
    finally:
        s.close()
    # the server keeps serving other connections
    c = gp.GoClientConn(path)
    try:
        assert c.unary(DP + "GetDevicePluginOptions", b"", 3.0)[0] == 0
    finally:
        c.close()


STREAM_CLOSED = 5


def _headers(enc, path, method="POST", ctype="application/grpc"):
    return enc.encode([(":method", method), (":scheme", "http"), (":path", path), (":authority", "localhost"),
                       ("content-type", ctype), ("te", "trailers")])


def _until(rd, dec, pred, timeout=5.0):
    """Frames until pred(frame) holds (that frame last). Every HEADERS block is
    decoded in arrival order (the HPACK dynamic table) and carried decoded."""
    seen, deadline = [], time.monotonic() + timeout
    while time.monotonic() < deadline:
        f = rd.read(0.2)
        if f is None:
            continue
        if f[0] == gp.HEADERS:
            f = (f[0], f[1], f[2], dec.decode(f[3]))
        seen.append(f)
        if pred(f):
            return seen
    raise AssertionError(f"no such frame in {[(x[0], x[1], x[2]) for x in seen]}")


def _rst_code(frames, sid):
    return [struct.unpack(">I", f[3])[0] for f in frames if f[0] == gp.RST_STREAM and f[2] == sid]


@pytest.mark.parametrize("case", ["content-type", "get-method", "data-after-end", "zero-window-update",
                                  "stream-window-overflow", "message-too-large"])
def test_native_server_stream_errors_keep_the_connection(daemon_node, case):
    """Stream-level errors (RFC 7540 5.4.2) end only their stream: the next call
    on the same connection is answered."""
    kdir, _, _ = daemon_node
    s, rd = _raw(os.path.join(kdir, "amd.com_gpu"))
    enc, dec = gp.GoHpackEncoder(), gp.HpackDecoder()
    opts = DP + "GetDevicePluginOptions"
    try:
        if case == "content-type":
            s.sendall(gp.frame(gp.HEADERS, gp.END_HEADERS | gp.END_STREAM, 1, _headers(enc, opts, ctype="text/plain")))
            fr = _until(rd, dec, lambda f: f[0] == gp.HEADERS and f[2] == 1)
            assert fr[-1][1] & gp.END_STREAM and (":status", "415") in fr[-1][3]
        elif case == "get-method":
            s.sendall(gp.frame(gp.HEADERS, gp.END_HEADERS | gp.END_STREAM, 1, _headers(enc, opts, method="GET")))
            assert _rst_code(_until(rd, dec, lambda f: f[0] == gp.RST_STREAM), 1) == [gp.PROTOCOL_ERROR]
        elif case == "data-after-end":
            s.sendall(gp.frame(gp.HEADERS, gp.END_HEADERS, 1, _headers(enc, opts)) +
                      gp.frame(gp.DATA, gp.END_STREAM, 1, gp.grpc_message(b"")) +
                      gp.frame(gp.DATA, 0, 1, gp.grpc_message(b"late")))
            assert STREAM_CLOSED in _rst_code(_until(rd, dec, lambda f: f[0] == gp.RST_STREAM), 1)
        elif case in ("zero-window-update", "stream-window-overflow"):
            _open_lw(s, 1)
            _until(rd, dec, lambda f: f[0] == gp.DATA and f[2] == 1)        # the list is streaming
            inc = 0 if case == "zero-window-update" else gp.MAX_WINDOW
            s.sendall(gp.frame(gp.WINDOW_UPDATE, 0, 1, struct.pack(">I", inc)))
            want = gp.PROTOCOL_ERROR if inc == 0 else gp.FLOW_CONTROL_ERROR
            assert _rst_code(_until(rd, dec, lambda f: f[0] == gp.RST_STREAM), 1) == [want]
        elif case == "message-too-large":
            # 4 MiB is the gRPC default receive limit; the server returns credit as DATA arrives
            chunk = b"\0" * 16384
            out = gp.frame(gp.HEADERS, gp.END_HEADERS, 1, _headers(enc, opts))
            s.sendall(out + b"".join(gp.frame(gp.DATA, 0, 1, chunk) for _ in range(257)))
            fr = _until(rd, dec, lambda f: f[0] == gp.RST_STREAM and f[2] == 1)
            trailers = [f[3] for f in fr if f[0] == gp.HEADERS and f[2] == 1]
            assert trailers and ("grpc-status", "8") in trailers[-1] and _rst_code(fr, 1) == [gp.CANCEL]
        # the connection is still good: a call on the next stream is answered
        s.sendall(gp.frame(gp.HEADERS, gp.END_HEADERS, 3, _headers(enc, opts)) +
                  gp.frame(gp.DATA, gp.END_STREAM, 3, gp.grpc_message(b"")))
        fr = _until(rd, dec, lambda f: f[0] == gp.HEADERS and f[2] == 3 and f[1] & gp.END_STREAM)
        assert not [f for f in fr if f[0] == gp.GOAWAY]
        assert ("grpc-status", "0") in fr[-1][3]
    finally:
        s.close()


# ------------------------------------------------------------------ transport watchdog (native daemon)

def _stray_clients(path):
    """What may poke a plugin socket besides kubelet: curl, a socket health
    check, a client with a bad preface, and each connection error above on a
    connection that made no DevicePlugin call."""
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)     # connect and leave
    s.connect(path)
    s.close()
    for payload in (b"GET / HTTP/1.1\r\nHost: x\r\n\r\n", b"PRI * HTTP/2.0\r\n\r\nXX\r\n\r\n" + b"\0" * 9):
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.connect(path)
        s.sendall(payload)
        s.settimeout(5)
        try:
            while s.recv(4096):    # until the server hangs up
                pass
        except OSError:
            pass
        s.close()
    for case in ("no-settings-first", "rst-idle", "window-update-idle", "enable-push-2"):
        s, rd = _raw(path, first_settings=case != "no-settings-first")
        try:
            s.sendall({"no-settings-first": gp.frame(gp.PING, 0, 0, b"\0" * 8),
                       "rst-idle": gp.frame(gp.RST_STREAM, 0, 7, struct.pack(">I", gp.CANCEL)),
                       "window-update-idle": gp.frame(gp.WINDOW_UPDATE, 0, 9, struct.pack(">I", 100)),
                       "enable-push-2": gp.frame(gp.SETTINGS, 0, 0, gp.settings_payload([(gp.S_ENABLE_PUSH, 2)]))}[case])
            assert _goaway_code(rd) is not None, case
        finally:
            s.close()


@pytest.mark.parametrize("daemon_node", [("-pulse", "1", "-send_every_pulse")], indirect=True)
def test_stray_clients_never_trip_the_watchdog(daemon_node):
    """Default -grpc_watchdog (10 s), kubelet listing: stray or malformed
    clients get GOAWAY and lose only their own connection (grpc-go
    server.go:984-998); the daemon stays up, kubelet's stream keeps receiving
    lists and nothing registers again."""
    kdir, kub, p = daemon_node
    path = os.path.join(kdir, "amd.com_gpu")
    _stray_clients(path)
    n = kub.updates()
    assert _wait(lambda: kub.updates() >= n + 2, 10), "kubelet's stream stopped receiving lists"
    assert p.poll() is None and len(kub.registrations) == 1 and not kub.stream_ended.is_set()
    assert list(kub.lists[-1].values()).count("Healthy") == 8
    c = gp.GoClientConn(path)
    try:
        assert c.unary(DP + "GetDevicePluginOptions", b"", 3.0)[0] == 0
    finally:
        c.close()


def test_watchdog_counts_a_list_opened_before_the_register_answer(tmp_path):
    """kubelet opens ListAndWatch inside its Register handler (eager GoKubelet):
    the stream exists before the daemon reads the Register answer. The
    watchdog's baseline is taken when Register is sent, so it is counted."""
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")
    kub = GoKubelet(kdir, eager=True)
    p = _daemon(kdir, fi, "-grpc_watchdog", "1")
    try:
        assert _wait(lambda: kub.updates(), 20)
        time.sleep(2.5)     # well past -grpc_watchdog
        assert p.poll() is None and len(kub.registrations) == 1
    finally:
        rc, err = _stop(p)
        kub.close()
    assert rc == 0 and "transport watchdog" not in err, err[-2000:]


def test_watchdog_trips_on_a_protocol_error_of_kubelets_connection(tmp_path):
    """Before the first ListAndWatch, a protocol error on a connection that has
    made a DevicePlugin call (kubelet's) means kubelet cannot use this
    transport: exit 3 so the DaemonSet restarts the plugin."""
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")
    kub = GoKubelet(kdir, list_and_watch=False)
    p = _daemon(kdir, fi, "-grpc_watchdog", "30")
    try:
        assert _wait(lambda: kub.registrations, 20)
        path = os.path.join(kdir, "amd.com_gpu")
        _stray_clients(path)                 # stray clients: still nothing
        time.sleep(0.5)
        assert p.poll() is None
        c = gp.GoClientConn(path)            # kubelet's connection: a call, then a protocol error
        try:
            assert c.unary(DP + "GetDevicePluginOptions", b"", 3.0)[0] == 0
            c._send(gp.frame(gp.RST_STREAM, 0, 99, struct.pack(">I", gp.CANCEL)), raw=True)
            assert p.wait(timeout=10) == 3
        finally:
            c.close()
    finally:
        rc, err = _stop(p)
        kub.close()
    assert rc == 3 and "protocol error(s) on kubelet's connection before its ListAndWatch" in err, err[-2000:]


def test_daemon_registers_again_when_kubelet_drops_the_stream(tmp_path):
    """kubelet ends ListAndWatch when it drops a plugin (runClient ->
    disconnectClient): with kubelet.sock unchanged the daemon registers again
    after -reregister s and the new stream gets the devices."""
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")
    kub = GoKubelet(kdir)
    p = _daemon(kdir, fi, "-reregister", "0.5")
    try:
        assert _wait(lambda: kub.updates(), 20)
        n = kub.updates()
        kub.end_stream()
        assert _wait(lambda: len(kub.registrations) == 2 and kub.updates() > n, 10), (kub.registrations, kub.errors)
        assert len(kub.lists[-1]) == 8
        time.sleep(1.0)      # one re-registration, not a loop
        assert len(kub.registrations) == 2 and p.poll() is None
    finally:
        rc, err = _stop(p)
        kub.close()
    assert rc == 0 and "registering again" in err, err[-2000:]



def test_native_client_connect_waits_out_a_full_listen_backlog(tmp_path):
    """A non-blocking AF_UNIX connect() answers EAGAIN while kubelet's listen
    backlog is full: the client retries until the deadline (or the abort fd),
    and gets in as soon as kubelet accepts one."""
    path = str(tmp_path / "busy.sock")
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(path)
    srv.listen(0)
    pending, accepted = [], []
    try:
        while True:
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            s.setblocking(False)
            try:
                s.connect(path)
            except BlockingIOError:
                s.close()
                break
            pending.append(s)
            if len(pending) > 64:
                pytest.skip("the listen backlog never filled")
        c = core().GrpcClient()
        t0 = time.monotonic()
        err = c.connect(path, 0.3)
        assert err.endswith("listen backlog full until the deadline"), err
        assert 0.25 < time.monotonic() - t0 < 10
        r, w = os.pipe()
        try:
            c.set_abort_fd(r)
            threading.Timer(0.2, os.write, (w, b"x")).start()
            assert c.connect(path, 30).endswith(": interrupted")
        finally:
            c.set_abort_fd(-1)
            os.close(r)
            os.close(w)
        threading.Timer(0.3, lambda: accepted.append(srv.accept()[0])).start()
        t0 = time.monotonic()
        assert c.connect(path, 30) == ""
        assert 0.2 < time.monotonic() - t0 < 15 and c.connected
        c.close()
    finally:
        for s in pending + accepted:
            s.close()
        srv.close()
