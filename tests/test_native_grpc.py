"""Native HTTP/2 gRPC server (native/src/rpc, plugin/native_server.py), CPU.

* HPACK conformance: RFC 7541 Appendix C vectors (Huffman both ways, decoder
  with a shared dynamic table) and the header blocks grpc's C-core client
  really sends (captured from the socket, decoded, compared with what was sent);
* interop: the grpcio client (sync and aio) against the native server, and
  byte-for-byte *parsed* equality of every admission RPC with the Python
  grpc.aio servicer on the same DeviceImpl (single / CPX / CDI strategies);
* error statuses and messages equal to the aio servicer's;
* ListAndWatch: first list, pushed health changes, client cancel, server stop;
* flow control (a list larger than the 64 KiB initial window), concurrency,
  malformed input (the server keeps serving), fallbacks to Python.
"""
import asyncio
import base64
import os
import random
import socket
import struct
import threading
import time

import grpc
import pytest

from rocm_k8s_device_plugin_amd import cdi
from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
from rocm_k8s_device_plugin_amd.ops.native import core
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.plugin.manager import ManagerConfig, PluginManager
from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node

N = core()


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


# ------------------------------------------------------------------ HPACK

RFC_HUFFMAN = {
    b"www.example.com": "f1e3c2e5f23a6ba0ab90f4ff",
    b"no-cache": "a8eb10649cbf",
    b"custom-key": "25a849e95ba97d7f",
    b"custom-value": "25a849e95bb8e8b4bf",
    b"302": "6402",
    b"private": "aec3771a4b",
    b"Mon, 21 Oct 2013 20:13:21 GMT": "d07abe941054d444a8200595040b8166e082a62d1bff",
    b"https://www.example.com": "9d29ad171863c78f0b97c8e9ae82ae43d3",
    b"307": "640eff",
    b"gzip": "9bd9ab",
    b"foo=ASDJKHQKBZXOQWEOPIUAXQWEOIU; max-age=3600; version=1":
        "94e7821dd7f2e6c7b335dfdfcd5b3960d5af27087f3672c1ab270fb5291f9587316065c003ed4ee5b1063d5007",
}


@pytest.mark.parametrize("plain,coded", sorted(RFC_HUFFMAN.items()))
def test_huffman_rfc7541_vectors(plain, coded):
    assert N.hpack_huffman_encode(plain).hex() == coded
    assert N.hpack_huffman_decode(bytes.fromhex(coded)) == plain


def test_huffman_roundtrip_every_byte_and_bad_padding():
    rng = random.Random(7)
    for _ in range(200):
        s = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 40)))
        assert N.hpack_huffman_decode(N.hpack_huffman_encode(s)) == s
    assert N.hpack_huffman_decode(b"\xff\xff\xff\xff") is None       # EOS inside the string
    # padding must be a prefix of EOS (all ones): '0' = 00000, then 000 padding is invalid
    assert N.hpack_huffman_decode(b"\x00") is None


def test_hpack_rfc7541_c3_request_blocks_without_huffman():
    blk = bytes.fromhex("828684410f7777772e6578616d706c652e636f6d")
    assert N.hpack_decode_block(blk) == [(b":method", b"GET"), (b":scheme", b"http"), (b":path", b"/"),
                                         (b":authority", b"www.example.com")]


# grpc C-core as an HPACK oracle: capture the first header block a real client sends

def _capture_client_headers(tmp_path, metadata):
    path = str(tmp_path / "cap.sock")
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(path)
    srv.listen(1)
    got = {}

    def serve():
        c, _ = srv.accept()
        c.settimeout(5)
        c.sendall(struct.pack(">I", 0)[1:] + bytes([4, 0]) + struct.pack(">I", 0))  # empty SETTINGS
        buf = b""
        block = b""
        try:
            while True:
                chunk = c.recv(65536)
                if not chunk:
                    break
                buf += chunk
                if buf.startswith(b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"):
                    buf = buf[24:]
                while len(buf) >= 9:
                    ln = int.from_bytes(buf[:3], "big")
                    if len(buf) < 9 + ln:
                        break
                    typ, flags, payload = buf[3], buf[4], buf[9:9 + ln]
                    buf = buf[9 + ln:]
                    if typ == 4 and not flags & 1:
                        c.sendall(bytes([0, 0, 0, 4, 1, 0, 0, 0, 0]))    # SETTINGS ACK
                    if typ in (1, 9):
                        if typ == 1 and flags & 0x8:
                            payload = payload[1:len(payload) - payload[0]]
                        if typ == 1 and flags & 0x20:
                            payload = payload[5:]
                        block += payload
                        if flags & 0x4:
                            got["block"] = block
                            return
        finally:
            c.close()

    t = threading.Thread(target=serve)
    t.start()
    ch = grpc.insecure_channel(f"unix:{path}")
    try:
        pb.DevicePluginStub(ch).GetDevicePluginOptions(pb.Empty(), timeout=2, metadata=metadata)
    except grpc.RpcError:
        pass
    t.join(10)
    ch.close()
    srv.close()
    return got.get("block")


def test_hpack_decodes_what_grpc_core_sends(tmp_path):
    """Printable ASCII and binary metadata (C-core sends -bin values base64 +
    Huffman when that is shorter): our decoder must recover every field."""
    rng = random.Random(3)
    blob = bytes(rng.randrange(256) for _ in range(300))
    ascii_all = "".join(chr(c) for c in range(0x20, 0x7f))
    md = [("x-ascii", ascii_all), ("x-ids", "0000:05:00.0,amdgpu_xcp_17,0000:f5:00.0"), ("x-blob-bin", blob)]
    block = _capture_client_headers(tmp_path, md)
    assert block, "no header block captured"
    fields = dict(N.hpack_decode_block(block))
    assert fields[b":path"] == b"/v1beta1.DevicePlugin/GetDevicePluginOptions"
    assert fields[b"content-type"].startswith(b"application/grpc")
    assert fields[b"x-ascii"].decode() == ascii_all
    assert fields[b"x-ids"] == b"0000:05:00.0,amdgpu_xcp_17,0000:f5:00.0"
    raw = fields[b"x-blob-bin"]
    assert base64.b64decode(raw + b"=" * (-len(raw) % 4)) == blob


# ------------------------------------------------------------------ plugin-level interop

def _impl(fi, **kw):
    return ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None), **kw)


async def _with_plugin(tmp_path, impl, grpc_server, fn, pulse=0.0):
    """`fn(kubelet, mgr, resource state)` against the plugin served by the C++
    server ("native": the Python oracle's manager) or by grpc.aio ("aio": the
    oracle servicer on grpcio's own HTTP/2 stack, testing/aio_plugin.py; `mgr`
    is then the AioPlugin)."""
    pdir = str(tmp_path / f"dp-{grpc_server}")
    k = FakeKubelet(pdir)
    await k.start()
    if grpc_server == "aio":
        from rocm_k8s_device_plugin_amd.testing.aio_plugin import AioPlugin
        ap = AioPlugin(impl, pdir, impl.resource_names()[0])
        try:
            await ap.start()
            st = await k.wait_for_resource(f"amd.com/{impl.resource_names()[0]}", 1)
            return await fn(k, ap, st)
        finally:
            await ap.stop()
            await k.stop()
    mgr = PluginManager(impl, ManagerConfig(pulse_s=pulse, plugin_dir=pdir, handle_signals=False))
    task = asyncio.create_task(mgr.run())
    try:
        st = await k.wait_for_resource(f"amd.com/{impl.resource_names()[0]}", 1)
        return await fn(k, mgr, st)
    finally:
        mgr.request_stop()
        await asyncio.wait_for(task, 20)
        await k.stop()


def _requests(ids, rng):
    out = []
    for size in (1, 2, 3, len(ids) // 2, len(ids)):
        avail = sorted(rng.sample(ids, max(size, min(len(ids), size + rng.randrange(0, 4)))))
        must = rng.sample(avail, rng.randrange(0, min(2, size) + 1))
        out.append((avail, must, size))
    return out


async def _drive(st, reqs):
    res = []
    opts = await st.stub.GetDevicePluginOptions(pb.Empty(), timeout=5)
    res.append(("options", opts))
    for avail, must, size in reqs:
        r = pb.PreferredAllocationRequest()
        r.container_requests.add(available_deviceIDs=avail, must_include_deviceIDs=must, allocation_size=size)
        pref = await st.stub.GetPreferredAllocation(r, timeout=5)
        res.append(("preferred", pref))
        a = pb.AllocateRequest()
        a.container_requests.add(devices_ids=list(pref.container_responses[0].deviceIDs))
        a.container_requests.add(devices_ids=avail[:1])
        res.append(("allocate", await st.stub.Allocate(a, timeout=5)))
    res.append(("prestart", await st.stub.PreStartContainer(pb.PreStartContainerRequest(), timeout=5)))
    return res


@pytest.mark.parametrize("mode,strategies", [("spx", (cdi.DEVICE_SPECS,)), ("cpx", (cdi.DEVICE_SPECS,)),
                                             ("spx", (cdi.DEVICE_SPECS, cdi.CDI_CRI, cdi.CDI_ANNOTATIONS)),
                                             ("spx-nodeview", (cdi.DEVICE_SPECS,))])
def test_native_answers_equal_the_aio_servicer(tmp_path, mode, strategies):
    fi = make_mi355x_node(tmp_path / "n", **({"compute_partition": "CPX"} if mode == "cpx" else {}))
    out = {}
    for server in ("aio", "native"):
        extra = {"node_view_dir": str(tmp_path / "nv")} if mode == "spx-nodeview" else {}
        impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None),
                             device_list_strategy=strategies, cdi_spec_dir=str(tmp_path / f"cdi-{server}"), **extra)

        async def fn(k, mgr, st):
            ids = sorted(st.devices)
            res = await _drive(st, _requests(ids, random.Random(11)))
            if server == "native":
                plugin = mgr.plugins[impl.resource_names()[0]]
                plugin.sync()
                assert plugin.native.calls >= len(res) and plugin.native.fallbacks == 0
            return res, dict(st.devices)

        out[server] = run(_with_plugin(tmp_path, impl, server, fn))
    (a_res, a_list), (n_res, n_list) = out["aio"], out["native"]
    assert a_list == n_list
    assert [k for k, _ in a_res] == [k for k, _ in n_res]
    for (kind, a), (_, b) in zip(a_res, n_res):
        assert a == b, kind          # protobuf equality of the parsed responses


def test_native_error_statuses_match_aio(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    got = {}
    for server in ("aio", "native"):
        impl = _impl(fi)

        async def fn(k, mgr, st):
            errs = []
            a = pb.AllocateRequest()
            a.container_requests.add(devices_ids=["0000:99:00.0"])
            r = pb.PreferredAllocationRequest()
            r.container_requests.add(available_deviceIDs=sorted(st.devices)[:2], allocation_size=3)
            for call, req in ((st.stub.Allocate, a), (st.stub.GetPreferredAllocation, r)):
                with pytest.raises(grpc.aio.AioRpcError) as ei:
                    await call(req, timeout=5)
                errs.append((ei.value.code(), ei.value.details()))
            return errs

        got[server] = run(_with_plugin(tmp_path, impl, server, fn))
    assert got["native"] == got["aio"]
    assert got["native"][0][0] == grpc.StatusCode.INVALID_ARGUMENT
    assert got["native"][1][0] == grpc.StatusCode.UNKNOWN
    assert got["native"][1][1].startswith("unable to get preferred allocation list. Error:")


def test_unknown_method_is_unimplemented(tmp_path):
    srv = N.DevicePluginServer()
    sock = str(tmp_path / "s.sock")
    assert srv.start(sock) == ""
    try:
        ch = grpc.insecure_channel(f"unix:{sock}")
        call = ch.unary_unary("/v1beta1.DevicePlugin/Bogus", request_serializer=lambda x: x,
                              response_deserializer=lambda x: x)
        with pytest.raises(grpc.RpcError) as ei:
            call(b"", timeout=5)
        assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED
        # no prepared state and no fallback: an explicit error, not a hang
        with pytest.raises(grpc.RpcError) as ei:
            pb.DevicePluginStub(ch).GetDevicePluginOptions(pb.Empty(), timeout=5)
        assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED
        ch.close()
    finally:
        srv.stop(0.1)


def test_listandwatch_push_cancel_and_stop(tmp_path):
    """Health flips reach an open stream; a cancelled stream is dropped by the
    server; stopping the plugin ends the stream with OK."""
    fi = make_mi355x_node(tmp_path / "n")
    impl = _impl(fi)

    async def go():
        pdir = str(tmp_path / "dp")
        os.makedirs(pdir, exist_ok=True)
        k = FakeKubelet(pdir)
        await k.start()
        mgr = PluginManager(impl, ManagerConfig(pulse_s=0.05, plugin_dir=pdir, handle_signals=False))
        task = asyncio.create_task(mgr.run())
        st = await k.wait_for_resource("amd.com/gpu", 8)
        native = mgr.plugins["gpu"].native
        # a second, independent stream from another client
        ch = grpc.aio.insecure_channel(f"unix:{mgr.plugins['gpu'].socket}")
        stream = pb.DevicePluginStub(ch).ListAndWatch(pb.Empty())
        first = await stream.read()
        assert len(first.devices) == 8
        for _ in range(50):
            if native.srv.open_streams() == 2:
                break
            await asyncio.sleep(0.02)
        assert native.srv.open_streams() == 2
        # flip one device Unhealthy: both streams get the new list
        victim = sorted(st.devices)[3]
        from rocm_k8s_device_plugin_amd.health.monitor import Verdict

        async def no_sweep():
            return False

        impl.monitor.check_once = no_sweep      # keep the injected verdict
        before = k.resources["amd.com/gpu"].updates
        snap = dict(impl.monitor.snapshot())
        snap[victim] = Verdict(pb.UNHEALTHY, ("test",))
        impl.monitor._snapshot = snap
        impl.monitor.version += 1
        upd = await asyncio.wait_for(stream.read(), 5)
        assert {d.ID: d.health for d in upd.devices}[victim] == pb.UNHEALTHY
        await k.wait_for_update("amd.com/gpu", before, timeout=5)
        assert k.resources["amd.com/gpu"].devices[victim] == pb.UNHEALTHY
        stream.cancel()
        for _ in range(100):
            if native.srv.open_streams() == 1:
                break
            await asyncio.sleep(0.02)
        assert native.srv.open_streams() == 1
        await ch.close()
        mgr.request_stop()
        await asyncio.wait_for(task, 20)
        await k.stop()

    run(go())


def test_flow_control_list_larger_than_the_initial_window(tmp_path):
    """A ListAndWatch message beyond the 64 KiB initial windows arrives intact
    (the server waits for the client's WINDOW_UPDATEs)."""
    srv = N.DevicePluginServer()
    devs = [pb.Device(ID=f"dev-{i:06d}-" + "x" * 40, health=pb.HEALTHY) for i in range(4000)]
    big = pb.ListAndWatchResponse(devices=devs).SerializeToString()
    assert len(big) > 3 * 65535
    srv.set_device_list(big)
    sock = str(tmp_path / "s.sock")
    assert srv.start(sock) == ""
    try:
        ch = grpc.insecure_channel(f"unix:{sock}")
        it = pb.DevicePluginStub(ch).ListAndWatch(pb.Empty(), timeout=10)
        msg = next(it)
        assert len(msg.devices) == 4000 and msg.devices[-1].ID == devs[-1].ID
        srv.publish_list(big)
        assert len(next(it).devices) == 4000
        it.cancel()
        ch.close()
    finally:
        srv.stop(0.1)


def test_concurrent_clients(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    impl = _impl(fi)

    async def fn(k, mgr, st):
        sock = mgr.plugins["gpu"].socket
        ids = sorted(st.devices)
        errors = []

        def worker(seed):
            rng = random.Random(seed)
            ch = grpc.insecure_channel(f"unix:{sock}")
            stub = pb.DevicePluginStub(ch)
            try:
                for _ in range(60):
                    size = rng.randrange(1, 9)
                    r = pb.PreferredAllocationRequest()
                    r.container_requests.add(available_deviceIDs=ids, allocation_size=size)
                    got = stub.GetPreferredAllocation(r, timeout=10).container_responses[0].deviceIDs
                    if len(got) != size:
                        errors.append(("size", size, list(got)))
                    a = pb.AllocateRequest()
                    a.container_requests.add(devices_ids=list(got))
                    car = stub.Allocate(a, timeout=10).container_responses[0]
                    if len(car.devices) != 1 + 2 * size:
                        errors.append(("specs", size, len(car.devices)))
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))
            finally:
                ch.close()

        ths = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
        await asyncio.gather(*(asyncio.to_thread(t.run) for t in ths))
        return errors

    assert run(_with_plugin(tmp_path, impl, "native", fn), timeout=120) == []


def test_malformed_input_does_not_take_the_server_down(tmp_path):
    srv = N.DevicePluginServer()
    srv.set_options(pb.DevicePluginOptions(get_preferred_allocation_available=True).SerializeToString())
    sock = str(tmp_path / "s.sock")
    assert srv.start(sock) == ""
    rng = random.Random(5)
    preface = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"
    frames = [
        b"GET / HTTP/1.1\r\nHost: x\r\n\r\n",                                   # not HTTP/2
        preface + b"\x00\x00\x00\x04\x00\x00\x00\x00\x00" + b"\xff\xff\xff\x00\x00\x00\x00\x00\x01",  # huge frame
        preface + bytes([0, 0, 3, 1, 5, 0, 0, 0, 1, 0xbf, 0xff, 0xff]),          # bad HPACK index
        preface + bytes([0, 0, 0, 0, 1, 0, 0, 0, 7]),                            # DATA on an idle stream
        preface + bytes([0, 0, 4, 8, 0, 0, 0, 0, 0, 0, 0, 0, 0]),                # zero WINDOW_UPDATE
    ] + [preface + bytes(rng.randrange(256) for _ in range(rng.randrange(1, 300))) for _ in range(40)]
    try:
        for payload in frames:
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            s.settimeout(2)
            s.connect(sock)
            try:
                s.sendall(payload)
                s.shutdown(socket.SHUT_WR)
                while s.recv(65536):
                    pass
            except OSError:
                pass
            s.close()
        ch = grpc.insecure_channel(f"unix:{sock}")
        opts = pb.DevicePluginStub(ch).GetDevicePluginOptions(pb.Empty(), timeout=5)
        assert opts.get_preferred_allocation_available
        ch.close()
        assert srv.stats()["protocol_errors"] >= 3
    finally:
        srv.stop(0.1)


def test_topology_view_allocate_goes_through_the_python_fallback(tmp_path):
    """Allocate mounts made per request (-topology_view) are not in the
    prepared fragments: the server calls the DeviceImpl for them."""
    fi = make_mi355x_node(tmp_path / "n")
    impl = _impl(fi, topology_view_dir=str(tmp_path / "views"))

    async def fn(k, mgr, st):
        adm = await k.admit("amd.com/gpu", 2)
        car = adm.response.container_responses[0]
        mgr.plugins["gpu"].sync()
        return car, mgr.plugins["gpu"].native.fallbacks

    car, fallbacks = run(_with_plugin(tmp_path, impl, "native", fn))
    assert any(m.container_path.endswith("topology") for m in car.mounts)
    assert fallbacks == 1                  # Allocate only; GetPreferredAllocation stayed native


def test_stop_while_a_fallback_waits_for_the_gil(tmp_path):
    """stop() releases the GIL, so a fallback running on the server thread can
    finish: no deadlock between the loop thread and the server thread."""
    srv = N.DevicePluginServer()
    entered = threading.Event()

    def slow(method, req):
        entered.set()
        time.sleep(0.3)
        return 0, "", b""

    srv.set_fallback(slow)
    sock = str(tmp_path / "s.sock")
    assert srv.start(sock) == ""
    ch = grpc.insecure_channel(f"unix:{sock}")
    fut = pb.DevicePluginStub(ch).GetDevicePluginOptions.future(pb.Empty(), timeout=5)
    assert entered.wait(5)
    t0 = time.perf_counter()
    srv.stop(0.5)
    assert time.perf_counter() - t0 < 3
    try:
        fut.result(timeout=5)
    except grpc.RpcError:
        pass
    ch.close()


def test_views_switched_at_run_time_reach_the_native_allocate(tmp_path):
    """Setting -node_view's view on a running plugin (what bench.py does for its
    comparison) updates the prepared Allocate fragments: the mounts come back
    without a Python fallback; a topology view switches Allocate to the fallback."""
    from rocm_k8s_device_plugin_amd.node_view import NodeView
    from rocm_k8s_device_plugin_amd.topology_view import TopologyViews
    fi = make_mi355x_node(tmp_path / "n")
    impl = _impl(fi)

    async def fn(k, mgr, st):
        a0 = await k.admit("amd.com/gpu", 1)
        assert not a0.response.container_responses[0].mounts
        k.release("amd.com/gpu", a0.device_ids)
        impl.node_view = NodeView(str(tmp_path / "nv"), str(fi.sysfs))
        a1 = await k.admit("amd.com/gpu", 1)
        k.release("amd.com/gpu", a1.device_ids)
        plugin = mgr.plugins["gpu"]
        plugin.sync()
        fb = plugin.native.fallbacks
        impl.topology_views = TopologyViews(str(tmp_path / "tv"), str(fi.sysfs / "class/kfd/kfd/topology"))
        a2 = await k.admit("amd.com/gpu", 1)
        plugin.sync()
        return a1, a2, fb, plugin.native.fallbacks

    a1, a2, fb_before, fb_after = run(_with_plugin(tmp_path, impl, "native", fn))
    m1 = a1.response.container_responses[0].mounts
    assert m1 and all(m.read_only for m in m1)
    assert fb_before == 0
    assert fb_after == 1 and any(m.container_path.endswith("topology") for m in a2.response.container_responses[0].mounts)


def _raw_server(tmp_path, fallback=None):
    srv = N.DevicePluginServer()
    if fallback is not None:
        srv.set_fallback(fallback)
    sock = str(tmp_path / "r.sock")
    assert srv.start(sock) == ""
    return srv, sock


def test_large_request_needs_server_window_updates(tmp_path):
    """A request larger than the 64 KiB initial windows (and a header block
    split into CONTINUATION frames) arrives intact."""
    seen = {}

    def fb(method, req):
        r = pb.PreferredAllocationRequest.FromString(req)
        seen["n"] = len(r.container_requests[0].available_deviceIDs)
        return 0, "", pb.PreferredAllocationResponse().SerializeToString()

    srv, sock = _raw_server(tmp_path, fb)
    try:
        ch = grpc.insecure_channel(f"unix:{sock}")
        r = pb.PreferredAllocationRequest()
        ids = [f"amdgpu_xcp_{i:06d}_" + "y" * 40 for i in range(5000)]
        r.container_requests.add(available_deviceIDs=ids, allocation_size=3)
        assert r.ByteSize() > 4 * 65535
        pb.DevicePluginStub(ch).GetPreferredAllocation(r, timeout=10, metadata=[("x-big", "z" * 30000)])
        assert seen["n"] == 5000
        ch.close()
    finally:
        srv.stop(0.1)


def test_client_keepalive_pings_on_a_long_stream(tmp_path):
    """kubelet-style long-lived ListAndWatch with client keepalive PINGs every
    100 ms: every PING is acknowledged and the stream stays open."""
    srv, sock = _raw_server(tmp_path)
    srv.set_device_list(pb.ListAndWatchResponse(devices=[pb.Device(ID="a", health=pb.HEALTHY)]).SerializeToString())
    try:
        ch = grpc.insecure_channel(f"unix:{sock}", options=[("grpc.keepalive_time_ms", 100),
                                                            ("grpc.keepalive_timeout_ms", 1000),
                                                            ("grpc.keepalive_permit_without_calls", 1),
                                                            ("grpc.http2.max_pings_without_data", 0)])
        it = pb.DevicePluginStub(ch).ListAndWatch(pb.Empty(), timeout=10)
        assert next(it).devices[0].ID == "a"
        time.sleep(1.0)                                  # ~10 keepalive PINGs
        srv.publish_list(pb.ListAndWatchResponse(devices=[pb.Device(ID="b", health=pb.UNHEALTHY)])
                         .SerializeToString())
        assert next(it).devices[0].ID == "b"
        assert srv.stats()["protocol_errors"] == 0
        it.cancel()
        ch.close()
    finally:
        srv.stop(0.1)


def test_server_restart_on_the_same_socket_path(tmp_path):
    """The plugin restarts its server on kubelet restarts: a new server binds the
    same path (stale socket file replaced) and clients reconnect."""
    srv, sock = _raw_server(tmp_path)
    srv.set_options(pb.DevicePluginOptions(get_preferred_allocation_available=True).SerializeToString())
    srv.stop(0.1)
    srv2 = N.DevicePluginServer()
    srv2.set_options(pb.DevicePluginOptions().SerializeToString())
    assert srv2.start(sock) == ""
    try:
        ch = grpc.insecure_channel(f"unix:{sock}")
        assert not pb.DevicePluginStub(ch).GetDevicePluginOptions(pb.Empty(), timeout=5).get_preferred_allocation_available
        ch.close()
    finally:
        srv2.stop(0.1)


def test_native_start_failure_is_retried_not_replaced(tmp_path, monkeypatch):
    """The server failing to start is retried (the reference's 3 tries, dpm
    manager.go:205-219) and, once it starts, serves the node; there is no
    second transport to fall back to."""
    from rocm_k8s_device_plugin_amd.plugin import native_server as ns_mod
    fi = make_mi355x_node(tmp_path / "n")
    real, tries = ns_mod.NativePluginServer.start, []

    async def flaky(self, socket):
        tries.append(socket)
        if len(tries) == 1:
            raise OSError("bind: injected")
        return await real(self, socket)

    monkeypatch.setattr(ns_mod.NativePluginServer, "start", flaky)

    async def go():
        pdir = str(tmp_path / "dp")
        k = FakeKubelet(pdir)
        await k.start()
        mgr = PluginManager(_impl(fi), ManagerConfig(plugin_dir=pdir, handle_signals=False, retry_wait_s=0.05))
        task = asyncio.create_task(mgr.run())
        try:
            await k.wait_for_resource("amd.com/gpu", 1)
            adm = await k.admit("amd.com/gpu", 2)
            return mgr.plugins["gpu"].native, adm
        finally:
            mgr.request_stop()
            await asyncio.wait_for(task, 20)
            await k.stop()

    native, adm = run(go())
    assert len(tries) == 2 and native is not None and len(adm.device_ids) == 2


@pytest.mark.parametrize("server", ["native", "aio"])
def test_native_client_on_a_worker_thread_works_with_either_server(tmp_path, server):
    """The fake kubelet's native client, called from a worker thread, admits
    against both servers (the inline native client would block the event loop
    that serves grpc.aio, so bench.py switches to the threaded one there)."""
    fi = make_mi355x_node(tmp_path / "n")

    async def fn(k, mgr, st):
        k.rpc_client = "native-thread"
        adms = [await k.admit("amd.com/gpu", n) for n in (1, 2, 4)]
        return [len(a.device_ids) for a in adms]

    assert run(_with_plugin(tmp_path, _impl(fi), server, fn)) == [1, 2, 4]
