"""grpc-go-shaped HTTP/2 peers for the native transport's interop tests.

The kubelet is a grpc-go program: it is the *client* of every DevicePlugin
RPC and the *server* of Registration (the metrics exporter is a grpc-go
server too). The native HTTP/2 stack (native/src/rpc/grpc_server.cpp, grpc_client.cpp) must
therefore interoperate with grpc-go's transport, which no Go toolchain here
can run. These peers replay, frame by frame, what that transport does, taken
from the vendored sources (reference paths below are under
/root/reference/vendor/):

client (``GoClientConn``, google.golang.org/grpc/internal/transport/http2_client.go)
  * connection preface, then a SETTINGS frame with no entries when the default
    windows are in use (``newHTTP2Client``, :419-454; a connection
    WINDOW_UPDATE only when InitialConnWindowSize is set);
  * waits for the server preface (its SETTINGS) and acknowledges it;
  * request headers ``:method :scheme :path :authority content-type
    user-agent te`` and ``grpc-timeout`` when the call has a deadline
    (``createHeaderFields``, :553-588), HPACK-encoded as golang.org/x/net/http2/
    hpack's Encoder does (encode.go: dynamic-table inserts for every field that
    fits, Huffman when strictly shorter, indexed references on repeats),
    split into HEADERS + CONTINUATION beyond the peer's max frame size
    (controlbuf.go writeHeader);
  * one DATA frame per message carrying END_STREAM for unary and
    server-streaming calls, within the connection and stream windows;
  * inbound flow control of ``trInFlow`` / ``inFlow`` (flowcontrol.go):
    connection WINDOW_UPDATE once a quarter of the window is consumed, stream
    WINDOW_UPDATE as the application reads;
  * the BDP estimator (bdp_estimator.go): on the first DATA of a sample a
    connection WINDOW_UPDATE then PING ``{2,4,16,16,9,14,7,7}``
    (``handleData``, :1140-1173); on its ACK, when the sample says the
    window is too small, ``updateFlowControl`` (:1119-1137): connection
    WINDOW_UPDATE plus SETTINGS{INITIAL_WINDOW_SIZE} mid-connection;
  * ``cancel()``: RST_STREAM(CANCEL), what a cancelled context sends.

server (``GoServer``, http2_server.go)
  * server preface SETTINGS{MAX_FRAME_SIZE: 16384} (+ MAX_CONCURRENT_STREAMS /
    INITIAL_WINDOW_SIZE when configured, ``NewServerTransport`` :166-210);
  * the client preface must be followed by a SETTINGS frame;
  * responses ``:status 200, content-type`` then DATA then trailers
    ``grpc-status, grpc-message`` (WriteStatus), HPACK as above;
  * ``too_many_pings``: GOAWAY(ENHANCE_YOUR_CALM, "too_many_pings") and close
    (:922); graceful shutdown: GOAWAY(2^31-1) + PING ``{1,6,1,8,0,3,3,9}``,
    then GOAWAY(last stream) (:1336-1379);
  * fault knobs for what a grpc-go server may legitimately do that the
    kubelet's tiny messages never trigger (header blocks split across
    CONTINUATION frames, small initial windows, server-initiated PINGs), plus
    the failure modes the daemons must survive (never answering, non-gRPC
    HTTP status).

The HPACK tables here are built independently of the C++ code under test
(canonical Huffman code from the RFC 7541 code lengths) and are checked
against x/net's own tables in tests/test_go_interop.py.
"""
from __future__ import annotations

import os
import socket
import struct
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

GRPC_GO_USER_AGENT = "grpc-go/1.65.0"   # vendor/google.golang.org/grpc/version.go
PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"
BDP_PING = bytes([2, 4, 16, 16, 9, 14, 7, 7])        # bdp_estimator.go:47
GOAWAY_PING = bytes([1, 6, 1, 8, 0, 3, 3, 9])        # http2_server.go:1336
DEFAULT_WINDOW = 65535
MAX_WINDOW = (1 << 31) - 1
BDP_LIMIT = 16 << 20

DATA, HEADERS, PRIORITY, RST_STREAM, SETTINGS, PUSH_PROMISE, PING, GOAWAY, WINDOW_UPDATE, CONTINUATION = range(10)
FRAME_NAMES = ("DATA", "HEADERS", "PRIORITY", "RST_STREAM", "SETTINGS", "PUSH_PROMISE", "PING", "GOAWAY",
               "WINDOW_UPDATE", "CONTINUATION")
END_STREAM = ACK = 0x1
END_HEADERS, PADDED, PRIORITY_FLAG = 0x4, 0x8, 0x20
NO_ERROR, PROTOCOL_ERROR, FLOW_CONTROL_ERROR, REFUSED_STREAM, CANCEL, ENHANCE_YOUR_CALM = 0, 1, 3, 7, 8, 11
S_HEADER_TABLE_SIZE, S_ENABLE_PUSH, S_MAX_CONCURRENT_STREAMS, S_INITIAL_WINDOW_SIZE, S_MAX_FRAME_SIZE, \
    S_MAX_HEADER_LIST_SIZE = range(1, 7)

# ----------------------------------------------------------------------- HPACK
# RFC 7541 Appendix B code length of symbols 0..255 and EOS (256). The code is
# canonical, so the lengths determine every code.
HUFF_LEN = (
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 30, 28, 28, 28, 28, 28,
    28, 28, 28, 28, 6, 10, 10, 12, 13, 6, 8, 11, 10, 10, 8, 11, 8, 6, 6, 6, 5, 5, 5, 6, 6, 6, 6, 6, 6, 6, 7, 8, 15,
    6, 12, 10, 13, 6, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 8, 7, 8, 13, 19, 13, 14, 6,
    15, 5, 6, 5, 6, 5, 6, 6, 6, 5, 7, 7, 6, 6, 6, 5, 6, 7, 6, 5, 5, 6, 7, 7, 7, 7, 7, 15, 11, 14, 13, 28, 20, 22, 20,
    20, 22, 22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23, 24, 24, 22, 23, 24, 23, 23, 23, 23, 21, 22, 23, 22, 23, 23,
    24, 22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22, 24, 21, 22, 23, 23, 21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22,
    22, 23, 22, 22, 23, 26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25, 19, 21, 26, 27, 27, 26, 27,
    24, 21, 21, 26, 26, 28, 27, 27, 27, 20, 24, 20, 21, 22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23, 26, 27, 26,
    26, 27, 27, 27, 27, 27, 28, 27, 27, 27, 27, 27, 26, 30)


def _canonical_codes(lengths: Sequence[int]) -> List[int]:
    codes = [0] * len(lengths)
    code = 0
    for ln in range(1, max(lengths) + 1):
        for sym, l2 in enumerate(lengths):
            if l2 == ln:
                codes[sym] = code
                code += 1
        code <<= 1
    return codes


HUFF_CODE = _canonical_codes(HUFF_LEN)
_HUFF_DECODE = {(HUFF_LEN[s], HUFF_CODE[s]): s for s in range(257)}


def huffman_encoded_len(data: bytes) -> int:
    return (sum(HUFF_LEN[b] for b in data) + 7) // 8


def huffman_encode(data: bytes) -> bytes:
    acc = nbits = 0
    out = bytearray()
    for b in data:
        acc = (acc << HUFF_LEN[b]) | HUFF_CODE[b]
        nbits += HUFF_LEN[b]
        while nbits >= 8:
            nbits -= 8
            out.append((acc >> nbits) & 0xFF)
        acc &= (1 << nbits) - 1
    if nbits:
        out.append(((acc << (8 - nbits)) | ((1 << (8 - nbits)) - 1)) & 0xFF)   # EOS-prefix padding
    return bytes(out)


def huffman_decode(data: bytes) -> bytes:
    out = bytearray()
    cur = ln = 0
    for byte in data:
        for i in range(7, -1, -1):
            cur = (cur << 1) | ((byte >> i) & 1)
            ln += 1
            sym = _HUFF_DECODE.get((ln, cur))
            if sym is not None:
                if sym == 256:
                    raise ValueError("EOS in a Huffman string")
                out.append(sym)
                cur = ln = 0
            elif ln > 30:
                raise ValueError("invalid Huffman code")
    if ln > 7 or cur != (1 << ln) - 1:
        raise ValueError("invalid Huffman padding")
    return bytes(out)


STATIC_TABLE: Tuple[Tuple[str, str], ...] = (
    (":authority", ""), (":method", "GET"), (":method", "POST"), (":path", "/"), (":path", "/index.html"),
    (":scheme", "http"), (":scheme", "https"), (":status", "200"), (":status", "204"), (":status", "206"),
    (":status", "304"), (":status", "400"), (":status", "404"), (":status", "500"), ("accept-charset", ""),
    ("accept-encoding", "gzip, deflate"), ("accept-language", ""), ("accept-ranges", ""), ("accept", ""),
    ("access-control-allow-origin", ""), ("age", ""), ("allow", ""), ("authorization", ""), ("cache-control", ""),
    ("content-disposition", ""), ("content-encoding", ""), ("content-language", ""), ("content-length", ""),
    ("content-location", ""), ("content-range", ""), ("content-type", ""), ("cookie", ""), ("date", ""),
    ("etag", ""), ("expect", ""), ("expires", ""), ("from", ""), ("host", ""), ("if-match", ""),
    ("if-modified-since", ""), ("if-none-match", ""), ("if-range", ""), ("if-unmodified-since", ""),
    ("last-modified", ""), ("link", ""), ("location", ""), ("max-forwards", ""), ("proxy-authenticate", ""),
    ("proxy-authorization", ""), ("range", ""), ("referer", ""), ("refresh", ""), ("retry-after", ""),
    ("server", ""), ("set-cookie", ""), ("strict-transport-security", ""), ("transfer-encoding", ""),
    ("user-agent", ""), ("vary", ""), ("via", ""), ("www-authenticate", ""))
# x/net's static search: exact (name, value) pairs, and per name the LAST entry
# with that name (its byName map is filled in table order)
_STATIC_PAIR = {e: i + 1 for i, e in enumerate(STATIC_TABLE)}
_STATIC_NAME: Dict[str, int] = {}
for _i, (_n, _v) in enumerate(STATIC_TABLE):
    _STATIC_NAME[_n] = _i + 1


def _put_int(v: int, prefix: int, first: int = 0) -> bytes:
    k = (1 << prefix) - 1
    if v < k:
        return bytes([first | v])
    out = bytearray([first | k])
    v -= k
    while v >= 128:
        out.append(0x80 | (v & 0x7F))
        v >>= 7
    out.append(v)
    return bytes(out)


def _get_int(buf: bytes, pos: int, prefix: int) -> Tuple[int, int]:
    if pos >= len(buf):
        raise ValueError("truncated integer")
    k = (1 << prefix) - 1
    v = buf[pos] & k
    pos += 1
    if v < k:
        return v, pos
    shift = 0
    while True:
        if pos >= len(buf) or shift > 56:
            raise ValueError("truncated integer")
        b = buf[pos]
        pos += 1
        v += (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            return v, pos


def _put_str(s: bytes) -> bytes:
    """appendHpackString: Huffman only when strictly shorter."""
    h = huffman_encoded_len(s)
    if h < len(s):
        return _put_int(h, 7, 0x80) + huffman_encode(s)
    return _put_int(len(s), 7) + s


def _entry_size(name: str, value: str) -> int:
    return len(name.encode()) + len(value.encode()) + 32


class GoHpackEncoder:
    """golang.org/x/net/http2/hpack Encoder (encode.go, tables.go)."""

    def __init__(self, max_size: int = 4096):
        self.ents: List[Tuple[str, str]] = []   # oldest first, like x/net's headerFieldTable.ents
        self.size = 0
        self.max_size = max_size
        self.max_size_limit = 4096
        self.min_size: Optional[int] = None
        self.table_size_update = False
        self.evictions = 0
        self.inserts = 0

    def set_max_dynamic_table_size(self, v: int) -> None:
        v = min(v, self.max_size_limit)
        if self.min_size is None or v < self.min_size:
            self.min_size = v
        self.table_size_update = True
        self._set_max(v)

    def _set_max(self, v: int) -> None:
        self.max_size = v
        self._evict()

    def _evict(self) -> None:
        n = 0
        while self.size > self.max_size and n < len(self.ents):
            self.size -= _entry_size(*self.ents[n])
            n += 1
        if n:
            del self.ents[:n]
            self.evictions += n

    def _dyn_search(self, name: str, value: str, sensitive: bool) -> Tuple[int, bool]:
        # newest entry has HPACK index 1; x/net's maps keep the newest id per key
        for pos in range(len(self.ents) - 1, -1, -1):
            if not sensitive and self.ents[pos] == (name, value):
                return len(self.ents) - pos, True
        for pos in range(len(self.ents) - 1, -1, -1):
            if self.ents[pos][0] == name:
                return len(self.ents) - pos, False
        return 0, False

    def write_field(self, name: str, value: str, sensitive: bool = False) -> bytes:
        out = bytearray()
        if self.table_size_update:
            self.table_size_update = False
            if self.min_size is not None and self.min_size < self.max_size:
                out += _put_int(self.min_size, 5, 0x20)
            self.min_size = None
            out += _put_int(self.max_size, 5, 0x20)
        # searchTable: static exact, then dynamic exact, then a name match
        i = 0 if sensitive else _STATIC_PAIR.get((name, value), 0)
        if i:
            return bytes(out + _put_int(i, 7, 0x80))
        i = _STATIC_NAME.get(name, 0)
        j, exact = self._dyn_search(name, value, sensitive)
        if exact:
            return bytes(out + _put_int(j + len(STATIC_TABLE), 7, 0x80))
        idx = i if i else (j + len(STATIC_TABLE) if j else 0)
        indexing = not sensitive and _entry_size(name, value) <= self.max_size
        if indexing:
            self.ents.append((name, value))
            self.size += _entry_size(name, value)
            self.inserts += 1
            self._evict()
        type_byte = 0x10 if sensitive else (0x40 if indexing else 0)
        if idx == 0:
            out.append(type_byte)
            out += _put_str(name.encode())
        else:
            out += _put_int(idx, 6 if indexing else 4, type_byte)
        out += _put_str(value.encode())
        return bytes(out)

    def encode(self, fields: Sequence[Tuple[str, str]]) -> bytes:
        return b"".join(self.write_field(n, v) for n, v in fields)


class HpackDecoder:
    """RFC 7541 decoder (dynamic table, size updates, Huffman)."""

    def __init__(self, max_size: int = 4096):
        self.limit = max_size
        self.max_size = max_size
        self.dyn: List[Tuple[str, str]] = []   # newest first
        self.size = 0

    def _entry(self, idx: int) -> Tuple[str, str]:
        if 1 <= idx <= len(STATIC_TABLE):
            return STATIC_TABLE[idx - 1]
        d = idx - len(STATIC_TABLE) - 1
        if idx <= 0 or d >= len(self.dyn):
            raise ValueError(f"bad HPACK index {idx}")
        return self.dyn[d]

    def _evict(self, limit: int) -> None:
        while self.size > limit and self.dyn:
            self.size -= _entry_size(*self.dyn.pop())

    def _insert(self, name: str, value: str) -> None:
        sz = _entry_size(name, value)
        if sz > self.max_size:
            self._evict(0)
            return
        self._evict(self.max_size - sz)
        self.dyn.insert(0, (name, value))
        self.size += sz

    def _string(self, buf: bytes, pos: int) -> Tuple[str, int]:
        huff = bool(buf[pos] & 0x80)
        n, pos = _get_int(buf, pos, 7)
        if pos + n > len(buf):
            raise ValueError("truncated string")
        raw = buf[pos:pos + n]
        return (huffman_decode(raw) if huff else raw).decode("latin-1"), pos + n

    def decode(self, block: bytes) -> List[Tuple[str, str]]:
        out: List[Tuple[str, str]] = []
        pos = 0
        while pos < len(block):
            b = block[pos]
            if b & 0x80:
                idx, pos = _get_int(block, pos, 7)
                out.append(self._entry(idx))
            elif b & 0xE0 == 0x20:
                if out:
                    raise ValueError("table size update after a field")
                sz, pos = _get_int(block, pos, 5)
                if sz > self.limit:
                    raise ValueError("table size update above the limit")
                self.max_size = sz
                self._evict(sz)
            else:
                indexing = b & 0xC0 == 0x40
                idx, pos = _get_int(block, pos, 6 if indexing else 4)
                if idx:
                    name = self._entry(idx)[0]
                else:
                    name, pos = self._string(block, pos)
                value, pos = self._string(block, pos)
                out.append((name, value))
                if indexing:
                    self._insert(name, value)
        return out


# ---------------------------------------------------------------------- frames
def frame(ftype: int, flags: int, sid: int, payload: bytes = b"") -> bytes:
    n = len(payload)
    return bytes([n >> 16 & 0xFF, n >> 8 & 0xFF, n & 0xFF, ftype, flags]) + struct.pack(">I", sid & 0x7FFFFFFF) + \
        payload


def settings_payload(settings: Sequence[Tuple[int, int]]) -> bytes:
    return b"".join(struct.pack(">HI", k, v) for k, v in settings)


def grpc_message(msg: bytes) -> bytes:
    return b"\x00" + struct.pack(">I", len(msg)) + msg


def encode_grpc_message(msg: str) -> str:
    """grpc-go's encodeGrpcMessage (internal/transport/http_util.go:224-262):
    printable ASCII but '%' passes through, every other byte is %XX."""
    out = []
    for b in msg.encode("utf-8", "surrogateescape"):
        out.append(chr(b) if 0x20 <= b <= 0x7E and b != 0x25 else "%%%02X" % b)
    return "".join(out)


def encode_duration(seconds: float) -> str:
    """grpcutil.EncodeDuration: the finest unit that fits in 8 digits, rounded up."""
    ns = int(round(seconds * 1e9))
    if ns <= 0:
        return "0n"
    for unit, scale in (("n", 1), ("u", 1000), ("m", 10 ** 6), ("S", 10 ** 9), ("M", 60 * 10 ** 9),
                        ("H", 3600 * 10 ** 9)):
        d = -(-ns // scale)
        if d <= 99999999:
            return f"{d}{unit}"
    return f"{-(-ns // (3600 * 10 ** 9))}H"


class FrameReader:
    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.buf = b""
        self.eof = False

    def read(self, timeout: float) -> Optional[Tuple[int, int, int, bytes]]:
        """One frame, None on timeout; EOFError when the peer closed."""
        deadline = time.monotonic() + timeout
        while True:
            if len(self.buf) >= 9:
                n = int.from_bytes(self.buf[:3], "big")
                if len(self.buf) >= 9 + n:
                    t, fl = self.buf[3], self.buf[4]
                    sid = struct.unpack(">I", self.buf[5:9])[0] & 0x7FFFFFFF
                    payload = self.buf[9:9 + n]
                    self.buf = self.buf[9 + n:]
                    return t, fl, sid, payload
            if self.eof:
                raise EOFError("peer closed the connection")
            left = deadline - time.monotonic()
            if left <= 0:
                return None
            self.sock.settimeout(left)
            try:
                chunk = self.sock.recv(65536)
            except socket.timeout:
                return None
            except (ConnectionResetError, BrokenPipeError):
                chunk = b""
            if not chunk:
                self.eof = True
                continue
            self.buf += chunk


# ---------------------------------------------------------------------- client
class _TrInFlow:
    """Connection-level inbound flow control (flowcontrol.go trInFlow)."""

    def __init__(self, limit: int):
        self.limit, self.unacked = limit, 0

    def new_limit(self, n: int) -> int:
        d, self.limit = n - self.limit, n
        return d

    def on_data(self, n: int) -> int:
        self.unacked += n
        if self.unacked >= self.limit // 4:
            w, self.unacked = self.unacked, 0
            return w
        return 0

    def reset(self) -> int:
        w, self.unacked = self.unacked, 0
        return w


class _InFlow:
    """Stream-level inbound flow control (flowcontrol.go inFlow)."""

    def __init__(self, limit: int):
        self.limit, self.pending_data, self.pending_update = limit, 0, 0

    def on_data(self, n: int) -> bool:
        self.pending_data += n
        return self.pending_data + self.pending_update <= self.limit

    def on_read(self, n: int) -> int:
        if self.pending_data == 0:
            return 0
        self.pending_data -= n
        self.pending_update += n
        if self.pending_update >= self.limit // 4:
            w, self.pending_update = self.pending_update, 0
            return w
        return 0


class _BdpEstimator:
    """bdp_estimator.go (alpha 0.9, beta 0.66, gamma 2, limit 16 MiB)."""

    def __init__(self):
        self.bdp, self.sample, self.bw_max, self.is_sent = DEFAULT_WINDOW, 0, 0.0, False
        self.sample_count, self.rtt, self.sent_at = 0, 0.0, 0.0

    def add(self, n: int) -> bool:
        if self.bdp == BDP_LIMIT:
            return False
        if not self.is_sent:
            self.is_sent, self.sample, self.sent_at = True, n, 0.0
            self.sample_count += 1
            return True
        self.sample += n
        return False

    def timesnap(self) -> None:
        self.sent_at = time.monotonic()

    def calculate(self) -> Optional[int]:
        rtt_sample = max(1e-9, time.monotonic() - self.sent_at)
        if self.sample_count < 10:
            self.rtt += (rtt_sample - self.rtt) / self.sample_count
        else:
            self.rtt += (rtt_sample - self.rtt) * 0.9
        self.is_sent = False
        bw = self.sample / (max(self.rtt, 1e-9) * 1.5)
        if bw > self.bw_max:
            self.bw_max = bw
        if self.sample >= 0.66 * self.bdp and bw == self.bw_max and self.bdp != BDP_LIMIT:
            self.bdp = min(int(2 * self.sample), BDP_LIMIT)
            return self.bdp
        return None


@dataclass
class GoStream:
    sid: int
    method: str
    send_window: int
    inflow: _InFlow
    headers: List[Tuple[str, str]] = field(default_factory=list)
    trailers: List[Tuple[str, str]] = field(default_factory=list)
    data: bytearray = field(default_factory=bytearray)
    messages: List[bytes] = field(default_factory=list)
    ended: bool = False
    rst_code: Optional[int] = None
    pending_body: bytes = b""

    def status(self) -> Tuple[Optional[int], str]:
        for src in (self.trailers, self.headers):
            d = dict(src)
            if "grpc-status" in d:
                return int(d["grpc-status"]), d.get("grpc-message", "")
        return None, ""


class GoClientConn:
    """A kubelet's grpc-go client connection to a device-plugin socket."""

    def __init__(self, path: str, user_agent: str = GRPC_GO_USER_AGENT, authority: str = "localhost",
                 bdp: bool = True, timeout: float = 5.0, header_table_size: Optional[int] = None):
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.settimeout(timeout)
        self.sock.connect(path)
        self.rd = FrameReader(self.sock)
        self.enc, self.dec = GoHpackEncoder(), HpackDecoder()
        self.user_agent, self.authority = user_agent, authority
        self.next_id = 1
        self.streams: Dict[int, GoStream] = {}
        self.initial_window = DEFAULT_WINDOW         # our receive window for new streams
        self.peer_initial_window = DEFAULT_WINDOW    # the server's, for what we send
        self.peer_max_frame = 16384
        self.conn_send_window = DEFAULT_WINDOW
        self.fc = _TrInFlow(DEFAULT_WINDOW)
        self.bdp = _BdpEstimator() if bdp else None
        self.sent: List[Tuple[str, int, int]] = []    # (frame name, flags, stream) in order
        self.received: List[Tuple[str, int, int]] = []
        self.settings_acks = 0
        self.ping_acks: List[bytes] = []
        self.goaway: Optional[Tuple[int, int, bytes]] = None
        self.window_updates_received = 0
        self._cont: Optional[Tuple[int, bytearray, bool]] = None
        self.server_settings: Dict[int, int] = {}
        # newHTTP2Client: preface + SETTINGS (no entries with default windows);
        # a connection WINDOW_UPDATE only with a non-default connection window
        self._send(PREFACE, raw=True)
        settings = [] if header_table_size is None else [(S_HEADER_TABLE_SIZE, header_table_size)]
        self._send(frame(SETTINGS, 0, 0, settings_payload(settings)))
        # reader: the server preface (its SETTINGS) comes first
        f = self.rd.read(timeout)
        if f is None or f[0] != SETTINGS or f[1] & ACK:
            raise ConnectionError(f"no server preface SETTINGS: {f}")
        self._on_frame(*f)

    # -------------------------------------------------------------- output
    def _send(self, data: bytes, raw: bool = False) -> None:
        if not raw:
            pos = 0
            while pos < len(data):
                n = int.from_bytes(data[pos:pos + 3], "big")
                self.sent.append((FRAME_NAMES[data[pos + 3]] if data[pos + 3] < 10 else str(data[pos + 3]),
                                  data[pos + 4], struct.unpack(">I", data[pos + 5:pos + 9])[0]))
                pos += 9 + n
        self.sock.sendall(data)

    def _header_frames(self, sid: int, block: bytes, end_stream: bool) -> bytes:
        """controlbuf.go writeHeader: HEADERS, then CONTINUATIONs of at most max frame."""
        out, first, pos = [], True, 0
        while True:
            chunk = block[pos:pos + self.peer_max_frame]
            pos += len(chunk)
            last = pos >= len(block)
            flags = (END_HEADERS if last else 0) | (END_STREAM if first and end_stream else 0)
            out.append(frame(HEADERS if first else CONTINUATION, flags, sid, chunk))
            first = False
            if last:
                return b"".join(out)

    def request_fields(self, method: str, timeout_s: Optional[float] = None,
                       metadata: Sequence[Tuple[str, str]] = ()) -> List[Tuple[str, str]]:
        f = [(":method", "POST"), (":scheme", "http"), (":path", method), (":authority", self.authority),
             ("content-type", "application/grpc"), ("user-agent", self.user_agent), ("te", "trailers")]
        if timeout_s is not None:
            f.append(("grpc-timeout", encode_duration(timeout_s)))
        return f + list(metadata)

    def start_call(self, method: str, msg: bytes, timeout_s: Optional[float] = None,
                   metadata: Sequence[Tuple[str, str]] = ()) -> int:
        sid = self.next_id
        self.next_id += 2
        st = GoStream(sid, method, self.peer_initial_window, _InFlow(self.initial_window))
        self.streams[sid] = st
        block = self.enc.encode(self.request_fields(method, timeout_s, metadata))
        self._send(self._header_frames(sid, block, False))
        st.pending_body = grpc_message(msg)
        self._flush_body(st)
        return sid

    def _flush_body(self, st: GoStream) -> None:
        """The loopy writer: DATA within the connection and stream quota; the
        last frame carries END_STREAM (unary / server-streaming requests)."""
        while st.pending_body:
            q = min(self.conn_send_window, st.send_window, self.peer_max_frame)
            if q <= 0:
                return
            chunk, st.pending_body = st.pending_body[:q], st.pending_body[q:]
            self.conn_send_window -= len(chunk)
            st.send_window -= len(chunk)
            self._send(frame(DATA, END_STREAM if not st.pending_body else 0, st.sid, chunk))

    def cancel(self, sid: int) -> None:
        """A cancelled call context: RST_STREAM(CANCEL)."""
        self._send(frame(RST_STREAM, 0, sid, struct.pack(">I", CANCEL)))
        self.streams[sid].ended = True

    def ping(self, data: bytes = b"\0" * 8) -> None:
        self._send(frame(PING, 0, 0, data))

    def update_flow_control(self, n: int) -> None:
        """http2_client.go updateFlowControl(n): new stream limit for every
        stream, connection WINDOW_UPDATE, SETTINGS{INITIAL_WINDOW_SIZE: n}."""
        self.initial_window = n
        for st in self.streams.values():
            st.inflow.limit = n
        inc = self.fc.new_limit(n)
        if inc > 0:
            self._send(frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", inc)))
        self._send(frame(SETTINGS, 0, 0, settings_payload([(S_INITIAL_WINDOW_SIZE, n)])))

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass

    # --------------------------------------------------------------- input
    def _on_frame(self, t: int, fl: int, sid: int, p: bytes) -> None:
        self.received.append((FRAME_NAMES[t] if t < 10 else str(t), fl, sid))
        if self._cont is not None and (t != CONTINUATION or sid != self._cont[0]):
            raise ConnectionError("header block interrupted")
        if t == SETTINGS:
            if fl & ACK:
                self.settings_acks += 1
                return
            for i in range(0, len(p), 6):
                k, v = struct.unpack(">HI", p[i:i + 6])
                self.server_settings[k] = v
                if k == S_INITIAL_WINDOW_SIZE:
                    delta = v - self.peer_initial_window
                    self.peer_initial_window = v
                    for st in self.streams.values():
                        st.send_window += delta
                elif k == S_MAX_FRAME_SIZE:
                    self.peer_max_frame = v
            self._send(frame(SETTINGS, ACK, 0))
            for st in self.streams.values():
                self._flush_body(st)
        elif t == PING:
            if fl & ACK:
                self.ping_acks.append(p)
                if p == BDP_PING and self.bdp is not None:
                    n = self.bdp.calculate()
                    if n is not None:
                        self.update_flow_control(n)
            else:
                self._send(frame(PING, ACK, 0, p))
        elif t == GOAWAY:
            last, code = struct.unpack(">II", p[:8])
            self.goaway = (last & 0x7FFFFFFF, code, p[8:])
        elif t == WINDOW_UPDATE:
            inc = struct.unpack(">I", p)[0] & 0x7FFFFFFF
            self.window_updates_received += 1
            if sid == 0:
                self.conn_send_window += inc
                for st in self.streams.values():
                    self._flush_body(st)
            elif sid in self.streams:
                self.streams[sid].send_window += inc
                self._flush_body(self.streams[sid])
        elif t == RST_STREAM:
            if sid in self.streams:
                self.streams[sid].rst_code = struct.unpack(">I", p)[0]
                self.streams[sid].ended = True
        elif t in (HEADERS, CONTINUATION):
            if t == HEADERS:
                if fl & PADDED:
                    pad = p[0]
                    p = p[1:len(p) - pad]
                if fl & PRIORITY_FLAG:
                    p = p[5:]
                self._cont = (sid, bytearray(), bool(fl & END_STREAM))
            assert self._cont is not None
            self._cont[1].extend(p)
            if fl & END_HEADERS:
                csid, block, end = self._cont
                self._cont = None
                fields = self.dec.decode(bytes(block))   # every block, in order (shared table)
                st = self.streams.get(csid)
                if st is not None:
                    if st.headers and not end:
                        raise ConnectionError("second header block without END_STREAM")
                    (st.trailers if st.headers else st.headers).extend(fields)
                    if end:
                        st.ended = True
        elif t == DATA:
            size = len(p)
            # handleData: BDP sample, connection credit, then the stream
            send_ping = self.bdp.add(size) if self.bdp is not None else False
            w = self.fc.on_data(size)
            if w:
                self._send(frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", w)))
            if send_ping:
                w = self.fc.reset()
                if w:
                    self._send(frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", w)))
                self._send(frame(PING, 0, 0, BDP_PING))
                self.bdp.timesnap()
            st = self.streams.get(sid)
            if st is None:
                return
            if fl & PADDED:
                pad = p[0]
                p = p[1:len(p) - pad]
            if size and not st.inflow.on_data(size):
                raise ConnectionError(f"stream {sid}: server exceeded the stream window")
            st.data.extend(p)
            # the application reads at once: stream WINDOW_UPDATE per inFlow.onRead
            if size:
                w = st.inflow.on_read(size)
                if w:
                    self._send(frame(WINDOW_UPDATE, 0, sid, struct.pack(">I", w)))
            while len(st.data) >= 5:
                n = struct.unpack(">I", st.data[1:5])[0]
                if len(st.data) < 5 + n:
                    break
                st.messages.append(bytes(st.data[5:5 + n]))
                del st.data[:5 + n]
            if fl & END_STREAM:
                st.ended = True

    def pump(self, timeout: float) -> bool:
        """Handle frames for up to `timeout` s (returns after the first batch)."""
        f = self.rd.read(timeout)
        if f is None:
            return False
        self._on_frame(*f)
        while True:
            f = self.rd.read(0.0)
            if f is None:
                return True
            self._on_frame(*f)

    def wait(self, cond: Callable[[], bool], timeout: float = 5.0) -> bool:
        deadline = time.monotonic() + timeout
        while not cond():
            left = deadline - time.monotonic()
            if left <= 0:
                return False
            self.pump(left)
        return True

    def unary(self, method: str, msg: bytes, timeout_s: Optional[float] = 10.0,
              wait_s: float = 5.0) -> Tuple[Optional[int], str, bytes]:
        sid = self.start_call(method, msg, timeout_s)
        st = self.streams[sid]
        if not self.wait(lambda: st.ended, wait_s):
            raise TimeoutError(f"{method}: no response")
        if st.rst_code is not None:
            return None, f"RST_STREAM {st.rst_code}", b""
        code, message = st.status()
        return code, message, st.messages[0] if st.messages else b""

    def next_message(self, sid: int, timeout: float = 5.0) -> Optional[bytes]:
        st = self.streams[sid]
        self.wait(lambda: bool(st.messages) or st.ended, timeout)
        return st.messages.pop(0) if st.messages else None


# ---------------------------------------------------------------------- server
@dataclass
class ServerCall:
    sid: int
    headers: List[Tuple[str, str]]
    body: bytes


@dataclass
class GoServerConfig:
    max_concurrent_streams: Optional[int] = None
    initial_window: int = DEFAULT_WINDOW            # SETTINGS_INITIAL_WINDOW_SIZE we announce (stream receive window)
    continuation_chunk: int = 0                     # > 0: split every header block into chunks of this size
    ping_before_response: bool = False              # a server PING (BDP-style) ahead of the response
    too_many_pings: bool = False                    # GOAWAY(ENHANCE_YOUR_CALM, "too_many_pings") + close on a call
    graceful_goaway: bool = False                   # GOAWAY(2^31-1) + PING, answer, then GOAWAY(last)
    http_status: int = 200                          # != 200: a non-gRPC HTTP error response
    never_answer: bool = False                      # read the call, never respond (hung exporter)
    settings_after_headers: Optional[List[Tuple[int, int]]] = None   # a SETTINGS change mid-call
    refuse_calls: int = 0                           # the first N calls get RST_STREAM(REFUSED_STREAM)
    # What other HTTP/2 servers (C++ gRPC, a proxy in front of an exporter) may
    # send and grpc-go never does. RFC 7540 allows all of it; the client must cope.
    pad: Optional[int] = None                       # not None: every HEADERS / DATA frame PADDED with this many
                                                    # bytes (0: the flag and the pad-length byte, no padding)
    priority_in_headers: bool = False               # HEADERS frames carry the PRIORITY flag (5 bytes)
    noise_frames: bool = False                      # a PRIORITY and an unknown-type frame ahead of the response
    rst_code: Optional[int] = None                  # answer every call with RST_STREAM(rst_code)
    goaway_first: Optional[int] = None              # GOAWAY(last stream 0, this code) instead of an answer
    # protocol violations the client must turn into a clean error
    oversized_data: bool = False                    # a 20000-byte DATA frame (above our 16384 maximum)
    interrupted_headers: bool = False               # HEADERS without END_HEADERS, then DATA
    orphan_continuation: bool = False               # CONTINUATION with no HEADERS before it


class GoServer:
    """A grpc-go server on a Unix socket (kubelet Registration / metrics exporter)."""

    def __init__(self, path: str, handlers: Dict[str, Callable[[bytes], Tuple[int, str, bytes]]],
                 config: Optional[GoServerConfig] = None):
        self.path = path
        self.handlers = handlers
        self.cfg = config or GoServerConfig()
        self.calls: List[ServerCall] = []
        self.violations: List[str] = []
        self.connections = 0
        self.refused = 0
        self.client_settings: List[Dict[int, int]] = []
        self.frames: List[Tuple[str, int, int]] = []
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self._conns: List[socket.socket] = []
        try:
            os.unlink(path)
        except FileNotFoundError:
            pass
        self.lsock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.lsock.bind(path)
        self.lsock.listen(16)
        self.lsock.settimeout(0.1)
        t = threading.Thread(target=self._accept_loop, daemon=True)
        t.start()
        self._threads.append(t)

    def close(self) -> None:
        self._stop.set()
        for c in list(self._conns):
            try:
                c.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
        for t in self._threads:
            t.join(timeout=5)
        self.lsock.close()
        try:
            os.unlink(self.path)
        except FileNotFoundError:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _accept_loop(self) -> None:
        while not self._stop.is_set():
            try:
                c, _ = self.lsock.accept()
            except socket.timeout:
                continue
            except OSError:
                return
            self.connections += 1
            self._conns.append(c)
            t = threading.Thread(target=self._serve_conn, args=(c,), daemon=True)
            t.start()
            self._threads.append(t)

    def _serve_conn(self, c: socket.socket) -> None:
        try:
            _ServerConn(self, c).run()
        except (EOFError, OSError, ConnectionError) as e:
            if not self._stop.is_set() and not isinstance(e, EOFError):
                self.violations.append(f"connection error: {e}")
        finally:
            try:
                c.close()
            except OSError:
                pass


class _ServerConn:
    def __init__(self, srv: GoServer, sock: socket.socket):
        self.srv, self.sock, self.cfg = srv, sock, srv.cfg
        self.rd = FrameReader(sock)
        self.enc, self.dec = GoHpackEncoder(), HpackDecoder()
        self.peer_initial_window = DEFAULT_WINDOW
        self.peer_max_frame = 16384
        self.conn_send_window = DEFAULT_WINDOW
        self.recv_conn = 0                  # bytes received on the connection since our last credit
        self.streams: Dict[int, dict] = {}
        self.stream_send: Dict[int, int] = {}
        self.last_sid = 0
        self._cont: Optional[Tuple[int, bytearray, bool]] = None

    def send(self, data: bytes) -> None:
        self.sock.sendall(data)

    def _padded(self, flags: int, payload: bytes, prio: bool = False) -> Tuple[int, bytes]:
        """(flags, payload) with the configured padding / priority fields added."""
        if prio:
            flags |= PRIORITY_FLAG
            payload = struct.pack(">IB", 0, 15) + payload      # no dependency, weight 16
        if self.cfg.pad is not None:
            flags |= PADDED
            payload = bytes([self.cfg.pad]) + payload + b"\0" * self.cfg.pad
        return flags, payload

    def _headers(self, sid: int, fields, end_stream: bool) -> None:
        block = self.enc.encode(fields)
        # padding and priority fields count against the frame size
        room = self.peer_max_frame - (1 + self.cfg.pad if self.cfg.pad is not None else 0) - \
            (5 if self.cfg.priority_in_headers else 0)
        chunk = self.cfg.continuation_chunk or room
        parts = [block[i:i + chunk] for i in range(0, len(block), chunk)] or [b""]
        out = []
        for i, part in enumerate(parts):
            last = i == len(parts) - 1
            flags = (END_HEADERS if last else 0) | (END_STREAM if i == 0 and end_stream else 0)
            if i == 0:
                flags, part = self._padded(flags, part, self.cfg.priority_in_headers)
            out.append(frame(HEADERS if i == 0 else CONTINUATION, flags, sid, part))
        self.send(b"".join(out))

    def _data(self, sid: int, payload: bytes) -> None:
        """DATA within the client's windows (waits for its WINDOW_UPDATEs)."""
        while payload:
            extra = 1 + self.cfg.pad if self.cfg.pad is not None else 0     # padding is flow-controlled too
            q = min(self.conn_send_window, self.stream_send.get(sid, self.peer_initial_window),
                    self.peer_max_frame) - extra
            if q <= 0:
                f = self.rd.read(5.0)
                if f is None:
                    raise ConnectionError("client never opened its window")
                self._on_frame(*f)
                continue
            chunk, payload = payload[:q], payload[q:]
            self.conn_send_window -= len(chunk) + extra
            self.stream_send[sid] = self.stream_send.get(sid, self.peer_initial_window) - len(chunk) - extra
            fl, pl = self._padded(0, chunk)
            self.send(frame(DATA, fl, sid, pl))

    def run(self) -> None:
        settings = [(S_MAX_FRAME_SIZE, 16384)]
        if self.cfg.max_concurrent_streams is not None:
            settings.append((S_MAX_CONCURRENT_STREAMS, self.cfg.max_concurrent_streams))
        if self.cfg.initial_window != DEFAULT_WINDOW:
            settings.append((S_INITIAL_WINDOW_SIZE, self.cfg.initial_window))
        self.send(frame(SETTINGS, 0, 0, settings_payload(settings)))
        pre = b""
        while len(pre) < len(PREFACE):
            self.sock.settimeout(10)
            chunk = self.sock.recv(len(PREFACE) - len(pre))
            if not chunk:
                raise EOFError
            pre += chunk
        if pre != PREFACE:
            raise ConnectionError(f"bad client preface {pre!r}")
        f = self.rd.read(10)
        if f is None or f[0] != SETTINGS or f[1] & ACK:
            raise ConnectionError(f"client preface not followed by SETTINGS: {f}")
        self._on_frame(*f)
        while not self.srv._stop.is_set():
            f = self.rd.read(0.2)
            if f is not None:
                self._on_frame(*f)

    def _on_frame(self, t: int, fl: int, sid: int, p: bytes) -> None:
        self.srv.frames.append((FRAME_NAMES[t] if t < 10 else str(t), fl, sid))
        if self._cont is not None and (t != CONTINUATION or sid != self._cont[0]):
            raise ConnectionError("client interrupted a header block")
        if len(p) > 16384:
            self.srv.violations.append(f"frame of {len(p)} bytes above our SETTINGS_MAX_FRAME_SIZE")
        if t == SETTINGS:
            if fl & ACK:
                return
            st = {}
            for i in range(0, len(p), 6):
                k, v = struct.unpack(">HI", p[i:i + 6])
                st[k] = v
                if k == S_INITIAL_WINDOW_SIZE:
                    delta = v - self.peer_initial_window
                    self.peer_initial_window = v
                    for s in self.stream_send:
                        self.stream_send[s] += delta
                elif k == S_MAX_FRAME_SIZE:
                    self.peer_max_frame = v
            self.srv.client_settings.append(st)
            self.send(frame(SETTINGS, ACK, 0))
        elif t == PING:
            if not fl & ACK:
                self.send(frame(PING, ACK, 0, p))
        elif t == WINDOW_UPDATE:
            inc = struct.unpack(">I", p)[0] & 0x7FFFFFFF
            if sid == 0:
                self.conn_send_window += inc
            else:
                self.stream_send[sid] = self.stream_send.get(sid, self.peer_initial_window) + inc
        elif t in (HEADERS, CONTINUATION):
            if t == HEADERS:
                if sid <= self.last_sid or not sid & 1:
                    self.srv.violations.append(f"bad new stream id {sid}")
                self.last_sid = sid
                if fl & PADDED:
                    p = p[1:len(p) - p[0]]
                if fl & PRIORITY_FLAG:
                    p = p[5:]
                self._cont = (sid, bytearray(), bool(fl & END_STREAM))
            self._cont[1].extend(p)
            if fl & END_HEADERS:
                csid, block, end = self._cont
                self._cont = None
                self.streams[csid] = {"headers": self.dec.decode(bytes(block)), "body": bytearray(), "recv": 0}
                if end:
                    self._dispatch(csid)
        elif t == DATA:
            s = self.streams.get(sid)
            self.recv_conn += len(p)
            if self.recv_conn > DEFAULT_WINDOW:
                self.srv.violations.append(f"client overran the connection window ({self.recv_conn} bytes)")
            if s is None:
                self.srv.violations.append(f"DATA on unknown stream {sid}")
                return
            s["recv"] += len(p)
            if s["recv"] > self.cfg.initial_window:
                self.srv.violations.append(
                    f"stream {sid}: client sent {s['recv']} bytes into a {self.cfg.initial_window}-byte window")
            s["body"].extend(p)
            # the handler reads as it arrives: credit back at once (onRead)
            if p:
                self.recv_conn -= len(p)
                s["recv"] -= len(p)
                self.send(frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", len(p))) +
                          frame(WINDOW_UPDATE, 0, sid, struct.pack(">I", len(p))))
            if fl & END_STREAM:
                self._dispatch(sid)
        elif t == RST_STREAM:
            self.streams.pop(sid, None)

    def _dispatch(self, sid: int) -> None:
        s = self.streams[sid]
        hdr = dict(s["headers"])
        body = bytes(s["body"])
        msg = body[5:] if len(body) >= 5 else b""
        self.srv.calls.append(ServerCall(sid, s["headers"], msg))
        cfg = self.cfg
        if cfg.never_answer:
            return
        if self.srv.refused < cfg.refuse_calls:
            self.srv.refused += 1
            self.send(frame(RST_STREAM, 0, sid, struct.pack(">I", REFUSED_STREAM)))
            return
        if cfg.too_many_pings:
            self.send(frame(GOAWAY, 0, 0, struct.pack(">II", self.last_sid, ENHANCE_YOUR_CALM) + b"too_many_pings"))
            raise EOFError("closed after too_many_pings")
        if cfg.graceful_goaway:
            self.send(frame(GOAWAY, 0, 0, struct.pack(">II", MAX_WINDOW, NO_ERROR)) + frame(PING, 0, 0, GOAWAY_PING))
        if cfg.ping_before_response:
            self.send(frame(PING, 0, 0, BDP_PING))
        if cfg.http_status != 200:
            self._headers(sid, [(":status", str(cfg.http_status)), ("content-type", "text/plain")], True)
            return
        if cfg.rst_code is not None:
            self.send(frame(RST_STREAM, 0, sid, struct.pack(">I", cfg.rst_code)))
            return
        if cfg.goaway_first is not None:
            self.send(frame(GOAWAY, 0, 0, struct.pack(">II", 0, cfg.goaway_first) + b"shutting down"))
            return
        if cfg.noise_frames:
            self.send(frame(PRIORITY, 0, sid, struct.pack(">IB", 0, 15)) + frame(0xFA, 0x3, sid, b"ext") +
                      frame(0xFB, 0, 0, b""))
        if cfg.oversized_data:
            self._headers(sid, [(":status", "200"), ("content-type", "application/grpc")], False)
            self.send(frame(DATA, 0, sid, b"\0" * 20000))
            return
        if cfg.interrupted_headers:
            block = self.enc.encode([(":status", "200"), ("content-type", "application/grpc")])
            self.send(frame(HEADERS, 0, sid, block) + frame(DATA, 0, sid, grpc_message(b"x")))
            return
        if cfg.orphan_continuation:
            self.send(frame(CONTINUATION, END_HEADERS, sid, self.enc.encode([(":status", "200")])))
            return
        h = self.srv.handlers.get(hdr.get(":path", ""))
        code, message, resp = h(msg) if h is not None else (12, f"unknown method {hdr.get(':path')}", b"")
        if code != 0:   # trailers-only
            self._headers(sid, [(":status", "200"), ("content-type", "application/grpc"),
                                ("grpc-status", str(code)), ("grpc-message", encode_grpc_message(message))],
                          True)
        else:
            self._headers(sid, [(":status", "200"), ("content-type", "application/grpc")], False)
            if cfg.settings_after_headers:
                self.send(frame(SETTINGS, 0, 0, settings_payload(cfg.settings_after_headers)))
            self._data(sid, grpc_message(resp))
            self._headers(sid, [("grpc-status", "0"), ("grpc-message", "")], True)
        if cfg.graceful_goaway:
            # A client that saw the first GOAWAY may close as soon as its last
            # stream ends (RFC 7540 6.8); grpc-go's loopy writer drops the
            # write error of the final GOAWAY in that case.
            try:
                self.send(frame(GOAWAY, 0, 0, struct.pack(">II", self.last_sid, NO_ERROR)))
            except (BrokenPipeError, ConnectionResetError):
                raise EOFError("client closed after the drain")
