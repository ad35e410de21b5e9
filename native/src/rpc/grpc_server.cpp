// Native HTTP/2 gRPC server (see mi355x/grpc_server.h).
//
// One I/O thread owns every connection: epoll over the listening Unix socket,
// the connections and an eventfd that other threads use to hand over
// streaming messages and the stop request. Frames are parsed in place; the
// per-connection HPACK decoder sees header blocks in arrival order (also for
// refused streams, so its dynamic table stays in sync with the client's).
// Responses use literal header fields only (no dynamic-table state on our
// side). Flow control: every DATA frame received is credited back at once
// (connection and stream); what we send waits for the peer's windows.
#include "mi355x/grpc_server.h"

#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>

#include "hpack.h"

namespace mi355x::rpc {
namespace {

enum FrameType : uint8_t {
  kData = 0,
  kHeaders = 1,
  kPriority = 2,
  kRstStream = 3,
  kSettings = 4,
  kPushPromise = 5,
  kPing = 6,
  kGoaway = 7,
  kWindowUpdate = 8,
  kContinuation = 9,
};
constexpr uint8_t kEndStream = 0x1, kAck = 0x1, kEndHeaders = 0x4, kPadded = 0x8, kPriorityFlag = 0x20;
enum H2Error : uint32_t {
  kNoError = 0,
  kProtocolError = 1,
  kFlowControlError = 3,
  kStreamClosed = 5,
  kFrameSizeError = 6,
  kRefusedStream = 7,
  kCancel = 8,
  kCompressionError = 9,
};

constexpr size_t kOurMaxFrame = 16384;  // SETTINGS_MAX_FRAME_SIZE we accept (the default)
constexpr size_t kMaxHeaderBlock = 64 * 1024;
constexpr size_t kMaxMessage = 4 * 1024 * 1024;
constexpr uint32_t kMaxConcurrentStreams = 128;
constexpr int64_t kMaxWindow = 0x7fffffff;
constexpr char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
constexpr size_t kPrefaceLen = 24;

uint32_t be32(const uint8_t* p) {
  return (static_cast<uint32_t>(p[0]) << 24) | (static_cast<uint32_t>(p[1]) << 16) |
         (static_cast<uint32_t>(p[2]) << 8) | p[3];
}

void put_be32(std::string* out, uint32_t v) {
  out->push_back(static_cast<char>(v >> 24));
  out->push_back(static_cast<char>(v >> 16));
  out->push_back(static_cast<char>(v >> 8));
  out->push_back(static_cast<char>(v));
}

void put_frame(std::string* out, uint8_t type, uint8_t flags, uint32_t sid, const char* payload, size_t len) {
  out->push_back(static_cast<char>(len >> 16));
  out->push_back(static_cast<char>(len >> 8));
  out->push_back(static_cast<char>(len));
  out->push_back(static_cast<char>(type));
  out->push_back(static_cast<char>(flags));
  put_be32(out, sid & 0x7fffffffu);
  if (len) out->append(payload, len);
}

std::string grpc_frame(const std::string& msg) {
  std::string f;
  f.reserve(5 + msg.size());
  f.push_back('\0');
  put_be32(&f, static_cast<uint32_t>(msg.size()));
  f.append(msg);
  return f;
}

std::string percent_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s.substr(0, 1024)) {
    if (c >= 0x20 && c <= 0x7E && c != '%') {
      o.push_back(static_cast<char>(c));
    } else {
      o.push_back('%');
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    }
  }
  return o;
}

// grpc-message as grpc-go sends it: percent-encoded (a malformed escape is kept as is)
std::string percent_decode(const std::string& s) {
  auto hexv = [](char h) {
    return h >= '0' && h <= '9' ? h - '0' : h >= 'a' && h <= 'f' ? h - 'a' + 10 : h >= 'A' && h <= 'F' ? h - 'A' + 10 : -1;
  };
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && hexv(s[i + 1]) >= 0 && hexv(s[i + 2]) >= 0) {
      o.push_back(static_cast<char>(hexv(s[i + 1]) * 16 + hexv(s[i + 2])));
      i += 2;
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

struct Stream {
  uint32_t id = 0;
  std::string header_block;
  bool headers_done = false;
  bool end_on_headers = false;
  bool refused = false;
  std::string path, method, content_type;
  std::string data;
  bool remote_closed = false;
  bool dispatched = false;
  int64_t send_window = 65535;
  std::string out;  // DATA payload waiting for flow-control credit
  size_t out_off = 0;
  bool trailers_queued = false;
  std::string trailers;  // header block sent (END_STREAM) once `out` has drained
  bool streaming = false;
  uint64_t call_id = 0;
  bool finished = false;
};

struct Conn {
  int fd = -1;
  std::string in;
  std::string out;
  size_t out_off = 0;
  bool preface_done = false;
  bool settings_seen = false;  // the client preface's SETTINGS (must be its first frame)
  HpackDecoder dec;
  int64_t send_window = 65535;
  int64_t peer_initial_window = 65535;
  size_t peer_max_frame = 16384;
  std::map<uint32_t, Stream> streams;
  uint32_t last_stream = 0;
  uint32_t cont_stream = 0;
  bool goaway_sent = false;
  bool errored = false;  // connection error: input is discarded, the connection ends once flushed
  bool closing = false;
  bool epollout = false;
  bool dead = false;
  bool made_call = false;  // a call on a served route (a device-plugin client, i.e. kubelet)
};

}  // namespace

struct GrpcServer::Impl {
  struct Route {
    bool streaming = false;
    UnaryFn unary;
    StreamOpenFn open;
    StreamCloseFn close;
  };
  struct CallRef {
    int fd;
    uint32_t sid;
    std::string route;
  };
  struct Outgoing {
    std::string route;  // broadcast to every stream of this route ("" = one call)
    uint64_t call_id;
    std::string msg;
  };

  std::unordered_map<std::string, Route> routes;
  std::string sock_path;
  int listen_fd = -1, epfd = -1, evfd = -1;
  std::thread thread;
  std::unordered_map<int, std::unique_ptr<Conn>> conns;

  mutable std::mutex mu;  // calls, outbox, stop request
  std::unordered_map<uint64_t, CallRef> calls;
  std::vector<Outgoing> outbox;
  bool stop_requested = false;
  double grace_s = 0.5;
  uint64_t next_call = 1;

  std::atomic<uint64_t> n_conns{0}, n_calls{0}, n_proto_err{0}, bytes_in{0}, bytes_out{0}, n_stream_opens{0};
  std::atomic<uint64_t> n_caller_err{0};  // protocol errors on connections that had made a served call

  // ------------------------------------------------------------------ output
  void send_settings(Conn& c) {
    std::string p;
    auto setting = [&](uint16_t id, uint32_t v) {
      p.push_back(static_cast<char>(id >> 8));
      p.push_back(static_cast<char>(id));
      put_be32(&p, v);
    };
    setting(0x3, kMaxConcurrentStreams);       // MAX_CONCURRENT_STREAMS
    setting(0x6, kMaxHeaderBlock);             // MAX_HEADER_LIST_SIZE
    put_frame(&c.out, kSettings, 0, 0, p.data(), p.size());
  }

  void goaway(Conn& c, uint32_t code, const char* debug = "") {
    if (c.goaway_sent) return;
    std::string p;
    put_be32(&p, c.last_stream);
    put_be32(&p, code);
    p.append(debug);
    put_frame(&c.out, kGoaway, 0, 0, p.data(), p.size());
    c.goaway_sent = true;
  }

  void conn_error(Conn& c, uint32_t code, const char* why) {
    n_proto_err++;
    if (c.made_call) n_caller_err++;
    goaway(c, code, why);
    c.closing = true;
    c.errored = true;
  }

  void rst(Conn& c, uint32_t sid, uint32_t code) {
    std::string p;
    put_be32(&p, code);
    put_frame(&c.out, kRstStream, 0, sid, p.data(), p.size());
  }

  void window_update(Conn& c, uint32_t sid, uint32_t inc) {
    std::string p;
    put_be32(&p, inc & 0x7fffffffu);
    put_frame(&c.out, kWindowUpdate, 0, sid, p.data(), p.size());
  }

  static std::string response_headers() {
    std::string h;
    hpack_put_indexed(&h, 8);                        // :status 200
    hpack_put_literal(&h, 31, "application/grpc");  // content-type
    return h;
  }

  static std::string trailer_block(int status, const std::string& message, bool trailers_only) {
    std::string h = trailers_only ? response_headers() : std::string();
    hpack_put_literal(&h, "grpc-status", std::to_string(status));
    if (!message.empty()) hpack_put_literal(&h, "grpc-message", percent_encode(message));
    return h;
  }

  void send_headers(Conn& c, uint32_t sid, const std::string& block, bool end_stream) {
    // header blocks here are far below any legal SETTINGS_MAX_FRAME_SIZE (>= 16384)
    put_frame(&c.out, kHeaders, static_cast<uint8_t>(kEndHeaders | (end_stream ? kEndStream : 0)), sid,
              block.data(), block.size());
  }

  // DATA within the windows, then the trailers; true once the stream is complete
  bool pump(Conn& c, Stream& s) {
    while (s.out_off < s.out.size()) {
      const int64_t w = std::min(c.send_window, s.send_window);
      if (w <= 0) return false;
      const size_t chunk = std::min({s.out.size() - s.out_off, static_cast<size_t>(w), c.peer_max_frame});
      put_frame(&c.out, kData, 0, s.id, s.out.data() + s.out_off, chunk);
      c.send_window -= static_cast<int64_t>(chunk);
      s.send_window -= static_cast<int64_t>(chunk);
      s.out_off += chunk;
    }
    s.out.clear();
    s.out_off = 0;
    if (s.trailers_queued) {
      send_headers(c, s.id, s.trailers, true);
      s.trailers_queued = false;
      s.finished = true;
      return true;
    }
    return false;
  }

  void finish_stream(Conn& c, uint32_t sid) {
    auto it = c.streams.find(sid);
    if (it == c.streams.end()) return;
    if (it->second.streaming) end_call(it->second.call_id);
    c.streams.erase(it);
  }

  void end_call(uint64_t call_id) {
    StreamCloseFn close;
    {
      std::lock_guard<std::mutex> lk(mu);
      auto it = calls.find(call_id);
      if (it == calls.end()) return;
      auto r = routes.find(it->second.route);
      if (r != routes.end()) close = r->second.close;
      calls.erase(it);
    }
    if (close) close(call_id);
  }

  void pump_all(Conn& c) {
    std::vector<uint32_t> done;
    for (auto& [sid, s] : c.streams)
      if (pump(c, s)) done.push_back(sid);
    for (uint32_t sid : done) finish_stream(c, sid);
  }

  void queue_message(Conn&, Stream& s, const std::string& msg) {
    s.out.append(grpc_frame(msg));
  }

  void trailers_only(Conn& c, Stream& s, int status, const std::string& message) {
    send_headers(c, s.id, trailer_block(status, message, true), true);
    s.finished = true;
  }

  // ------------------------------------------------------------------ calls
  void dispatch(Conn& c, Stream& s) {
    if (s.dispatched) return;
    s.dispatched = true;
    n_calls++;
    auto r = routes.find(s.path);
    if (r == routes.end()) return trailers_only(c, s, kUnimplemented, "unknown method " + s.path);
    c.made_call = true;
    if (s.data.size() < 5) return trailers_only(c, s, kInternal, "missing request message");
    const auto* d = reinterpret_cast<const uint8_t*>(s.data.data());
    if (d[0] != 0) return trailers_only(c, s, kUnimplemented, "grpc compression is not supported");
    const uint32_t len = be32(d + 1);
    if (static_cast<size_t>(len) + 5 != s.data.size())
      return trailers_only(c, s, kInternal, "expected exactly one request message");
    std::string req = s.data.substr(5);
    s.data.clear();
    s.data.shrink_to_fit();
    Reply rep;
    uint64_t call_id = 0;
    if (r->second.streaming) {
      {
        std::lock_guard<std::mutex> lk(mu);
        call_id = next_call++;
        calls[call_id] = CallRef{c.fd, s.id, s.path};
      }
      try {
        rep = r->second.open(call_id, req);
      } catch (const std::exception& e) {
        rep = Reply{kUnknown, e.what(), ""};
      }
      if (rep.status != kOk) {
        std::lock_guard<std::mutex> lk(mu);
        calls.erase(call_id);
        return trailers_only(c, s, rep.status, rep.message);
      }
      s.streaming = true;
      s.call_id = call_id;
      n_stream_opens++;
      send_headers(c, s.id, response_headers(), false);
      queue_message(c, s, rep.body);
      pump(c, s);
      return;
    }
    try {
      rep = r->second.unary(req);
    } catch (const std::exception& e) {
      rep = Reply{kUnknown, e.what(), ""};
    }
    if (rep.status != kOk) return trailers_only(c, s, rep.status, rep.message);
    send_headers(c, s.id, response_headers(), false);
    queue_message(c, s, rep.body);
    s.trailers = trailer_block(kOk, "", false);
    s.trailers_queued = true;
    pump(c, s);
  }

  bool finish_headers(Conn& c, Stream& s) {
    HeaderList hl;
    const bool ok = c.dec.decode(reinterpret_cast<const uint8_t*>(s.header_block.data()), s.header_block.size(), &hl);
    s.header_block.clear();
    if (!ok) {
      conn_error(c, kCompressionError, "hpack");
      return false;
    }
    if (s.refused) {
      rst(c, s.id, kRefusedStream);
      s.finished = true;
      return true;
    }
    if (!s.headers_done) {
      s.headers_done = true;
      for (auto& [k, v] : hl) {
        if (k == ":path") s.path = v;
        else if (k == ":method") s.method = v;
        else if (k == "content-type") s.content_type = v;
      }
      if (s.method != "POST" || s.path.empty()) {
        rst(c, s.id, kProtocolError);
        s.finished = true;
        return true;
      }
      if (s.content_type.compare(0, 16, "application/grpc") != 0) {
        std::string h;
        hpack_put_literal(&h, 8, "415");  // :status 415 (gRPC: not a gRPC request)
        send_headers(c, s.id, h, true);
        s.finished = true;
        return true;
      }
    }
    if (s.end_on_headers) {
      s.remote_closed = true;
      dispatch(c, s);
    }
    return true;
  }

  // ------------------------------------------------------------------ input
  // false: the connection is finished (error or GOAWAY sent)
  bool frame(Conn& c, uint8_t type, uint8_t flags, uint32_t sid, const uint8_t* p, size_t len) {
    if (c.cont_stream && (type != kContinuation || sid != c.cont_stream)) {
      conn_error(c, kProtocolError, "expected CONTINUATION");
      return false;
    }
    if (!c.settings_seen) {  // RFC 7540 3.5: the preface ends with a SETTINGS frame
      if (type != kSettings || (flags & kAck)) return conn_error(c, kProtocolError, "preface without SETTINGS"), false;
      c.settings_seen = true;
    }
    switch (type) {
      case kData: {
        if (sid == 0) return conn_error(c, kProtocolError, "DATA on stream 0"), false;
        const size_t flow = len;  // flow-controlled size: the whole payload, padding included
        if (flow) window_update(c, 0, static_cast<uint32_t>(flow));  // connection credit back at once
        size_t pad = 0;
        if (flags & kPadded) {
          if (len < 1 || p[0] >= len) return conn_error(c, kProtocolError, "bad padding"), false;
          pad = p[0];
          ++p;
          --len;
        }
        auto it = c.streams.find(sid);
        if (it == c.streams.end() || it->second.remote_closed) {
          if (sid > c.last_stream) return conn_error(c, kProtocolError, "DATA on idle stream"), false;
          rst(c, sid, kStreamClosed);
          return true;
        }
        Stream& s = it->second;
        const size_t body = len - pad;
        if (s.data.size() + body > kMaxMessage) {
          trailers_only(c, s, kResourceExhausted, "request message too large");
          rst(c, sid, kCancel);
          finish_stream(c, sid);
          return true;
        }
        s.data.append(reinterpret_cast<const char*>(p), body);
        if (flags & kEndStream) {
          s.remote_closed = true;
          dispatch(c, s);
        } else if (flow) {
          window_update(c, sid, static_cast<uint32_t>(flow));
        }
        if (s.finished) finish_stream(c, sid);
        return true;
      }
      case kHeaders: {
        if (sid == 0 || !(sid & 1)) return conn_error(c, kProtocolError, "bad stream id"), false;
        size_t pad = 0;
        if (flags & kPadded) {
          if (len < 1) return conn_error(c, kProtocolError, "bad padding"), false;
          pad = p[0];
          ++p;
          --len;
        }
        if (flags & kPriorityFlag) {
          if (len < 5) return conn_error(c, kProtocolError, "short priority"), false;
          p += 5;
          len -= 5;
        }
        if (pad > len) return conn_error(c, kProtocolError, "bad padding"), false;
        len -= pad;
        auto it = c.streams.find(sid);
        Stream* s;
        if (it == c.streams.end()) {
          if (sid <= c.last_stream) return conn_error(c, kStreamClosed, "stream id reused"), false;
          c.last_stream = sid;
          Stream& ns = c.streams[sid];
          ns.id = sid;
          ns.send_window = c.peer_initial_window;
          ns.refused = c.closing || c.streams.size() > kMaxConcurrentStreams;
          s = &ns;
        } else {
          s = &it->second;  // trailers from the client (gRPC clients send none)
        }
        if (s->header_block.size() + len > kMaxHeaderBlock)
          return conn_error(c, kProtocolError, "header block too large"), false;
        s->header_block.append(reinterpret_cast<const char*>(p), len);
        if (flags & kEndStream) s->end_on_headers = true;
        if (flags & kEndHeaders) {
          if (!finish_headers(c, *s)) return false;
          if (s->finished) finish_stream(c, sid);
        } else {
          c.cont_stream = sid;
        }
        return true;
      }
      case kContinuation: {
        // only right after a HEADERS / CONTINUATION of the same stream without END_HEADERS
        if (!c.cont_stream) return conn_error(c, kProtocolError, "CONTINUATION without HEADERS"), false;
        auto it = c.streams.find(sid);
        if (it == c.streams.end()) return conn_error(c, kProtocolError, "CONTINUATION without HEADERS"), false;
        Stream& s = it->second;
        if (s.header_block.size() + len > kMaxHeaderBlock)
          return conn_error(c, kProtocolError, "header block too large"), false;
        s.header_block.append(reinterpret_cast<const char*>(p), len);
        if (flags & kEndHeaders) {
          c.cont_stream = 0;
          if (!finish_headers(c, s)) return false;
          if (s.finished) finish_stream(c, sid);
        }
        return true;
      }
      case kPriority:
        return true;
      case kRstStream:
        if (sid == 0) return conn_error(c, kProtocolError, "RST_STREAM on stream 0"), false;
        if (len != 4) return conn_error(c, kFrameSizeError, "bad RST_STREAM"), false;
        if (sid > c.last_stream) return conn_error(c, kProtocolError, "RST_STREAM on an idle stream"), false;
        finish_stream(c, sid);
        return true;
      case kSettings: {
        if (sid != 0) return conn_error(c, kProtocolError, "SETTINGS on a stream"), false;
        if (flags & kAck) return true;
        if (len % 6) return conn_error(c, kFrameSizeError, "SETTINGS length"), false;
        for (size_t i = 0; i < len; i += 6) {
          const uint16_t id = static_cast<uint16_t>((p[i] << 8) | p[i + 1]);
          const uint32_t v = be32(p + i + 2);
          if (id == 0x4) {  // INITIAL_WINDOW_SIZE
            if (v > static_cast<uint32_t>(kMaxWindow)) return conn_error(c, kFlowControlError, "window"), false;
            const int64_t delta = static_cast<int64_t>(v) - c.peer_initial_window;
            c.peer_initial_window = v;
            for (auto& [k, s] : c.streams) {
              s.send_window += delta;  // RFC 7540 6.9.2: an overflow is a connection error
              if (s.send_window > kMaxWindow) return conn_error(c, kFlowControlError, "stream window overflow"), false;
            }
          } else if (id == 0x2) {  // ENABLE_PUSH
            if (v > 1) return conn_error(c, kProtocolError, "ENABLE_PUSH"), false;
          } else if (id == 0x5) {  // MAX_FRAME_SIZE
            if (v < 16384 || v > 16777215) return conn_error(c, kProtocolError, "max frame size"), false;
            c.peer_max_frame = v;
          }
        }
        put_frame(&c.out, kSettings, kAck, 0, nullptr, 0);
        pump_all(c);
        return true;
      }
      case kPushPromise:
        return conn_error(c, kProtocolError, "PUSH_PROMISE from a client"), false;
      case kPing:
        if (sid != 0 || len != 8) return conn_error(c, kFrameSizeError, "bad PING"), false;
        if (!(flags & kAck)) put_frame(&c.out, kPing, kAck, 0, reinterpret_cast<const char*>(p), 8);
        return true;
      case kGoaway:
        c.closing = true;
        return true;
      case kWindowUpdate: {
        if (len != 4) return conn_error(c, kFrameSizeError, "bad WINDOW_UPDATE"), false;
        const uint32_t inc = be32(p) & 0x7fffffffu;
        if (sid == 0) {
          if (inc == 0) return conn_error(c, kProtocolError, "zero window increment"), false;
          c.send_window += inc;
          if (c.send_window > kMaxWindow) return conn_error(c, kFlowControlError, "window overflow"), false;
          pump_all(c);
          return true;
        }
        if (sid > c.last_stream) return conn_error(c, kProtocolError, "WINDOW_UPDATE on an idle stream"), false;
        auto it = c.streams.find(sid);
        if (it == c.streams.end()) return true;
        if (inc == 0) {
          rst(c, sid, kProtocolError);
          finish_stream(c, sid);
          return true;
        }
        it->second.send_window += inc;
        if (it->second.send_window > kMaxWindow) {
          rst(c, sid, kFlowControlError);
          finish_stream(c, sid);
          return true;
        }
        if (pump(c, it->second)) finish_stream(c, sid);
        return true;
      }
      default:
        return true;  // unknown frame types are ignored
    }
  }

  void process(Conn& c) {
    size_t off = 0;
    if (!c.preface_done) {
      if (c.in.size() < kPrefaceLen) return;
      if (std::memcmp(c.in.data(), kPreface, kPrefaceLen) != 0) {
        n_proto_err++;
        c.closing = true;
        c.dead = true;
        return;
      }
      off = kPrefaceLen;
      c.preface_done = true;
    }
    while (!c.errored) {
      if (c.in.size() - off < 9) break;
      const auto* h = reinterpret_cast<const uint8_t*>(c.in.data() + off);
      const size_t len = (static_cast<size_t>(h[0]) << 16) | (static_cast<size_t>(h[1]) << 8) | h[2];
      if (len > kOurMaxFrame) {
        conn_error(c, kFrameSizeError, "frame too large");
        return;
      }
      if (c.in.size() - off < 9 + len) break;
      const uint8_t type = h[3], flags = h[4];
      const uint32_t sid = be32(h + 5) & 0x7fffffffu;
      off += 9 + len;
      if (!frame(c, type, flags, sid, h + 9, len)) break;
    }
    if (c.errored)
      c.in.clear();
    else
      c.in.erase(0, off);
  }

  // ------------------------------------------------------------------ I/O
  void set_events(Conn& c, bool out) {
    if (c.epollout == out) return;
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP | (out ? static_cast<uint32_t>(EPOLLOUT) : 0u);
    ev.data.fd = c.fd;
    epoll_ctl(epfd, EPOLL_CTL_MOD, c.fd, &ev);
    c.epollout = out;
  }

  void flush(Conn& c) {
    while (c.out_off < c.out.size()) {
      const ssize_t n = ::send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
      if (n > 0) {
        c.out_off += static_cast<size_t>(n);
        bytes_out += static_cast<uint64_t>(n);
        continue;
      }
      if (n < 0 && errno == EINTR) continue;
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        set_events(c, true);
        return;
      }
      c.dead = true;
      return;
    }
    c.out.clear();
    c.out_off = 0;
    set_events(c, false);
  }

  void close_conn(int fd) {
    auto it = conns.find(fd);
    if (it == conns.end()) return;
    Conn& c = *it->second;
    std::vector<uint32_t> sids;
    for (auto& [sid, s] : c.streams) sids.push_back(sid);
    for (uint32_t sid : sids) finish_stream(c, sid);
    epoll_ctl(epfd, EPOLL_CTL_DEL, fd, nullptr);
    ::close(fd);
    conns.erase(it);
  }

  void accept_all() {
    while (true) {
      const int fd = ::accept4(listen_fd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.fd = fd;
      epoll_ctl(epfd, EPOLL_CTL_ADD, fd, &ev);
      send_settings(*c);
      n_conns++;
      Conn& ref = *c;
      conns[fd] = std::move(c);
      flush(ref);
    }
  }

  void read_conn(Conn& c) {
    char buf[65536];
    while (true) {
      const ssize_t n = ::read(c.fd, buf, sizeof(buf));
      if (n > 0) {
        bytes_in += static_cast<uint64_t>(n);
        if (!c.errored) c.in.append(buf, static_cast<size_t>(n));
        if (static_cast<size_t>(n) < sizeof(buf)) break;
        continue;
      }
      if (n < 0 && errno == EINTR) continue;
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      c.dead = true;  // EOF or error
      break;
    }
    if (!c.in.empty()) process(c);
  }

  void drain_outbox() {
    std::vector<Outgoing> todo;
    std::vector<std::pair<uint64_t, CallRef>> targets;
    {
      std::lock_guard<std::mutex> lk(mu);
      todo.swap(outbox);
    }
    for (auto& o : todo) {
      targets.clear();
      {
        std::lock_guard<std::mutex> lk(mu);
        if (o.route.empty()) {
          auto it = calls.find(o.call_id);
          if (it != calls.end()) targets.emplace_back(it->first, it->second);
        } else {
          for (auto& [id, ref] : calls)
            if (ref.route == o.route) targets.emplace_back(id, ref);
        }
      }
      for (auto& [id, ref] : targets) {
        auto ci = conns.find(ref.fd);
        if (ci == conns.end()) continue;
        Conn& c = *ci->second;
        auto si = c.streams.find(ref.sid);
        if (si == c.streams.end() || si->second.trailers_queued) continue;
        queue_message(c, si->second, o.msg);
        if (pump(c, si->second)) finish_stream(c, ref.sid);
      }
    }
  }

  void begin_stop() {
    if (listen_fd >= 0) {
      epoll_ctl(epfd, EPOLL_CTL_DEL, listen_fd, nullptr);
      ::close(listen_fd);
      listen_fd = -1;
    }
    for (auto& [fd, c] : conns) {
      std::vector<uint32_t> done;
      for (auto& [sid, s] : c->streams) {
        if (s.streaming && !s.trailers_queued && !s.finished) {
          s.trailers = trailer_block(kOk, "", false);
          s.trailers_queued = true;
          if (pump(*c, s)) done.push_back(sid);
        }
      }
      for (uint32_t sid : done) finish_stream(*c, sid);
      goaway(*c, kNoError);
      c->closing = true;
    }
  }

  void run() {
    epoll_event evs[64];
    bool stopping = false;
    std::chrono::steady_clock::time_point deadline{};
    while (true) {
      const int n = epoll_wait(epfd, evs, 64, stopping ? 10 : -1);
      for (int i = 0; i < n; ++i) {
        const int fd = evs[i].data.fd;
        if (fd == listen_fd) {
          accept_all();
        } else if (fd == evfd) {
          uint64_t v;
          while (::read(evfd, &v, sizeof(v)) > 0) {
          }
          drain_outbox();
          bool stop;
          {
            std::lock_guard<std::mutex> lk(mu);
            stop = stop_requested;
          }
          if (stop && !stopping) {
            stopping = true;
            deadline = std::chrono::steady_clock::now() +
                       std::chrono::microseconds(static_cast<int64_t>(grace_s * 1e6));
            begin_stop();
          }
        } else {
          auto it = conns.find(fd);
          if (it == conns.end()) continue;
          Conn& c = *it->second;
          if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) read_conn(c);
        }
      }
      // write what the handlers produced; reap finished connections
      std::vector<int> dead;
      for (auto& [fd, c] : conns) {
        if (!c->out.empty()) flush(*c);
        const bool drained = c->out.empty();
        if (c->dead || (c->closing && drained && (c->goaway_sent || c->streams.empty()))) dead.push_back(fd);
      }
      for (int fd : dead) close_conn(fd);
      if (after_io) after_io();
      if (stopping) {
        bool all_drained = true;
        for (auto& [fd, c] : conns) all_drained = all_drained && c->out.empty();
        if (all_drained || std::chrono::steady_clock::now() > deadline) break;
      }
    }
    std::vector<int> fds;
    for (auto& [fd, c] : conns) fds.push_back(fd);
    for (int fd : fds) close_conn(fd);
  }

  std::function<void()> after_io;

  void wake() {
    const uint64_t one = 1;
    ssize_t r = ::write(evfd, &one, sizeof(one));
    (void)r;
  }
};

GrpcServer::GrpcServer() : impl_(new Impl) {}

GrpcServer::~GrpcServer() { stop(0.0); }

void GrpcServer::set_after_io(std::function<void()> fn) { impl_->after_io = std::move(fn); }

void GrpcServer::add_unary(const std::string& path, UnaryFn fn) {
  Impl::Route r;
  r.unary = std::move(fn);
  impl_->routes[path] = std::move(r);
}

void GrpcServer::add_server_stream(const std::string& path, StreamOpenFn open, StreamCloseFn close) {
  Impl::Route r;
  r.streaming = true;
  r.open = std::move(open);
  r.close = std::move(close);
  impl_->routes[path] = std::move(r);
}

std::string GrpcServer::start(const std::string& unix_path) {
  if (running_.load()) return "already running";
  Impl& I = *impl_;
  sockaddr_un addr{};
  if (unix_path.size() >= sizeof(addr.sun_path)) return "socket path too long: " + unix_path;
  addr.sun_family = AF_UNIX;
  std::memcpy(addr.sun_path, unix_path.c_str(), unix_path.size() + 1);
  const int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) return std::string("socket: ") + std::strerror(errno);
  ::unlink(unix_path.c_str());
  if (::bind(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0 || ::listen(fd, 64) != 0) {
    const std::string err = std::string("bind/listen ") + unix_path + ": " + std::strerror(errno);
    ::close(fd);
    return err;
  }
  I.listen_fd = fd;
  I.sock_path = unix_path;
  I.epfd = ::epoll_create1(EPOLL_CLOEXEC);
  I.evfd = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (I.epfd < 0 || I.evfd < 0) {
    const std::string err = std::string("epoll/eventfd: ") + std::strerror(errno);
    ::close(fd);
    if (I.epfd >= 0) ::close(I.epfd);
    if (I.evfd >= 0) ::close(I.evfd);
    I.listen_fd = I.epfd = I.evfd = -1;
    return err;
  }
  for (int f : {I.listen_fd, I.evfd}) {
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = f;
    epoll_ctl(I.epfd, EPOLL_CTL_ADD, f, &ev);
  }
  {
    std::lock_guard<std::mutex> lk(I.mu);
    I.stop_requested = false;
  }
  running_.store(true);
  I.thread = std::thread([&I] { I.run(); });
  return "";
}

void GrpcServer::stop(double grace_s) {
  Impl& I = *impl_;
  if (!running_.exchange(false)) return;
  {
    std::lock_guard<std::mutex> lk(I.mu);
    I.stop_requested = true;
    I.grace_s = grace_s;
  }
  I.wake();
  if (I.thread.joinable()) I.thread.join();
  if (I.listen_fd >= 0) ::close(I.listen_fd);
  ::close(I.epfd);
  ::close(I.evfd);
  I.listen_fd = I.epfd = I.evfd = -1;
  std::lock_guard<std::mutex> lk(I.mu);
  I.calls.clear();
  I.outbox.clear();
}

size_t GrpcServer::broadcast(const std::string& path, const std::string& msg) {
  Impl& I = *impl_;
  size_t n = 0;
  {
    std::lock_guard<std::mutex> lk(I.mu);
    if (!running_.load()) return 0;
    for (auto& [id, ref] : I.calls) n += ref.route == path;
    if (!n) return 0;
    I.outbox.push_back(Impl::Outgoing{path, 0, msg});
  }
  I.wake();
  return n;
}

bool GrpcServer::send(uint64_t call_id, const std::string& msg) {
  Impl& I = *impl_;
  {
    std::lock_guard<std::mutex> lk(I.mu);
    if (!running_.load() || !I.calls.count(call_id)) return false;
    I.outbox.push_back(Impl::Outgoing{"", call_id, msg});
  }
  I.wake();
  return true;
}

size_t GrpcServer::open_streams(const std::string& path) const {
  std::lock_guard<std::mutex> lk(impl_->mu);
  size_t n = 0;
  for (auto& [id, ref] : impl_->calls) n += path.empty() || ref.route == path;
  return n;
}

ServerStats GrpcServer::stats() const {
  ServerStats s;
  s.connections = impl_->n_conns.load();
  s.calls = impl_->n_calls.load();
  s.streams_open = open_streams("");
  s.streams_opened = impl_->n_stream_opens.load();
  s.protocol_errors = impl_->n_proto_err.load();
  s.caller_protocol_errors = impl_->n_caller_err.load();
  s.bytes_in = impl_->bytes_in.load();
  s.bytes_out = impl_->bytes_out.load();
  return s;
}

}  // namespace mi355x::rpc

// ---------------------------------------------------------------- client
namespace mi355x::rpc {

namespace {

const char* h2_error_name(uint32_t code) {
  static const char* kNames[] = {"NO_ERROR",      "PROTOCOL_ERROR",     "INTERNAL_ERROR",     "FLOW_CONTROL_ERROR",
                                 "SETTINGS_TIMEOUT", "STREAM_CLOSED",   "FRAME_SIZE_ERROR",   "REFUSED_STREAM",
                                 "CANCEL",        "COMPRESSION_ERROR",  "CONNECT_ERROR",      "ENHANCE_YOUR_CALM",
                                 "INADEQUATE_SECURITY", "HTTP_1_1_REQUIRED"};
  return code < sizeof(kNames) / sizeof(kNames[0]) ? kNames[code] : "UNKNOWN";
}

// RST_STREAM code -> gRPC status (grpc-go http2ErrConvTab, internal/transport/http_util.go)
int rst_to_status(uint32_t code) {
  switch (code) {
    case 7: return kUnavailable;          // REFUSED_STREAM: not processed, safe to retry
    case 8: return kCancelled;            // CANCEL
    case 11: return kResourceExhausted;   // ENHANCE_YOUR_CALM
    case 12: return kPermissionDenied;    // INADEQUATE_SECURITY
    default: return kInternal;
  }
}

// HTTP status of a response that is not gRPC -> gRPC status (grpc-go HTTPStatusConvTab)
int http_to_status(int http) {
  switch (http) {
    case 400: return kInternal;
    case 401: return kUnauthenticated;
    case 403: return kPermissionDenied;
    case 404: return kUnimplemented;
    case 429: case 502: case 503: case 504: return kUnavailable;
    default: return kUnknown;
  }
}

}  // namespace

struct ClientState {
  HpackDecoder dec;
  int64_t conn_window = 65535;       // what we may still send on the connection
  int64_t peer_initial_window = 65535;
  size_t peer_max_frame = 16384;
  uint64_t recv_unacked = 0;         // DATA received and not yet credited back on the connection
  uint32_t cont_sid = 0;             // header block in progress (CONTINUATION expected)
  bool cont_end_stream = false;
  std::string cont_block;
  bool going_away = false;
  uint32_t goaway_last = 0x7fffffffu;
  uint32_t goaway_code = 0;
  std::string goaway_debug;
};

// One call's view of the connection while it runs.
struct Call {
  uint32_t sid = 0;
  int64_t send_window = 65535;
  bool headers_seen = false;
  int http_status = 0;
  std::string content_type;
  int grpc_status = -1;
  std::string grpc_message;
  std::string data;
  uint32_t recv_unacked = 0;  // stream bytes received since our last WINDOW_UPDATE for it
  bool done = false;
  bool failed = false;
  Reply fail;
};

GrpcClient::GrpcClient() = default;
GrpcClient::~GrpcClient() { close(); }

bool GrpcClient::going_away() const { return st_ && st_->going_away; }

void GrpcClient::close() {
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
  in_.clear();
  st_.reset();
}

namespace {

using Clock = std::chrono::steady_clock;

enum class Ready { kOk, kTimeout, kAbort, kError };

// Waits for `events` on fd (or the abort fd); EINTR re-polls with the time left.
Ready wait_fd(int fd, short events, int abort_fd, Clock::time_point deadline) {
  while (true) {
    const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count();
    if (left <= 0) return Ready::kTimeout;
    pollfd p[2] = {{fd, events, 0}, {abort_fd, POLLIN, 0}};
    const int r = ::poll(p, abort_fd >= 0 ? 2 : 1, static_cast<int>(std::min<long long>(left, 1 << 30)));
    if (r < 0) {
      if (errno == EINTR) continue;
      return Ready::kError;
    }
    if (r == 0) continue;  // re-check the deadline
    if (abort_fd >= 0 && (p[1].revents & POLLIN)) return Ready::kAbort;
    if (p[0].revents & (events | POLLHUP | POLLERR)) return Ready::kOk;
  }
}

const char* ready_error(Ready r) {
  return r == Ready::kTimeout ? "deadline exceeded" : r == Ready::kAbort ? "interrupted" : "poll failed";
}

}  // namespace

std::string GrpcClient::connect(const std::string& unix_path, double timeout_s) {
  close();
  sockaddr_un addr{};
  if (unix_path.size() >= sizeof(addr.sun_path)) return "socket path too long";
  addr.sun_family = AF_UNIX;
  std::memcpy(addr.sun_path, unix_path.c_str(), unix_path.size() + 1);
  const int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) return std::string("socket: ") + std::strerror(errno);
  const auto deadline = Clock::now() + std::chrono::microseconds(static_cast<int64_t>(timeout_s * 1e6));
  // A non-blocking AF_UNIX connect() never completes later: EAGAIN means the
  // listen backlog is full and the socket stays unconnected (poll() would
  // report it at once with SO_ERROR 0). So try again until it succeeds, in
  // short steps bounded by the deadline and the abort fd.
  while (::connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
    if (errno == EINTR) continue;
    if (errno != EAGAIN) {
      const std::string err = std::string("connect ") + unix_path + ": " + std::strerror(errno);
      ::close(fd);
      return err;
    }
    const auto step = std::min<Clock::duration>(std::chrono::milliseconds(5), deadline - Clock::now());
    if (step <= Clock::duration::zero()) {
      ::close(fd);
      return std::string("connect ") + unix_path + ": listen backlog full until the deadline";
    }
    if (abort_fd_ >= 0) {
      pollfd p{abort_fd_, POLLIN, 0};
      if (::poll(&p, 1, static_cast<int>(std::chrono::duration_cast<std::chrono::milliseconds>(step).count()) + 1) > 0) {
        ::close(fd);
        return std::string("connect ") + unix_path + ": interrupted";
      }
    } else {
      std::this_thread::sleep_for(step);
    }
  }
  fd_ = fd;
  st_ = std::make_unique<ClientState>();
  next_sid_ = 1;
  std::string out(kPreface, kPrefaceLen);
  put_frame(&out, kSettings, 0, 0, nullptr, 0);
  // a large connection window: responses never wait for our credit
  std::string wu;
  put_be32(&wu, (1u << 30) - 65535);
  put_frame(&out, kWindowUpdate, 0, 0, wu.data(), wu.size());
  size_t off = 0;
  while (off < out.size()) {
    const ssize_t n = ::send(fd_, out.data() + off, out.size() - off, MSG_NOSIGNAL);
    if (n > 0) {
      off += static_cast<size_t>(n);
      continue;
    }
    if (n < 0 && errno == EINTR) continue;
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK) && wait_fd(fd_, POLLOUT, abort_fd_, deadline) == Ready::kOk)
      continue;
    close();
    return "handshake write failed";
  }
  return "";
}

Reply GrpcClient::unary(const std::string& path, const std::string& request, double timeout_s) {
  if (fd_ < 0) return Reply{-1, "not connected", ""};
  if (st_->going_away) return Reply{-1, "connection is going away (server sent GOAWAY)", ""};
  ClientState& st = *st_;
  const auto deadline = Clock::now() + std::chrono::microseconds(static_cast<int64_t>(timeout_s * 1e6));
  Call call;
  call.sid = next_sid_;
  next_sid_ += 2;
  call.send_window = st.peer_initial_window;

  std::string pending_out;  // control frames (ACKs, credit) + request frames, flushed as we go
  auto fail = [&](int status, std::string msg, bool drop_conn) {
    if (drop_conn) close();
    return Reply{status, std::move(msg), ""};
  };
  // Writes pending_out completely (non-blocking socket, bounded by the deadline).
  auto flush = [&](std::string* err) -> bool {
    size_t off = 0;
    while (off < pending_out.size()) {
      const ssize_t n = ::send(fd_, pending_out.data() + off, pending_out.size() - off, MSG_NOSIGNAL);
      if (n > 0) {
        off += static_cast<size_t>(n);
        continue;
      }
      if (n < 0 && errno == EINTR) continue;
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        const Ready r = wait_fd(fd_, POLLOUT, abort_fd_, deadline);
        if (r == Ready::kOk) continue;
        *err = ready_error(r);
        return false;
      }
      *err = "write failed";
      // the server may have closed right after a GOAWAY that says why (e.g.
      // ENHANCE_YOUR_CALM for too many pings): read what it sent and name it
      char buf[65536];
      ssize_t r;
      while ((r = ::read(fd_, buf, sizeof(buf))) > 0) in_.append(buf, static_cast<size_t>(r));
      for (size_t o = 0; in_.size() - o >= 9;) {
        const auto* f = reinterpret_cast<const uint8_t*>(in_.data() + o);
        const size_t len = (static_cast<size_t>(f[0]) << 16) | (static_cast<size_t>(f[1]) << 8) | f[2];
        if (in_.size() - o < 9 + len) break;
        if (f[3] == kGoaway && len >= 8) {
          st.going_away = true;
          st.goaway_code = be32(f + 13);
          st.goaway_debug.assign(reinterpret_cast<const char*>(f + 17), std::min<size_t>(len - 8, 256));
          *err = "connection closed after GOAWAY " + std::string(h2_error_name(st.goaway_code)) +
                 (st.goaway_debug.empty() ? "" : " (" + st.goaway_debug + ")");
        }
        o += 9 + len;
      }
      return false;
    }
    pending_out.clear();
    return true;
  };
  // Reads what is there (waiting up to the deadline for something).
  auto read_more = [&](std::string* err) -> bool {
    const Ready r = wait_fd(fd_, POLLIN, abort_fd_, deadline);
    if (r != Ready::kOk) {
      *err = ready_error(r);
      return false;
    }
    char buf[65536];
    while (true) {
      const ssize_t n = ::read(fd_, buf, sizeof(buf));
      if (n > 0) {
        in_.append(buf, static_cast<size_t>(n));
        return true;
      }
      if (n < 0 && errno == EINTR) continue;
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return true;  // spurious wake-up
      *err = st.going_away ? "connection closed after GOAWAY " + std::string(h2_error_name(st.goaway_code)) +
                                 (st.goaway_debug.empty() ? "" : " (" + st.goaway_debug + ")")
                           : "connection closed";
      return false;
    }
  };

  // A complete header block of stream `sid` (every block is decoded, in order:
  // the HPACK dynamic table is shared by all streams of the connection).
  auto on_header_block = [&](uint32_t sid, const std::string& block, bool end_stream) -> bool {
    HeaderList hl;
    if (!st.dec.decode(reinterpret_cast<const uint8_t*>(block.data()), block.size(), &hl)) return false;
    if (sid != call.sid) return true;
    for (auto& [k, v] : hl) {
      if (k == ":status") call.http_status = std::atoi(v.c_str());
      else if (k == "content-type") call.content_type = v;
      else if (k == "grpc-status") call.grpc_status = std::atoi(v.c_str());
      else if (k == "grpc-message") call.grpc_message = percent_decode(v);
    }
    call.headers_seen = true;
    if (end_stream) call.done = true;
    return true;
  };

  // Handles one frame; false = connection-level failure (call.fail set).
  auto on_frame = [&](uint8_t type, uint8_t flags, uint32_t sid, const uint8_t* p, size_t len) -> bool {
    auto conn_fail = [&](std::string why) {
      call.failed = true;
      call.fail = Reply{-1, std::move(why), ""};
      return false;
    };
    if (st.cont_sid && (type != kContinuation || sid != st.cont_sid))
      return conn_fail("protocol error: header block interrupted (CONTINUATION expected)");
    switch (type) {
      case kSettings: {
        if (sid != 0) return conn_fail("protocol error: SETTINGS on a stream");
        if (flags & kAck) return true;
        if (len % 6) return conn_fail("protocol error: SETTINGS length");
        for (size_t i = 0; i < len; i += 6) {
          const uint16_t id = static_cast<uint16_t>((p[i] << 8) | p[i + 1]);
          const uint32_t v = be32(p + i + 2);
          if (id == 0x4) {  // INITIAL_WINDOW_SIZE: applies to the open stream too (RFC 7540 6.9.2)
            if (v > static_cast<uint32_t>(kMaxWindow)) return conn_fail("flow control error: initial window");
            const int64_t delta = static_cast<int64_t>(v) - st.peer_initial_window;
            st.peer_initial_window = v;
            call.send_window += delta;
            if (call.send_window > kMaxWindow) return conn_fail("flow control error: stream window overflow");
          } else if (id == 0x5) {  // MAX_FRAME_SIZE
            if (v < 16384 || v > 16777215) return conn_fail("protocol error: max frame size");
            st.peer_max_frame = v;
          }
        }
        put_frame(&pending_out, kSettings, kAck, 0, nullptr, 0);
        return true;
      }
      case kPing:
        if (sid != 0 || len != 8) return conn_fail("protocol error: bad PING");
        if (!(flags & kAck)) put_frame(&pending_out, kPing, kAck, 0, reinterpret_cast<const char*>(p), 8);
        return true;
      case kGoaway: {
        if (len < 8) return conn_fail("protocol error: short GOAWAY");
        st.going_away = true;
        st.goaway_last = std::min(st.goaway_last, be32(p) & 0x7fffffffu);
        st.goaway_code = be32(p + 4);
        st.goaway_debug.assign(reinterpret_cast<const char*>(p + 8), std::min<size_t>(len - 8, 256));
        if (st.goaway_last < call.sid)  // our stream was not processed
          return conn_fail(std::string("server sent GOAWAY ") + h2_error_name(st.goaway_code) +
                           (st.goaway_debug.empty() ? "" : " (" + st.goaway_debug + ")") + " before the call");
        return true;
      }
      case kWindowUpdate: {
        if (len != 4) return conn_fail("frame size error: WINDOW_UPDATE");
        const uint32_t inc = be32(p) & 0x7fffffffu;
        if (sid == 0) {
          if (inc == 0) return conn_fail("protocol error: zero connection window increment");
          st.conn_window += inc;
          if (st.conn_window > kMaxWindow) return conn_fail("flow control error: connection window overflow");
        } else if (sid == call.sid) {
          call.send_window += inc;
          if (call.send_window > kMaxWindow) return conn_fail("flow control error: stream window overflow");
        }
        return true;
      }
      case kRstStream:
        if (len != 4 || sid == 0) return conn_fail("protocol error: bad RST_STREAM");
        if (sid == call.sid) {
          const uint32_t code = be32(p);
          call.failed = true;
          call.fail = Reply{rst_to_status(code), std::string("stream terminated by RST_STREAM with error code: ") +
                                                     h2_error_name(code), ""};
          call.done = true;
        }
        return true;
      case kHeaders:
      case kContinuation: {
        if (sid == 0) return conn_fail("protocol error: header block on stream 0");
        size_t pad = 0;
        if (type == kHeaders) {
          if (flags & kPadded) {
            if (len < 1) return conn_fail("protocol error: bad padding");
            pad = p[0];
            ++p;
            --len;
          }
          if (flags & kPriorityFlag) {
            if (len < 5) return conn_fail("protocol error: short priority");
            p += 5;
            len -= 5;
          }
          if (pad > len) return conn_fail("protocol error: bad padding");
          len -= pad;
          st.cont_block.clear();
          st.cont_end_stream = (flags & kEndStream) != 0;
        } else if (!st.cont_sid) {
          return conn_fail("protocol error: CONTINUATION without HEADERS");
        }
        if (st.cont_block.size() + len > kMaxHeaderBlock) return conn_fail("header block too large");
        st.cont_block.append(reinterpret_cast<const char*>(p), len);
        if (!(flags & kEndHeaders)) {
          st.cont_sid = sid;
          return true;
        }
        st.cont_sid = 0;
        if (!on_header_block(sid, st.cont_block, st.cont_end_stream)) return conn_fail("bad response headers (HPACK)");
        st.cont_block.clear();
        return true;
      }
      case kData: {
        if (sid == 0) return conn_fail("protocol error: DATA on stream 0");
        // connection credit for everything received (padding included), in batches
        st.recv_unacked += len;
        if (st.recv_unacked >= (1u << 28)) {
          std::string wu;
          put_be32(&wu, static_cast<uint32_t>(st.recv_unacked));
          put_frame(&pending_out, kWindowUpdate, 0, 0, wu.data(), wu.size());
          st.recv_unacked = 0;
        }
        size_t pad = 0;
        if (flags & kPadded) {
          if (len < 1 || p[0] >= len) return conn_fail("protocol error: bad padding");
          pad = p[0];
        }
        if (sid != call.sid) return true;  // a stream we gave up on
        if (len) call.data.append(reinterpret_cast<const char*>(p + (pad ? 1 : 0)), len - (pad ? pad + 1 : 0));
        if (call.data.size() > kMaxMessage + 5) return conn_fail("response message too large");
        if (flags & kEndStream) {
          call.done = true;  // a closed stream needs no credit
        } else {
          // stream credit in batches of half the initial window (grpc-go's inFlow
          // acks at a quarter): a unary reply of a few hundred bytes costs the
          // server no extra wakeup
          call.recv_unacked += static_cast<uint32_t>(len);
          if (call.recv_unacked >= 32768) {
            std::string wu;
            put_be32(&wu, call.recv_unacked);
            put_frame(&pending_out, kWindowUpdate, 0, call.sid, wu.data(), wu.size());
            call.recv_unacked = 0;
          }
        }
        return true;
      }
      default:
        return true;  // PRIORITY, unknown extension frames
    }
  };
  auto process = [&]() -> bool {
    size_t off = 0;
    bool ok = true;
    while (ok && !call.done && in_.size() - off >= 9) {
      const auto* f = reinterpret_cast<const uint8_t*>(in_.data() + off);
      const size_t len = (static_cast<size_t>(f[0]) << 16) | (static_cast<size_t>(f[1]) << 8) | f[2];
      if (len > kOurMaxFrame) {  // we announce the default SETTINGS_MAX_FRAME_SIZE
        call.failed = true;
        call.fail = Reply{-1, "frame size error: frame larger than 16384", ""};
        ok = false;
        break;
      }
      if (in_.size() - off < 9 + len) break;
      off += 9 + len;
      ok = on_frame(f[3], f[4], be32(f + 5) & 0x7fffffffu, f + 9, len);
    }
    in_.erase(0, off);
    return ok;
  };

  // request: HEADERS (+ CONTINUATION beyond the peer's max frame), then DATA within the windows
  std::string h;
  hpack_put_indexed(&h, 3);  // :method POST
  hpack_put_indexed(&h, 6);  // :scheme http
  hpack_put_literal(&h, 4, path);
  hpack_put_literal(&h, 1, "localhost");  // :authority
  hpack_put_literal(&h, 31, "application/grpc");
  hpack_put_literal(&h, "te", "trailers");
  {
    const size_t maxf = std::min(st.peer_max_frame, kOurMaxFrame);
    for (size_t off = 0; off < h.size() || off == 0; off += maxf) {
      const size_t n = std::min(maxf, h.size() - off);
      const bool last = off + n >= h.size();
      put_frame(&pending_out, off == 0 ? kHeaders : kContinuation, last ? kEndHeaders : 0, call.sid, h.data() + off, n);
      if (last) break;
    }
  }
  const std::string body = grpc_frame(request);
  std::string err;
  size_t sent = 0;
  while (sent < body.size()) {
    const int64_t w = std::min({st.conn_window, call.send_window,
                                static_cast<int64_t>(std::min(st.peer_max_frame, kOurMaxFrame))});
    if (w > 0) {
      const size_t n = std::min(body.size() - sent, static_cast<size_t>(w));
      put_frame(&pending_out, kData, sent + n >= body.size() ? kEndStream : 0, call.sid, body.data() + sent, n);
      st.conn_window -= static_cast<int64_t>(n);
      call.send_window -= static_cast<int64_t>(n);
      sent += n;
      continue;
    }
    // out of credit: send what we have, then wait for WINDOW_UPDATE / SETTINGS
    if (!flush(&err)) return fail(-1, err, true);
    if (!read_more(&err)) return fail(-1, err, true);
    if (!process()) return fail(call.fail.status, call.fail.message, true);
    if (call.done) break;  // answered (or reset) before the request was complete
  }
  while (!call.done) {
    if (!process()) return fail(call.fail.status, call.fail.message, true);
    if (call.done) break;
    // everything process() queued (WINDOW_UPDATE, SETTINGS / PING acks) goes out
    // before we wait: the peer may be blocked on exactly that credit
    if (!flush(&err)) return fail(-1, err, true);
    if (!read_more(&err)) return fail(-1, err, true);
  }
  if (!flush(&err)) return fail(-1, err, true);
  if (call.failed) return fail(call.fail.status, call.fail.message, false);
  if (!call.headers_seen) return fail(kInternal, "server closed the stream without sending trailers", false);
  // not a gRPC response: the HTTP status decides (grpc-go operateHeaders)
  if (call.http_status != 200 || call.content_type.compare(0, 16, "application/grpc") != 0) {
    if (call.grpc_status >= 0 && call.http_status == 200) return Reply{call.grpc_status, call.grpc_message, ""};
    return fail(call.http_status == 200 ? kUnknown : http_to_status(call.http_status),
                "unexpected HTTP status code " + std::to_string(call.http_status) + " (content-type \"" +
                    call.content_type + "\")",
                false);
  }
  if (call.grpc_status < 0) return fail(kInternal, "server closed the stream without sending trailers", false);
  Reply rep{call.grpc_status, call.grpc_message, ""};
  if (rep.status == 0) {
    if (call.data.size() < 5) return Reply{kInternal, "missing response message", ""};
    const auto* d = reinterpret_cast<const uint8_t*>(call.data.data());
    if (d[0] != 0) return Reply{kInternal, "compressed response message", ""};
    const uint32_t mlen = be32(d + 1);
    if (static_cast<size_t>(mlen) + 5 != call.data.size()) return Reply{kInternal, "expected exactly one response message", ""};
    rep.body = call.data.substr(5);
  }
  return rep;
}

}  // namespace mi355x::rpc
