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

#include "h2_wire.h"
#include "hpack.h"

namespace mi355x::rpc {
namespace {

using namespace h2;  // NOLINT(build/namespaces)

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
  bool deferred = false;  // a deferrable unary call waiting for complete()
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
    DeferrableUnaryFn deferrable;
    StreamOpenFn open;
    StreamCloseFn close;
  };
  struct CallRef {
    int fd;
    uint32_t sid;
    std::string route;
    bool deferred = false;  // a deferrable unary call, not a stream
  };
  struct Outgoing {
    std::string route;  // broadcast to every stream of this route ("" = one call)
    uint64_t call_id;
    std::string msg;
    std::optional<Reply> reply;  // the answer of a deferred unary call
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
    if (it->second.streaming || it->second.deferred) end_call(it->second.call_id);
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
    if (r->second.deferrable) {
      {
        std::lock_guard<std::mutex> lk(mu);
        call_id = next_call++;
        calls[call_id] = CallRef{c.fd, s.id, s.path, true};
      }
      s.deferred = true;
      s.call_id = call_id;
      std::optional<Reply> now;
      try {
        now = r->second.deferrable(call_id, req);
      } catch (const std::exception& e) {
        now = Reply{kUnknown, e.what(), ""};
      }
      if (!now) return;  // complete(call_id, ...) answers it
      {
        std::lock_guard<std::mutex> lk(mu);
        calls.erase(call_id);
      }
      s.deferred = false;
      rep = std::move(*now);
    } else {
      try {
        rep = r->second.unary(req);
      } catch (const std::exception& e) {
        rep = Reply{kUnknown, e.what(), ""};
      }
    }
    answer(c, s, rep);
  }

  // a unary call's response: headers, the message and OK trailers, or trailers only
  void answer(Conn& c, Stream& s, const Reply& rep) {
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
      if (o.reply) {  // a deferred unary call's answer
        CallRef ref{};
        {
          std::lock_guard<std::mutex> lk(mu);
          auto it = calls.find(o.call_id);
          if (it == calls.end()) continue;  // reset or its connection ended meanwhile
          ref = it->second;
          calls.erase(it);
        }
        auto ci = conns.find(ref.fd);
        if (ci == conns.end()) continue;
        Conn& c = *ci->second;
        auto si = c.streams.find(ref.sid);
        if (si == c.streams.end() || !si->second.deferred) continue;
        si->second.deferred = false;
        answer(c, si->second, *o.reply);
        if (pump(c, si->second) || si->second.finished) finish_stream(c, ref.sid);
        continue;
      }
      targets.clear();
      {
        std::lock_guard<std::mutex> lk(mu);
        if (o.route.empty()) {
          auto it = calls.find(o.call_id);
          if (it != calls.end()) targets.emplace_back(it->first, it->second);
        } else {
          for (auto& [id, ref] : calls)
            if (!ref.deferred && ref.route == o.route) targets.emplace_back(id, ref);
        }
      }
      for (auto& [id, ref] : targets) {
        auto ci = conns.find(ref.fd);
        if (ci == conns.end()) continue;
        Conn& c = *ci->second;
        auto si = c.streams.find(ref.sid);
        if (si == c.streams.end() || si->second.trailers_queued || si->second.deferred) continue;
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
        } else if (s.deferred && !s.finished) {  // a deferred answer that will not come
          s.deferred = false;
          trailers_only(*c, s, kUnavailable, "server stopping");
          done.push_back(sid);
          {
            std::lock_guard<std::mutex> lk(mu);
            calls.erase(s.call_id);
          }
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

void GrpcServer::add_unary_deferrable(const std::string& path, DeferrableUnaryFn fn) {
  Impl::Route r;
  r.deferrable = std::move(fn);
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
    for (auto& [id, ref] : I.calls) n += !ref.deferred && ref.route == path;
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

bool GrpcServer::complete(uint64_t call_id, Reply reply) {
  Impl& I = *impl_;
  {
    std::lock_guard<std::mutex> lk(I.mu);
    if (!running_.load() || !I.calls.count(call_id)) return false;
    I.outbox.push_back(Impl::Outgoing{"", call_id, "", std::move(reply)});
  }
  I.wake();
  return true;
}

size_t GrpcServer::open_streams(const std::string& path) const {
  std::lock_guard<std::mutex> lk(impl_->mu);
  size_t n = 0;
  for (auto& [id, ref] : impl_->calls) n += !ref.deferred && (path.empty() || ref.route == path);
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
