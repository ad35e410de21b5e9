// Native HTTP/2 gRPC client (see mi355x/grpc_server.h): one blocking unary call
// at a time over a Unix socket, as the daemon's Register call and the
// metrics-exporter health query need. Non-blocking socket, every wait bounded
// by the call's deadline and an optional abort fd; the HPACK decoder sees every
// response header block in order, so its dynamic table follows the server's.
#include "mi355x/grpc_server.h"

#include <errno.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "h2_wire.h"
#include "hpack.h"

namespace mi355x::rpc {

using namespace h2;  // NOLINT(build/namespaces)

namespace {

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
      // ENHANCE_YOUR_CALM for too many pings): read what it sent and name it.
      // The GOAWAY may also have been processed already, in the same read as
      // the frames whose answer (a SETTINGS ack) this write carried.
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
        }
        o += 9 + len;
      }
      if (st.going_away)
        *err = "connection closed after GOAWAY " + std::string(h2_error_name(st.goaway_code)) +
               (st.goaway_debug.empty() ? "" : " (" + st.goaway_debug + ")");
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
        // the payload without the pad-length byte and the padding (RFC 7540 6.1;
        // PADDED with a pad length of 0 still carries the length byte)
        const uint8_t* body = p;
        size_t body_len = len;
        if (flags & kPadded) {
          if (len < 1 || p[0] >= len) return conn_fail("protocol error: bad padding");
          body_len = len - 1 - p[0];
          ++body;
        }
        if (sid != call.sid) return true;  // a stream we gave up on
        if (body_len) call.data.append(reinterpret_cast<const char*>(body), body_len);
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
