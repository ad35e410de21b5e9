// Native gRPC server (HTTP/2 over a Unix socket) for the kubelet-facing
// device-plugin API.
//
// The kubelet is a Go gRPC client; the reference answers it from grpc-go. A
// Python grpc.aio server puts ~0.6-0.9 ms of interpreter and event-loop work
// on every GetPreferredAllocation / Allocate (profiles/archive/measurements_r1_r3.md §6).
// This server speaks the subset of HTTP/2 + gRPC a kubelet uses (unary and
// server-streaming calls, HPACK with Huffman, flow control, PING, GOAWAY) on
// one I/O thread with epoll; handlers run on that thread.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <optional>
#include <string>
#include <vector>

namespace mi355x::rpc {

// gRPC status codes used by the device-plugin service
enum GrpcStatus : int {
  kOk = 0,
  kCancelled = 1,
  kUnknown = 2,
  kInvalidArgument = 3,
  kDeadlineExceeded = 4,
  kPermissionDenied = 7,
  kResourceExhausted = 8,
  kFailedPrecondition = 9,
  kUnimplemented = 12,
  kInternal = 13,
  kUnavailable = 14,
  kUnauthenticated = 16,
};

struct Reply {
  int status = kOk;
  std::string message;  // grpc-message for status != 0
  std::string body;     // serialized response message (status == 0)
};

// unary: request bytes -> reply
using UnaryFn = std::function<Reply(const std::string& request)>;
// server streaming: called when a call opens; status == 0 sends `body` as the
// first message and keeps the stream open for broadcast()/send()
using StreamOpenFn = std::function<Reply(uint64_t call_id, const std::string& request)>;
using StreamCloseFn = std::function<void(uint64_t call_id)>;
// unary that may answer later: a reply now, or nullopt and complete(call_id, reply)
// from any thread once the answer is known (e.g. after a GPU probe). A call the
// client resets or whose connection ends meanwhile is forgotten; complete() then
// returns false. Stopping the server answers a pending call UNAVAILABLE.
using DeferrableUnaryFn = std::function<std::optional<Reply>(uint64_t call_id, const std::string& request)>;

struct ServerStats {
  uint64_t connections = 0;
  uint64_t calls = 0;
  uint64_t streams_open = 0;
  uint64_t streams_opened = 0;  // server-streaming calls ever opened (ListAndWatch)
  uint64_t protocol_errors = 0;
  // protocol errors on connections that had made a call on a served route:
  // kubelet's connection, as opposed to a stray client (a health checker, curl)
  uint64_t caller_protocol_errors = 0;
  uint64_t bytes_in = 0;
  uint64_t bytes_out = 0;
};

class GrpcServer {
 public:
  GrpcServer();
  ~GrpcServer();
  GrpcServer(const GrpcServer&) = delete;
  GrpcServer& operator=(const GrpcServer&) = delete;

  // Registration happens before start().
  void add_unary(const std::string& path, UnaryFn fn);
  void add_server_stream(const std::string& path, StreamOpenFn open, StreamCloseFn close = nullptr);
  void add_unary_deferrable(const std::string& path, DeferrableUnaryFn fn);
  // called on the I/O thread after each round's responses are written (before start())
  void set_after_io(std::function<void()> fn);

  // Binds the Unix socket (an existing file at `path` is replaced) and starts
  // the I/O thread. Returns "" or an error message.
  std::string start(const std::string& unix_path);
  // GOAWAY to every connection, open streams end with status OK, pending
  // output is flushed for up to `grace_s`, then the thread is joined.
  void stop(double grace_s = 0.5);
  bool running() const { return running_.load(); }

  // Queue `msg` on every open stream of `path` / on one call (thread-safe).
  // Returns the number of streams it was queued on.
  size_t broadcast(const std::string& path, const std::string& msg);
  bool send(uint64_t call_id, const std::string& msg);
  // the answer of a deferred unary call (thread-safe); false when the call is gone
  bool complete(uint64_t call_id, Reply reply);
  size_t open_streams(const std::string& path) const;
  ServerStats stats() const;

  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
  std::atomic<bool> running_{false};
};

// Blocking unary client over a Unix socket: the daemons' Registration and
// metrics-exporter client, and the benchmark's kubelet stand-in (kubelet's own
// client is grpc-go, not an interpreter). One call at a time per client; the
// connection is reused across calls until the server sends GOAWAY.
//
// HTTP/2 as a grpc-go server expects it (vendor/google.golang.org/grpc/
// internal/transport/http2_server.go): header blocks of any stream are decoded
// in arrival order (HEADERS + CONTINUATION, dynamic-table inserts), request
// DATA waits for the peer's connection and stream windows and never exceeds
// its SETTINGS_MAX_FRAME_SIZE, SETTINGS and PING are acknowledged, a GOAWAY
// that leaves the call unprocessed fails it, RST_STREAM and a non-200 :status
// map to gRPC codes as grpc-go does. Every wait is bounded by the call's
// deadline and ends early when `abort_fd` (a daemon's signal pipe) becomes
// readable; EINTR never turns into a blocking read.
class GrpcClient {
 public:
  GrpcClient();
  ~GrpcClient();
  GrpcClient(const GrpcClient&) = delete;
  GrpcClient& operator=(const GrpcClient&) = delete;

  std::string connect(const std::string& unix_path, double timeout_s = 10.0);  // "" or an error
  // status -1: transport error / timeout / interrupted (message says which)
  Reply unary(const std::string& path, const std::string& request, double timeout_s);
  void close();
  bool connected() const { return fd_ >= 0; }
  void set_abort_fd(int fd) { abort_fd_ = fd; }
  // the server announced GOAWAY: the next call needs a new connection
  bool going_away() const;

 private:
  int fd_ = -1;
  int abort_fd_ = -1;
  uint32_t next_sid_ = 1;
  std::string in_;
  std::unique_ptr<struct ClientState> st_;
};

}  // namespace mi355x::rpc
