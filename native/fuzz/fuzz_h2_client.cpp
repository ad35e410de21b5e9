// Native gRPC client (GrpcClient in src/rpc/grpc_client.cpp): the daemons'
// Register call to kubelet and List call to the metrics exporter. The input
// is everything the server side sends on the connection (SETTINGS, HEADERS /
// CONTINUATION with HPACK, DATA, PING, GOAWAY, RST_STREAM, WINDOW_UPDATE, ...),
// then the server closes. Invariants: the call returns a status, within its
// deadline (plus scheduling slack), and a second call on a reused connection
// does the same.
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <string>

#include "fuzz_common.h"
#include "mi355x/grpc_server.h"

using namespace mi355x::fuzz;
namespace rpc = mi355x::rpc;

namespace {

int listener() {
  static int fd = uds_listen(scratch_dir() + "/kubelet.sock");
  return fd;
}

void call(rpc::GrpcClient& c, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  const rpc::Reply r = c.unary("/v1beta1.Registration/Register", std::string("\x0a\x07v1beta1", 9), 1.0);
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (s > 3.0) fail("client call outlived its 1 s deadline", what);
  if (r.status == 0 && r.body.size() > (16u << 20)) fail("absurd response body");
}

}  // namespace

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  listener();
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size > 64 * 1024) return 0;
  rpc::GrpcClient c;
  if (const std::string e = c.connect(scratch_dir() + "/kubelet.sock", 2.0); !e.empty()) fail("connect", e);
  const int peer = ::accept4(listener(), nullptr, nullptr, SOCK_CLOEXEC);
  if (peer < 0) fail("accept");
  const int big = 4 << 20;
  ::setsockopt(peer, SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
  write_all(peer, data, size);
  ::shutdown(peer, SHUT_WR);
  call(c, "first call");
  if (c.connected() && !c.going_away()) call(c, "second call on the same connection");
  ::close(peer);
  return 0;
}
