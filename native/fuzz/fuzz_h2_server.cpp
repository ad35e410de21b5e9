// Native gRPC server (src/rpc/grpc_server.cpp + dp_service.cpp) against raw
// HTTP/2 bytes after the client preface: what kubelet's grpc-go client, or
// anything else that can open the plugin socket, may send. Each input is one
// connection that half-closes after its bytes. Invariants: the server closes
// that connection within 3 s (no wedged connection, no busy loop), and every
// 64 inputs a fresh well-formed call is still answered.
#include <sys/socket.h>
#include <unistd.h>

#include <string>

#include "dp_fixture.h"

using namespace mi355x::fuzz;

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  dp_server();
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  static uint64_t n = 0;
  DpServer& s = dp_server();
  const int fd = uds_connect(s.sock);
  if (fd < 0) fail("connect to the plugin socket");
  static const char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
  bool ok = write_all(fd, kPreface, sizeof(kPreface) - 1) && write_all(fd, data, size);
  (void)ok;  // the server may close early on a protocol error: that is an answer too
  ::shutdown(fd, SHUT_WR);
  if (!drain(fd, 3000)) fail("server kept a half-closed connection open for 3 s");
  ::close(fd);
  s.service->drain_events();
  if (++n % 64 == 0) check_server_alive("a fuzzed connection");
  return 0;
}
