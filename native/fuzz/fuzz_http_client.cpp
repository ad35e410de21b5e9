// HTTP/1.1 client of the native labeller (src/kube/http.cpp): the apiserver's
// responses to GET / PATCH / PUT and its streamed watch (status line, headers,
// Content-Length / chunked / to-EOF bodies, newline-delimited events). A local
// plain-HTTP server answers each request with the input bytes and closes.
// Byte 0 picks a one-shot request or a watch stream. Invariants: every call
// ends within its 1 s deadline (plus slack); a decoded body or the watch lines
// never hold more bytes than the server sent; a JSON event line that parses
// serialises again.
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>

#include "../src/kube/http.h"
#include "../src/kube/json.h"
#include "fuzz_common.h"

using namespace mi355x::fuzz;
namespace http = mi355x::http;

namespace {

struct Server {
  int fd = -1;
  int port = 0;
  std::mutex mu;
  std::string reply;  // what the next connection gets
};

Server& server() {
  static Server* s = [] {
    auto* sv = new Server;
    sv->fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (sv->fd < 0) fail("socket");
    const int one = 1;
    ::setsockopt(sv->fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (::bind(sv->fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(sv->fd, 64) != 0)
      fail("bind 127.0.0.1");
    socklen_t len = sizeof(a);
    ::getsockname(sv->fd, reinterpret_cast<sockaddr*>(&a), &len);
    sv->port = ntohs(a.sin_port);
    std::thread([sv] {
      for (;;) {
        const int c = ::accept4(sv->fd, nullptr, nullptr, SOCK_CLOEXEC);
        if (c < 0) continue;
        std::string reply;
        {
          std::lock_guard<std::mutex> lk(sv->mu);
          reply = sv->reply;
        }
        // the request head first, as a server would, then the reply and a close
        std::string req;
        char b[4096];
        while (req.find("\r\n\r\n") == std::string::npos && req.size() < 65536) {
          const ssize_t n = ::recv(c, b, sizeof(b), 0);
          if (n <= 0) break;
          req.append(b, static_cast<size_t>(n));
        }
        write_all(c, reply.data(), reply.size());
        ::shutdown(c, SHUT_WR);
        drain(c, 3000);
        ::close(c);
      }
    }).detach();
    return sv;
  }();
  return *s;
}

}  // namespace

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  server();
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size == 0 || size > 256 * 1024) return 0;
  Server& s = server();
  {
    std::lock_guard<std::mutex> lk(s.mu);
    s.reply.assign(reinterpret_cast<const char*>(data) + 1, size - 1);
  }
  http::Config cfg;
  cfg.server = "http://127.0.0.1:" + std::to_string(s.port);
  cfg.timeout_s = 1.0;
  const http::Headers hdr = {{"Authorization", "Bearer fuzz"}, {"Accept", "application/json"}};
  const auto t0 = std::chrono::steady_clock::now();
  if (data[0] & 1) {
    http::Stream st;
    int status = 0;
    std::string ebody;
    const std::string e = st.open(cfg, "/api/v1/nodes?watch=1&fieldSelector=metadata.name%3Dn", hdr, &status, &ebody,
                                  1000, -1);
    size_t total = 0;
    if (e.empty()) {
      std::string line;
      for (int i = 0; i < 100000; ++i) {
        const int rc = st.next_line(&line, 1000, -1);
        if (rc != 1) break;
        total += line.size() + 1;
        if (auto v = mi355x::json::parse(line)) {
          if (!mi355x::json::parse(mi355x::json::serialize(*v))) fail("watch event does not re-serialise");
        }
      }
      st.close();
    }
    if (total > size + 1) fail("watch lines hold more bytes than the server sent");
  } else {
    const http::Response r = http::request(cfg, "PATCH", "/api/v1/nodes/n", hdr, "{}");
    if (r.body.size() > size) fail("decoded body larger than the response");
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (secs > 4.0) fail("HTTP call outlived its deadline");
  return 0;
}
