// Shared helpers of the coverage-guided fuzz targets (libFuzzer + ASan/UBSan).
//
// Every target feeds bytes an untrusted or merely unexpected peer controls into
// the native daemons' parsers: kubelet's and the metrics exporter's HTTP/2
// frames and HPACK blocks, DevicePlugin protobuf requests, the apiserver's
// HTTP/1.1 responses and JSON, kubeconfig / -config YAML, and kfd sysfs text.
// A target aborts (a finding) on a crash, a sanitizer report, a hang past its
// own bound, or a broken invariant it checks after the input.
#pragma once

#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

// Leak checking on (a leak per input is a finding too). Defined here: every
// fuzz target is one translation unit that includes this header.
extern "C" __attribute__((used)) const char* __asan_default_options() { return "detect_leaks=1"; }

namespace mi355x::fuzz {

[[noreturn]] inline void fail(const char* what, const std::string& detail = "") {
  std::fprintf(stderr, "FUZZ INVARIANT BROKEN: %s %s\n", what, detail.c_str());
  std::fflush(stderr);
  std::abort();
}

inline std::string env_or_die(const char* name) {
  const char* v = std::getenv(name);
  if (!v || !*v) {
    std::fprintf(stderr, "%s is not set (tools/fuzz_native.py sets it)\n", name);
    std::exit(2);
  }
  return v;
}

// a scratch directory for sockets and files, removed by the runner
inline std::string scratch_dir() {
  static std::string dir = [] {
    const char* base = std::getenv("MI355X_FUZZ_TMP");
    std::string tmpl = std::string(base && *base ? base : "/tmp") + "/mi355x-fuzz-XXXXXX";
    if (!::mkdtemp(tmpl.data())) fail("mkdtemp", tmpl);
    return tmpl;
  }();
  return dir;
}

inline int uds_connect(const std::string& path) {
  const int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  std::snprintf(a.sun_path, sizeof(a.sun_path), "%s", path.c_str());
  if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
    ::close(fd);
    return -1;
  }
  return fd;
}

inline int uds_listen(const std::string& path) {
  ::unlink(path.c_str());
  const int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) fail("socket");
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  std::snprintf(a.sun_path, sizeof(a.sun_path), "%s", path.c_str());
  if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(fd, 64) != 0) fail("bind", path);
  return fd;
}

inline bool write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

// Reads until EOF; false when the peer neither closes nor goes quiet within `limit_ms`
// (quiet = no byte for `idle_ms` while the connection stays open counts as done too
// when `idle_ok`).
inline bool drain(int fd, int limit_ms, int idle_ms = -1, size_t* got = nullptr) {
  using Clock = std::chrono::steady_clock;
  const auto end = Clock::now() + std::chrono::milliseconds(limit_ms);
  char buf[16384];
  size_t total = 0;
  for (;;) {
    const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(end - Clock::now()).count();
    if (left <= 0) return false;
    pollfd p{fd, POLLIN, 0};
    const int wait = idle_ms >= 0 ? std::min<int>(idle_ms, static_cast<int>(left)) : static_cast<int>(left);
    const int r = ::poll(&p, 1, wait);
    if (r < 0 && errno == EINTR) continue;
    if (r == 0) {
      if (idle_ms >= 0) break;
      continue;
    }
    const ssize_t n = ::read(fd, buf, sizeof(buf));
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) break;
    total += static_cast<size_t>(n);
  }
  if (got) *got = total;
  return true;
}

}  // namespace mi355x::fuzz
