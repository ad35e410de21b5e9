#pragma once
// ioctl timing for measurement builds (never linked into shipped binaries).
//
// The executable exports its own ioctl() (-rdynamic); ROCr's thunk, dlopen()ed
// later, resolves ioctl against the executable first, so every kfd / drm
// ioctl the runtime issues is timed here (wall time per call, by type and
// command number) before being forwarded to libc. ioctl_trace_mark() returns
// a cursor; ioctl_trace_json(since) summarises the calls made after it:
//   {"K02":{"n":1,"ms":4.61,"max_ms":4.61},...}   K = kfd ('K'), d = drm ('d')
// (kfd: 0x02 CREATE_QUEUE, 0x03 DESTROY_QUEUE, 0x16 ALLOC_MEMORY_OF_GPU,
//  0x17 FREE_MEMORY_OF_GPU, 0x18 MAP_MEMORY_TO_GPU, 0x0c WAIT_EVENTS, ...)
#include <dlfcn.h>
#include <stdarg.h>
#include <sys/ioctl.h>
#include <time.h>

#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace ioctl_trace {

struct Call {
  unsigned char type, nr;
  double ms;
};

inline std::mutex& mu() {
  static std::mutex m;
  return m;
}
inline std::vector<Call>& calls() {
  static std::vector<Call>* v = new std::vector<Call>();  // never destroyed: ioctls may run at exit
  return *v;
}

inline double now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

}  // namespace ioctl_trace

extern "C" int ioctl(int fd, unsigned long request, ...) {
  using fn_t = int (*)(int, unsigned long, ...);
  static fn_t real = reinterpret_cast<fn_t>(dlsym(RTLD_NEXT, "ioctl"));
  va_list ap;
  va_start(ap, request);
  void* arg = va_arg(ap, void*);
  va_end(ap);
  const double t0 = ioctl_trace::now_ms();
  const int r = real(fd, request, arg);
  const double ms = ioctl_trace::now_ms() - t0;
  const unsigned char type = static_cast<unsigned char>(_IOC_TYPE(request));
  const unsigned char nr = static_cast<unsigned char>(_IOC_NR(request));
  if (!(type == 'K' && nr == 0x0c)) {  // WAIT_EVENTS blocks on ROCr's event thread by design
    std::lock_guard<std::mutex> lk(ioctl_trace::mu());
    ioctl_trace::calls().push_back({type, nr, ms});
  }
  return r;
}

inline size_t ioctl_trace_mark() {
  std::lock_guard<std::mutex> lk(ioctl_trace::mu());
  return ioctl_trace::calls().size();
}

inline std::string ioctl_trace_json(size_t since) {
  struct Agg {
    int n = 0;
    double ms = 0, max_ms = 0;
  };
  std::map<std::string, Agg> agg;
  {
    std::lock_guard<std::mutex> lk(ioctl_trace::mu());
    const auto& v = ioctl_trace::calls();
    for (size_t i = since; i < v.size(); ++i) {
      char key[8];
      std::snprintf(key, sizeof(key), "%c%02x", v[i].type >= 32 && v[i].type < 127 ? v[i].type : '?', v[i].nr);
      Agg& a = agg[key];
      ++a.n;
      a.ms += v[i].ms;
      if (v[i].ms > a.max_ms) a.max_ms = v[i].ms;
    }
  }
  std::string o = "{";
  bool first = true;
  for (const auto& kv : agg) {
    char buf[128];
    std::snprintf(buf, sizeof(buf), "%s\"%s\":{\"n\":%d,\"ms\":%.3f,\"max_ms\":%.3f}", first ? "" : ",",
                  kv.first.c_str(), kv.second.n, kv.second.ms, kv.second.max_ms);
    o += buf;
    first = false;
  }
  return o + "}";
}
