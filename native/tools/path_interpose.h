#pragma once
// Path interposition for measurement builds (never linked into shipped binaries).
//
// The executable exports its own open/openat/fopen/opendir (-rdynamic). ROCr
// (dlopen()ed below) resolves those symbols against the executable first, so
// every path its thunk opens passes through here: counted per path template
// (digit runs folded to N) and, if it matches a prefix in
// $MI355X_INITPROF_HIDE (colon separated, 'N' stands for a digit run), refused with ENOENT — an in-process
// stand-in for a container view that lacks those files (bind mounts need root).
//
// $MI355X_DEV_ALLOW (';'-separated exact paths) emulates the container's /dev
// as the Allocate DeviceSpecs build it: under /dev/dri/ only the listed nodes
// exist, every other open there fails with ENOENT — so ROCr's thunk skips the
// GPUs the pod was not given, as it does for render nodes a container lacks.
// $MI355X_INITPROF_COUNT=0 turns the per-path counting off (no lock, no map:
// the container entrypoint build pays two string compares per open).
//
// Include in exactly ONE translation unit of an executable linked with
// -rdynamic; call path_interpose_configure() at the top of main().
#include <dirent.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

std::mutex g_mu;
std::map<std::string, long>* g_counts = nullptr;  // allocated lazily (interposers run before main)
std::vector<std::string>* g_hide = nullptr;
// $MI355X_INITPROF_REDIRECT="<from>=<to>[;<from>=<to>...]": path prefix rewrites
std::vector<std::pair<std::string, std::string>>* g_redir = nullptr;
std::atomic<long> g_redirected{0};
std::vector<std::string>* g_dev_allow = nullptr;   // $MI355X_DEV_ALLOW
bool g_count = true;                               // $MI355X_INITPROF_COUNT != 0
thread_local std::string t_path;
std::atomic<long> g_hidden{0};
thread_local bool t_in_hook = false;
// lock-free, always on: what the container view changed (the probe's "view" field)
std::atomic<long> g_seen{0};             // paths through the hooks
std::atomic<long> g_node_cache_ok{0};    // successful opens under /sys/devices/system/node/node*/cpu*/cache
std::atomic<long> g_kfd_open_ns{0};      // time in open("/dev/kfd"): it waits for other processes' kfd teardown

bool is_kfd(const char* p) { return p && std::strcmp(p, "/dev/kfd") == 0; }

long mono_ns_now() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000000000L + ts.tv_nsec;
}

// a path under the NUMA-node tree's per-CPU cache descriptors (the -node_view hides them)
bool node_cpu_cache(const char* p) {
  static const char kNode[] = "/sys/devices/system/node/node";
  if (!p || std::strncmp(p, kNode, sizeof(kNode) - 1) != 0) return false;
  const char* cpu = std::strstr(p + sizeof(kNode) - 1, "/cpu");
  return cpu && std::strstr(cpu, "/cache") != nullptr;
}

template <typename R>
R tally(const char* path, R r, bool ok) {
  g_seen.fetch_add(1, std::memory_order_relaxed);
  if (ok && node_cpu_cache(path)) g_node_cache_ok.fetch_add(1, std::memory_order_relaxed);
  return r;
}


std::string fold(const char* p) {
  std::string o;
  for (; p && *p && o.size() < 160; ++p) {
    if (*p >= '0' && *p <= '9') {
      if (o.empty() || o.back() != 'N') o += 'N';
    } else {
      o += *p;
    }
  }
  return o;
}

// redirect `path` if it starts with the configured prefix (emulates a bind mount)
const char* map_path(const char* path) {
  if (!path || !g_redir) return path;
  for (const auto& r : *g_redir) {
    if (std::strncmp(path, r.first.c_str(), r.first.size()) == 0) {
      t_path = r.second + (path + r.first.size());
      g_redirected.fetch_add(1);
      return t_path.c_str();
    }
  }
  return path;
}

// true -> refuse this path
bool dev_hidden(const char* path) {
  if (!g_dev_allow || std::strncmp(path, "/dev/dri/", 9) != 0) return false;
  for (const auto& a : *g_dev_allow)
    if (a == path) return false;
  return true;
}

bool note(const char* path) {
  if (!path || t_in_hook) return false;
  if (dev_hidden(path)) {
    g_hidden.fetch_add(1);
    return true;
  }
  if (!g_count && !g_hide) return false;
  t_in_hook = true;
  bool hide = false;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_counts) g_counts = new std::map<std::string, long>();
    const std::string f = fold(path);
    if (g_count) ++(*g_counts)[f];
    if (g_hide)  // prefixes are matched against the folded path ('N' = any digits)
      for (const auto& h : *g_hide)
        if (!h.empty() && f.compare(0, h.size(), h) == 0) hide = true;
  }
  t_in_hook = false;
  if (hide) g_hidden.fetch_add(1);
  return hide;
}

template <typename F>
F real(const char* name) {
  return reinterpret_cast<F>(dlsym(RTLD_NEXT, name));
}

}  // namespace

extern "C" {

int open(const char* path, int flags, ...) {
  static auto fn = real<int (*)(const char*, int, ...)>("open");
  mode_t mode = 0;
  if (flags & (O_CREAT | O_TMPFILE)) {
    va_list ap;
    va_start(ap, flags);
    mode = va_arg(ap, mode_t);
    va_end(ap);
  }
  if (note(path)) {
    errno = ENOENT;
    return -1;
  }
  const long t0 = is_kfd(path) ? mono_ns_now() : 0;
  const int fd = fn(map_path(path), flags, mode);
  if (t0) g_kfd_open_ns.fetch_add(mono_ns_now() - t0, std::memory_order_relaxed);
  return tally(path, fd, fd >= 0);
}

int open64(const char* path, int flags, ...) {
  static auto fn = real<int (*)(const char*, int, ...)>("open64");
  mode_t mode = 0;
  if (flags & (O_CREAT | O_TMPFILE)) {
    va_list ap;
    va_start(ap, flags);
    mode = va_arg(ap, mode_t);
    va_end(ap);
  }
  if (note(path)) {
    errno = ENOENT;
    return -1;
  }
  const long t0 = is_kfd(path) ? mono_ns_now() : 0;
  const int fd = fn(map_path(path), flags, mode);
  if (t0) g_kfd_open_ns.fetch_add(mono_ns_now() - t0, std::memory_order_relaxed);
  return tally(path, fd, fd >= 0);
}

int openat(int dirfd, const char* path, int flags, ...) {
  static auto fn = real<int (*)(int, const char*, int, ...)>("openat");
  mode_t mode = 0;
  if (flags & (O_CREAT | O_TMPFILE)) {
    va_list ap;
    va_start(ap, flags);
    mode = va_arg(ap, mode_t);
    va_end(ap);
  }
  if (note(path)) {
    errno = ENOENT;
    return -1;
  }
  const long t0 = is_kfd(path) ? mono_ns_now() : 0;
  const int fd = fn(dirfd, map_path(path), flags, mode);
  if (t0) g_kfd_open_ns.fetch_add(mono_ns_now() - t0, std::memory_order_relaxed);
  return tally(path, fd, fd >= 0);
}

FILE* fopen(const char* path, const char* mode) {
  static auto fn = real<FILE* (*)(const char*, const char*)>("fopen");
  if (note(path)) {
    errno = ENOENT;
    return nullptr;
  }
  FILE* f = fn(map_path(path), mode);
  return tally(path, f, f != nullptr);
}

FILE* fopen64(const char* path, const char* mode) {
  static auto fn = real<FILE* (*)(const char*, const char*)>("fopen64");
  if (note(path)) {
    errno = ENOENT;
    return nullptr;
  }
  FILE* f = fn(map_path(path), mode);
  return tally(path, f, f != nullptr);
}

DIR* opendir(const char* path) {
  static auto fn = real<DIR* (*)(const char*)>("opendir");
  if (note(path)) {
    errno = ENOENT;
    return nullptr;
  }
  DIR* d = fn(map_path(path));
  return tally(path, d, d != nullptr);
}

}  // extern "C"


// Reads $MI355X_INITPROF_HIDE / $MI355X_INITPROF_REDIRECT and resets the counters.
inline void path_interpose_configure() {
  if (const char* h = std::getenv("MI355X_INITPROF_HIDE")) {
    g_hide = new std::vector<std::string>();
    std::string s = h;
    size_t pos = 0;
    while (pos <= s.size()) {
      size_t c = s.find(':', pos);
      if (c == std::string::npos) c = s.size();
      g_hide->push_back(s.substr(pos, c - pos));
      pos = c + 1;
    }
  }
  if (const char* a = std::getenv("MI355X_DEV_ALLOW")) {
    g_dev_allow = new std::vector<std::string>();
    std::string s = a;
    size_t pos = 0;
    while (pos < s.size()) {
      size_t c = s.find(';', pos);
      if (c == std::string::npos) c = s.size();
      if (c > pos) g_dev_allow->push_back(s.substr(pos, c - pos));
      pos = c + 1;
    }
  }
  if (const char* c = std::getenv("MI355X_INITPROF_COUNT")) g_count = std::strcmp(c, "0") != 0;
  if (const char* r = std::getenv("MI355X_INITPROF_REDIRECT")) {
    g_redir = new std::vector<std::pair<std::string, std::string>>();
    std::string s = r;
    size_t pos = 0;
    while (pos < s.size()) {
      size_t c = s.find(';', pos);
      if (c == std::string::npos) c = s.size();
      const std::string item = s.substr(pos, c - pos);
      const size_t eq = item.find('=');
      if (eq != std::string::npos) g_redir->emplace_back(item.substr(0, eq), item.substr(eq + 1));
      pos = c + 1;
    }
  }
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_counts) g_counts->clear();  // ignore the dynamic loader's own opens
  }
}

// {"paths":N,"node_cpu_cache_opens":N,"redirected":N,"hidden":N,"kfd_open_us":X}: cheap enough for every container
inline std::string path_interpose_view_json() {
  char kfd[32];
  std::snprintf(kfd, sizeof(kfd), "%.1f", g_kfd_open_ns.load() / 1e3);
  return "{\"paths\":" + std::to_string(g_seen.load()) + ",\"node_cpu_cache_opens\":" +
         std::to_string(g_node_cache_ok.load()) + ",\"redirected\":" + std::to_string(g_redirected.load()) +
         ",\"hidden\":" + std::to_string(g_hidden.load()) + ",\"kfd_open_us\":" + kfd + "}";
}

// {"opens":N,"hidden":N,"redirected":N,"by_template":{...top 40...}}
inline std::string path_interpose_json() {
  std::lock_guard<std::mutex> lk(g_mu);
  long total = 0;
  std::vector<std::pair<long, std::string>> top;
  if (g_counts)
    for (const auto& kv : *g_counts) {
      total += kv.second;
      top.emplace_back(kv.second, kv.first);
    }
  std::sort(top.rbegin(), top.rend());
  std::string o;
  for (size_t i = 0; i < top.size() && i < 40; ++i) {
    if (i) o += ",";
    o += "\"" + top[i].second + "\":" + std::to_string(top[i].first);
  }
  return "{\"opens\":" + std::to_string(total) + ",\"hidden\":" + std::to_string(g_hidden.load()) +
         ",\"redirected\":" + std::to_string(g_redirected.load()) + ",\"by_template\":{" + o + "}}";
}
