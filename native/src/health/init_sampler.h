// Poor man's wall-clock profiler for GPU-runtime start-up (probe --sample-init).
//
// strace/perf are not available in the deployment image and ptrace is often
// blocked in pods, but a process may read its own /proc/self/task/*/{stat,syscall}.
// A sampler thread polls every thread of the process at a fixed period and
// histograms (thread role, scheduler state, current syscall). That splits the
// start-up wall time into "on a CPU", "runnable but waiting for a
// CPU" (host contention), "blocked in ioctl" (driver work), "reading sysfs", ...
#pragma once

#include <dirent.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>

namespace mi355x {

class InitSampler {
 public:
  explicit InitSampler(int period_us) : period_us_(period_us), main_tid_(static_cast<int>(::syscall(SYS_gettid))) {}

  void start() {
    th_ = std::thread([this] { run(); });
  }

  void stop() {
    stop_.store(true, std::memory_order_relaxed);
    if (th_.joinable()) th_.join();
  }

  // {"period_us":P,"ticks":N,"threads_max":T,"buckets":{"main R oncpu":n,...}}
  std::string json() const {
    std::string o = "{\"period_us\":" + std::to_string(period_us_) + ",\"ticks\":" + std::to_string(ticks_) +
                    ",\"threads_max\":" + std::to_string(threads_max_) + ",\"buckets\":{";
    bool first = true;
    for (const auto& kv : buckets_) {
      if (!first) o += ",";
      first = false;
      o += "\"" + kv.first + "\":" + std::to_string(kv.second);
    }
    return o + "}}";
  }

 private:
  static const char* syscall_name(long nr) {
    switch (nr) {  // x86_64 numbers of the calls a GPU runtime start-up makes
      case 0: return "read";
      case 1: return "write";
      case 2: return "open";
      case 3: return "close";
      case 4: return "stat";
      case 5: return "fstat";
      case 7: return "poll";
      case 8: return "lseek";
      case 9: return "mmap";
      case 10: return "mprotect";
      case 11: return "munmap";
      case 16: return "ioctl";
      case 17: return "pread64";
      case 21: return "access";
      case 28: return "madvise";
      case 35: return "nanosleep";
      case 56: return "clone";
      case 89: return "readlink";
      case 202: return "futex";
      case 217: return "getdents64";
      case 230: return "clock_nanosleep";
      case 232: return "epoll_wait";
      case 257: return "openat";
      case 262: return "newfstatat";
      case 318: return "getrandom";
      case 332: return "statx";
      case 435: return "clone3";
      default: return nullptr;
    }
  }

  // For a thread blocked in open/openat the path argument is still live in our
  // own address space; process_vm_readv copes with a stale pointer (EFAULT).
  // Digit runs are folded to 'N' so per-node sysfs files pool together.
  static std::string open_path(unsigned long addr) {
    char raw[256] = {0};
    iovec local{raw, sizeof(raw) - 1};
    iovec remote{reinterpret_cast<void*>(addr), sizeof(raw) - 1};
    // a read that crosses into an unmapped page fails as a whole: retry short
    if (process_vm_readv(getpid(), &local, 1, &remote, 1, 0) <= 0) {
      local.iov_len = remote.iov_len = 64;
      if (process_vm_readv(getpid(), &local, 1, &remote, 1, 0) <= 0) return "?";
    }
    std::string o;
    for (const char* c = raw; *c && o.size() < 120; ++c) {
      if (*c >= '0' && *c <= '9') {
        if (o.empty() || o.back() != 'N') o += 'N';
      } else if (*c == '"' || *c == '\\' || static_cast<unsigned char>(*c) < 0x20) {
        o += '_';
      } else {
        o += *c;
      }
    }
    return o;
  }

  static std::string fd_path(long fd) {
    char link[64], target[256];
    std::snprintf(link, sizeof(link), "/proc/self/fd/%ld", fd);
    const ssize_t k = readlink(link, target, sizeof(target) - 1);
    if (k <= 0) return "?";
    target[k] = 0;
    std::string o;
    for (const char* c = target; *c && o.size() < 120; ++c) {
      if (*c >= '0' && *c <= '9') {
        if (o.empty() || o.back() != 'N') o += 'N';
      } else if (*c == '"' || *c == '\\') {
        o += '_';
      } else {
        o += *c;
      }
    }
    return o;
  }

  static bool read_small(const char* path, char* buf, size_t n) {
    FILE* f = std::fopen(path, "r");
    if (!f) return false;
    size_t got = std::fread(buf, 1, n - 1, f);
    std::fclose(f);
    buf[got] = 0;
    return got > 0;
  }

  void sample_task(int tid) {
    char path[96], buf[512];
    std::snprintf(path, sizeof(path), "/proc/self/task/%d/stat", tid);
    if (!read_small(path, buf, sizeof(buf))) return;
    const char* rp = std::strrchr(buf, ')');
    if (!rp || !rp[1] || !rp[2]) return;
    const char state = rp[2];
    std::string what;
    std::snprintf(path, sizeof(path), "/proc/self/task/%d/syscall", tid);
    if (read_small(path, buf, sizeof(buf))) {
      if (std::strncmp(buf, "running", 7) == 0) {
        what = "oncpu";  // "running": on a CPU right now (user or kernel mode)
      } else {
        char* p = nullptr;
        const long nr = std::strtol(buf, &p, 10);
        const char* nm = nr >= 0 ? syscall_name(nr) : nullptr;
        what = nr < 0 ? "kernel" : nm ? nm : "sys" + std::to_string(nr);
        if (nr == 2 || nr == 257) {  // open(path, ..) / openat(dirfd, path, ..)
          unsigned long a0 = std::strtoul(p, &p, 16);
          unsigned long a1 = std::strtoul(p, &p, 16);
          what += " " + open_path(nr == 2 ? a0 : a1);
        } else if (nr == 0 || nr == 17 || nr == 16 || nr == 3) {  // read/pread64/ioctl/close(fd, ..)
          const long fd = static_cast<long>(std::strtoul(p, &p, 16));
          what += " " + fd_path(fd);
          if (nr == 16) {  // ioctl(fd, cmd): the command's number byte names the kfd/drm call
            const unsigned long cmd = std::strtoul(p, &p, 16);
            char c[16];
            std::snprintf(c, sizeof(c), " #%02lx", cmd & 0xFF);
            what += c;
          }
        }
      }
    } else {
      what = "?";
    }
    if (state == 'D') {
      // uninterruptible sleep: name the kernel function it waits in
      // (/proc/self/task/<tid>/wchan is readable by the task's owner)
      std::snprintf(path, sizeof(path), "/proc/self/task/%d/wchan", tid);
      if (read_small(path, buf, sizeof(buf)) && buf[0] && std::strcmp(buf, "0") != 0) {
        what += " @";
        for (const char* c = buf; *c && *c != '\n' && what.size() < 200; ++c) what += *c;
      }
    }
    std::string key = tid == main_tid_ ? "main " : "aux ";
    key += state;
    key += ' ';
    key += what;
    ++buckets_[key];
  }

  void run() {
    const int self = static_cast<int>(::syscall(SYS_gettid));
    while (!stop_.load(std::memory_order_relaxed)) {
      DIR* d = opendir("/proc/self/task");
      if (d) {
        int threads = 0;
        while (dirent* e = readdir(d)) {
          const int tid = std::atoi(e->d_name);
          if (tid <= 0 || tid == self) continue;
          ++threads;
          sample_task(tid);
        }
        closedir(d);
        if (threads > threads_max_) threads_max_ = threads;
      }
      ++ticks_;
      timespec ts{0, static_cast<long>(period_us_) * 1000};
      nanosleep(&ts, nullptr);
    }
  }

  const int period_us_;
  const int main_tid_;
  std::atomic<bool> stop_{false};
  std::thread th_;
  long ticks_ = 0;
  int threads_max_ = 0;
  std::map<std::string, long> buckets_;
};

}  // namespace mi355x
