// inotify directory watch (see mi355x/dir_watch.h).
#include "mi355x/dir_watch.h"

#include <errno.h>
#include <sys/inotify.h>
#include <unistd.h>

#include <cstring>

namespace mi355x {

DirWatcher::~DirWatcher() { close(); }

void DirWatcher::close() {
  if (fd_ >= 0) ::close(fd_);
  fd_ = wd_ = -1;
}

std::string DirWatcher::open(const std::string& dir) {
  close();
  fd_ = ::inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
  if (fd_ < 0) return std::string("inotify_init1: ") + std::strerror(errno);
  wd_ = ::inotify_add_watch(fd_, dir.c_str(),
                            IN_CREATE | IN_DELETE | IN_MOVED_FROM | IN_MOVED_TO | IN_ATTRIB | IN_DELETE_SELF |
                                IN_MOVE_SELF);
  if (wd_ < 0) {
    const std::string err = "inotify_add_watch " + dir + ": " + std::strerror(errno);
    close();
    return err;
  }
  return "";
}

std::vector<std::pair<std::string, uint32_t>> DirWatcher::read_events() {
  std::vector<std::pair<std::string, uint32_t>> out;
  if (fd_ < 0) return out;
  alignas(inotify_event) char buf[8192];
  while (true) {
    const ssize_t n = ::read(fd_, buf, sizeof(buf));
    if (n <= 0) break;
    for (ssize_t off = 0; off + static_cast<ssize_t>(sizeof(inotify_event)) <= n;) {
      const auto* ev = reinterpret_cast<const inotify_event*>(buf + off);
      out.emplace_back(ev->len ? std::string(ev->name) : std::string(), ev->mask);
      off += static_cast<ssize_t>(sizeof(inotify_event)) + ev->len;
    }
  }
  return out;
}

}  // namespace mi355x
