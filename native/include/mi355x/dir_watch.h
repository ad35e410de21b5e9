// inotify watch of one directory (the kubelet's device-plugin directory).
//
// Reference: the vendored kubevirt device-plugin-manager watches
// /var/lib/kubelet/device-plugins/ with fsnotify to notice kubelet.sock being
// re-created (a kubelet restart) and re-register at once
// (vendor/github.com/kubevirt/device-plugin-manager/pkg/dpm/manager.go).
// The plugin's manager waits on this fd from its event loop instead of polling.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace mi355x {

class DirWatcher {
 public:
  DirWatcher() = default;
  ~DirWatcher();
  DirWatcher(const DirWatcher&) = delete;
  DirWatcher& operator=(const DirWatcher&) = delete;

  // "" or an error; entries created / deleted / moved / attribute-changed and
  // the directory itself going away are reported
  std::string open(const std::string& dir);
  int fd() const { return fd_; }
  // drains pending events: (entry name, inotify mask); name "" = the directory itself
  std::vector<std::pair<std::string, uint32_t>> read_events();
  void close();

 private:
  int fd_ = -1;
  int wd_ = -1;
};

}  // namespace mi355x
