// Health sweeps of the native daemon, off the control loop.
//
// Reference: UpdateHealth on every pulse (internal/pkg/amdgpu/amdgpu.go:
// 322-345 container, amdgpu_sriov.go:217-308 VF, amdgpu_pf.go:210-229 PF),
// called from ListAndWatch's loop. Here a sweep runs on a worker thread, and
// the job it gets owns everything it touches:
//   * container driver: a shared_ptr to the health engine (mi355x/
//     health_engine.h) that was current when the sweep started - a topology
//     reload that builds a new engine cannot free it under the sweep;
//   * passthrough: an immutable snapshot of the IOMMU groups and their PFs.
// Each engine has a generation; a sweep result from an older engine (a
// reload happened meanwhile) is dropped instead of applied to the new devices.
// At most one sweep is in flight (a pulse that finds one running is skipped),
// and a topology reload waits until none is (may_reload()).
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "flags.h"
#include "resources.h"
#include "mi355x/health_engine.h"

namespace mi355x::daemon {

struct SweepResult {
  uint64_t engine_gen = 0;
  std::map<std::string, bool> health;  // device id / IOMMU group -> healthy
  double sweep_ms = 0;
  // container driver: xGMI fabric state after the sweep
  uint64_t fabric_version = 0;
  std::vector<std::pair<std::string, std::string>> degraded;
  uint64_t health_version = 0;
};

// passthrough input of one sweep (copied when the sweep starts)
struct PassthroughSnapshot {
  Driver driver = Driver::Vf;
  std::string sysfs_root;
  std::string exporter_socket;
  std::vector<std::pair<std::string, std::vector<std::string>>> groups;  // group -> parent PF BDFs
};

// gim gone -> every group Unhealthy; else a group is Unhealthy if any parent PF is (amdgpu_sriov.go:217-308);
// vfio-pci present -> Healthy (amdgpu_pf.go:210-229)
std::map<std::string, bool> passthrough_health(const PassthroughSnapshot& s, int abort_fd);

class HealthController {
 public:
  // `abort_fd`: the daemon's shutdown pipe (ends every wait of a sweep)
  HealthController(const Flags& f, int abort_fd) : f_(f), abort_fd_(abort_fd) {}
  ~HealthController() { close(); }

  // a new engine (generation) for these devices; none for passthrough drivers or no devices
  void rebuild(Driver drv, const std::vector<GpuDevice>& devices, const KfdTopology& topo,
               const std::vector<Resource>& resources);
  // the work of one sweep, for a worker thread (self-contained, see above)
  std::function<SweepResult()> job() const;
  // run a sweep on this thread (start-up: verdicts before the first registration)
  SweepResult sweep_now() const { return job()(); }

  bool inflight() const { return inflight_; }
  void started() { inflight_ = true; }
  // a sweep finished; false when it was for an engine that has been replaced
  bool finished(const SweepResult& r);
  bool may_reload() const { return !inflight_; }

  // xGMI fabric: true once per change of the engine's degraded-link set
  bool fabric_changed(const SweepResult& r);

  uint64_t generation() const { return gen_; }
  std::shared_ptr<health::Engine> engine() const { return engine_; }
  void close();

 private:
  const Flags& f_;
  int abort_fd_;
  Driver driver_ = Driver::Container;
  std::shared_ptr<health::Engine> engine_;
  PassthroughSnapshot pt_;
  uint64_t gen_ = 0;
  uint64_t fabric_seen_ = 0;
  bool inflight_ = false;
};

}  // namespace mi355x::daemon
