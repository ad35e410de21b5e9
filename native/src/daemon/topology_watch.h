// -topology_watch: when to re-discover the node's GPUs.
//
// An amd-smi partition switch (SPX -> CPX, NPS1 -> NPS2) changes the devices
// under a running plugin; the reference only notices at its next start. The
// daemon polls a cheap signature of the topology (gpu_discovery.h
// topology_signature) every period. A reload happens when a new signature
// has held for one whole period (a switch passes through states with devices
// half gone) and no health sweep is running (the sweep's engine was built for
// the old devices; HealthController::may_reload()).
#pragma once

#include <string>

namespace mi355x::daemon {

class TopologyWatch {
 public:
  explicit TopologyWatch(const std::string& sig = "") : applied_(sig), seen_(sig) {}

  // one periodic reading; true = reload now (then call applied())
  bool observe(const std::string& cur, bool may_reload) {
    if (cur != seen_) {  // changed since the last reading: wait one period
      seen_ = cur;
      return false;
    }
    return cur != applied_ && may_reload;
  }
  void applied(const std::string& sig) { applied_ = sig; }
  const std::string& current() const { return applied_; }

 private:
  std::string applied_;  // what the advertised resources were built from
  std::string seen_;     // the previous reading
};

}  // namespace mi355x::daemon
