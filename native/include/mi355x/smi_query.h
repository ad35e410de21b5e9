// amd-smi (libamd_smi.so, ROCm 7.x) cross-check and health source.
//
// No reference counterpart: the reference reads partition modes and health
// from sysfs and an external exporter. amd-smi gives
// per-processor xGMI hive id, partition modes, ECC counters and — crucially
// for the liveness probe — the render-node <-> HIP ordinal mapping
// (amdsmi_get_gpu_enumeration_info). The library is dlopen()ed; every field is
// best-effort and `ok=false` simply means "not available here".
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace mi355x {

struct SmiGpu {
  std::string bdf;              // dddd:bb:dd.f
  std::string uuid;
  std::string market_name;
  uint64_t device_id = 0;
  uint64_t target_graphics_version = 0;  // e.g. 0x950 style value as reported
  uint32_t num_compute_units = 0;
  uint64_t kfd_id = 0;
  int kfd_node_id = -1;
  int partition_id = -1;
  uint64_t xgmi_hive_id = 0;
  std::string compute_partition;
  std::string memory_partition;
  uint64_t vram_mb = 0;
  uint64_t ecc_correctable = 0;
  uint64_t ecc_uncorrectable = 0;
  bool ecc_ok = false;
  int drm_render = -1;
  int drm_card = -1;
  int hsa_id = -1;
  int hip_id = -1;
  std::string hip_uuid;
  std::string driver_name;      // amdsmi_get_gpu_driver_info
  std::string driver_version;
  int gfx_activity = -1;        // amdsmi_get_gpu_activity, % (-1 = unavailable)
};

struct SmiSnapshot {
  bool ok = false;
  std::string error;
  std::vector<SmiGpu> gpus;
};

bool smi_available();
// Keep amd-smi initialised between queries (a reference on the shared
// amdsmi_init): each query otherwise pays a full init/shut_down cycle, ~26 ms
// on an MI355X node. The health loop holds one while amd-smi sources are on.
bool smi_hold();
void smi_unhold();
// amdsmi_init(AMD_GPUS) -> enumerate every GPU processor -> amdsmi_shut_down
// (init/shut_down are reference-counted across this file's users).
SmiSnapshot smi_snapshot();

// xGMI link state of one GPU (amdsmi_get_gpu_xgmi_link_status: up / down /
// disabled per link) and the per-link peers it is wired to
// (amdsmi_get_link_metrics: destination BDF, bit rate, max bandwidth, type,
// traffic counters). The health loop watches for links that go down; the
// allocator then stops treating that GPU pair as xGMI-connected.
struct SmiLinkPeer {
  std::string peer_bdf;
  int link_type = -1;          // amdsmi_link_type_t: 1 PCIe, 2 xGMI
  uint32_t bit_rate_gbps = 0;  // current
  uint32_t max_bandwidth_gbps = 0;
  uint64_t read_kb = 0, write_kb = 0;
};

struct SmiXgmiLinks {
  std::string bdf;
  bool status_ok = false;       // link status query answered
  std::vector<int> status;      // per link: 0 down, 1 up, 2 disabled
  bool metrics_ok = false;
  std::vector<SmiLinkPeer> peers;
  std::string error;
};

struct SmiXgmiSnapshot {
  bool ok = false;
  std::string error;
  std::vector<SmiXgmiLinks> gpus;
};

SmiXgmiSnapshot smi_xgmi_links();

// Push-style GPU events from the driver (amdsmi_*_gpu_event_notification):
// resets, VM faults, thermal throttling, queue evictions. SURVEY §5 "failure
// detection": the health loop drains them every pulse instead of waiting for
// a probe to fail.
struct SmiEvent {
  std::string bdf;
  int type = 0;            // amdsmi_evt_notification_type_t
  std::string name;        // "gpu_pre_reset", ...
  std::string message;
};

class SmiEventWatcher {
 public:
  SmiEventWatcher() = default;
  ~SmiEventWatcher();
  SmiEventWatcher(const SmiEventWatcher&) = delete;
  SmiEventWatcher& operator=(const SmiEventWatcher&) = delete;
  // Subscribe every GPU to `mask` (bit i-1 = event type i). Returns "" or an error.
  std::string start(uint64_t mask);
  // Events that arrived within `timeout_ms` (0 = just drain what is queued).
  std::vector<SmiEvent> poll(int timeout_ms);
  void stop();
  bool running() const { return running_; }
  size_t devices() const { return handles_.size(); }

 private:
  bool running_ = false;
  std::vector<void*> handles_;
  std::vector<std::string> bdfs_;
};

const char* smi_event_name(int type);

}  // namespace mi355x
