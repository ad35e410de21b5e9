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
};

struct SmiSnapshot {
  bool ok = false;
  std::string error;
  std::vector<SmiGpu> gpus;
};

bool smi_available();
// amdsmi_init(AMD_GPUS) -> enumerate every GPU processor -> amdsmi_shut_down.
SmiSnapshot smi_snapshot();

}  // namespace mi355x
