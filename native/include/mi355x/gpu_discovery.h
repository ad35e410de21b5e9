// Physical GPU / partition discovery: joins the amdgpu PCI driver view,
// the amdgpu_xcp_* platform devices (partitions beyond the first) and the kfd
// topology into one device list.
//
// Behavioural parity with the reference GetAMDGPUs
// (internal/pkg/amdgpu/amdgpu.go:448-568):
//   * PCI functions under module/amdgpu/drivers/pci:amdgpu/<BDF> with a readable
//     numa_node become devices with ID = BDF;
//   * amdgpu_xcp_<N> platform devices become devices with ID "amdgpu_xcp_<N>",
//     inheriting partition modes and NUMA node from their parent (matched by kfd
//     unique_id) and kept only if their render node is known to kfd.
// Fixed relative to the reference: card / renderD /
// unique_id / node id are reset per device instead of leaking from the
// previous loop iteration, and every path is rooted at an injectable sysfs root.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "mi355x/kfd_topology.h"

namespace mi355x {

struct GpuDevice {
  std::string id;              // PCI BDF or "amdgpu_xcp_<N>" (kubelet device ID)
  std::string bdf;             // PCI BDF of the physical GPU that owns this device
  bool is_partition = false;   // came from an amdgpu_xcp_* platform device
  int xcp_index = -1;          // <N> of amdgpu_xcp_<N>, else -1
  int card = -1;               // /dev/dri/card<N>
  int render_minor = -1;       // /dev/dri/renderD<N>
  std::string unique_id;       // kfd unique_id: identity of the physical GPU
  std::string compute_partition;  // lower-case, e.g. "spx", "cpx"
  std::string memory_partition;   // lower-case, e.g. "nps1"
  int numa_node = -1;
  int node_id = -1;            // kfd topology node index

  // enrichment from the kfd node (0 when unknown)
  int gfx_target_version = 0;  // gfx950 -> 90500
  int simd_count = 0;
  int simd_per_cu = 0;
  int num_xcc = 0;
  int pci_device_id = 0;       // kfd device_id (e.g. 0x75a3)
  int location_id = 0;
  int domain = 0;
  uint64_t hive_id = 0;        // xGMI hive; 0 = not in a hive
  uint64_t vram_bytes = 0;
  // Where the identity (unique_id / hive / partition membership) came from:
  //   "kfd"   - the device's kfd topology node (reference behaviour);
  //   "sysfs" - kfd denied the read (EPERM under a device cgroup), recovered
  //             from PCI sysfs: <dev>/unique_id, xgmi_hive_info/xgmi_hive_id,
  //             and for partitions the amdgpu_xcp_* drm-minor block layout;
  //   ""      - unknown: no kfd node and no recoverable sysfs identity.
  std::string identity;

  std::string partition_type() const {
    if (compute_partition.empty() || memory_partition.empty()) return "";
    return compute_partition + "_" + memory_partition;
  }
  int cu_count() const { return simd_per_cu > 0 ? simd_count / simd_per_cu : 0; }
};

struct DiscoveryResult {
  std::vector<GpuDevice> devices;  // sorted: PCI BDFs first (lexicographic), then xcp by N
  bool driver_loaded = false;      // <sysfs>/module/amdgpu/drivers exists
  bool kfd_present = false;        // <sysfs>/class/kfd exists
  std::vector<std::string> warnings;
  std::vector<int> kfd_unreadable_nodes;  // kfd node dirs whose properties could not be read
  int recovered_devices = 0;              // devices whose identity came from sysfs instead of kfd
  std::vector<std::string> unresolved;    // device IDs with no identity (placement must not trust them)
};

// Cheap fingerprint of the node's GPU topology: kfd's generation_id (bumped
// when kfd nodes come or go) and every amdgpu function's current compute /
// memory partition (topology.py topology_signature). Polled by both daemons'
// -topology_watch; a change is followed by a full re-discovery.
std::string topology_signature(const std::string& sysfs_root);

// Logical devices one physical GPU splits into in compute mode `mode`
// (lower-case); CPX = one per XCC. 0 = unknown mode or XCC count.
int partitions_for_mode(const std::string& mode, int total_xcc);
// XCCs per physical GPU by PCI device id (MI355X 0x75a3, MI300X 0x74a1: 8;
// MI308X 0x74a2: 4); 0 = unknown. Mirrors rocm_k8s_device_plugin_amd/models.
int xcc_count_for_device_id(int pci_device_id);

DiscoveryResult discover_gpus(const std::string& sysfs_root, const KfdTopology& topo);
DiscoveryResult discover_gpus(const std::string& sysfs_root);

// partition type ("<compute>_<memory>") -> device count; devices with unknown
// partition info are not counted (reference UniquePartitionConfigCount, amdgpu.go:570-585)
std::map<std::string, int> partition_config_count(const std::vector<GpuDevice>& devs);
// reference IsHomogeneous (amdgpu.go:588-592)
bool is_homogeneous(const std::vector<GpuDevice>& devs);
// reference IsComputePartitionSupported / IsMemoryPartitionSupported
// (amdgpu.go:594-627): presence of available_*_partition on the first GPU.
bool compute_partition_supported(const std::string& sysfs_root);
bool memory_partition_supported(const std::string& sysfs_root);

// debugfs amdgpu_firmware_info parser: "<FW> feature version: N, firmware version: 0xH"
// (reference parseDebugFSFirmwareInfo, amdgpu.go:791-816)
struct FirmwareInfo {
  std::map<std::string, uint32_t> feature;
  std::map<std::string, uint32_t> firmware;
};
FirmwareInfo parse_debugfs_firmware_info(const std::string& path);

}  // namespace mi355x
