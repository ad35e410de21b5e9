// KFD topology model: every node under <sysfs>/class/kfd/kfd/topology/nodes,
// parsed once, with io_links / p2p_links / mem_banks.
//
// Replaces the reference's per-key regex scans, which open every kfd
// properties file 3-4 times per startup (internal/pkg/amdgpu/amdgpu.go:406-445,
// 821-863; internal/pkg/allocator/device.go:107-133,159-252). Here each file
// is read exactly once into a key/value map, and the gfx950-relevant fields
// the reference ignores (hive_id, num_xcc, location_id, link weight and
// bandwidth) are first-class.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "mi355x/sysfs.h"

namespace mi355x {

// kfd io_link "type" values (include/uapi/linux/kfd_sysfs.h). The reference
// only distinguishes 11 (xGMI) and 2 (PCIe) (internal/pkg/allocator/device.go:144-150).
enum KfdLinkType : int {
  kLinkUndefined = 0,
  kLinkHyperTransport = 1,
  kLinkPcie = 2,
  kLinkOther = 3,
  kLinkXgmi = 11,
};

struct KfdLink {
  int type = kLinkUndefined;
  int node_from = -1;
  int node_to = -1;
  int weight = 0;           // kfd NUMA-distance style link weight
  int64_t min_bandwidth = 0;  // MB/s
  int64_t max_bandwidth = 0;  // MB/s
  int flags = 0;
  bool p2p = false;         // came from p2p_links/ (indirect) rather than io_links/
};

struct KfdMemBank {
  int heap_type = 0;
  uint64_t size_in_bytes = 0;
  int flags = 0;
  int width = 0;
  int mem_clk_max = 0;
};

struct KfdNode {
  int id = -1;
  KeyValues props;
  std::string name;
  int64_t gpu_id = 0;
  std::vector<KfdLink> io_links;
  std::vector<KfdLink> p2p_links;
  std::vector<KfdMemBank> mem_banks;

  int64_t prop(const char* key, int64_t fallback = 0) const { return kv_i64(props, key, fallback); }
  uint64_t prop_u64(const char* key, uint64_t fallback = 0) const { return kv_u64(props, key, fallback); }
  std::string prop_str(const char* key) const { return kv_str(props, key); }

  int cpu_cores_count() const { return static_cast<int>(prop("cpu_cores_count")); }
  int simd_count() const { return static_cast<int>(prop("simd_count")); }
  int simd_per_cu() const { return static_cast<int>(prop("simd_per_cu")); }
  int gfx_target_version() const { return static_cast<int>(prop("gfx_target_version")); }
  int drm_render_minor() const { return static_cast<int>(prop("drm_render_minor", -1)); }
  int num_xcc() const { return static_cast<int>(prop("num_xcc", 1)); }
  int device_id() const { return static_cast<int>(prop("device_id")); }
  int vendor_id() const { return static_cast<int>(prop("vendor_id")); }
  int location_id() const { return static_cast<int>(prop("location_id")); }
  int domain() const { return static_cast<int>(prop("domain")); }
  uint64_t hive_id() const { return prop_u64("hive_id"); }
  // unique_id as the decimal string kfd prints (the reference keys partitions
  // of one physical GPU by this string, amdgpu.go:433-441).
  std::string unique_id() const { return prop_str("unique_id"); }
  uint64_t local_mem_bytes() const;  // sum of mem_banks (falls back to local_mem_size)

  // A compute-capable GPU agent. kfd reports CPU nodes with simd_count 0.
  bool is_gpu() const { return cpu_cores_count() == 0 && simd_count() > 0; }
  // The reference's node-global health predicate (amdgpu.go:902).
  bool is_live_gpu() const { return cpu_cores_count() == 0 && gfx_target_version() > 0; }
  // The reference's pair-weight scan only walks nodes with a render node (device.go:238-241).
  bool has_render_node() const { return drm_render_minor() > 0; }
};

class KfdTopology {
 public:
  // nodes_dir is ".../topology/nodes". Missing directory => empty topology.
  static KfdTopology load(const std::string& nodes_dir);
  // Convenience: <sysfs_root>/class/kfd/kfd/topology/nodes
  static KfdTopology load_sysfs(const std::string& sysfs_root);

  const std::vector<KfdNode>& nodes() const { return nodes_; }
  const KfdNode* node(int id) const;
  const KfdNode* node_by_render_minor(int minor) const;

  // render minor -> unique_id (reference GetDevIdsFromTopology, amdgpu.go:406-445)
  std::map<int, std::string> render_to_unique_id() const;
  // render minor -> kfd node index (reference GetNodeIdsFromTopology, amdgpu.go:821-863)
  std::map<int, int> render_to_node_id() const;
  // GPU nodes in node-id order. ROCr enumerates agents in this order, so the
  // position in this list is the ROCr/HIP ordinal when every node is visible.
  std::vector<const KfdNode*> gpu_nodes() const;
  // number of nodes with simd_count > 0 (reference countGPUDevFromTopology, amdgpu.go:914-950)
  int count_gpu_nodes() const;
  // reference simpleHealthCheck predicate (amdgpu.go:865-910)
  bool any_live_gpu() const;
  // all links (io + p2p) originating from GPU nodes with a render node
  std::vector<KfdLink> all_gpu_links() const;

  const std::string& nodes_dir() const { return nodes_dir_; }
  // Node directories whose properties file exists but cannot be read. kfd
  // answers EPERM for GPUs the reader's device cgroup denies (measured on the
  // gpurun box: 7 of 8 GPU nodes, profiles/archive/sysfs_access_box.json), so these
  // are GPUs the process cannot see through kfd, not missing GPUs.
  const std::vector<int>& unreadable_node_ids() const { return unreadable_; }

 private:
  std::string nodes_dir_;
  std::vector<KfdNode> nodes_;
  std::vector<int> unreadable_;
  std::map<int, size_t> index_;
};

// Parse one link properties file.
bool parse_kfd_link(const std::string& properties_path, bool p2p, KfdLink* out);

}  // namespace mi355x
