// Hive-aware device-subset allocator (GetPreferredAllocation policy).
//
// Reference: BestEffortPolicy (internal/pkg/allocator/besteffort_policy.go:45-151)
// over the pair-weight graph and candidate enumeration in
// internal/pkg/allocator/device.go:135-442.
//
// The reference scores a candidate subset by the sum of pairwise weights
// (same physical GPU / link type / same NUMA) and enumerates candidates by a
// BFS over *ordered* sequences of physical GPUs: every GPU but the last is
// taken whole, the last contributes a prefix. That is 8!/(8-k)! sequences for k
// whole GPUs, with every set visited many times.
//
// This allocator searches the same candidate family — (set S of whole GPUs,
// one partial GPU p) — but over *sets*, by depth-first search with
// precomputed group-level weight aggregates and a non-negative-weight bound,
// so each distinct candidate costs O(|S|) and no set is visited twice. The
// reference's first-found tie-break is reproduced exactly: among equal weights
// the winner is the candidate with the fewest GPUs, then the lexicographically
// smallest GPU sequence in the (free-count asc, parent-id asc) group order —
// which is precisely the order in which the reference BFS emits candidates.
// `reference_allocate` keeps a faithful re-implementation of the ordered BFS
// for parity tests and for the side-by-side benchmark.
//
// Deliberate differences:
//   * a pair with no kfd link scores as the worst link, not 0 (configurable);
//   * pairs in different xGMI hives pay an extra penalty, so a request that
//     fits in one hive never straddles two;
//   * no nil-dereference when no candidate exists: an error is returned.
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "mi355x/kfd_topology.h"

namespace mi355x {

struct AllocDevice {
  std::string id;         // kubelet device ID (BDF / amdgpu_xcp_N / test ids)
  int node_id = -1;       // kfd node index
  int numa_node = -1;
  std::string unique_id;  // physical GPU identity ("DevId" in the reference)
  uint64_t hive_id = 0;   // 0 = unknown; filled from kfd when possible
  // The device's kfd node is unreadable (EPERM) but its identity was
  // recovered from PCI sysfs (GpuDevice::identity == "sysfs"): links to it are
  // inferred from unique_id / hive_id instead of kfd io_links.
  bool inferred_links = false;
};

struct AllocatorOptions {
  // reference behaviour: a pair without any kfd link weighs 0 (device.go:266)
  bool missing_pair_is_worst = true;
  // extra weight for a pair whose endpoints sit in different (known) xGMI hives
  int cross_hive_penalty = 100;
  // physical-GPU pairs (AllocDevice::unique_id keys) whose direct xGMI link is
  // down at run time (amd-smi link state, health/fabric.py): their kfd link
  // still reads xGMI, but traffic between them now takes another path, so the
  // pair scores as the worst link ("other") and packing avoids it
  std::vector<std::pair<std::string, std::string>> degraded_links;
  // Off (default): the reference's candidate family (whole GPUs + one partial
  // prefix), exact reference tie-breaks. On: an exact search over how many
  // devices to take from every class of interchangeable devices (several
  // partial GPUs allowed), minimising the same total pair weight; ties go to
  // fewer physical GPUs, then the better kfd links between them (lower kfd
  // link weight, then higher max_bandwidth), then the anti-fragmentation order.
  bool extended_search = false;
  // Auto (the plugins' default): extended search on nodes where some physical
  // GPU is split into several devices (partition modes), the reference family
  // on whole-GPU nodes, where it already enumerates every GPU subset. Measured:
  // on fragmented partitioned nodes the reference family was never heavier than
  // the optimum, but broke ties onto more physical GPUs (profiles/
  // allocator_default_vs_optimum.json); every Appendix A.1 row is unchanged.
  bool extended_search_auto = false;
  // extended search: node budget before falling back to the reference family
  uint64_t extended_node_limit = 2000000;
};

struct AllocResult {
  std::vector<std::string> ids;
  std::string error;                 // empty on success
  int64_t weight = -1;               // total pair weight of the chosen set (-1: short-circuit)
  uint64_t candidates = 0;           // candidate subsets scored
  bool short_circuit = false;
};

class HiveAllocator {
 public:
  HiveAllocator() = default;

  // Builds the pair-weight matrix from kfd io_links/p2p_links of the nodes in
  // `devs` (reference fetchAllPairWeights, device.go:220-252) and groups
  // devices by physical GPU (groupPartitionsByDevId, device.go:287-304).
  // Returns "" or an error message.
  std::string init(const std::vector<AllocDevice>& devs, const KfdTopology& topo,
                   const AllocatorOptions& opt = AllocatorOptions());

  // Optimal allocation; same validations, short-circuits and error strings as
  // BestEffortPolicy.Allocate (besteffort_policy.go:88-151).
  AllocResult allocate(const std::vector<std::string>& available,
                       const std::vector<std::string>& required, int size) const;

  // Faithful ordered-BFS enumeration (reference getCandidateDeviceSubsets,
  // device.go:353-442) over the same weight matrix. For parity tests and
  // benchmarks only: cost grows factorially with the number of GPUs.
  AllocResult reference_allocate(const std::vector<std::string>& available,
                                 const std::vector<std::string>& required, int size) const;

  bool initialized() const { return !devs_.empty(); }
  size_t num_devices() const { return devs_.size(); }
  size_t num_groups() const { return groups_.size(); }
  // number of (from<to) node pairs that had a kfd link (reference len(p2pWeights) counts 'from' keys)
  size_t num_linked_pairs() const { return linked_pairs_; }
  size_t num_from_keys() const { return from_keys_; }
  // number of (i<j) device pairs whose link was inferred from sysfs identity
  size_t num_inferred_pairs() const { return inferred_pairs_; }
  int pair_weight(const std::string& a, const std::string& b) const;
  int link_type(const std::string& a, const std::string& b) const;
  const AllocatorOptions& options() const { return opt_; }
  // effective search mode after init (extended_search, or auto resolved)
  bool extended() const { return opt_.extended_search; }

 private:
  struct Group {
    std::string key;        // unique_id
    std::string parent_id;  // ID of the non-xcp device of this GPU ("" if none)
    std::vector<int> members;  // device indices, by node id
  };
  std::string validate(const std::vector<std::string>& available, const std::vector<std::string>& required,
                       int size, AllocResult* out, std::vector<int>* avail_idx,
                       std::vector<int>* req_idx) const;
  // groups restricted to available-and-not-required members, in reference order
  std::vector<std::vector<int>> filtered_groups(const std::vector<int>& avail_idx,
                                                const std::vector<int>& req_idx) const;
  // extended_search: false when the node budget ran out (caller falls back)
  bool allocate_extended(const std::vector<int>& avail_idx, const std::vector<int>& req_idx, int size,
                         AllocResult* out) const;

  AllocatorOptions opt_;
  std::vector<AllocDevice> devs_;
  std::unordered_map<std::string, int> index_;
  std::vector<int> w_;         // n*n pair weights
  std::vector<int> link_;      // n*n best link type (0 = none)
  std::vector<int> link_kw_;   // n*n kfd link weight of that link (0 = unknown)
  std::vector<int64_t> link_bw_;  // n*n kfd max_bandwidth of that link (MB/s, 0 = unknown)
  std::vector<Group> groups_;
  std::vector<int> dev_group_;  // device index -> group index
  size_t linked_pairs_ = 0;
  size_t from_keys_ = 0;
  size_t inferred_pairs_ = 0;
};

// Reference pair-weight formula (device.go:135-157) plus the hive term.
int pair_weight_formula(bool same_gpu, int link_type, bool same_numa, bool cross_hive,
                        const AllocatorOptions& opt, bool has_link);

}  // namespace mi355x
