// Container start-up views returned as Allocate mounts (opt-in, both
// experimental): the native daemon's -node_view and -topology_view, with the
// same layout as the Python CLI's node_view.py / topology_view.py.
//
//   node view      /sys/devices/system/node without the per-CPU cache
//                  descriptors ROCr walks at start-up (7,650 of hsa_init's 9,486
//                  sysfs opens on a 256-CPU MI355X host; hsa_init 48 -> 14-16 ms
//                  in emulation, profiles/archive/measurements_r1_r3.md §3e). Everything else stays
//                  live: symlinks into the real node directory, bind-mounted
//                  read-only at an alias path, and into /sys/devices/system/cpu.
//   topology view  per distinct allocated GPU set, a copy of the kfd topology
//                  holding the CPU nodes and those GPU nodes only (renumbered,
//                  links re-targeted and filtered, *_links_count fixed),
//                  mounted over /sys/devices/virtual/kfd/kfd/topology: ROCr
//                  reads ~1/8 of the files for a 1-GPU pod and sees exactly its
//                  GPUs. gpu_id files are copied verbatim (kfd ioctls address
//                  GPUs by gpu_id).
#pragma once

#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace mi355x::views {

constexpr const char* kNodeContainerPath = "/sys/devices/system/node";
constexpr const char* kNodeAlias = "/run/mi355x/sys-node";
constexpr const char* kCpuContainerPath = "/sys/devices/system/cpu";
constexpr const char* kKfdTopologyContainerPath = "/sys/devices/virtual/kfd/kfd/topology";

// Writes the node view of `src` into `dst`; "" or the error. *links / *hidden:
// symlinks written and per-CPU cache directories left out.
std::string build_node_view(const std::string& src, const std::string& dst, const std::string& alias,
                            const std::string& cpu_root, const std::string& src_cpu_root, int* links, int* hidden);

class NodeView {
 public:
  // `alias`: where the real node directory is visible in the container (a
  // runtime that cannot mount passes the host path itself: no alias mount)
  NodeView(std::string root, const std::string& sysfs_root, std::string alias = kNodeAlias);
  // builds once; "" or the error
  std::string build();
  // (host path, container path) pairs in mount order; empty before build()
  std::vector<std::pair<std::string, std::string>> mounts() const;
  int links = 0, hidden = 0;

 private:
  std::string root_, alias_, src_, src_cpu_, path_;
};

// Writes the filtered topology of `src_topology` (…/kfd/kfd/topology) for the
// GPU nodes `gpu_nodes` into `dst`; "" or the error.
std::string build_topology_view(const std::string& src_topology, const std::string& dst,
                                const std::vector<int>& gpu_nodes);

class TopologyViews {
 public:
  TopologyViews(std::string base_dir, std::string src_topology)
      : base_(std::move(base_dir)), src_(std::move(src_topology)) {}
  // the view directory for this GPU node set (built on first use); "" + err
  std::string get(std::vector<int> gpu_nodes, std::string* err);
  int built() const { return built_; }

 private:
  std::string base_, src_;
  std::mutex mu_;
  int built_ = 0;
};

}  // namespace mi355x::views
