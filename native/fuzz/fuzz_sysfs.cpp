// kfd topology + GPU discovery + hive allocator (src/topology/*, src/alloc/*)
// over a generated MI355X sysfs tree ($MI355X_FUZZ_SYSFS_MUT, a private copy)
// whose files the input rewrites or removes (sysfs_mutator.h): what a driver
// in a strange state, a partition switch caught half-way, or a newer kernel's
// format looks like to the daemons. Invariants: discovery returns (devices
// with unique IDs), the allocator either refuses or answers every request with
// exactly `size` distinct available IDs, and the topology signature is a pure
// function of the tree.
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "mi355x/allocator.h"
#include "mi355x/gpu_discovery.h"
#include "mi355x/kfd_topology.h"
#include "sysfs_mutator.h"

using namespace mi355x;
using mi355x::fuzz::fail;

namespace {
std::unique_ptr<fuzz::SysfsMutator> g_tree;
}

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  g_tree = std::make_unique<fuzz::SysfsMutator>(fuzz::env_or_die("MI355X_FUZZ_SYSFS_MUT"));
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size > 64 * 1024) return 0;
  g_tree->apply(data, size);
  const std::string& root = g_tree->root();

  const KfdTopology topo = KfdTopology::load_sysfs(root);
  const DiscoveryResult res = discover_gpus(root, topo);
  std::set<std::string> ids;
  for (const auto& d : res.devices)
    if (!ids.insert(d.id).second) fail("duplicate device ID", d.id);
  (void)partition_config_count(res.devices);
  (void)is_homogeneous(res.devices);
  const std::string sig = topology_signature(root);
  if (sig != topology_signature(root)) fail("topology signature not deterministic");

  std::vector<AllocDevice> ad;
  for (const auto& d : res.devices) {
    AllocDevice a;
    a.id = d.id;
    a.node_id = d.node_id;
    a.numa_node = d.numa_node;
    a.unique_id = !d.unique_id.empty() ? d.unique_id : "bdf:" + d.bdf;
    a.hive_id = d.hive_id;
    a.inferred_links = d.node_id < 0 && d.identity == "sysfs";
    ad.push_back(a);
  }
  for (const bool ext : {false, true}) {
    HiveAllocator alloc;
    AllocatorOptions opt;
    opt.extended_search_auto = ext;
    opt.extended_node_limit = 50000;
    if (!alloc.init(ad, topo, opt).empty()) continue;
    const std::vector<std::string> avail(ids.begin(), ids.end());
    for (int k : {1, 2, 3, 4, 8, static_cast<int>(avail.size())}) {
      if (k < 1 || k > static_cast<int>(avail.size())) continue;
      const std::vector<std::string> must = {avail.front()};
      const AllocResult r = alloc.allocate(avail, must, k);
      if (!r.error.empty()) fail("allocation over every device failed", r.error);
      const std::set<std::string> got(r.ids.begin(), r.ids.end());
      if (static_cast<int>(got.size()) != k || r.ids.size() != got.size()) fail("wrong allocation size");
      for (const auto& id : got)
        if (!ids.count(id)) fail("allocated an unknown ID", id);
      if (!got.count(avail.front())) fail("must-include ID dropped");
    }
  }

  g_tree->restore();
  return 0;
}
