// kfd topology + GPU discovery + hive allocator (src/topology/*, src/alloc/*)
// over a generated MI355X sysfs tree ($MI355X_FUZZ_SYSFS_MUT, a private copy)
// whose files the input rewrites or removes: what a driver in a strange state,
// a partition switch caught half-way, or a newer kernel's format looks like to
// the daemons. Input: records of [u16 file index][u16 length][bytes]; length
// 0xFFFF removes the file. The tree is restored after every input.
// Invariants: discovery returns (devices with unique IDs), the allocator either
// refuses or answers every request with exactly `size` distinct available IDs,
// and the topology signature is a pure function of the tree.
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <map>
#include <memory>
#include <optional>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "fuzz_common.h"
#include "mi355x/allocator.h"
#include "mi355x/gpu_discovery.h"
#include "mi355x/kfd_topology.h"
#include "mi355x/sysfs.h"

using namespace mi355x;
using mi355x::fuzz::fail;

namespace {

std::string g_root;
std::vector<std::string> g_files;  // regular files the input may rewrite (relative)

void walk(const std::string& rel) {
  const std::string abs = rel.empty() ? g_root : g_root + "/" + rel;
  for (const auto& name : list_dir(abs)) {
    const std::string r = rel.empty() ? name : rel + "/" + name;
    struct stat st {};
    if (::lstat((g_root + "/" + r).c_str(), &st) != 0 || S_ISLNK(st.st_mode)) continue;
    if (S_ISDIR(st.st_mode)) {
      if (r == "devices/system") continue;  // CPU / NUMA trees: views only, not discovery
      walk(r);
    } else if (S_ISREG(st.st_mode)) {
      g_files.push_back(r);
    }
  }
}

std::optional<std::string> slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) return std::nullopt;
  std::ostringstream o;
  o << f.rdbuf();
  return o.str();
}

void put(const std::string& p, const std::string& data) {
  std::ofstream f(p, std::ios::binary | std::ios::trunc);
  f << data;
}

}  // namespace

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  g_root = fuzz::env_or_die("MI355X_FUZZ_SYSFS_MUT");
  walk("");
  std::sort(g_files.begin(), g_files.end());
  if (g_files.size() < 100) fail("fixture tree too small", g_root);
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size > 64 * 1024) return 0;
  std::map<std::string, std::optional<std::string>> saved;  // original content (nullopt: absent)
  size_t i = 0;
  while (i + 4 <= size) {
    const size_t idx = (data[i] | (data[i + 1] << 8)) % g_files.size();
    const size_t len = data[i + 2] | (data[i + 3] << 8);
    i += 4;
    const std::string p = g_root + "/" + g_files[idx];
    if (!saved.count(p)) saved[p] = slurp(p);
    if (len == 0xFFFF) {
      ::unlink(p.c_str());
      continue;
    }
    const size_t n = std::min(len, size - i);
    put(p, std::string(reinterpret_cast<const char*>(data) + i, n));
    i += n;
  }

  const KfdTopology topo = KfdTopology::load_sysfs(g_root);
  const DiscoveryResult res = discover_gpus(g_root, topo);
  std::set<std::string> ids;
  for (const auto& d : res.devices)
    if (!ids.insert(d.id).second) fail("duplicate device ID", d.id);
  (void)partition_config_count(res.devices);
  (void)is_homogeneous(res.devices);
  const std::string sig = topology_signature(g_root);
  if (sig != topology_signature(g_root)) fail("topology signature not deterministic");

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

  for (const auto& [p, orig] : saved) {
    if (orig) put(p, *orig);
    else ::unlink(p.c_str());
  }
  return 0;
}
