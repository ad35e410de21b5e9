// C++ unit tests for the native core (ctest). Built plain and under
// -fsanitize=address,undefined / thread (MI355X_SANITIZE) — the reference has
// no race or sanitizer coverage at all.
//
//   test_core <repo testdata dir> [<reference testdata dir>]
//
// Reference fixtures are optional: missing => those cases are skipped.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "mi355x/allocator.h"
#include "mi355x/gpu_discovery.h"
#include "mi355x/kfd_topology.h"
#include "mi355x/pci_scan.h"
#include "mi355x/sysfs.h"

using namespace mi355x;

static int g_fail = 0, g_pass = 0, g_skip = 0;
#define CHECK(cond)                                                   \
  do {                                                                \
    if (cond) {                                                       \
      ++g_pass;                                                       \
    } else {                                                          \
      ++g_fail;                                                       \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                 \
  } while (0)

static std::vector<AllocDevice> synthetic_devices(int dev_count, int parts, int numa_count, int start, int end) {
  // mirrors the reference test-device generator semantics (device_test.go:43-67):
  // first partition of GPU i is "test<i+1>", the rest "amdgpu_xcp_<8i+j>"
  std::vector<AllocDevice> out;
  int node = start;
  for (int i = 0; i < dev_count; ++i) {
    int per_numa = dev_count / numa_count;
    for (int j = 0; j < parts; ++j) {
      if (node > end) break;
      std::string id = j == 0 ? "test" + std::to_string(i + 1) : "amdgpu_xcp_" + std::to_string(i * 8 + j);
      out.push_back(AllocDevice{id, node, i / per_numa, std::to_string(i), 0});
      ++node;
    }
  }
  return out;
}

static std::vector<std::string> ids_of(const std::vector<AllocDevice>& d) {
  std::vector<std::string> o;
  for (auto& x : d) o.push_back(x.id);
  return o;
}

static std::set<std::string> as_set(const std::vector<std::string>& v) { return {v.begin(), v.end()}; }

static void test_parsers(const std::string& ref) {
  auto kv = parse_kv_file(ref + "/topology-parsing/topology/nodes/2/properties");
  if (!kv) {
    ++g_skip;
    return;
  }
  CHECK(kv_i64(*kv, "simd_count", 0) == 256);
  CHECK(kv_i64(*kv, "simd_id_base", 0) == 2147487744LL);
  CHECK(kv->find("asdf") == kv->end());
  auto mb = parse_kv_file(ref + "/topology-parsing/topology/nodes/1/mem_banks/0/properties");
  CHECK(mb && kv_u64(*mb, "size_in_bytes", 0) == 17163091968ULL);
  auto t = KfdTopology::load(ref + "/topology-parsing/topology/nodes");
  CHECK(t.count_gpu_nodes() == 2);
  auto fw = parse_debugfs_firmware_info(ref + "/debugfs-parsing/amdgpu_firmware_info");
  CHECK(fw.feature.size() == 14 && fw.firmware.size() == 14);
  CHECK(fw.firmware["VCE"] == 0x352d0400u && fw.feature["MEC2"] == 33u);
  auto m = KfdTopology::load(ref + "/topology-parsing-mi308/topology/nodes");
  auto r2u = m.render_to_unique_id();
  CHECK(r2u.size() == 32);
  CHECK(r2u[128] == "598046273873802902" && r2u[187] == "6576958293045616595");
}

static void test_allocator_reference_contract(const std::string& ref) {
  auto topo = KfdTopology::load(ref + "/topo-mi300-cpx/topology/nodes");
  if (topo.nodes().empty()) {
    ++g_skip;
    return;
  }
  auto devs = synthetic_devices(8, 8, 2, 2, 64);
  HiveAllocator a;
  CHECK(a.init(devs, topo).empty());
  auto all = ids_of(devs);
  auto r = a.allocate(all, {}, 1);
  CHECK(r.error.empty() && r.ids == std::vector<std::string>{"test8"});
  r = a.allocate(all, {}, 8);
  CHECK(as_set(r.ids) == as_set({"test1", "amdgpu_xcp_1", "amdgpu_xcp_2", "amdgpu_xcp_3", "amdgpu_xcp_4",
                                 "amdgpu_xcp_5", "amdgpu_xcp_6", "amdgpu_xcp_7"}));
  r = a.allocate({"test3", "test4", "test5", "test6", "test7", "test8"}, {"test5"}, 3);
  CHECK(as_set(r.ids) == as_set({"test5", "test6", "test7"}));
  // exact search and the ordered BFS agree on every size
  for (int k = 1; k <= 40; k += 3) {
    auto e = a.allocate(all, {}, k);
    auto b = a.reference_allocate(all, {}, k);
    CHECK(e.error.empty() && b.error.empty());
    CHECK(e.weight == b.weight);
    CHECK(e.ids == b.ids);
  }
  // reentrancy: concurrent allocate() on a shared const allocator
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&] {
      for (int i = 0; i < 50; ++i)
        if (a.allocate(all, {}, 10).ids.size() != 10) ++bad;
    });
  for (auto& x : th) x.join();
  CHECK(bad == 0);
}

static void test_errors() {
  KfdTopology empty;
  HiveAllocator a;
  CHECK(!a.init({}, empty).empty());
  CHECK(a.allocate({"a", "b"}, {}, 1).error == "Init method must be called before Allocate");
  auto devs = synthetic_devices(4, 1, 1, 2, 5);
  CHECK(a.init(devs, empty).empty());
  CHECK(a.allocate({"test1"}, {}, 0).error == "allocation size can not be negative");
  CHECK(a.allocate({"test1"}, {}, 2).error == "available devices count less than allocation size");
  CHECK(a.allocate({"test1", "test2"}, {"test1", "test2", "test3"}, 2).error ==
        "must_include devices size is more than allocation size");
  CHECK(a.allocate({"test1", "test2", "test3"}, {"test4"}, 2).error ==
        "No candidate subset found with matching criteria");
  auto r = a.allocate({"test1", "test2"}, {}, 2);
  CHECK(r.short_circuit && r.ids.size() == 2);
}

// xGMI link down at run time (AllocatorOptions::degraded_links): the pair
// scores as the worst link, so packing avoids it; the search and the
// reference BFS still agree on the re-weighted matrix.
static void test_degraded_links(const std::string& ref) {
  auto topo = KfdTopology::load(ref + "/topo-mi210-xgmi-pcie/nodes");
  if (topo.nodes().empty()) {
    ++g_skip;
    return;
  }
  auto devs = synthetic_devices(8, 1, 2, 1, 8);
  HiveAllocator a;
  CHECK(a.init(devs, topo).empty());
  auto all = ids_of(devs);
  auto before = a.allocate(all, {}, 2);
  CHECK(before.error.empty() && before.ids.size() == 2);
  // degrade the chosen pair (physical GPU keys = unique_id = GPU index here)
  AllocatorOptions opt;
  std::string ka, kb;
  for (auto& d : devs) {
    if (d.id == before.ids[0]) ka = d.unique_id;
    if (d.id == before.ids[1]) kb = d.unique_id;
  }
  opt.degraded_links = {{kb, ka}};  // order does not matter
  CHECK(a.init(devs, topo, opt).empty());
  auto after = a.allocate(all, {}, 2);
  CHECK(after.error.empty() && as_set(after.ids) != as_set(before.ids));
  CHECK(after.weight <= before.weight);  // another same-hive pair is as good
  auto forced = a.allocate(before.ids, {}, 2);  // only the degraded pair available
  CHECK(forced.short_circuit && as_set(forced.ids) == as_set(before.ids));
  for (int k = 2; k <= 7; ++k) {
    auto e = a.allocate(all, {}, k);
    auto b = a.reference_allocate(all, {}, k);
    CHECK(e.weight == b.weight);
  }
}

int main(int argc, char** argv) {
  std::string repo = argc > 1 ? argv[1] : "testdata";
  std::string ref = argc > 2 ? argv[2] : "/root/reference/testdata";
  (void)repo;
  test_parsers(ref);
  test_allocator_reference_contract(ref);
  test_errors();
  test_degraded_links(ref);
  std::printf("test_core: %d passed, %d failed, %d skipped\n", g_pass, g_fail, g_skip);
  return g_fail ? 1 : 0;
}
