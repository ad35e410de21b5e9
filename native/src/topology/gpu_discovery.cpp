#include "mi355x/gpu_discovery.h"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <set>

namespace mi355x {

namespace {

bool looks_like_bdf(const std::string& n) {
  // dddd:bb:dd.f — the reference globs "[0-9a-fA-F]{4}:*" (amdgpu.go:455)
  if (n.size() < 5) return false;
  for (int i = 0; i < 4; ++i)
    if (!std::isxdigit(static_cast<unsigned char>(n[i]))) return false;
  return n[4] == ':';
}

struct DrmNodes {
  int card = -1;
  int render = -1;
};

DrmNodes scan_drm(const std::string& dev_dir) {
  DrmNodes d;
  for (auto& name : list_dir(path_join(dev_dir, "drm"))) {
    if (name.rfind("card", 0) == 0 && is_all_digits(name.substr(4))) {
      d.card = static_cast<int>(parse_i64(name.substr(4), -1));
    } else if (name.rfind("renderD", 0) == 0 && is_all_digits(name.substr(7))) {
      d.render = static_cast<int>(parse_i64(name.substr(7), -1));
    }
  }
  return d;
}

void enrich(GpuDevice* g, const KfdTopology& topo) {
  const KfdNode* n = topo.node(g->node_id);
  if (!n) return;
  g->gfx_target_version = n->gfx_target_version();
  g->simd_count = n->simd_count();
  g->simd_per_cu = n->simd_per_cu();
  g->num_xcc = n->num_xcc();
  g->pci_device_id = n->device_id();
  g->location_id = n->location_id();
  g->domain = n->domain();
  g->hive_id = n->hive_id();
  g->vram_bytes = n->local_mem_bytes();
  g->identity = "kfd";
}

// "dddd:bb:dd.f" -> kfd-style location_id ((bus << 8) | (dev << 3) | fn) and domain
bool bdf_location(const std::string& bdf, int* domain, int* location) {
  unsigned d = 0, b = 0, dv = 0, f = 0;
  if (std::sscanf(bdf.c_str(), "%x:%x:%x.%x", &d, &b, &dv, &f) != 4) return false;
  *domain = static_cast<int>(d);
  *location = static_cast<int>((b << 8) | (dv << 3) | f);
  return true;
}

// Identity of a GPU whose kfd node this process cannot read. amdgpu prints
// unique_id as hex on the PCI device ("%016llx") and kfd prints the same
// value in decimal; the xGMI hive id is the same decimal number kfd shows as
// hive_id. Both are plain device attributes (no device-cgroup check), unlike
// every file under a kfd GPU node (profiles/archive/sysfs_access_box.json).
void recover_from_sysfs(GpuDevice* g, const std::string& dev_dir) {
  if (auto v = read_trimmed(path_join(dev_dir, "unique_id"))) {
    std::string hex = *v;
    if (hex.rfind("0x", 0) != 0 && hex.rfind("0X", 0) != 0) hex = "0x" + hex;
    uint64_t uid = parse_u64(hex, 0);
    if (uid != 0) {
      g->unique_id = std::to_string(uid);
      g->identity = "sysfs";
    }
  }
  if (auto v = read_trimmed(path_join(dev_dir, "xgmi_hive_info/xgmi_hive_id"))) g->hive_id = parse_u64(*v, 0);
  if (auto v = read_trimmed(path_join(dev_dir, "device"))) g->pci_device_id = static_cast<int>(parse_i64(*v, 0));
  if (auto v = read_trimmed(path_join(dev_dir, "mem_info_vram_total"))) g->vram_bytes = parse_u64(*v, 0);
  bdf_location(g->bdf, &g->domain, &g->location_id);
}

}  // namespace

int partitions_for_mode(const std::string& mode, int total_xcc) {
  if (mode == "spx") return 1;
  if (mode == "dpx") return 2;
  if (mode == "tpx") return 3;
  if (mode == "qpx") return 4;
  if (mode == "cpx") return total_xcc > 0 ? total_xcc : 0;
  return 0;
}

int xcc_count_for_device_id(int pci_device_id) {
  switch (pci_device_id) {
    case 0x75a3: return 8;  // MI355X (measured: num_xcc 8 in SPX)
    case 0x74a1: return 8;  // MI300X (reference testdata/topo-mi300-cpx: 8 partitions per GPU)
    case 0x74a2: return 4;  // MI308X (reference testdata/topology-parsing-mi308: 4 per GPU)
    default: return 0;
  }
}

DiscoveryResult discover_gpus(const std::string& sysfs_root) {
  return discover_gpus(sysfs_root, KfdTopology::load_sysfs(sysfs_root));
}

DiscoveryResult discover_gpus(const std::string& sysfs_root, const KfdTopology& topo) {
  DiscoveryResult res;
  res.kfd_present = path_exists(path_join(sysfs_root, "class/kfd"));
  res.driver_loaded = path_exists(path_join(sysfs_root, "module/amdgpu/drivers"));
  res.kfd_unreadable_nodes = topo.unreadable_node_ids();
  if (!res.driver_loaded) {
    res.warnings.push_back("amdgpu driver unavailable: " + path_join(sysfs_root, "module/amdgpu/drivers"));
    return res;
  }
  const auto render_uid = topo.render_to_unique_id();
  const auto render_node = topo.render_to_node_id();

  const std::string pci_dir = path_join(sysfs_root, "module/amdgpu/drivers/pci:amdgpu");
  std::vector<GpuDevice> pci_devs;
  for (auto& bdf : list_dir(pci_dir)) {
    if (!looks_like_bdf(bdf)) continue;
    std::string dev_dir = path_join(pci_dir, bdf);
    GpuDevice g;
    g.id = bdf;
    g.bdf = bdf;
    if (auto v = read_trimmed(path_join(dev_dir, "current_compute_partition")))
      g.compute_partition = to_lower(*v);
    if (auto v = read_trimmed(path_join(dev_dir, "current_memory_partition")))
      g.memory_partition = to_lower(*v);
    auto numa = read_trimmed(path_join(dev_dir, "numa_node"));
    if (!numa) {
      res.warnings.push_back("Failed to read 'numa_node' for " + bdf);
      continue;
    }
    int64_t nn = parse_i64(*numa, INT64_MIN);
    if (nn == INT64_MIN) {
      res.warnings.push_back("Failed to convert 'numa_node' for " + bdf);
      continue;
    }
    g.numa_node = static_cast<int>(nn);
    DrmNodes d = scan_drm(dev_dir);
    g.card = d.card;
    g.render_minor = d.render;
    if (auto it = render_uid.find(d.render); it != render_uid.end()) g.unique_id = it->second;
    if (auto it = render_node.find(d.render); it != render_node.end()) g.node_id = it->second;
    enrich(&g, topo);
    if (g.identity.empty()) {
      recover_from_sysfs(&g, dev_dir);
    } else if (g.unique_id.empty()) {
      // kfd node without a unique_id line (older kernels; the reference's
      // topology-parsing capture): the PCI attribute may still carry it
      GpuDevice probe = g;
      recover_from_sysfs(&probe, dev_dir);
      g.unique_id = probe.unique_id;
    }
    pci_devs.push_back(std::move(g));
  }

  // Devices recovered from sysfs take the per-partition compute shape of a
  // kfd-readable GPU of the same part and mode (same XCC split, same CUs).
  // total_xcc: XCCs of the physical GPU (sum of num_xcc over its kfd nodes).
  std::map<std::string, int> total_xcc_by_uid;
  for (auto& n : topo.nodes())
    if (n.is_gpu() && !n.unique_id().empty()) total_xcc_by_uid[n.unique_id()] += n.num_xcc();
  std::map<int, int> total_xcc_by_devid;
  for (auto& p : pci_devs)
    if (p.identity == "kfd" && total_xcc_by_uid.count(p.unique_id))
      total_xcc_by_devid[p.pci_device_id] = total_xcc_by_uid[p.unique_id];
  auto total_xcc_of = [&](const GpuDevice& g) {
    auto it = total_xcc_by_devid.find(g.pci_device_id);
    return it != total_xcc_by_devid.end() ? it->second : xcc_count_for_device_id(g.pci_device_id);
  };
  for (auto& g : pci_devs) {
    if (g.identity == "kfd") continue;
    for (auto& s : pci_devs) {
      if (s.identity != "kfd" || s.pci_device_id != g.pci_device_id) continue;
      g.gfx_target_version = s.gfx_target_version;
      g.simd_per_cu = s.simd_per_cu;
      if (s.compute_partition == g.compute_partition) {
        g.simd_count = s.simd_count;
        g.num_xcc = s.num_xcc;
      }
      break;
    }
  }

  // The partitions beyond the first live on amdgpu_xcp_<N> platform devices,
  // which have no sysfs link to their GPU. amdgpu allocates them in a block
  // right after the GPU's own drm device (amdgpu_xcp_dev_alloc): the block
  // that follows a GPU's primary card/render minor belongs to that GPU, and
  // partition i (i >= 1) of it uses the block's i-th xcp device. On the
  // MI355X box: GPU card0 -> amdgpu_xcp_0..6 = card1..7, card8 -> xcp_7..13 =
  // card9..15 (profiles/archive/sysfs_access_box.json). Used only for GPUs whose kfd
  // nodes are unreadable; kfd's own render-minor map decides otherwise.
  std::vector<const GpuDevice*> primaries;
  for (auto& p : pci_devs)
    if (p.card >= 0 && p.render_minor >= 0) primaries.push_back(&p);
  std::sort(primaries.begin(), primaries.end(), [](auto* a, auto* b) { return a->card < b->card; });
  auto block_parent = [&](const DrmNodes& d, int* slot) -> const GpuDevice* {
    const GpuDevice* best = nullptr;
    for (auto* p : primaries)
      if (p->card < d.card) best = p;
    if (!best) return nullptr;
    int s = d.card - best->card;
    // card and render minors are allocated together: both offsets must agree
    if (d.render - best->render_minor != s) return nullptr;
    *slot = s;
    return best;
  };
  std::map<std::string, int> block_base;  // parent BDF -> xcp index - slot (constant within a block)
  std::set<std::string> inconsistent, unknown_mode;

  std::vector<std::pair<int, GpuDevice>> xcp_devs;
  const std::string plat_dir = path_join(sysfs_root, "devices/platform");
  for (auto& name : list_dir_prefix(plat_dir, "amdgpu_xcp_")) {
    std::string num = name.substr(std::strlen("amdgpu_xcp_"));
    if (!is_all_digits(num)) continue;
    DrmNodes d = scan_drm(path_join(plat_dir, name));
    if (d.render < 0) continue;
    GpuDevice g;
    g.id = name;
    g.is_partition = true;
    g.xcp_index = static_cast<int>(parse_i64(num, -1));
    g.card = d.card;
    g.render_minor = d.render;
    auto uit = render_uid.find(d.render);
    if (uit != render_uid.end()) {
      // Only render nodes known to kfd are real partitions (amdgpu.go:555-560).
      g.unique_id = uit->second;
      if (auto it = render_node.find(d.render); it != render_node.end()) g.node_id = it->second;
      // inherit partition modes + NUMA from the physical GPU with the same unique_id
      for (auto& p : pci_devs) {
        if (p.unique_id == g.unique_id && !p.compute_partition.empty() && !p.memory_partition.empty()) {
          g.compute_partition = p.compute_partition;
          g.memory_partition = p.memory_partition;
          g.numa_node = p.numa_node;
          g.bdf = p.bdf;
          break;
        }
      }
      if (g.numa_node == -1) continue;
      enrich(&g, topo);
      xcp_devs.emplace_back(g.xcp_index, std::move(g));
      continue;
    }
    // Not a kfd render node: an inactive xcp slot, or a partition of a GPU
    // whose kfd nodes this process cannot read.
    int slot = 0;
    const GpuDevice* parent = d.card >= 0 ? block_parent(d, &slot) : nullptr;
    if (!parent || parent->identity == "kfd") continue;
    auto [bit, fresh] = block_base.emplace(parent->bdf, g.xcp_index - slot);
    if (!fresh && bit->second != g.xcp_index - slot) {
      inconsistent.insert(parent->bdf);
      continue;
    }
    int parts = partitions_for_mode(parent->compute_partition, total_xcc_of(*parent));
    if (parts == 0) {
      unknown_mode.insert(parent->bdf);
      continue;
    }
    if (slot >= parts) continue;  // inactive slot of that GPU's block
    g.bdf = parent->bdf;
    g.unique_id = parent->unique_id;
    g.identity = parent->identity;
    g.compute_partition = parent->compute_partition;
    g.memory_partition = parent->memory_partition;
    g.numa_node = parent->numa_node;
    g.hive_id = parent->hive_id;
    g.pci_device_id = parent->pci_device_id;
    g.domain = parent->domain;
    g.location_id = parent->location_id + slot;  // kfd: partition index in the function bits
    g.gfx_target_version = parent->gfx_target_version;
    g.simd_count = parent->simd_count;
    g.simd_per_cu = parent->simd_per_cu;
    g.num_xcc = parent->num_xcc;
    g.vram_bytes = parent->vram_bytes;
    xcp_devs.emplace_back(g.xcp_index, std::move(g));
  }
  std::sort(xcp_devs.begin(), xcp_devs.end(),
            [](const auto& a, const auto& b) { return a.first < b.first; });
  if (!inconsistent.empty() || !unknown_mode.empty()) {
    std::set<std::string> drop(inconsistent.begin(), inconsistent.end());
    drop.insert(unknown_mode.begin(), unknown_mode.end());
    std::vector<std::pair<int, GpuDevice>> keep;
    for (auto& e : xcp_devs)
      if (!drop.count(e.second.bdf) || e.second.identity == "kfd") keep.push_back(std::move(e));
    xcp_devs = std::move(keep);
    for (auto& b : inconsistent)
      res.warnings.push_back(b + ": kfd nodes unreadable and its amdgpu_xcp_* devices are not one contiguous "
                                 "drm-minor block; its partitions beyond the first are not advertised");
    for (auto& b : unknown_mode)
      res.warnings.push_back(b + ": kfd nodes unreadable and the partition count of its compute mode is "
                                 "unknown; its partitions beyond the first are not advertised");
  }

  res.devices = std::move(pci_devs);
  for (auto& [n, g] : xcp_devs) res.devices.push_back(std::move(g));
  for (auto& g : res.devices) {
    if (g.identity == "sysfs") ++res.recovered_devices;
    if (g.unique_id.empty() && g.node_id < 0) res.unresolved.push_back(g.id);
  }
  if (!res.kfd_unreadable_nodes.empty()) {
    std::string ids;
    for (int n : res.kfd_unreadable_nodes) ids += (ids.empty() ? "" : ",") + std::to_string(n);
    res.warnings.push_back("kfd topology: " + std::to_string(res.kfd_unreadable_nodes.size()) +
                           " node(s) unreadable [" + ids + "] (EPERM: the device cgroup denies those GPUs); " +
                           std::to_string(res.recovered_devices) + " device(s) identified from PCI sysfs instead");
  }
  for (auto& id : res.unresolved)
    res.warnings.push_back(id + ": no kfd node and no sysfs unique_id; physical-GPU identity unknown");
  return res;
}

std::map<std::string, int> partition_config_count(const std::vector<GpuDevice>& devs) {
  std::map<std::string, int> out;
  for (auto& d : devs) {
    auto t = d.partition_type();
    if (!t.empty()) out[t]++;
  }
  return out;
}

bool is_homogeneous(const std::vector<GpuDevice>& devs) { return partition_config_count(devs).size() <= 1; }

static bool first_gpu_has(const std::string& sysfs_root, const char* file) {
  const std::string pci_dir = path_join(sysfs_root, "module/amdgpu/drivers/pci:amdgpu");
  for (auto& bdf : list_dir(pci_dir)) {
    if (!looks_like_bdf(bdf)) continue;
    return path_exists(path_join(path_join(pci_dir, bdf), file));
  }
  return false;
}

bool compute_partition_supported(const std::string& sysfs_root) {
  return first_gpu_has(sysfs_root, "available_compute_partition");
}

bool memory_partition_supported(const std::string& sysfs_root) {
  return first_gpu_has(sysfs_root, "available_memory_partition");
}

FirmwareInfo parse_debugfs_firmware_info(const std::string& path) {
  FirmwareInfo fi;
  auto content = read_file(path);
  if (!content) return fi;
  size_t pos = 0;
  const std::string& s = *content;
  const std::string kFeat = " feature version: ";
  const std::string kFw = ", firmware version: ";
  while (pos < s.size()) {
    size_t eol = s.find('\n', pos);
    if (eol == std::string::npos) eol = s.size();
    std::string line = s.substr(pos, eol - pos);
    pos = eol + 1;
    size_t f = line.find(kFeat);
    size_t w = line.find(kFw);
    if (f == std::string::npos || w == std::string::npos || w < f) continue;
    // name = last word before " feature version"
    size_t ne = f;
    size_t nb = ne;
    while (nb > 0 && (std::isalnum(static_cast<unsigned char>(line[nb - 1])) || line[nb - 1] == '_')) --nb;
    if (nb == ne) continue;
    std::string name = line.substr(nb, ne - nb);
    std::string feat = trim(line.substr(f + kFeat.size(), w - f - kFeat.size()));
    std::string fw = line.substr(w + kFw.size());
    size_t fe = 0;
    if (fw.rfind("0x", 0) != 0 && fw.rfind("0X", 0) != 0) continue;
    fe = 2;
    while (fe < fw.size() && std::isxdigit(static_cast<unsigned char>(fw[fe]))) ++fe;
    if (!is_all_digits(feat) || fe == 2) continue;
    fi.feature[name] = static_cast<uint32_t>(parse_u64(feat, 0));
    fi.firmware[name] = static_cast<uint32_t>(parse_u64(fw.substr(0, fe), 0));
  }
  return fi;
}

std::string topology_signature(const std::string& sysfs_root) {
  std::string sig = read_trimmed(path_join(sysfs_root, "class/kfd/kfd/topology/generation_id")).value_or("-");
  const std::string drv = path_join(sysfs_root, "module/amdgpu/drivers/pci:amdgpu");
  auto bdfs = list_dir(drv);
  std::sort(bdfs.begin(), bdfs.end());
  for (const auto& b : bdfs) {
    if (b.find(':') == std::string::npos) continue;
    sig += "|" + b + "=" + read_trimmed(path_join(drv, b + "/current_compute_partition")).value_or("-") + "," +
           read_trimmed(path_join(drv, b + "/current_memory_partition")).value_or("-");
  }
  return sig;
}

}  // namespace mi355x
