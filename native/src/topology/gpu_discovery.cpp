#include "mi355x/gpu_discovery.h"

#include <algorithm>
#include <cctype>
#include <cstring>

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
}

}  // namespace

DiscoveryResult discover_gpus(const std::string& sysfs_root) {
  return discover_gpus(sysfs_root, KfdTopology::load_sysfs(sysfs_root));
}

DiscoveryResult discover_gpus(const std::string& sysfs_root, const KfdTopology& topo) {
  DiscoveryResult res;
  res.kfd_present = path_exists(path_join(sysfs_root, "class/kfd"));
  res.driver_loaded = path_exists(path_join(sysfs_root, "module/amdgpu/drivers"));
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
    pci_devs.push_back(std::move(g));
  }

  std::vector<std::pair<int, GpuDevice>> xcp_devs;
  const std::string plat_dir = path_join(sysfs_root, "devices/platform");
  for (auto& name : list_dir_prefix(plat_dir, "amdgpu_xcp_")) {
    std::string num = name.substr(std::strlen("amdgpu_xcp_"));
    if (!is_all_digits(num)) continue;
    DrmNodes d = scan_drm(path_join(plat_dir, name));
    // Only render nodes known to kfd are real partitions (amdgpu.go:555-560).
    auto uit = render_uid.find(d.render);
    if (d.render < 0 || uit == render_uid.end()) continue;
    GpuDevice g;
    g.id = name;
    g.is_partition = true;
    g.xcp_index = static_cast<int>(parse_i64(num, -1));
    g.card = d.card;
    g.render_minor = d.render;
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
  }
  std::sort(xcp_devs.begin(), xcp_devs.end(),
            [](const auto& a, const auto& b) { return a.first < b.first; });

  res.devices = std::move(pci_devs);
  for (auto& [n, g] : xcp_devs) res.devices.push_back(std::move(g));
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

}  // namespace mi355x
