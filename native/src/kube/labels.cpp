// Label generation (labels.h). Reference: cmd/k8s-node-labeller/main.go:85-505.
#include "labels.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <optional>
#include <set>

#include "mi355x/drm_query.h"
#include "mi355x/glog.h"
#include "mi355x/gpu_discovery.h"
#include "mi355x/kfd_topology.h"
#include "mi355x/pci_scan.h"
#include "mi355x/smi_query.h"
#include "mi355x/sysfs.h"

namespace mi355x::labeller {

namespace {

const char* kAmd = "amd.com";
const char* kBeta = "beta.amd.com";

bool on(const LabelOptions& f, const std::string& kind) {
  auto it = f.enabled.find(kind);
  return it != f.enabled.end() && it->second;
}

void create_labels(const std::string& kind, const std::map<std::string, int>& entries, Labels* out) {
  for (const bool experimental : {true, false}) {
    const std::string p = prefix_of(kind, experimental);
    for (const auto& [k, v] : entries) {
      (*out)[p + "." + k] = std::to_string(v);
      if (entries.size() == 1) (*out)[p] = k;
    }
  }
}

bool alnum(char c) { return std::isalnum(static_cast<unsigned char>(c)) != 0; }

std::string gfx_name(int v) {
  char b[32];
  std::snprintf(b, sizeof(b), "gfx%d%x%x", v / 10000, (v / 100) % 100, v % 100);
  return b;
}

// ---- container-mode generators (main.go:123-385) --------------------------------
struct Ctx {
  std::string sysfs, dev;
  KfdTopology topo;
  std::vector<GpuDevice> gpus;
  std::map<std::string, DrmGpuInfo> drm_info;
  std::map<std::string, DrmFirmware> drm_fw;

  std::optional<std::string> drm_node(const GpuDevice& g) const {
    if (g.card >= 0 && path_exists(path_join(dev, "dri/card" + std::to_string(g.card))))
      return "card" + std::to_string(g.card);
    if (g.render_minor >= 0 && path_exists(path_join(dev, "dri/renderD" + std::to_string(g.render_minor))))
      return "renderD" + std::to_string(g.render_minor);
    if (g.card >= 0) return "card" + std::to_string(g.card);
    return std::nullopt;
  }
  std::optional<std::string> card_attr(const GpuDevice& g, const std::string& attr) const {
    return read_trimmed(path_join(sysfs, "class/drm/card" + std::to_string(g.card) + "/device/" + attr));
  }
  const KfdNode* kfd_node(const GpuDevice& g) const { return g.node_id < 0 ? nullptr : topo.node(g.node_id); }
};

void gen_firmware(Ctx& c, Labels* out) {
  std::map<std::string, int> counts;
  for (const auto& g : c.gpus) {
    const auto node = c.drm_node(g);
    if (!node) {
      MI_LOG(kError, "Fail to get firmware versions: no drm node");
      continue;
    }
    auto it = c.drm_fw.find(*node);
    if (it == c.drm_fw.end()) it = c.drm_fw.emplace(*node, drm_query_firmware(c.dev, c.sysfs, *node)).first;
    if (!it->second.ok) {
      MI_LOG(kError, "Fail to get firmware versions: %s", it->second.error.c_str());
      continue;
    }
    for (const auto& [name, ver] : it->second.feature) counts[name + ".feat." + std::to_string(ver)]++;
    for (const auto& [name, ver] : it->second.firmware) counts[name + ".fw." + std::to_string(ver)]++;
  }
  const std::string p = prefix_of("firmware", true);
  for (const auto& [k, v] : counts) (*out)[p + "." + k] = std::to_string(v);
}

void gen_family(Ctx& c, Labels* out) {
  std::map<std::string, int> counts;
  for (const auto& g : c.gpus) {
    const auto node = c.drm_node(g);
    if (!node) {
      MI_LOG(kError, "Fail to get card family name: no drm node");
      continue;
    }
    auto it = c.drm_info.find(*node);
    if (it == c.drm_info.end()) it = c.drm_info.emplace(*node, drm_query_gpu_info(c.dev, c.sysfs, *node)).first;
    if (!it->second.ok) {
      MI_LOG(kError, "Fail to get card family name: %s", it->second.error.c_str());
      continue;
    }
    counts[it->second.family]++;
  }
  create_labels("family", counts, out);
}

std::string module_attr(const Ctx& c, const std::string& attr) {
  for (const auto& g : c.gpus)
    if (auto v = c.card_attr(g, "driver/module/" + attr)) return *v;
  return "";
}

void gen_driver_version(Ctx& c, Labels* out) {
  std::string v = module_attr(c, "version");
  if (v.empty()) {
    // built-in amdgpu / no module version string: /sys/module/amdgpu/version, then amd-smi
    if (auto m = read_trimmed(path_join(c.sysfs, "module/amdgpu/version")); m && !m->empty()) {
      v = *m;
    } else if (!c.gpus.empty() && smi_available()) {
      const SmiSnapshot s = smi_snapshot();
      std::set<std::string> mine;
      for (const auto& g : c.gpus) mine.insert(to_lower(g.bdf));
      if (s.ok)
        for (const auto& g : s.gpus)
          if (mine.count(to_lower(g.bdf)) && !g.driver_version.empty()) {
            v = driver_version_value(g.driver_version);
            break;
          }
    }
  }
  (*out)[prefix_of("driver-version", false)] = v;
}

void gen_driver_src_version(Ctx& c, Labels* out) {
  (*out)[prefix_of("driver-src-version", false)] = module_attr(c, "srcversion");
}

void gen_device_id(Ctx& c, Labels* out) {
  std::map<std::string, int> counts;
  for (const auto& g : c.gpus) {
    auto v = c.card_attr(g, "device");
    if (!v) continue;
    std::string s = *v;
    if (s.compare(0, 2, "0x") == 0) s = s.substr(2);
    counts[s]++;
  }
  create_labels("device-id", counts, out);
}

void gen_product_name(Ctx& c, Labels* out) {
  std::map<std::string, int> counts;
  for (const auto& g : c.gpus) {
    auto v = c.card_attr(g, "product_name");
    if (!v) continue;
    std::string s;
    for (const char ch : trim(*v)) {
      if (ch == ' ') s.push_back('_');
      else if (ch != '(' && ch != ')') s.push_back(ch);
    }
    if (!s.empty()) counts[s]++;
  }
  create_labels("product-name", counts, out);
}

// A GPU whose kfd node this process may not read (a device cgroup denies it)
// is still counted in vram / simd-count / cu-count from what discovery
// recovered from PCI sysfs: its own mem_info_vram_total, and the SIMD shape of
// a readable GPU of the same part and partition mode. The counts then agree
// with device-id. The reference's labeller runs privileged and reads every
// node (k8s-ds-amdgpu-labeller.yaml:66-67); unprivileged it would drop such
// GPUs from these counts (cmd/k8s-node-labeller/main.go:237-277).
bool recovered(const GpuDevice& g) { return g.identity == "sysfs"; }

void gen_vram(Ctx& c, Labels* out) {
  std::map<std::string, int> counts;
  for (const auto& g : c.gpus) {
    const KfdNode* n = c.kfd_node(g);
    uint64_t size = 0;
    if (n && !n->mem_banks.empty()) size = n->mem_banks[0].size_in_bytes;
    else if (!n && recovered(g) && g.vram_bytes > 0) size = g.vram_bytes;
    else continue;
    const uint64_t mib = size / (1024 * 1024);
    // Go math.Round: half away from zero
    counts[std::to_string(static_cast<long long>(std::floor(static_cast<double>(mib) / 1024.0 + 0.5))) + "G"]++;
  }
  create_labels("vram", counts, out);
}

void gen_simd_count(Ctx& c, Labels* out) {
  std::map<std::string, int> counts;
  for (const auto& g : c.gpus) {
    const KfdNode* n = c.kfd_node(g);
    if (n && n->props.count("simd_count")) counts[std::to_string(n->simd_count())]++;
    else if (!n && recovered(g) && g.simd_count > 0) counts[std::to_string(g.simd_count)]++;
  }
  create_labels("simd-count", counts, out);
}

void gen_cu_count(Ctx& c, Labels* out) {
  std::map<std::string, int> counts;
  for (const auto& g : c.gpus) {
    const KfdNode* n = c.kfd_node(g);
    if (n && n->simd_per_cu() != 0) counts[std::to_string(n->simd_count() / n->simd_per_cu())]++;
    else if (!n && recovered(g) && g.cu_count() > 0) counts[std::to_string(g.cu_count())]++;
  }
  create_labels("cu-count", counts, out);
}

void gen_compute_memory_partition(Ctx& c, Labels* out) {
  if (!is_homogeneous(c.gpus)) return;
  for (const auto& [t, n] : partition_config_count(c.gpus))
    if (n > 0) {
      (*out)[prefix_of("compute-memory-partition", false)] = t;
      return;
    }
}

void gen_compute_partitioning_supported(Ctx& c, Labels* out) {
  (*out)[prefix_of("compute-partitioning-supported", false)] =
      compute_partition_supported(c.sysfs) ? "true" : "false";
}

void gen_memory_partitioning_supported(Ctx& c, Labels* out) {
  (*out)[prefix_of("memory-partitioning-supported", false)] = memory_partition_supported(c.sysfs) ? "true" : "false";
}

void gen_mode(Ctx&, Labels* out) {
  (*out)[prefix_of("mode", true)] = "container";
  (*out)[prefix_of("mode", false)] = "container";
}

void gen_gfx_target(Ctx& c, Labels* out) {
  std::map<std::string, int> counts;
  for (const auto& g : c.gpus)
    if (g.gfx_target_version > 0) counts[gfx_name(g.gfx_target_version)]++;
  create_labels("gfx-target", counts, out);
}

void gen_xgmi_hive_count(Ctx& c, Labels* out) {
  if (c.gpus.empty()) return;
  std::set<uint64_t> hives;
  for (const auto& g : c.gpus)
    if (g.hive_id) hives.insert(g.hive_id);
  (*out)[prefix_of("xgmi-hive-count", false)] = std::to_string(hives.size());
}

void gen_xgmi_links_down(Ctx& c, Labels* out) {
  if (c.gpus.empty()) return;
  const SmiXgmiSnapshot s = smi_xgmi_links();
  if (!s.ok) return;
  std::set<std::string> mine;
  for (const auto& g : c.gpus) mine.insert(to_lower(g.bdf));
  int seen = 0, down = 0;
  for (const auto& g : s.gpus) {
    if (!mine.count(to_lower(g.bdf)) || !g.status_ok) continue;
    ++seen;
    for (const int st : g.status) down += st == 0;
  }
  if (seen) (*out)[prefix_of("xgmi-links-down", false)] = std::to_string(down);
}

using Gen = void (*)(Ctx&, Labels*);
const std::vector<std::pair<std::string, Gen>> kGenerators = {
    {"firmware", gen_firmware},
    {"family", gen_family},
    {"driver-version", gen_driver_version},
    {"driver-src-version", gen_driver_src_version},
    {"device-id", gen_device_id},
    {"product-name", gen_product_name},
    {"vram", gen_vram},
    {"simd-count", gen_simd_count},
    {"cu-count", gen_cu_count},
    {"compute-memory-partition", gen_compute_memory_partition},
    {"compute-partitioning-supported", gen_compute_partitioning_supported},
    {"memory-partitioning-supported", gen_memory_partitioning_supported},
    {"mode", gen_mode},
    {"gfx-target", gen_gfx_target},
    {"xgmi-hive-count", gen_xgmi_hive_count},
    {"xgmi-links-down", gen_xgmi_links_down},
};

Labels container_labels(const LabelOptions& f) {
  Labels out;
  Ctx c;
  c.sysfs = f.sysfs_root;
  c.dev = f.dev_root;
  if (is_dir(path_join(f.sysfs_root, "module/amdgpu/drivers"))) {
    c.topo = KfdTopology::load_sysfs(f.sysfs_root);
    c.gpus = discover_gpus(f.sysfs_root, c.topo).devices;
  }
  if (c.gpus.empty()) {
    MI_LOG(kInfo, "No AMD GPUs found, skipping label generation");
    return out;
  }
  for (const auto& [name, gen] : kGenerators)
    if (on(f, name)) gen(c, &out);
  return out;
}

void count_functions(const PciScanResult& r, Labels* out) {
  std::map<std::string, int> counts;
  for (const auto& [group, fns] : r.groups)
    for (const auto& fn : fns) counts[fn.device_id]++;
  create_labels("device-id", counts, out);
}

// VF passthrough (main.go:438-475)
Labels vf_labels(const LabelOptions& f) {
  Labels out;
  const PciScanResult r = scan_vf_mapping(f.sysfs_root);
  if (!r.ok || r.groups.empty()) return out;
  const GimVersions gim = read_gim_versions(f.sysfs_root);
  if (!gim.ok) return out;
  if (on(f, "driver-version")) out[prefix_of("driver-version", false)] = gim.version;
  if (on(f, "driver-src-version")) out[prefix_of("driver-src-version", false)] = gim.srcversion;
  if (on(f, "mode")) {
    out[prefix_of("mode", false)] = "vf-passthrough";
    out[prefix_of("mode", true)] = "vf-passthrough";
  }
  if (on(f, "device-id")) count_functions(r, &out);
  return out;
}

// PF passthrough (main.go:477-505)
Labels pf_labels(const LabelOptions& f) {
  Labels out;
  const PciScanResult r = scan_pf_mapping(f.sysfs_root);
  if (!r.ok || r.groups.empty()) return out;
  if (on(f, "mode")) out[prefix_of("mode", false)] = "pf-passthrough";
  if (on(f, "device-id")) count_functions(r, &out);
  return out;
}

}  // namespace

// ---- label helpers (main.go:85-116) ----------------------------------------------
std::string prefix_of(const std::string& kind, bool experimental) {
  return std::string(experimental ? kBeta : kAmd) + "/gpu." + kind;
}

// apimachinery IsValidLabelValue: <= 63 chars, alphanumeric at both ends, [-_.A-Za-z0-9] between
bool valid_label_value(const std::string& v) {
  if (v.size() > 63) return false;
  if (v.empty()) return true;
  if (!alnum(v.front()) || !alnum(v.back())) return false;
  for (const char c : v)
    if (!alnum(c) && c != '-' && c != '_' && c != '.') return false;
  return true;
}

std::string sanitize_label_value(const std::string& v) {
  if (valid_label_value(v)) return v;
  std::string out;
  for (const char c : v) out.push_back(alnum(c) || c == '-' || c == '_' || c == '.' ? c : '_');
  if (out.size() > 63) out.resize(63);
  size_t b = 0, e = out.size();
  while (b < e && !alnum(out[b])) ++b;
  while (e > b && !alnum(out[e - 1])) --e;
  return out.substr(b, e - b);
}

// amd-smi reports an in-tree amdgpu's version as the kernel banner with its spaces
// removed ("Linuxversion6.18.54-ant.1(nixbld@...)"): the kernel release is the version
std::string driver_version_value(const std::string& raw) {
  size_t i = 0;
  auto skip_ws = [&] {
    while (i < raw.size() && std::isspace(static_cast<unsigned char>(raw[i]))) ++i;
  };
  if (raw.compare(0, 5, "Linux") != 0) return raw;
  i = 5;
  skip_ws();
  if (raw.compare(i, 7, "version") != 0) return raw;
  i += 7;
  skip_ws();
  if (i >= raw.size() || !std::isdigit(static_cast<unsigned char>(raw[i]))) return raw;
  size_t e = i;
  while (e < raw.size() && !std::isspace(static_cast<unsigned char>(raw[e])) && raw[e] != '(') ++e;
  return raw.substr(i, e - i);
}

// generateLabels (main.go:389-408): explicit mode, else container -> VF -> PF
Labels generate_labels(const LabelOptions& f) {
  Labels out;
  if (f.driver_type == "container" || f.driver_type.empty()) out = container_labels(f);
  if (f.driver_type == "vf-passthrough" || (f.driver_type.empty() && out.empty())) out = vf_labels(f);
  if (f.driver_type == "pf-passthrough" || (f.driver_type.empty() && out.empty())) out = pf_labels(f);
  return clean_labels(out);
}

// constants.go:21 order, then the opt-in additions
const std::vector<std::string>& label_kinds() {
  static const std::vector<std::string> kinds = {
      "mode", "firmware", "family", "driver-version", "driver-src-version", "device-id", "product-name", "vram",
      "simd-count", "cu-count", "compute-memory-partition", "compute-partitioning-supported",
      "memory-partitioning-supported", "gfx-target", "xgmi-hive-count", "xgmi-links-down"};
  return kinds;
}

bool valid_label_key(const std::string& k) {
  const size_t slash = k.find('/');
  const std::string name = slash == std::string::npos ? k : k.substr(slash + 1);
  if (name.empty() || !valid_label_value(name)) return false;
  if (slash == std::string::npos) return true;
  const std::string prefix = k.substr(0, slash);
  // DNS-1123 subdomain: <= 253, dot-separated lower-case alphanumeric labels with inner '-'
  if (prefix.empty() || prefix.size() > 253) return false;
  size_t a = 0;
  while (a <= prefix.size()) {
    size_t b = prefix.find('.', a);
    if (b == std::string::npos) b = prefix.size();
    const std::string part = prefix.substr(a, b - a);
    if (part.empty() || part.size() > 63 || part.front() == '-' || part.back() == '-') return false;
    for (const char c : part)
      if (!((c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '-')) return false;
    a = b + 1;
  }
  return true;
}

Labels clean_labels(const Labels& in) {
  Labels out;
  for (const auto& [k, v] : in) {
    if (!valid_label_key(k)) {
      MI_LOG(kWarning, "dropping label %s: not a valid Kubernetes label key", k.c_str());
      continue;
    }
    out[k] = sanitize_label_value(v);
  }
  return out;
}

}  // namespace mi355x::labeller
