#include "mi355x/pci_scan.h"

#include <algorithm>

#include "mi355x/constants.h"
#include "mi355x/sysfs.h"

namespace mi355x {

namespace {

bool numeric_less(const std::string& a, const std::string& b) {
  if (is_all_digits(a) && is_all_digits(b)) return parse_i64(a, 0) < parse_i64(b, 0);
  return a < b;
}

// Bound driver name of a PCI function, or "" if unbound.
std::string bound_driver(const std::string& dev_path) {
  auto l = read_link(path_join(dev_path, "driver"));
  return l ? basename(*l) : std::string();
}

bool is_amd(const std::string& dev_path) {
  auto v = read_trimmed(path_join(dev_path, "vendor"));
  return v && to_lower(*v) == kAmdVendorId;
}

}  // namespace

PciScanResult scan_vf_mapping(const std::string& sysfs_root) {
  PciScanResult r;
  const std::string devs = path_join(sysfs_root, "bus/pci/devices");
  if (!is_dir(devs)) {
    r.ok = false;
    r.error = "error reading " + devs;
    return r;
  }
  for (auto& pf : list_dir(devs)) {
    std::string pf_path = path_join(devs, pf);
    if (!is_amd(pf_path) || bound_driver(pf_path) != kGimDriverName) continue;
    auto vfs = list_dir_prefix(pf_path, "virtfn");
    std::sort(vfs.begin(), vfs.end(), [](const std::string& a, const std::string& b) {
      return numeric_less(a.substr(6), b.substr(6));
    });
    for (auto& vfn : vfs) {
      auto target = read_link(path_join(pf_path, vfn));
      if (!target) continue;
      std::string vf = basename(*target);
      std::string vf_path = path_join(devs, vf);
      auto grp = read_link(path_join(vf_path, "iommu_group"));
      if (!grp) continue;
      auto dev_id = read_trimmed(path_join(vf_path, "device"));
      if (!dev_id) continue;
      r.groups[basename(*grp)].push_back(PciFunctionInfo{pf, vf, *dev_id});
    }
  }
  return r;
}

PciScanResult scan_pf_mapping(const std::string& sysfs_root) {
  PciScanResult r;
  const std::string devs = path_join(sysfs_root, "bus/pci/devices");
  if (!is_dir(devs)) {
    r.ok = false;
    r.error = "error reading " + devs;
    return r;
  }
  for (auto& pf : list_dir(devs)) {
    std::string pf_path = path_join(devs, pf);
    if (!is_amd(pf_path) || bound_driver(pf_path) != kVfioDriverName) continue;
    auto grp = read_link(path_join(pf_path, "iommu_group"));
    if (!grp) continue;
    auto dev_id = read_trimmed(path_join(pf_path, "device"));
    if (!dev_id) continue;
    r.groups[basename(*grp)].push_back(PciFunctionInfo{pf, "", *dev_id});
  }
  return r;
}

GimVersions read_gim_versions(const std::string& sysfs_root) {
  GimVersions g;
  auto v = read_trimmed(path_join(sysfs_root, "module/gim/version"));
  auto s = read_trimmed(path_join(sysfs_root, "module/gim/srcversion"));
  if (!v || !s) return g;
  g.version = v->substr(0, v->find('+'));
  g.srcversion = *s;
  g.ok = true;
  return g;
}

}  // namespace mi355x
