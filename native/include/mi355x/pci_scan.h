// PCI scan for the passthrough modes.
//
// SR-IOV VF mode (reference GetVFMapping, internal/pkg/amdgpu/amdgpu_sriov.go:323-402):
//   AMD (0x1002) PFs bound to the "gim" driver -> virtfn* -> VF BDF -> iommu_group.
// PF passthrough (reference GetPFMapping, internal/pkg/amdgpu/amdgpu_pf.go:244-305):
//   AMD PCI functions bound to "vfio-pci" -> iommu_group.
// One kubelet device per IOMMU group; the group number is the device ID.
// All paths are relative to an injectable sysfs root.
#pragma once

#include <map>
#include <string>
#include <vector>

namespace mi355x {

struct PciFunctionInfo {
  std::string pf;         // parent PF BDF (for PF mode: the function itself)
  std::string vf;         // VF BDF (empty in PF mode)
  std::string device_id;  // contents of <dev>/device, e.g. "0x75a3"
};

// iommu group -> functions in it (ordered by group number, then discovery order)
using IommuMap = std::map<std::string, std::vector<PciFunctionInfo>>;

struct PciScanResult {
  IommuMap groups;
  bool ok = true;
  std::string error;
};

PciScanResult scan_vf_mapping(const std::string& sysfs_root);
PciScanResult scan_pf_mapping(const std::string& sysfs_root);

// gim module version/srcversion (reference GetGIMVersions, amdgpu_sriov.go:404-422):
// version is cut at the first '+'.
struct GimVersions {
  bool ok = false;
  std::string version;
  std::string srcversion;
};
GimVersions read_gim_versions(const std::string& sysfs_root);

}  // namespace mi355x
