// libdrm_amdgpu queries used by the node labeller (family, firmware, marketing
// name) and by hardware tests (device open).
//
// Reference: cgo bindings in internal/pkg/amdgpu/amdgpu.go:21-27,349-404,629-736.
// Differences: libdrm_amdgpu is dlopen()ed, so the plugin and labeller start
// (and degrade to sysfs-only labels) on hosts without it; family IDs newer than
// the system header are defined locally (this image's amdgpu_drm.h
// stops at AMDGPU_FAMILY_YC); the device path is rooted at an injectable /dev.
#pragma once

#include <cstdint>
#include <map>
#include <string>

namespace mi355x {

// AMDGPU_FAMILY_* -> name ("AI", "GC_11_0_0", ...); "" if unknown.
std::string family_id_to_string(uint32_t family_id);

struct DrmGpuInfo {
  bool ok = false;
  std::string error;
  uint32_t drm_major = 0, drm_minor = 0;
  uint32_t family_id = 0;
  uint32_t asic_id = 0;      // PCI device id
  uint32_t chip_rev = 0;
  uint32_t chip_external_rev = 0;
  uint64_t ids_flags = 0;
  std::string family;        // family_id_to_string(family_id)
  std::string marketing_name;
};

struct DrmFirmware {
  bool ok = false;
  std::string error;
  // keys: VCE UVD MC ME PFP CE RLC MEC SMC SDMA0 (the reference set, amdgpu.go:704-733)
  std::map<std::string, uint32_t> feature;
  std::map<std::string, uint32_t> firmware;
};

// True if libdrm_amdgpu could be loaded.
bool drm_available();
// <sysfs_root>/class/drm/<card>/device/vendor == 0x1002 (reference AMDGPU(), amdgpu.go:630-644)
bool drm_is_amd_card(const std::string& sysfs_root, const std::string& card);
// open + amdgpu_device_initialize + deinitialize (reference DevFunctional, amdgpu.go:678-687)
bool drm_dev_functional(const std::string& dev_root, const std::string& sysfs_root, const std::string& card,
                        std::string* error);
DrmGpuInfo drm_query_gpu_info(const std::string& dev_root, const std::string& sysfs_root, const std::string& card);
DrmFirmware drm_query_firmware(const std::string& dev_root, const std::string& sysfs_root, const std::string& card);

}  // namespace mi355x
