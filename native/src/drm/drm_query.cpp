#include "mi355x/drm_query.h"

#include <dlfcn.h>
#include <fcntl.h>
#include <unistd.h>

#include <mutex>

#include "mi355x/constants.h"
#include "mi355x/sysfs.h"

namespace mi355x {

namespace {

// ABI mirror of struct amdgpu_gpu_info (libdrm amdgpu.h). Only the leading
// fields are read; the tail is padded generously because the library
// memcpy()s its own (possibly newer, larger) definition into it.
struct GpuInfoAbi {
  uint32_t asic_id;
  uint32_t chip_rev;
  uint32_t chip_external_rev;
  uint32_t family_id;
  uint64_t ids_flags;
  uint64_t max_engine_clk;
  uint64_t max_memory_clk;
  unsigned char tail[8192];
};

// AMDGPU_FAMILY_* (include/uapi/drm/amdgpu_drm.h in the kernel tree). The
// system header here predates GC_11+, so the table is local.
struct FamilyName {
  uint32_t id;
  const char* name;
};
constexpr FamilyName kFamilies[] = {
    {110, "SI"},        {120, "CI"},        {125, "KV"},        {130, "VI"},
    {135, "CZ"},        {141, "AI"},        {142, "RV"},        {143, "NV"},
    {144, "VGH"},       {145, "GC_11_0_0"}, {146, "YC"},        {148, "GC_11_0_1"},
    {149, "GC_10_3_6"}, {150, "GC_11_5_0"}, {151, "GC_10_3_7"}, {152, "GC_12_0_0"},
};

// AMDGPU_INFO_FW_* selectors, in the reference's label order (amdgpu.go:704-733).
struct FwSel {
  const char* name;
  unsigned type;
};
constexpr FwSel kFirmware[] = {
    {"VCE", 0x01}, {"UVD", 0x02}, {"MC", 0x03},  {"ME", 0x04},  {"PFP", 0x05},
    {"CE", 0x06},  {"RLC", 0x07}, {"MEC", 0x08}, {"SMC", 0x0a}, {"SDMA0", 0x0b},
};

using amdgpu_device_handle = void*;
using fn_init_t = int (*)(int, uint32_t*, uint32_t*, amdgpu_device_handle*);
using fn_deinit_t = int (*)(amdgpu_device_handle);
using fn_gpu_info_t = int (*)(amdgpu_device_handle, GpuInfoAbi*);
using fn_fw_t = int (*)(amdgpu_device_handle, unsigned, unsigned, unsigned, uint32_t*, uint32_t*);
using fn_name_t = const char* (*)(amdgpu_device_handle);

struct Lib {
  void* h = nullptr;
  fn_init_t init = nullptr;
  fn_deinit_t deinit = nullptr;
  fn_gpu_info_t gpu_info = nullptr;
  fn_fw_t fw = nullptr;
  fn_name_t name = nullptr;
};

const Lib& lib() {
  static Lib l;
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* so : {"libdrm_amdgpu.so.1", "libdrm_amdgpu.so"}) {
      l.h = ::dlopen(so, RTLD_NOW | RTLD_LOCAL);
      if (l.h) break;
    }
    if (!l.h) return;
    l.init = reinterpret_cast<fn_init_t>(::dlsym(l.h, "amdgpu_device_initialize"));
    l.deinit = reinterpret_cast<fn_deinit_t>(::dlsym(l.h, "amdgpu_device_deinitialize"));
    l.gpu_info = reinterpret_cast<fn_gpu_info_t>(::dlsym(l.h, "amdgpu_query_gpu_info"));
    l.fw = reinterpret_cast<fn_fw_t>(::dlsym(l.h, "amdgpu_query_firmware_version"));
    l.name = reinterpret_cast<fn_name_t>(::dlsym(l.h, "amdgpu_get_marketing_name"));
  });
  return l;
}

// RAII open of /dev/dri/<card> + amdgpu_device_initialize.
class DrmDevice {
 public:
  DrmDevice(const std::string& dev_root, const std::string& sysfs_root, const std::string& card) {
    const Lib& L = lib();
    if (!L.init || !L.deinit) {
      error_ = "libdrm_amdgpu unavailable";
      return;
    }
    if (!drm_is_amd_card(sysfs_root, card)) {
      error_ = card + " is not an AMD GPU";
      return;
    }
    std::string path = path_join(path_join(dev_root, "dri"), card);
    fd_ = ::open(path.c_str(), O_RDWR | O_CLOEXEC);
    if (fd_ < 0) {
      error_ = "Fail to open " + path;
      return;
    }
    int rc = L.init(fd_, &major_, &minor_, &handle_);
    if (rc < 0) {
      error_ = "Fail to initialize " + path + ": rc=" + std::to_string(rc);
      handle_ = nullptr;
    }
  }
  ~DrmDevice() {
    if (handle_) lib().deinit(handle_);
    if (fd_ >= 0) ::close(fd_);  // libdrm dup()s the fd it keeps
  }
  bool ok() const { return handle_ != nullptr; }
  const std::string& error() const { return error_; }
  amdgpu_device_handle handle() const { return handle_; }
  uint32_t major() const { return major_; }
  uint32_t minor() const { return minor_; }

 private:
  int fd_ = -1;
  amdgpu_device_handle handle_ = nullptr;
  uint32_t major_ = 0, minor_ = 0;
  std::string error_;
};

}  // namespace

std::string family_id_to_string(uint32_t family_id) {
  for (auto& f : kFamilies)
    if (f.id == family_id) return f.name;
  return "";
}

bool drm_available() { return lib().init != nullptr; }

bool drm_is_amd_card(const std::string& sysfs_root, const std::string& card) {
  auto v = read_trimmed(path_join(sysfs_root, "class/drm/" + card + "/device/vendor"));
  return v && to_lower(*v) == kAmdVendorId;
}

bool drm_dev_functional(const std::string& dev_root, const std::string& sysfs_root, const std::string& card,
                        std::string* error) {
  DrmDevice d(dev_root, sysfs_root, card);
  if (!d.ok() && error) *error = d.error();
  return d.ok();
}

DrmGpuInfo drm_query_gpu_info(const std::string& dev_root, const std::string& sysfs_root, const std::string& card) {
  DrmGpuInfo out;
  DrmDevice d(dev_root, sysfs_root, card);
  if (!d.ok()) {
    out.error = d.error();
    return out;
  }
  out.drm_major = d.major();
  out.drm_minor = d.minor();
  const Lib& L = lib();
  if (!L.gpu_info) {
    out.error = "amdgpu_query_gpu_info unavailable";
    return out;
  }
  GpuInfoAbi info{};
  int rc = L.gpu_info(d.handle(), &info);
  if (rc < 0) {
    out.error = "Fail to get FamilyID " + card + ": " + std::to_string(rc);
    return out;
  }
  out.family_id = info.family_id;
  out.asic_id = info.asic_id;
  out.chip_rev = info.chip_rev;
  out.chip_external_rev = info.chip_external_rev;
  out.ids_flags = info.ids_flags;
  out.family = family_id_to_string(info.family_id);
  if (L.name) {
    const char* n = L.name(d.handle());
    if (n) out.marketing_name = n;
  }
  if (out.family.empty()) {
    out.error = "Unknown Family ID: " + std::to_string(info.family_id);
    return out;
  }
  out.ok = true;
  return out;
}

DrmFirmware drm_query_firmware(const std::string& dev_root, const std::string& sysfs_root, const std::string& card) {
  DrmFirmware out;
  DrmDevice d(dev_root, sysfs_root, card);
  if (!d.ok()) {
    out.error = d.error();
    return out;
  }
  const Lib& L = lib();
  if (!L.fw) {
    out.error = "amdgpu_query_firmware_version unavailable";
    return out;
  }
  for (auto& f : kFirmware) {
    uint32_t ver = 0, feat = 0;
    // like the reference, a failing query reports 0/0 rather than dropping the key
    L.fw(d.handle(), f.type, 0, 0, &ver, &feat);
    out.feature[f.name] = feat;
    out.firmware[f.name] = ver;
  }
  out.ok = true;
  return out;
}

}  // namespace mi355x
