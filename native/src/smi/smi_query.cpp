#include "mi355x/smi_query.h"

#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <mutex>

#if __has_include(<amd_smi/amdsmi.h>)
#include <amd_smi/amdsmi.h>
#define MI355X_HAVE_AMDSMI_HEADER 1
#else
#define MI355X_HAVE_AMDSMI_HEADER 0
#endif

namespace mi355x {

#if MI355X_HAVE_AMDSMI_HEADER

namespace {

struct SmiLib {
  void* h = nullptr;
  decltype(&amdsmi_init) init = nullptr;
  decltype(&amdsmi_shut_down) shut_down = nullptr;
  decltype(&amdsmi_get_socket_handles) sockets = nullptr;
  decltype(&amdsmi_get_processor_handles) processors = nullptr;
  decltype(&amdsmi_get_gpu_device_bdf) bdf = nullptr;
  decltype(&amdsmi_get_gpu_device_uuid) uuid = nullptr;
  decltype(&amdsmi_get_gpu_asic_info) asic = nullptr;
  decltype(&amdsmi_get_gpu_kfd_info) kfd = nullptr;
  decltype(&amdsmi_get_xgmi_info) xgmi = nullptr;
  decltype(&amdsmi_get_gpu_compute_partition) cpart = nullptr;
  decltype(&amdsmi_get_gpu_memory_partition) mpart = nullptr;
  decltype(&amdsmi_get_gpu_vram_info) vram = nullptr;
  decltype(&amdsmi_get_gpu_total_ecc_count) ecc = nullptr;
  decltype(&amdsmi_get_gpu_enumeration_info) enumeration = nullptr;
};

template <typename T>
void bind(void* h, const char* name, T* out) {
  *out = reinterpret_cast<T>(::dlsym(h, name));
}

const SmiLib& smi() {
  static SmiLib l;
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* so : {"libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so"}) {
      l.h = ::dlopen(so, RTLD_NOW | RTLD_LOCAL);
      if (l.h) break;
    }
    if (!l.h) return;
    bind(l.h, "amdsmi_init", &l.init);
    bind(l.h, "amdsmi_shut_down", &l.shut_down);
    bind(l.h, "amdsmi_get_socket_handles", &l.sockets);
    bind(l.h, "amdsmi_get_processor_handles", &l.processors);
    bind(l.h, "amdsmi_get_gpu_device_bdf", &l.bdf);
    bind(l.h, "amdsmi_get_gpu_device_uuid", &l.uuid);
    bind(l.h, "amdsmi_get_gpu_asic_info", &l.asic);
    bind(l.h, "amdsmi_get_gpu_kfd_info", &l.kfd);
    bind(l.h, "amdsmi_get_xgmi_info", &l.xgmi);
    bind(l.h, "amdsmi_get_gpu_compute_partition", &l.cpart);
    bind(l.h, "amdsmi_get_gpu_memory_partition", &l.mpart);
    bind(l.h, "amdsmi_get_gpu_vram_info", &l.vram);
    bind(l.h, "amdsmi_get_gpu_total_ecc_count", &l.ecc);
    bind(l.h, "amdsmi_get_gpu_enumeration_info", &l.enumeration);
  });
  return l;
}

std::string lower(const char* s) {
  std::string o(s);
  for (auto& c : o) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return o;
}

}  // namespace

bool smi_available() {
  const auto& L = smi();
  return L.init && L.sockets && L.processors;
}

SmiSnapshot smi_snapshot() {
  SmiSnapshot snap;
  const auto& L = smi();
  if (!smi_available()) {
    snap.error = "libamd_smi unavailable";
    return snap;
  }
  if (L.init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) {
    snap.error = "amdsmi_init failed";
    return snap;
  }
  uint32_t nsock = 0;
  if (L.sockets(&nsock, nullptr) == AMDSMI_STATUS_SUCCESS && nsock > 0) {
    std::vector<amdsmi_socket_handle> socks(nsock);
    L.sockets(&nsock, socks.data());
    for (uint32_t s = 0; s < nsock; ++s) {
      uint32_t nproc = 0;
      if (L.processors(socks[s], &nproc, nullptr) != AMDSMI_STATUS_SUCCESS || nproc == 0) continue;
      std::vector<amdsmi_processor_handle> procs(nproc);
      L.processors(socks[s], &nproc, procs.data());
      for (uint32_t p = 0; p < nproc; ++p) {
        SmiGpu g;
        auto h = procs[p];
        amdsmi_bdf_t bdf{};
        if (L.bdf && L.bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) {
          char buf[64];
          std::snprintf(buf, sizeof(buf), "%04llx:%02llx:%02llx.%llx",
                        static_cast<unsigned long long>(bdf.domain_number),
                        static_cast<unsigned long long>(bdf.bus_number),
                        static_cast<unsigned long long>(bdf.device_number),
                        static_cast<unsigned long long>(bdf.function_number));
          g.bdf = buf;
        }
        if (L.uuid) {
          char ubuf[AMDSMI_MAX_STRING_LENGTH] = {0};
          unsigned int len = sizeof(ubuf);
          if (L.uuid(h, &len, ubuf) == AMDSMI_STATUS_SUCCESS) g.uuid = ubuf;
        }
        amdsmi_asic_info_t asic{};
        if (L.asic && L.asic(h, &asic) == AMDSMI_STATUS_SUCCESS) {
          g.market_name = asic.market_name;
          g.device_id = asic.device_id;
          g.target_graphics_version = asic.target_graphics_version;
          g.num_compute_units = asic.num_of_compute_units;
        }
        amdsmi_kfd_info_t kfd{};
        if (L.kfd && L.kfd(h, &kfd) == AMDSMI_STATUS_SUCCESS) {
          g.kfd_id = kfd.kfd_id;
          g.kfd_node_id = kfd.node_id == 0xFFFFFFFFu ? -1 : static_cast<int>(kfd.node_id);
          g.partition_id = kfd.current_partition_id == 0xFFFFFFFFu ? -1 : static_cast<int>(kfd.current_partition_id);
        }
        amdsmi_xgmi_info_t x{};
        if (L.xgmi && L.xgmi(h, &x) == AMDSMI_STATUS_SUCCESS) g.xgmi_hive_id = x.xgmi_hive_id;
        char part[AMDSMI_MAX_STRING_LENGTH] = {0};
        if (L.cpart && L.cpart(h, part, sizeof(part)) == AMDSMI_STATUS_SUCCESS) g.compute_partition = lower(part);
        std::memset(part, 0, sizeof(part));
        if (L.mpart && L.mpart(h, part, sizeof(part)) == AMDSMI_STATUS_SUCCESS) g.memory_partition = lower(part);
        amdsmi_vram_info_t v{};
        if (L.vram && L.vram(h, &v) == AMDSMI_STATUS_SUCCESS) g.vram_mb = v.vram_size;
        amdsmi_error_count_t ec{};
        if (L.ecc && L.ecc(h, &ec) == AMDSMI_STATUS_SUCCESS) {
          g.ecc_ok = true;
          g.ecc_correctable = ec.correctable_count;
          g.ecc_uncorrectable = ec.uncorrectable_count;
        }
        amdsmi_enumeration_info_t en{};
        if (L.enumeration && L.enumeration(h, &en) == AMDSMI_STATUS_SUCCESS) {
          g.drm_render = static_cast<int>(en.drm_render);
          g.drm_card = static_cast<int>(en.drm_card);
          g.hsa_id = static_cast<int>(en.hsa_id);
          g.hip_id = static_cast<int>(en.hip_id);
          g.hip_uuid = en.hip_uuid;
        }
        snap.gpus.push_back(std::move(g));
      }
    }
  }
  if (L.shut_down) L.shut_down();
  snap.ok = true;
  return snap;
}

#else  // no amd-smi header at build time

bool smi_available() { return false; }
SmiSnapshot smi_snapshot() {
  SmiSnapshot s;
  s.error = "built without amd_smi/amdsmi.h";
  return s;
}

#endif

}  // namespace mi355x
