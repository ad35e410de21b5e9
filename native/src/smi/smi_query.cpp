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
  decltype(&amdsmi_init_gpu_event_notification) evt_init = nullptr;
  decltype(&amdsmi_set_gpu_event_notification_mask) evt_mask = nullptr;
  decltype(&amdsmi_get_gpu_event_notification) evt_get = nullptr;
  decltype(&amdsmi_stop_gpu_event_notification) evt_stop = nullptr;
  decltype(&amdsmi_get_gpu_xgmi_link_status) link_status = nullptr;
  decltype(&amdsmi_get_link_metrics) link_metrics = nullptr;
  decltype(&amdsmi_get_gpu_driver_info) driver = nullptr;
  decltype(&amdsmi_get_gpu_activity) activity = nullptr;
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
    bind(l.h, "amdsmi_init_gpu_event_notification", &l.evt_init);
    bind(l.h, "amdsmi_set_gpu_event_notification_mask", &l.evt_mask);
    bind(l.h, "amdsmi_get_gpu_event_notification", &l.evt_get);
    bind(l.h, "amdsmi_stop_gpu_event_notification", &l.evt_stop);
    bind(l.h, "amdsmi_get_gpu_xgmi_link_status", &l.link_status);
    bind(l.h, "amdsmi_get_link_metrics", &l.link_metrics);
    bind(l.h, "amdsmi_get_gpu_driver_info", &l.driver);
    bind(l.h, "amdsmi_get_gpu_activity", &l.activity);
  });
  return l;
}

// amdsmi_init / amdsmi_shut_down shared by snapshots and the event watcher
std::mutex g_init_mu;
int g_init_refs = 0;

bool acquire() {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (g_init_refs == 0 && smi().init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return false;
  ++g_init_refs;
  return true;
}

void release() {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (g_init_refs > 0 && --g_init_refs == 0 && smi().shut_down) smi().shut_down();
}

std::string bdf_of(amdsmi_processor_handle h) {
  amdsmi_bdf_t bdf{};
  if (!smi().bdf || smi().bdf(h, &bdf) != AMDSMI_STATUS_SUCCESS) return "";
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%04llx:%02llx:%02llx.%llx", static_cast<unsigned long long>(bdf.domain_number),
                static_cast<unsigned long long>(bdf.bus_number), static_cast<unsigned long long>(bdf.device_number),
                static_cast<unsigned long long>(bdf.function_number));
  return buf;
}

std::vector<amdsmi_processor_handle> all_gpus() {
  std::vector<amdsmi_processor_handle> out;
  uint32_t nsock = 0;
  if (smi().sockets(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS || nsock == 0) return out;
  std::vector<amdsmi_socket_handle> socks(nsock);
  smi().sockets(&nsock, socks.data());
  for (uint32_t s = 0; s < nsock; ++s) {
    uint32_t nproc = 0;
    if (smi().processors(socks[s], &nproc, nullptr) != AMDSMI_STATUS_SUCCESS || nproc == 0) continue;
    std::vector<amdsmi_processor_handle> procs(nproc);
    smi().processors(socks[s], &nproc, procs.data());
    out.insert(out.end(), procs.begin(), procs.end());
  }
  return out;
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

bool smi_hold() { return smi_available() && acquire(); }
void smi_unhold() {
  if (smi_available()) release();
}

SmiSnapshot smi_snapshot() {
  SmiSnapshot snap;
  const auto& L = smi();
  if (!smi_available()) {
    snap.error = "libamd_smi unavailable";
    return snap;
  }
  if (!acquire()) {
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
        amdsmi_driver_info_t di{};
        amdsmi_engine_usage_t eu{};
        if (L.activity && L.activity(h, &eu) == AMDSMI_STATUS_SUCCESS) g.gfx_activity = static_cast<int>(eu.gfx_activity);
        if (L.driver && L.driver(h, &di) == AMDSMI_STATUS_SUCCESS) {
          g.driver_name = di.driver_name;
          g.driver_version = di.driver_version;
        }
        snap.gpus.push_back(std::move(g));
      }
    }
  }
  release();
  snap.ok = true;
  return snap;
}

SmiXgmiSnapshot smi_xgmi_links() {
  SmiXgmiSnapshot snap;
  const auto& L = smi();
  if (!smi_available()) {
    snap.error = "libamd_smi unavailable";
    return snap;
  }
  if (!L.link_status && !L.link_metrics) {
    snap.error = "libamd_smi has no xGMI link queries";
    return snap;
  }
  if (!acquire()) {
    snap.error = "amdsmi_init failed";
    return snap;
  }
  for (auto h : all_gpus()) {
    SmiXgmiLinks g;
    g.bdf = bdf_of(h);
    if (L.link_status) {
      amdsmi_xgmi_link_status_t st{};
      const amdsmi_status_t rc = L.link_status(h, &st);
      if (rc == AMDSMI_STATUS_SUCCESS) {
        g.status_ok = true;
        const uint32_t n = st.total_links < AMDSMI_MAX_NUM_XGMI_LINKS ? st.total_links : AMDSMI_MAX_NUM_XGMI_LINKS;
        for (uint32_t i = 0; i < n; ++i) g.status.push_back(static_cast<int>(st.status[i]));
      } else {
        g.error = "xgmi_link_status rc=" + std::to_string(static_cast<int>(rc));
      }
    }
    if (L.link_metrics) {
      amdsmi_link_metrics_t lm{};
      const amdsmi_status_t rc = L.link_metrics(h, &lm);
      if (rc == AMDSMI_STATUS_SUCCESS) {
        g.metrics_ok = true;
        const uint32_t n =
            lm.num_links < AMDSMI_MAX_NUM_XGMI_PHYSICAL_LINK ? lm.num_links : AMDSMI_MAX_NUM_XGMI_PHYSICAL_LINK;
        for (uint32_t i = 0; i < n; ++i) {
          const auto& l = lm.links[i];
          SmiLinkPeer p;
          char buf[64];
          std::snprintf(buf, sizeof(buf), "%04llx:%02llx:%02llx.%llx",
                        static_cast<unsigned long long>(l.bdf.domain_number),
                        static_cast<unsigned long long>(l.bdf.bus_number),
                        static_cast<unsigned long long>(l.bdf.device_number),
                        static_cast<unsigned long long>(l.bdf.function_number));
          p.peer_bdf = buf;
          p.link_type = static_cast<int>(l.link_type);
          p.bit_rate_gbps = l.bit_rate;
          p.max_bandwidth_gbps = l.max_bandwidth;
          p.read_kb = l.read;
          p.write_kb = l.write;
          g.peers.push_back(p);
        }
      } else if (g.error.empty()) {
        g.error = "link_metrics rc=" + std::to_string(static_cast<int>(rc));
      }
    }
    snap.gpus.push_back(std::move(g));
  }
  release();
  snap.ok = true;
  return snap;
}

const char* smi_event_name(int type) {
  switch (type) {
    case AMDSMI_EVT_NOTIF_VMFAULT: return "vmfault";
    case AMDSMI_EVT_NOTIF_THERMAL_THROTTLE: return "thermal_throttle";
    case AMDSMI_EVT_NOTIF_GPU_PRE_RESET: return "gpu_pre_reset";
    case AMDSMI_EVT_NOTIF_GPU_POST_RESET: return "gpu_post_reset";
    case AMDSMI_EVT_NOTIF_MIGRATE_START: return "migrate_start";
    case AMDSMI_EVT_NOTIF_MIGRATE_END: return "migrate_end";
    case AMDSMI_EVT_NOTIF_PAGE_FAULT_START: return "page_fault_start";
    case AMDSMI_EVT_NOTIF_PAGE_FAULT_END: return "page_fault_end";
    case AMDSMI_EVT_NOTIF_QUEUE_EVICTION: return "queue_eviction";
    case AMDSMI_EVT_NOTIF_QUEUE_RESTORE: return "queue_restore";
    case AMDSMI_EVT_NOTIF_UNMAP_FROM_GPU: return "unmap_from_gpu";
    case AMDSMI_EVT_NOTIF_PROCESS_START: return "process_start";
    case AMDSMI_EVT_NOTIF_PROCESS_END: return "process_end";
    default: return "unknown";
  }
}

SmiEventWatcher::~SmiEventWatcher() { stop(); }

std::string SmiEventWatcher::start(uint64_t mask) {
  stop();
  const auto& L = smi();
  if (!smi_available() || !L.evt_init || !L.evt_mask || !L.evt_get || !L.evt_stop)
    return "libamd_smi event notification unavailable";
  if (!acquire()) return "amdsmi_init failed";
  for (auto h : all_gpus()) {
    if (L.evt_init(h) != AMDSMI_STATUS_SUCCESS) continue;
    if (L.evt_mask(h, mask) != AMDSMI_STATUS_SUCCESS) {
      L.evt_stop(h);
      continue;
    }
    handles_.push_back(h);
    bdfs_.push_back(bdf_of(h));
  }
  if (handles_.empty()) {
    release();
    return "no GPU accepted event notification";
  }
  running_ = true;
  return "";
}

std::vector<SmiEvent> SmiEventWatcher::poll(int timeout_ms) {
  std::vector<SmiEvent> out;
  if (!running_) return out;
  for (;;) {
    amdsmi_evt_notification_data_t data[32];
    uint32_t n = 32;
    const amdsmi_status_t st = smi().evt_get(timeout_ms, &n, data);
    if (st != AMDSMI_STATUS_SUCCESS || n == 0) break;
    for (uint32_t i = 0; i < n; ++i) {
      SmiEvent e;
      for (size_t k = 0; k < handles_.size(); ++k)
        if (handles_[k] == data[i].processor_handle) e.bdf = bdfs_[k];
      if (e.bdf.empty()) e.bdf = bdf_of(data[i].processor_handle);
      e.type = static_cast<int>(data[i].event);
      e.name = smi_event_name(e.type);
      e.message = data[i].message;
      out.push_back(std::move(e));
    }
    if (n < 32) break;
    timeout_ms = 0;  // drain the rest without waiting again
  }
  return out;
}

void SmiEventWatcher::stop() {
  if (!running_) return;
  for (auto h : handles_) smi().evt_stop(h);
  handles_.clear();
  bdfs_.clear();
  running_ = false;
  release();
}

#else  // no amd-smi header at build time

bool smi_available() { return false; }
bool smi_hold() { return false; }
void smi_unhold() {}
SmiSnapshot smi_snapshot() {
  SmiSnapshot s;
  s.error = "built without amd_smi/amdsmi.h";
  return s;
}
SmiXgmiSnapshot smi_xgmi_links() {
  SmiXgmiSnapshot s;
  s.error = "built without amd_smi/amdsmi.h";
  return s;
}
const char* smi_event_name(int) { return "unknown"; }
SmiEventWatcher::~SmiEventWatcher() = default;
std::string SmiEventWatcher::start(uint64_t) { return "built without amd_smi/amdsmi.h"; }
std::vector<SmiEvent> SmiEventWatcher::poll(int) { return {}; }
void SmiEventWatcher::stop() {}

#endif

}  // namespace mi355x
