// HSA-direct launcher for the gfx950 MFMA liveness kernel.
//
// A HIP program pays ~60 ms of runtime start-up and ~21 ms of per-device
// queue set-up before its first kernel (MI355X, profiles/r4/bench100_hip.json
// extra.container_phases_p50_ms), pure overhead for a few-us liveness dispatch
// that the plugin runs on every device every pulse. This path talks to ROCr
// directly:
//
//   hsa_init -> GPU agents (ROCR_VISIBLE_DEVICES honoured)
//   code object: the embedded liveness_gfx950.hsaco -> executable -> kernel object
//   AQL kernel-dispatch packet on a private queue, completion signal,
//   dispatch timestamps from hsa_amd_profiling
//   outputs in fine-grained system memory (host reads them directly),
//   scratch in the device's coarse-grained HBM pool.
//
// Exactly one dispatch per probe; the agent's kfd node id comes from
// HSA_AMD_AGENT_INFO_DRIVER_NODE_ID, so the verdict maps to the kubelet
// device ID without guessing.
#include <dlfcn.h>
#include <fcntl.h>
#include <unistd.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "hsa_runtime.h"
#include "probe_verify.h"

// The gfx950 code object, embedded at build time (declared in hsa_runtime.h).
#ifndef MI355X_HSACO_PATH
#error "MI355X_HSACO_PATH must name the gfx950 code object to embed"
#endif
asm(".section .rodata.mi355x_hsaco,\"a\",@progbits\n"
    ".p2align 12\n"
    ".globl mi355x_hsaco_start\n"
    "mi355x_hsaco_start:\n"
    ".incbin \"" MI355X_HSACO_PATH "\"\n"
    ".globl mi355x_hsaco_end\n"
    "mi355x_hsaco_end:\n"
    ".byte 0\n"
    ".previous\n");

namespace mi355x {

const HsaApi& hsa_api() {
  static HsaApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    const auto t0 = std::chrono::steady_clock::now();
    // RTLD_NOLOAD first: in a process that already has ROCr (torch, the HIP
    // runtime) reuse that copy rather than loading a second one
    void* h = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
    if (!h) h = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      std::snprintf(api.error, sizeof(api.error), "dlopen libhsa-runtime64.so.1: %s", dlerror());
      return;
    }
#define MI355X_HSA_SYM(name)                                                                  \
  api.name = reinterpret_cast<decltype(&::name)>(dlsym(h, #name));                            \
  if (!api.name) {                                                                            \
    std::snprintf(api.error, sizeof(api.error), "libhsa-runtime64.so.1 lacks %s", #name);     \
    return;                                                                                   \
  }
    MI355X_HSA_FUNCS(MI355X_HSA_SYM)
#undef MI355X_HSA_SYM
    api.loaded = true;
    api.load_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  });
  return api;
}

}  // namespace mi355x

using namespace mi355x::hsa_rt;  // NOLINT(build/namespaces)

namespace mi355x::hsa_rt {



Runtime g_rt;

hsa_status_t collect_agent(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  if (H().hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_GPU) {
    Agent ag;
    ag.agent = a;
    g_rt.gpus.push_back(ag);
  } else if (t == HSA_DEVICE_TYPE_CPU && g_rt.cpu.handle == 0) {
    g_rt.cpu = a;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t cpu_pool(hsa_amd_memory_pool_t p, void*) {
  hsa_amd_segment_t seg;
  H().hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  H().hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !g_rt.has_kernarg) {
    g_rt.kernarg = p;
    g_rt.has_kernarg = true;
  }
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !g_rt.has_fine) {
    g_rt.fine = p;
    g_rt.has_fine = true;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t gpu_pool(hsa_amd_memory_pool_t p, void* data) {
  auto* ag = static_cast<Agent*>(data);
  hsa_amd_segment_t seg;
  H().hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  H().hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  bool alloc_ok = false;
  H().hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc_ok);
  if (alloc_ok && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !ag->has_coarse) {
    ag->coarse = p;
    ag->has_coarse = true;
  }
  return HSA_STATUS_SUCCESS;
}

void set_status(mi355x_probe_result* r, hsa_status_t s, const char* what) {
  if (r->hip_error == 0) r->hip_error = static_cast<int>(s);
  const char* msg = nullptr;
  if (!H().loaded) {
    std::snprintf(r->error, sizeof(r->error), "%s: %.120s", what, H().error);
    return;
  }
  H().hsa_status_string(s, &msg);
  std::snprintf(r->error, sizeof(r->error), "%s: %s", what, msg ? msg : "hsa error");
}

void fill_identity(const Agent& ag, int ordinal, mi355x_probe_result* out) {
  out->ordinal = ordinal;
  std::snprintf(out->runtime, sizeof(out->runtime), "hsa");
  char name[64] = {0};
  H().hsa_agent_get_info(ag.agent, HSA_AGENT_INFO_NAME, name);
  std::snprintf(out->arch, sizeof(out->arch), "%s", name);
  char product[64] = {0};
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_PRODUCT_NAME), product);
  std::snprintf(out->name, sizeof(out->name), "%s", product);
  uint32_t node = 0, bdf = 0, domain = 0, cus = 0;
  if (H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DRIVER_NODE_ID), &node) ==
      HSA_STATUS_SUCCESS)
    out->kfd_node_id = static_cast<int>(node);
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &domain);
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT), &cus);
  out->pci_domain = static_cast<int>(domain);
  out->pci_bus = static_cast<int>((bdf >> 8) & 0xFF);
  out->pci_device = static_cast<int>((bdf >> 3) & 0x1F);
  out->cu_count = static_cast<int>(cus);
  std::snprintf(out->pci_bus_id, sizeof(out->pci_bus_id), "%04x:%02x:%02x.%x", domain, (bdf >> 8) & 0xFF,
                (bdf >> 3) & 0x1F, bdf & 0x7);
  char uuid[24] = {0};
  if (H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_UUID), uuid) ==
      HSA_STATUS_SUCCESS)
    std::snprintf(out->uuid, sizeof(out->uuid), "%s", uuid);
  if (ag.has_coarse) {
    size_t sz = 0;
    H().hsa_amd_memory_pool_get_info(ag.coarse, HSA_AMD_MEMORY_POOL_INFO_SIZE, &sz);
    out->total_mem = sz;
  }
}

}  // namespace mi355x::hsa_rt

extern "C" int mi355x_hsa_probe_init(void) {
  std::lock_guard<std::mutex> lk(g_rt.mu);
  if (g_rt.inited) return g_rt.init_status == HSA_STATUS_SUCCESS ? static_cast<int>(g_rt.gpus.size())
                                                                  : -static_cast<int>(g_rt.init_status);
  g_rt.inited = true;
  g_rt.init_status = HSA_STATUS_SUCCESS;  // a shut-down runtime may be initialised again
  using clk = std::chrono::steady_clock;
  auto us = [](clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
  };
  // Create this process' kfd process (kernel side) while ROCr's constructors
  // run on this thread; hsa_init's own open() then finds it (hsa_api.h).
  const auto tk = clk::now();
  std::thread preopen([tk] {
    g_rt.kfd_fd = open("/dev/kfd", O_RDWR | O_CLOEXEC);
    g_rt.init_us[1] = std::chrono::duration<double, std::micro>(clk::now() - tk).count();
  });
  const mi355x::HsaApi& api = H();
  preopen.join();
  g_rt.init_us[0] = api.load_us;
  if (!api.loaded) {
    g_rt.init_status = HSA_STATUS_ERROR;
    return -static_cast<int>(HSA_STATUS_ERROR);
  }
  const auto t0 = clk::now();
  hsa_status_t s = H().hsa_init();
  const auto t1 = clk::now();
  g_rt.init_us[2] = us(t0, t1);
  if (s != HSA_STATUS_SUCCESS) {
    g_rt.init_status = s;
    return -static_cast<int>(s);
  }
  H().hsa_iterate_agents(collect_agent, nullptr);
  const auto t2 = clk::now();
  if (g_rt.cpu.handle) H().hsa_amd_agent_iterate_memory_pools(g_rt.cpu, cpu_pool, nullptr);
  for (auto& ag : g_rt.gpus) H().hsa_amd_agent_iterate_memory_pools(ag.agent, gpu_pool, &ag);
  H().hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &g_rt.ts_freq);
  g_rt.init_us[3] = us(t1, t2);
  g_rt.init_us[4] = us(t2, clk::now());
  return static_cast<int>(g_rt.gpus.size());
}

extern "C" void mi355x_hsa_init_phases(double out_us[5]) {
  for (int i = 0; i < 5; ++i) out_us[i] = g_rt.init_us[i];
}


extern "C" void mi355x_hsa_probe_shutdown(void) {
  mi355x_hsa_probe_release();
  release_residents();
  forget_in_flight_sweeps();
  std::lock_guard<std::mutex> lk(g_rt.mu);
  if (g_rt.inited && g_rt.init_status == HSA_STATUS_SUCCESS) H().hsa_shut_down();
  if (g_rt.kfd_fd >= 0) close(g_rt.kfd_fd);
  g_rt.kfd_fd = -1;
  g_rt.inited = false;
  g_rt.gpus.clear();
  g_rt.has_kernarg = g_rt.has_fine = false;
  g_rt.cpu = hsa_agent_t{};
}

extern "C" int mi355x_hsa_probe_identify(int ordinal, mi355x_probe_result* out) {
  std::memset(out, 0, sizeof(*out));
  out->kfd_node_id = -1;
  int n = mi355x_hsa_probe_init();
  if (n < 0) {
    set_status(out, static_cast<hsa_status_t>(-n), "hsa_init");
    return 1;
  }
  if (ordinal < 0 || ordinal >= n) {
    std::snprintf(out->error, sizeof(out->error), "no such GPU agent (count=%d)", n);
    return 1;
  }
  fill_identity(g_rt.gpus[ordinal], ordinal, out);
  return 0;
}

namespace mi355x::hsa_rt {



std::mutex g_deferred_mu;
bool g_defer_release = false;
std::vector<ProbeResources> g_deferred;


struct Step {
  hsa_status_t s = HSA_STATUS_SUCCESS;
  const char* what = nullptr;
  bool ok() const { return s == HSA_STATUS_SUCCESS; }
};

#define STEP(st, expr, label)         \
  do {                                \
    (st).s = (expr);                  \
    if ((st).s != HSA_STATUS_SUCCESS) { \
      (st).what = (label);            \
      return st;                      \
    }                                 \
  } while (0)

// Queue, completion signal and buffers: independent of the code object, so it
// runs on a helper thread while the main thread loads the executable (both are
// a few ms of driver work each on MI355X).
Step make_queue_and_buffers(const Agent& ag, ProbeResources& r) {
  Step st;
  STEP(st, H().hsa_queue_create(ag.agent, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &r.queue),
       "queue create");
  H().hsa_amd_profiling_set_profiler_enabled(r.queue, 1);
  STEP(st, H().hsa_signal_create(1, 0, nullptr, &r.sig), "signal create");
  STEP(st, H().hsa_amd_memory_pool_allocate(g_rt.fine, MI355X_PROBE_OUT * sizeof(float), 0,
                                        reinterpret_cast<void**>(&r.h_out)), "alloc out");
  STEP(st, H().hsa_amd_memory_pool_allocate(g_rt.fine, 64, 0, reinterpret_cast<void**>(&r.h_meta)), "alloc meta");
  STEP(st, H().hsa_amd_memory_pool_allocate(ag.coarse, MI355X_SCRATCH_FLOATS * sizeof(float), 0,
                                        reinterpret_cast<void**>(&r.d_scratch)), "alloc scratch");
  STEP(st, H().hsa_amd_memory_pool_allocate(g_rt.kernarg, kKernargBytes, 0, reinterpret_cast<void**>(&r.kargs)),
       "alloc kernarg");
  STEP(st, H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, r.h_out), "allow out");
  STEP(st, H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, r.h_meta), "allow meta");
  STEP(st, H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, r.kargs), "allow kernarg");
  return st;
}


Step load_kernel(const Agent& ag, ProbeResources& r, KernelInfo& k) {
  Step st;
  const size_t co_size = static_cast<size_t>(mi355x_hsaco_end - mi355x_hsaco_start);
  STEP(st, H().hsa_code_object_reader_create_from_memory(mi355x_hsaco_start, co_size, &r.reader), "code object reader");
  STEP(st, H().hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &r.exe),
       "executable create");
  STEP(st, H().hsa_executable_load_agent_code_object(r.exe, ag.agent, r.reader, nullptr, nullptr), "load code object");
  STEP(st, H().hsa_executable_freeze(r.exe, nullptr), "executable freeze");
  hsa_executable_symbol_t sym{};
  STEP(st, H().hsa_executable_get_symbol_by_name(r.exe, "mi355x_mfma_liveness.kd", &ag.agent, &sym), "kernel symbol");
  H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.kobj);
  H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kseg);
  H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.gseg);
  H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.pseg);
  return st;
}
#undef STEP

}  // namespace mi355x::hsa_rt

extern "C" void mi355x_hsa_probe_defer_release(int on) {
  std::lock_guard<std::mutex> lk(g_deferred_mu);
  g_defer_release = on != 0;
}

extern "C" void mi355x_hsa_probe_release(void) {
  std::vector<ProbeResources> todo;
  {
    std::lock_guard<std::mutex> lk(g_deferred_mu);
    todo.swap(g_deferred);
  }
  for (auto& r : todo) r.release();
}

namespace mi355x::hsa_rt {

// Queue + buffers (helper thread) and the executable (this thread), overlapped.
// Fills out->phase_us[0..1] and out->setup_us; false with out->error on failure.
bool setup_resources(const Agent& ag, ProbeResources& r, KernelInfo& k, mi355x_probe_result* out) {
  using clk = std::chrono::steady_clock;
  auto us_since = [](clk::time_point a) { return std::chrono::duration<double, std::micro>(clk::now() - a).count(); };
  const auto t0 = clk::now();
  Step qst, kst;
  double queue_us = 0;
  std::thread qthread([&] {
    const auto tq = clk::now();
    qst = make_queue_and_buffers(ag, r);
    queue_us = us_since(tq);
  });
  kst = load_kernel(ag, r, k);
  out->phase_us[0] = us_since(t0);  // code object load + freeze
  qthread.join();
  out->phase_us[1] = queue_us;      // queue + signal + buffers (overlapped with phase 0)
  out->setup_us = us_since(t0);
  if (!kst.ok() || !qst.ok()) {
    const Step& bad = !kst.ok() ? kst : qst;
    set_status(out, bad.s, bad.what);
    return false;
  }
  if (k.kseg < sizeof(mi355x_liveness_args) || k.kseg > kKernargBytes) {
    std::snprintf(out->error, sizeof(out->error), "kernarg segment %u outside [%zu, %u]: code object / host ABI mismatch",
                  k.kseg, sizeof(mi355x_liveness_args), kKernargBytes);
    return false;
  }
  return true;
}

// Submits one AQL dispatch of the liveness kernel on r's queue (no wait).
void submit_dispatch(ProbeResources& r, const KernelInfo& k, uint32_t nonce, int iters, mi355x_probe_result* out) {
  std::memset(r.h_out, 0xFF, MI355X_PROBE_OUT * sizeof(float));
  std::memset(r.h_meta, 0, 64);
  std::memset(r.kargs, 0, kKernargBytes);
  r.kargs->out = r.h_out;
  r.kargs->meta = r.h_meta;
  r.kargs->scratch = r.d_scratch;
  r.kargs->nonce = nonce;
  r.kargs->iters = iters;
  H().hsa_signal_store_screlease(r.sig, 1);  // a kept signal was left at 0 by the previous dispatch

  const uint64_t idx = H().hsa_queue_add_write_index_screlease(r.queue, 1);
  auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(r.queue->base_address) + (idx & (r.queue->size - 1));
  std::memset(reinterpret_cast<char*>(pkt) + 4, 0, sizeof(*pkt) - 4);
  pkt->workgroup_size_x = 64;
  pkt->workgroup_size_y = 1;
  pkt->workgroup_size_z = 1;
  pkt->grid_size_x = 64;
  pkt->grid_size_y = 1;
  pkt->grid_size_z = 1;
  pkt->private_segment_size = k.pseg;
  pkt->group_segment_size = k.gseg;
  pkt->kernel_object = k.kobj;
  pkt->kernarg_address = r.kargs;
  pkt->completion_signal = r.sig;
  const uint16_t header = static_cast<uint16_t>(
      (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
      (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
      (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), header | (static_cast<uint32_t>(setup) << 16),
                   __ATOMIC_RELEASE);
  H().hsa_signal_store_screlease(r.queue->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
  out->dispatches += 1;
}

// Bounded wait for the dispatch submitted on r (nonce / iters as submitted),
// then the verdict. Returns false, with out->hip_error = -1, if it has not
// completed yet: r must then never be freed (the kernel may still write to it).
// Debug fault injection (mi355x_hsa_probe_corrupt): flip one bit of output
// word `word` of probes on `ordinal` (-1 = every device) after the dispatch
// completed and before the tile is verified -- a stand-in for a wrong MFMA
// result that drives the real verdict path end to end.
std::atomic<int> g_corrupt_word{-1};
std::atomic<int> g_corrupt_ordinal{-1};

bool wait_and_verify(const Agent& ag, ProbeResources& r, uint32_t nonce, int iters, double timeout_s,
                     mi355x_probe_result* out) {
  using clk = std::chrono::steady_clock;
  const auto t_wait = clk::now();
  const bool done = wait_signal(r.sig, timeout_s);
  out->phase_us[3] = std::chrono::duration<double, std::micro>(clk::now() - t_wait).count();
  if (!done) {
    std::snprintf(out->error, sizeof(out->error), "dispatch did not complete within %.1fs", timeout_s);
    out->hip_error = -1;
    return false;
  }
  hsa_amd_profiling_dispatch_time_t dt{};
  if (H().hsa_amd_profiling_get_dispatch_time(ag.agent, r.sig, &dt) == HSA_STATUS_SUCCESS && g_rt.ts_freq)
    out->kernel_us = static_cast<double>(dt.end - dt.start) * 1e6 / static_cast<double>(g_rt.ts_freq);
  out->nonce = nonce;
  out->iters = iters;
  const int cw = g_corrupt_word.load(std::memory_order_relaxed);
  const int co = g_corrupt_ordinal.load(std::memory_order_relaxed);
  if (cw >= 0 && cw < MI355X_PROBE_OUT && (co < 0 || co == out->ordinal)) {
    uint32_t bits;
    std::memcpy(&bits, &r.h_out[cw], sizeof(bits));
    bits ^= 1u;
    std::memcpy(&r.h_out[cw], &bits, sizeof(bits));
  }
  mi355x::verify_tile(r.h_out, r.h_meta, nonce, iters, out);
  return true;
}

// One dispatch, bounded wait, verdict (out->hip_error = -1 when it did not complete).
void dispatch_and_verify(const Agent& ag, ProbeResources& r, const KernelInfo& k, uint32_t nonce, double timeout_s,
                         mi355x_probe_result* out) {
  submit_dispatch(r, k, nonce, out->iters, out);
  wait_and_verify(ag, r, nonce, out->iters, timeout_s, out);
}

std::mutex g_resident_mu;
bool g_keep = false;
std::vector<std::pair<int, std::unique_ptr<Resident>>> g_resident;

// Frees every kept device's resources (runtime shutdown); a slot whose
// dispatch is still pending goes with the runtime itself.
void release_residents() {
  std::lock_guard<std::mutex> lk(g_resident_mu);
  for (auto& e : g_resident) {
    std::lock_guard<std::timed_mutex> lk2(e.second->mu);
    if (e.second->ready && !e.second->pending && !e.second->blocker) e.second->r.release();
    if (e.second->blocker && e.second->blocker->s.handle &&
        H().hsa_signal_load_scacquire(e.second->blocker->s) >= 1)
      e.second->blocker->s = hsa_signal_t{};  // still running: leave it to the runtime's teardown
    e.second->ready = false;
  }
  g_resident.clear();
}

Resident* resident_slot(int ordinal) {
  std::lock_guard<std::mutex> lk(g_resident_mu);
  for (auto& e : g_resident)
    if (e.first == ordinal) return e.second.get();
  g_resident.emplace_back(ordinal, std::make_unique<Resident>());
  return g_resident.back().second.get();
}

}  // namespace mi355x::hsa_rt

extern "C" void mi355x_hsa_probe_corrupt(int word, int ordinal) {
  g_corrupt_word.store(word, std::memory_order_relaxed);
  g_corrupt_ordinal.store(ordinal, std::memory_order_relaxed);
}

extern "C" void mi355x_hsa_probe_keep(int on) {
  std::lock_guard<std::mutex> lk(g_resident_mu);
  g_keep = on != 0;
}

extern "C" int mi355x_hsa_probe_device(int ordinal, uint32_t nonce, int iters, double timeout_s,
                                       mi355x_probe_result* out) {
  using clk = std::chrono::steady_clock;
  std::memset(out, 0, sizeof(*out));
  out->kfd_node_id = -1;
  out->nonce = nonce;
  out->iters = iters < 1 ? 1 : iters;
  const auto t0 = clk::now();
  auto finish = [&] {
    out->total_us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
    return out->ok ? 0 : 1;
  };
  int n = mi355x_hsa_probe_init();
  if (n < 0) {
    set_status(out, static_cast<hsa_status_t>(-n), "hsa_init");
    return 1;
  }
  if (ordinal < 0 || ordinal >= n) {
    out->ordinal = ordinal;
    std::snprintf(out->error, sizeof(out->error), "no such GPU agent (count=%d)", n);
    return 1;
  }
  const Agent& ag = g_rt.gpus[ordinal];
  fill_identity(ag, ordinal, out);
  if (!g_rt.has_kernarg || !g_rt.has_fine || !ag.has_coarse) {
    std::snprintf(out->error, sizeof(out->error), "missing memory pool (kernarg=%d fine=%d coarse=%d)",
                  g_rt.has_kernarg, g_rt.has_fine, ag.has_coarse);
    return 1;
  }
  bool keep;
  {
    std::lock_guard<std::mutex> lk(g_resident_mu);
    keep = g_keep;
  }

  if (keep) {
    Resident* slot = resident_slot(ordinal);
    // another request's probe, chip sweep or throughput check holds this
    // device's kept queue (concurrent --serve requests): wait for it no longer
    // than this probe's own deadline, then answer pending without a dispatch
    std::unique_lock<std::timed_mutex> lk(slot->mu, std::defer_lock);
    if (!lk.try_lock_for(std::chrono::duration<double>(timeout_s > 0 ? timeout_s : 5.0))) {
      const double s_out = std::max(1e-3, std::chrono::duration<double>(clk::now() - t0).count());
      std::snprintf(out->error, sizeof(out->error),
                    "another request on this device's queue still running after %.2fs (not dispatched)", s_out);
      out->pending_s = s_out;
      out->hip_error = -1;
      return finish();
    }
    // the deadline counts from the request, the wait for the slot included
    const double left_s =
        std::max(1e-3, (timeout_s > 0 ? timeout_s : 5.0) - std::chrono::duration<double>(clk::now() - t0).count());
    if (!slot->ready) {
      if (!setup_resources(ag, slot->r, slot->k, out)) {
        slot->r.release();
        return finish();
      }
      slot->ready = true;
    }
    if (slot->blocker) {
      if (H().hsa_signal_load_scacquire(slot->blocker->s) >= 1) {
        // > 0 however recent: pending_s > 0 is what marks the verdict inconclusive
        const double s_out =
            std::max(1e-3, std::chrono::duration<double>(clk::now() - slot->blocked_since).count());
        std::snprintf(out->error, sizeof(out->error),
                      "chip sweep / throughput check on this device's queue pending for %.1fs (not completed)", s_out);
        out->pending_s = s_out;
        out->hip_error = -1;
        return finish();
      }
      slot->blocker.reset();
      in_flight_for(ordinal);  // frees the completed sweep / check's buffers now, not at the next one
    }
    if (slot->pending) {
      // the previous probe's dispatch is still outstanding: wait for it (it
      // carries its own nonce), never stack a second one behind it
      if (!wait_and_verify(ag, slot->r, slot->pending_nonce, slot->pending_iters, left_s, out)) {
        const double s_out = std::max(1e-3, std::chrono::duration<double>(clk::now() - slot->pending_since).count());
        std::snprintf(out->error, sizeof(out->error), "dispatch pending for %.1fs (not completed)", s_out);
        out->pending_s = s_out;
        return finish();
      }
      slot->pending = false;
      out->late = 1;  // verdict of the dispatch submitted by an earlier probe
    } else {
      submit_dispatch(slot->r, slot->k, nonce, out->iters, out);
      if (!wait_and_verify(ag, slot->r, nonce, out->iters, left_s, out)) {
        slot->pending = true;
        slot->pending_nonce = nonce;
        slot->pending_iters = out->iters;
        slot->pending_since = t0;
        out->pending_s = std::max(1e-3, std::chrono::duration<double>(clk::now() - t0).count());
        return finish();
      }
    }
    if (!out->ok) {  // wrong tile or error: start from fresh resources next time
      slot->r.release();
      slot->ready = false;
    }
    return finish();
  }

  ProbeResources r;
  KernelInfo k;
  if (setup_resources(ag, r, k, out)) dispatch_and_verify(ag, r, k, nonce, timeout_s, out);
  const int rc = finish();
  {
    std::unique_lock<std::mutex> lk(g_deferred_mu);
    // a timed-out dispatch may still be running: never free what it can write
    if (g_defer_release || out->hip_error == -1) {
      if (out->hip_error != -1) g_deferred.push_back(r);
      return rc;
    }
  }
  r.release();
  return rc;
}

namespace mi355x::hsa_rt {

// Bounded wait for a completion signal (value 1 -> 0): true when it completed.
// hsa_signal_wait's BLOCKED wait (interrupt-driven: returns as soon as the
// dispatch completes) overshoots its timeout hint by up to ~20 ms on MI355X
// (a 50 ms deadline came back after 69 ms p50, tools/probe_deadline_tenant.py),
// so it is used only while more than kBlockedMargin is left, with the hint
// cut to leave that margin; the rest of the deadline is polled every 200 us.
// The first wait lasts at least 1 ms: no dispatch completes faster than its
// launch, so a shorter deadline would only abandon work that is about to finish.
bool wait_signal(hsa_signal_t sig, double timeout_s) {
  using clk = std::chrono::steady_clock;
  constexpr double kBlockedMargin = 0.025;
  const auto t0 = clk::now();
  const auto deadline = t0 + std::chrono::duration<double>(std::max(1e-3, timeout_s > 0 ? timeout_s : 5.0));
  const double ticks_per_s = g_rt.ts_freq ? static_cast<double>(g_rt.ts_freq) : 1e9;
  while (true) {
    const double left = std::chrono::duration<double>(deadline - clk::now()).count();
    if (left <= 0) return H().hsa_signal_load_scacquire(sig) < 1;
    if (left > kBlockedMargin + 1e-3) {
      const double hint_s = std::min(0.02, left - kBlockedMargin);
      const uint64_t hint = static_cast<uint64_t>(std::max(1.0, hint_s * ticks_per_s));
      if (H().hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, hint, HSA_WAIT_STATE_BLOCKED) < 1) return true;
      continue;
    }
    if (H().hsa_signal_load_scacquire(sig) < 1) return true;
    std::this_thread::sleep_for(std::chrono::duration<double>(std::min(left, 2e-4)));
  }
}

void bus_id(const Agent& ag, char* out, size_t n) {
  uint32_t bdf = 0, domain = 0;
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &domain);
  std::snprintf(out, n, "%04x:%02x:%02x.%x", domain, (bdf >> 8) & 0xFF, (bdf >> 3) & 0x1F, bdf & 0x7);
}

}  // namespace mi355x::hsa_rt
