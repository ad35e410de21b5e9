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

#include "hsa_api.h"
#include "liveness_kernel.h"
#include "mi355x/liveness_probe.h"
#include "probe_verify.h"

// The gfx950 code object, embedded at build time.
extern "C" const unsigned char mi355x_hsaco_start[];
extern "C" const unsigned char mi355x_hsaco_end[];
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

namespace {

inline const mi355x::HsaApi& H() { return mi355x::hsa_api(); }

struct Agent {
  hsa_agent_t agent{};
  hsa_amd_memory_pool_t coarse{};  // device HBM
  bool has_coarse = false;
};

struct Runtime {
  std::mutex mu;
  bool inited = false;
  hsa_status_t init_status = HSA_STATUS_SUCCESS;
  std::vector<Agent> gpus;
  hsa_agent_t cpu{};
  hsa_amd_memory_pool_t kernarg{};
  hsa_amd_memory_pool_t fine{};
  bool has_kernarg = false, has_fine = false;
  uint64_t ts_freq = 0;
  // dlopen(ROCr), pre-open of /dev/kfd (overlapped with dlopen), hsa_init,
  // agent enumeration, pool discovery
  double init_us[5] = {0, 0, 0, 0, 0};
  int kfd_fd = -1;
} g_rt;

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

}  // namespace

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

namespace {
void release_residents();
}  // namespace

namespace {
void forget_in_flight_sweeps();
double in_flight_for(int ordinal);
}  // namespace

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

namespace {

// A completion signal shared by whoever may still need it: a chip sweep or
// throughput check whose dispatch outlived its deadline is referenced both by
// the in-flight registry and by the kept queue it was submitted on.
struct SigRef {
  hsa_signal_t s{};
  SigRef() = default;
  SigRef(const SigRef&) = delete;
  SigRef& operator=(const SigRef&) = delete;
  ~SigRef() {
    if (s.handle) H().hsa_signal_destroy(s);
  }
};

// Everything one probe allocates. Released right after the verdict, or — for
// the container entrypoint, which reports "ready" as soon as the verdict is
// known — after the JSON line is out (mi355x_hsa_probe_defer_release).
struct ProbeResources {
  hsa_code_object_reader_t reader{};
  hsa_executable_t exe{};
  hsa_queue_t* queue = nullptr;
  hsa_signal_t sig{};
  float* h_out = nullptr;
  uint32_t* h_meta = nullptr;
  float* d_scratch = nullptr;
  mi355x_liveness_args* kargs = nullptr;

  void release() {
    if (kargs) H().hsa_amd_memory_pool_free(kargs);
    if (d_scratch) H().hsa_amd_memory_pool_free(d_scratch);
    if (h_meta) H().hsa_amd_memory_pool_free(h_meta);
    if (h_out) H().hsa_amd_memory_pool_free(h_out);
    if (sig.handle) H().hsa_signal_destroy(sig);
    if (queue) H().hsa_queue_destroy(queue);
    if (exe.handle) H().hsa_executable_destroy(exe);
    if (reader.handle) H().hsa_code_object_reader_destroy(reader);
    *this = ProbeResources{};
  }
};

std::mutex g_deferred_mu;
bool g_defer_release = false;
std::vector<ProbeResources> g_deferred;

// kernarg buffer size; the code object's segment size is checked against it
constexpr uint32_t kKernargBytes = 256;

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

struct KernelInfo {
  uint64_t kobj = 0;
  uint32_t kseg = 0, gseg = 0, pseg = 0;
};

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

}  // namespace

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

namespace {

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
  const auto deadline = t_wait + std::chrono::duration<double>(timeout_s > 0 ? timeout_s : 5.0);
  hsa_signal_value_t v = 1;
  while ((v = H().hsa_signal_wait_scacquire(r.sig, HSA_SIGNAL_CONDITION_LT, 1, 20 * 1000 * 1000ull,
                                        HSA_WAIT_STATE_BLOCKED)) >= 1) {
    if (clk::now() > deadline) break;
  }
  out->phase_us[3] = std::chrono::duration<double, std::micro>(clk::now() - t_wait).count();
  if (v >= 1) {
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

// Kept ("resident") per-device resources for mi355x_hsa_probe_keep(1).
struct Resident {
  std::mutex mu;  // one probe at a time per device
  bool ready = false;
  ProbeResources r;
  KernelInfo k;
  // a dispatch that has not completed yet (a tenant's long kernel holds every
  // CU, or the device hangs): the next probe waits for it instead of
  // submitting another or abandoning the queue with its 181 MB save area
  bool pending = false;
  uint32_t pending_nonce = 0;
  int pending_iters = 1;
  std::chrono::steady_clock::time_point pending_since{};
  // a chip sweep / throughput check submitted on this kept queue that did not
  // complete within its deadline: probes report pending until it has
  std::shared_ptr<SigRef> blocker;
  std::chrono::steady_clock::time_point blocked_since{};
};
std::mutex g_resident_mu;
bool g_keep = false;
std::vector<std::pair<int, std::unique_ptr<Resident>>> g_resident;

// Frees every kept device's resources (runtime shutdown); a slot whose
// dispatch is still pending goes with the runtime itself.
void release_residents() {
  std::lock_guard<std::mutex> lk(g_resident_mu);
  for (auto& e : g_resident) {
    std::lock_guard<std::mutex> lk2(e.second->mu);
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

}  // namespace

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
    std::lock_guard<std::mutex> lk(slot->mu);
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
      if (!wait_and_verify(ag, slot->r, slot->pending_nonce, slot->pending_iters, timeout_s, out)) {
        const double s_out = std::max(1e-3, std::chrono::duration<double>(clk::now() - slot->pending_since).count());
        std::snprintf(out->error, sizeof(out->error), "dispatch pending for %.1fs (not completed)", s_out);
        out->pending_s = s_out;
        return finish();
      }
      slot->pending = false;
      out->late = 1;  // verdict of the dispatch submitted by an earlier probe
    } else {
      submit_dispatch(slot->r, slot->k, nonce, out->iters, out);
      if (!wait_and_verify(ag, slot->r, nonce, out->iters, timeout_s, out)) {
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

namespace {

// Bounded wait for a DMA completion signal (value 1 -> 0).
bool wait_signal(hsa_signal_t sig, double timeout_s) {
  using clk = std::chrono::steady_clock;
  const auto deadline = clk::now() + std::chrono::duration<double>(timeout_s > 0 ? timeout_s : 5.0);
  while (H().hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 20 * 1000 * 1000ull,
                                       HSA_WAIT_STATE_BLOCKED) >= 1) {
    if (clk::now() > deadline) return false;
  }
  return true;
}

void bus_id(const Agent& ag, char* out, size_t n) {
  uint32_t bdf = 0, domain = 0;
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &domain);
  std::snprintf(out, n, "%04x:%02x:%02x.%x", domain, (bdf >> 8) & 0xFF, (bdf >> 3) & 0x1F, bdf & 0x7);
}

}  // namespace

extern "C" int mi355x_hsa_peer_probe(int src, int dst, uint32_t nonce, uint64_t bytes, int reps, double timeout_s,
                                     mi355x_peer_result* out) {
  using clk = std::chrono::steady_clock;
  std::memset(out, 0, sizeof(*out));
  out->src = src;
  out->dst = dst;
  out->reps = reps < 1 ? 1 : reps;
  bytes = (bytes < 4096 ? 4096 : bytes) & ~static_cast<uint64_t>(3);
  out->bytes = bytes;
  out->value = (nonce * 0x9E3779B1u) ^ 0xA5C3F00Du;
  const auto t0 = clk::now();
  const int n = mi355x_hsa_probe_init();
  if (n < 0) {
    out->hsa_error = n;
    std::snprintf(out->error, sizeof(out->error), "hsa_init: %.140s", H().loaded ? "runtime init failed" : H().error);
    return 1;
  }
  if (src < 0 || src >= n || dst < 0 || dst >= n) {
    std::snprintf(out->error, sizeof(out->error), "no such GPU agent pair %d->%d (count=%d)", src, dst, n);
    return 1;
  }
  const Agent& A = g_rt.gpus[src];
  const Agent& B = g_rt.gpus[dst];
  bus_id(A, out->src_bus_id, sizeof(out->src_bus_id));
  bus_id(B, out->dst_bus_id, sizeof(out->dst_bus_id));
  if (!A.has_coarse || !B.has_coarse || !g_rt.has_fine || !g_rt.cpu.handle) {
    std::snprintf(out->error, sizeof(out->error), "missing memory pool or CPU agent");
    return 1;
  }
  hsa_amd_memory_pool_access_t access = HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED;
  H().hsa_amd_agent_memory_pool_get_info(A.agent, B.coarse, HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &access);
  out->access = static_cast<int>(access);
  uint32_t hops = 0;
  H().hsa_amd_agent_memory_pool_get_info(A.agent, B.coarse, HSA_AMD_AGENT_MEMORY_POOL_INFO_NUM_LINK_HOPS, &hops);
  out->hops = hops;
  if (hops > 0 && hops <= 16) {
    std::vector<hsa_amd_memory_pool_link_info_t> li(hops);
    if (H().hsa_amd_agent_memory_pool_get_info(A.agent, B.coarse, HSA_AMD_AGENT_MEMORY_POOL_INFO_LINK_INFO,
                                               li.data()) == HSA_STATUS_SUCCESS) {
      out->link_type = static_cast<int>(li[0].link_type);
      out->numa_distance = li[0].numa_distance;
      out->link_max_bw_mbps = li[0].max_bandwidth;
    }
  }
  if (src != dst && access == HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED) {
    std::snprintf(out->error, sizeof(out->error), "peer access %s -> %s never allowed", out->src_bus_id,
                  out->dst_bus_id);
    return 1;
  }

  void* a_buf = nullptr;
  void* b_buf = nullptr;
  uint32_t* h_buf = nullptr;
  hsa_signal_t sig{};
  bool in_flight = false;  // a timed-out copy may still write: then nothing is freed
  hsa_status_t s = HSA_STATUS_SUCCESS;
  const hsa_agent_t both[2] = {A.agent, B.agent};
  const uint32_t n_agents = src == dst ? 1 : 2;
  auto fail = [&](hsa_status_t st, const char* what) {
    out->hsa_error = static_cast<int>(st);
    const char* msg = nullptr;
    H().hsa_status_string(st, &msg);
    std::snprintf(out->error, sizeof(out->error), "%s: %s", what, msg ? msg : "hsa error");
  };
#define PEER_CHECK(expr, what) \
  if ((s = (expr)) != HSA_STATUS_SUCCESS) { fail(s, what); goto done; }

  PEER_CHECK(H().hsa_amd_memory_pool_allocate(A.coarse, bytes, 0, &a_buf), "alloc src HBM");
  PEER_CHECK(H().hsa_amd_memory_pool_allocate(B.coarse, bytes, 0, &b_buf), "alloc dst HBM");
  PEER_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.fine, bytes, 0, reinterpret_cast<void**>(&h_buf)), "alloc host");
  PEER_CHECK(H().hsa_amd_agents_allow_access(n_agents, both, nullptr, a_buf), "allow src");
  PEER_CHECK(H().hsa_amd_agents_allow_access(n_agents, both, nullptr, b_buf), "allow dst");
  PEER_CHECK(H().hsa_amd_agents_allow_access(n_agents, both, nullptr, h_buf), "allow host");
  PEER_CHECK(H().hsa_amd_memory_fill(a_buf, out->value, bytes / 4), "fill src");
  PEER_CHECK(H().hsa_amd_memory_fill(b_buf, ~out->value, bytes / 4), "fill dst");
  std::memset(h_buf, 0, bytes);
  PEER_CHECK(H().hsa_signal_create(1, 0, nullptr, &sig), "signal create");
  out->copy_us_best = 1e30;
  for (int r = 0; r < out->reps; ++r) {
    H().hsa_signal_store_screlease(sig, 1);
    const auto tc = clk::now();
    PEER_CHECK(H().hsa_amd_memory_async_copy(b_buf, B.agent, a_buf, A.agent, bytes, 0, nullptr, sig), "peer copy");
    if (!wait_signal(sig, timeout_s)) {
      in_flight = true;
      std::snprintf(out->error, sizeof(out->error), "peer copy %s -> %s did not complete within %.1fs",
                    out->src_bus_id, out->dst_bus_id, timeout_s);
      out->hsa_error = -1;
      goto done;
    }
    const double us = std::chrono::duration<double, std::micro>(clk::now() - tc).count();
    if (us < out->copy_us_best) out->copy_us_best = us;
  }
  out->gbps_best = static_cast<double>(bytes) / (out->copy_us_best * 1e3);
  H().hsa_signal_store_screlease(sig, 1);
  PEER_CHECK(H().hsa_amd_memory_async_copy(h_buf, g_rt.cpu, b_buf, B.agent, bytes, 0, nullptr, sig), "readback");
  if (!wait_signal(sig, timeout_s)) {
    in_flight = true;
    std::snprintf(out->error, sizeof(out->error), "readback from %s did not complete within %.1fs", out->dst_bus_id,
                  timeout_s);
    out->hsa_error = -1;
    goto done;
  }
  for (uint64_t i = 0; i < bytes / 4; ++i) out->mismatches += h_buf[i] != out->value;
  out->ok = out->mismatches == 0;
  if (!out->ok)
    std::snprintf(out->error, sizeof(out->error), "%llu/%llu words differ after %s -> %s copy",
                  static_cast<unsigned long long>(out->mismatches), static_cast<unsigned long long>(bytes / 4),
                  out->src_bus_id, out->dst_bus_id);
#undef PEER_CHECK
done:
  if (!in_flight) {
    if (sig.handle) H().hsa_signal_destroy(sig);
    if (h_buf) H().hsa_amd_memory_pool_free(h_buf);
    if (b_buf) H().hsa_amd_memory_pool_free(b_buf);
    if (a_buf) H().hsa_amd_memory_pool_free(a_buf);
  }
  if (out->copy_us_best >= 1e29) out->copy_us_best = 0;
  out->total_us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
  return out->ok ? 0 : 1;
}

namespace {

// A chip sweep whose completion signal did not fire within its deadline: the
// dispatch may still write its records, so none of its resources can be freed
// until it completes. One per device at most (mi355x_hsa_chip_sweep refuses to
// submit another while it is outstanding).
struct SweepInFlight {
  hsa_code_object_reader_t reader{};  // null when the kept queue / executable were borrowed
  hsa_executable_t exe{};
  hsa_queue_t* queue = nullptr;
  std::shared_ptr<SigRef> sig;
  void* bufs[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  std::chrono::steady_clock::time_point since{};

  void release() {
    for (void* b : bufs)
      if (b) H().hsa_amd_memory_pool_free(b);
    if (queue) H().hsa_queue_destroy(queue);
    if (exe.handle) H().hsa_executable_destroy(exe);
    if (reader.handle) H().hsa_code_object_reader_destroy(reader);
    sig.reset();
  }
};
std::mutex g_sweep_mu;
std::vector<std::pair<int, SweepInFlight>> g_sweep_in_flight;

// > 0 (seconds outstanding) when an earlier sweep or throughput check on
// `ordinal` is still running; a completed one is freed here.
double in_flight_for(int ordinal) {
  std::lock_guard<std::mutex> lk(g_sweep_mu);
  for (auto it = g_sweep_in_flight.begin(); it != g_sweep_in_flight.end(); ++it) {
    if (it->first != ordinal) continue;
    if (H().hsa_signal_load_scacquire(it->second.sig->s) < 1) {
      it->second.release();
      g_sweep_in_flight.erase(it);
      return 0;
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - it->second.since).count();
    return s > 0 ? s : 1e-9;
  }
  return 0;
}

template <typename R>
bool sweep_still_in_flight(int ordinal, R* out) {
  const double s = in_flight_for(ordinal);
  if (s <= 0) return false;
  out->in_flight_s = s;
  out->hsa_error = -1;
  std::snprintf(out->error, sizeof(out->error), "earlier chip sweep / check still in flight for %.1fs (not completed)",
                s);
  return true;
}

// runtime shutdown: an outstanding sweep's resources go with the runtime
void forget_in_flight_sweeps() {
  std::lock_guard<std::mutex> lk(g_sweep_mu);
  // a dispatch still running may yet decrement its completion signal: leave
  // the signal to the runtime's own teardown instead of destroying it here
  for (auto& e : g_sweep_in_flight)
    if (e.second.sig && e.second.sig->s.handle && H().hsa_signal_load_scacquire(e.second.sig->s) >= 1)
      e.second.sig->s = hsa_signal_t{};
  g_sweep_in_flight.clear();
}

}  // namespace

namespace {

// One AQL kernel dispatch (barrier bit, system-scope fences), no wait.
void submit_kernel(hsa_queue_t* queue, uint64_t kobj, uint32_t gseg, uint32_t pseg, void* kargs, uint32_t wgs,
                   uint32_t wg_threads, hsa_signal_t sig) {
  H().hsa_signal_store_screlease(sig, 1);
  const uint64_t idx = H().hsa_queue_add_write_index_screlease(queue, 1);
  auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(queue->base_address) + (idx & (queue->size - 1));
  std::memset(reinterpret_cast<char*>(pkt) + 4, 0, sizeof(*pkt) - 4);
  pkt->workgroup_size_x = static_cast<uint16_t>(wg_threads);
  pkt->workgroup_size_y = 1;
  pkt->workgroup_size_z = 1;
  pkt->grid_size_x = wgs * wg_threads;
  pkt->grid_size_y = 1;
  pkt->grid_size_z = 1;
  pkt->private_segment_size = pseg;
  pkt->group_segment_size = gseg;
  pkt->kernel_object = kobj;
  pkt->kernarg_address = kargs;
  pkt->completion_signal = sig;
  const uint16_t header = static_cast<uint16_t>(
      (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
      (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
      (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), header | (static_cast<uint32_t>(setup) << 16), __ATOMIC_RELEASE);
  H().hsa_signal_store_screlease(queue->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
}

double dispatch_us(const Agent& ag, hsa_signal_t sig) {
  hsa_amd_profiling_dispatch_time_t dt{};
  if (H().hsa_amd_profiling_get_dispatch_time(ag.agent, sig, &dt) != HSA_STATUS_SUCCESS || !g_rt.ts_freq) return 0;
  return static_cast<double>(dt.end - dt.start) * 1e6 / static_cast<double>(g_rt.ts_freq);
}

double median_of(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

struct KernelSym {
  uint64_t kobj = 0;
  uint32_t kseg = 0, gseg = 0, pseg = 0;
};

// The queue and executable a chip sweep or throughput check runs on. With kept
// resources (--serve --keep) the device's kept queue and executable are
// borrowed -- set up here if no probe has yet -- so the check adds no kfd
// queue: no 181 MB context-save area, no HWS runlist update. The slot's mutex
// is held meanwhile, so no probe packet interleaves. Otherwise a private queue
// and executable are created for the check and destroyed after it.
struct DeviceWork {
  explicit DeviceWork(const Agent& a) : ag(a) {}
  DeviceWork(const DeviceWork&) = delete;
  DeviceWork& operator=(const DeviceWork&) = delete;
  ~DeviceWork() {
    if (abandoned || borrowed()) return;
    if (queue) H().hsa_queue_destroy(queue);
    if (exe.handle) H().hsa_executable_destroy(exe);
    if (reader.handle) H().hsa_code_object_reader_destroy(reader);
  }
  bool borrowed() const { return slot != nullptr; }

  hsa_status_t open(int ordinal, const char** what) {
    bool keep;
    {
      std::lock_guard<std::mutex> lk(g_resident_mu);
      keep = g_keep;
    }
    if (keep) {
      Resident* s = resident_slot(ordinal);
      std::unique_lock<std::mutex> lk(s->mu);
      if (!s->ready && !s->pending && !s->blocker) {
        mi355x_probe_result scratch;
        std::memset(&scratch, 0, sizeof(scratch));
        if (setup_resources(ag, s->r, s->k, &scratch))
          s->ready = true;
        else
          s->r.release();
      }
      if (s->ready && !s->pending && !s->blocker) {
        slot = s;
        slot_lk = std::move(lk);
        exe = s->r.exe;
        queue = s->r.queue;
      }
    }
    hsa_status_t st = HSA_STATUS_SUCCESS;
    if (!borrowed()) {
      const size_t co_size = static_cast<size_t>(mi355x_hsaco_end - mi355x_hsaco_start);
      if ((st = H().hsa_code_object_reader_create_from_memory(mi355x_hsaco_start, co_size, &reader)) != 0)
        return *what = "code object", st;
      if ((st = H().hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr,
                                              &exe)) != 0)
        return *what = "executable create", st;
      if ((st = H().hsa_executable_load_agent_code_object(exe, ag.agent, reader, nullptr, nullptr)) != 0)
        return *what = "load code object", st;
      if ((st = H().hsa_executable_freeze(exe, nullptr)) != 0) return *what = "freeze", st;
      if ((st = H().hsa_queue_create(ag.agent, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX,
                                     &queue)) != 0)
        return *what = "queue create", st;
      H().hsa_amd_profiling_set_profiler_enabled(queue, 1);
    }
    if ((st = H().hsa_signal_create(1, 0, nullptr, &sig->s)) != 0) return *what = "signal create", st;
    return st;
  }

  hsa_status_t symbol(const char* name, KernelSym* k) {
    hsa_executable_symbol_t sym{};
    const hsa_status_t st = H().hsa_executable_get_symbol_by_name(exe, name, &ag.agent, &sym);
    if (st != HSA_STATUS_SUCCESS) return st;
    H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->kobj);
    H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->kseg);
    H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->gseg);
    H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->pseg);
    return st;
  }

  void submit(const KernelSym& k, void* kargs, uint32_t wgs, uint32_t wg_threads) {
    submit_kernel(queue, k.kobj, k.gseg, k.pseg, kargs, wgs, wg_threads, sig->s);
  }

  // A dispatch did not complete within its deadline: everything it may still
  // write goes to the in-flight registry (at most one per device: later sweeps
  // and checks fail fast until it completes), and a borrowed kept queue blocks
  // probes until then.
  void abandon(int ordinal, std::initializer_list<void*> bufs, std::chrono::steady_clock::time_point since) {
    abandoned = true;
    SweepInFlight f;
    if (!borrowed()) {
      f.reader = reader;
      f.exe = exe;
      f.queue = queue;
    }
    f.sig = sig;
    int i = 0;
    for (void* b : bufs)
      if (i < 6) f.bufs[i++] = b;
    f.since = since;
    {
      std::lock_guard<std::mutex> lk(g_sweep_mu);
      g_sweep_in_flight.emplace_back(ordinal, f);
    }
    if (borrowed()) {
      slot->blocker = sig;
      slot->blocked_since = since;  // when the sweep / check was submitted
    }
  }

  const Agent& ag;
  Resident* slot = nullptr;
  std::unique_lock<std::mutex> slot_lk;
  hsa_code_object_reader_t reader{};
  hsa_executable_t exe{};
  hsa_queue_t* queue = nullptr;
  std::shared_ptr<SigRef> sig = std::make_shared<SigRef>();
  bool abandoned = false;
};

void set_hsa_error(int* err, char* buf, size_t n, hsa_status_t st, const char* what) {
  *err = static_cast<int>(st);
  const char* msg = nullptr;
  H().hsa_status_string(st, &msg);
  std::snprintf(buf, n, "%s: %s", what, msg ? msg : "hsa error");
}

}  // namespace

extern "C" int mi355x_hsa_chip_sweep(int ordinal, uint32_t nonce, int iters, double timeout_s,
                                     mi355x_sweep_result* out) {
  using clk = std::chrono::steady_clock;
  std::memset(out, 0, sizeof(*out));
  out->ordinal = ordinal;
  out->nonce = nonce;
  out->iters = iters < 1 ? 1 : (iters > 64 ? 64 : iters);
  const auto t0 = clk::now();
  auto finish = [&] {
    out->total_us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
    return out->ok ? 0 : 1;
  };
  const int n = mi355x_hsa_probe_init();
  if (n < 0) {
    out->hsa_error = n;
    std::snprintf(out->error, sizeof(out->error), "hsa_init: %.140s", H().loaded ? "runtime init failed" : H().error);
    return 1;
  }
  if (ordinal < 0 || ordinal >= n) {
    std::snprintf(out->error, sizeof(out->error), "no such GPU agent (count=%d)", n);
    return 1;
  }
  if (sweep_still_in_flight(ordinal, out)) return finish();
  const Agent& ag = g_rt.gpus[ordinal];
  uint32_t cus = 0, xcc = 0;
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT), &cus);
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NUM_XCC), &xcc);
  out->cu_count = static_cast<int>(cus);
  out->num_xcc = static_cast<int>(xcc);
  if (cus == 0 || cus > 1024 || !g_rt.has_fine || !g_rt.has_kernarg || !ag.has_coarse) {
    std::snprintf(out->error, sizeof(out->error), "unexpected agent (cus=%u) or missing memory pool", cus);
    return 1;
  }
  const uint32_t grid = cus;
  out->grid = static_cast<int>(grid);

  DeviceWork dw(ag);
  const char* what = "";
  hsa_status_t s = dw.open(ordinal, &what);
  if (s != HSA_STATUS_SUCCESS) {
    set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, what);
    return finish();
  }
  out->kept_queue = dw.borrowed() ? 1 : 0;
  KernelSym ksym;
  if ((s = dw.symbol("mi355x_chip_sweep.kd", &ksym)) != HSA_STATUS_SUCCESS) {
    set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, "kernel symbol");
    return finish();
  }
  if (ksym.kseg < sizeof(mi355x_sweep_args) || ksym.kseg > kKernargBytes) {
    std::snprintf(out->error, sizeof(out->error), "sweep kernarg segment %u: code object / host ABI mismatch", ksym.kseg);
    return finish();
  }
  uint32_t* records = nullptr;
  float* tiles = nullptr;
  uint32_t* arrive = nullptr;
  mi355x_sweep_args* kargs = nullptr;
  const size_t rec_bytes = static_cast<size_t>(grid) * MI355X_SWEEP_REC_WORDS * sizeof(uint32_t);
  const size_t tile_bytes = static_cast<size_t>(grid) * MI355X_PROBE_OUT * sizeof(float);
  auto free_bufs = [&] {
    if (kargs) H().hsa_amd_memory_pool_free(kargs);
    if (arrive) H().hsa_amd_memory_pool_free(arrive);
    if (tiles) H().hsa_amd_memory_pool_free(tiles);
    if (records) H().hsa_amd_memory_pool_free(records);
  };
#define SWEEP_CHECK(expr, label)                                                              \
  if ((s = (expr)) != HSA_STATUS_SUCCESS) {                                                   \
    set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, label);                 \
    free_bufs();                                                                              \
    return finish();                                                                          \
  }
  SWEEP_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.fine, rec_bytes, 0, reinterpret_cast<void**>(&records)),
              "alloc records");
  SWEEP_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.fine, tile_bytes, 0, reinterpret_cast<void**>(&tiles)),
              "alloc tiles");
  SWEEP_CHECK(H().hsa_amd_memory_pool_allocate(ag.coarse, 4096, 0, reinterpret_cast<void**>(&arrive)), "alloc arrive");
  SWEEP_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.kernarg, kKernargBytes, 0, reinterpret_cast<void**>(&kargs)),
              "alloc kernarg");
  SWEEP_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, records), "allow records");
  SWEEP_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, tiles), "allow tiles");
  SWEEP_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, kargs), "allow kernarg");
  SWEEP_CHECK(H().hsa_amd_memory_fill(arrive, 0u, 4096 / 4), "zero arrive");
#undef SWEEP_CHECK
  std::memset(records, 0, rec_bytes);
  std::memset(tiles, 0xFF, tile_bytes);
  std::memset(kargs, 0, kKernargBytes);
  kargs->records = records;
  kargs->tiles = tiles;
  kargs->arrive = arrive;
  kargs->nonce = nonce;
  kargs->iters = out->iters;
  kargs->grid = grid;
  kargs->wait_ticks = 2000000;  // 20 ms at the 100 MHz s_memrealtime clock
  dw.submit(ksym, kargs, grid, MI355X_SWEEP_THREADS);
  if (!wait_signal(dw.sig->s, timeout_s)) {
    std::snprintf(out->error, sizeof(out->error), "chip sweep did not complete within %.1fs", timeout_s);
    out->hsa_error = -1;
    dw.abandon(ordinal, {kargs, arrive, tiles, records}, t0);
    return finish();
  }
  out->kernel_us = dispatch_us(ag, dw.sig->s);
  {
    std::vector<uint32_t> keys;
    keys.reserve(grid);
    uint64_t tmin = UINT64_MAX, tmax = 0;
    uint32_t xmask = 0;
    bool all_res = true;
    std::vector<float> want(MI355X_PROBE_OUT);
    for (uint32_t w = 0; w < grid; ++w) {
      const uint32_t* r = records + static_cast<size_t>(w) * MI355X_SWEEP_REC_WORDS;
      const bool present = r[MI355X_REC_MAGIC] == MI355X_SWEEP_MAGIC && r[MI355X_REC_WG] == w &&
                           r[MI355X_REC_NONCE] == (nonce ^ w);
      if (!present) continue;
      out->mfma_bad += r[MI355X_REC_MFMA_BAD];
      out->lds_bad += r[MI355X_REC_LDS_BAD];
      const uint32_t x = r[MI355X_REC_XCC] & 0xF;
      xmask |= 1u << x;
      ++out->wgs_per_xcc[x];
      keys.push_back((x << 16) | ((r[MI355X_REC_HWID] >> 8) & 0xFF));
      all_res = all_res && r[MI355X_REC_ARRIVED] >= grid;
      const uint64_t t = (static_cast<uint64_t>(r[MI355X_REC_T0_HI]) << 32) | r[MI355X_REC_T0_LO];
      tmin = t < tmin ? t : tmin;
      tmax = t > tmax ? t : tmax;
      // wave 0's tile against the host reference
      const uint32_t nw = sweep_nonce(nonce, w, 0);
      uint32_t tb = 0;
      const float* tile = tiles + static_cast<size_t>(w) * MI355X_PROBE_OUT;
      for (int i = 0; i < MI355X_PROBE_M; ++i)
        for (int j = 0; j < MI355X_PROBE_N; ++j) {
          float dot = 0.f;
          for (int k = 0; k < MI355X_PROBE_K; ++k) dot += probe_a(i, k, nw) * probe_b(k, j, nw);
          const float e = probe_c(i, j, nw) + static_cast<float>(out->iters) * dot;
          tb += tile[i * MI355X_PROBE_N + j] != e;
        }
      out->tile_bad += tb;
      if (r[MI355X_REC_MFMA_BAD] == 0 && r[MI355X_REC_LDS_BAD] == 0 && tb == 0) ++out->records_ok;
    }
    std::sort(keys.begin(), keys.end());
    out->cus_covered = static_cast<int>(std::unique(keys.begin(), keys.end()) - keys.begin());
    out->xccs_covered = __builtin_popcount(xmask);
    out->all_resident = all_res && out->records_ok == static_cast<int>(grid);
    if (tmax >= tmin && tmin != UINT64_MAX) out->arrival_spread_us = static_cast<double>(tmax - tmin) / 100.0;
    out->ok = out->records_ok == static_cast<int>(grid) &&
              (out->num_xcc <= 0 || out->xccs_covered == out->num_xcc);
    if (!out->ok)
      std::snprintf(out->error, sizeof(out->error),
                    "%d/%d workgroups correct (mfma_bad=%u lds_bad=%u tile_bad=%u), %d/%d XCDs ran", out->records_ok,
                    grid, out->mfma_bad, out->lds_bad, out->tile_bad, out->xccs_covered, out->num_xcc);
  }
  free_bufs();
  return finish();
}

namespace {
std::atomic<uint64_t> g_perf_poison{~0ull};
}  // namespace

extern "C" void mi355x_hsa_perf_poison(uint64_t unit) { g_perf_poison.store(unit, std::memory_order_relaxed); }

extern "C" int mi355x_hsa_perf_check(int ordinal, uint32_t nonce, uint64_t bytes, int mfma_iters, double timeout_s,
                                     mi355x_perf_result* out) {
  using clk = std::chrono::steady_clock;
  std::memset(out, 0, sizeof(*out));
  out->ordinal = ordinal;
  out->nonce = nonce;
  out->hbm_first_bad = -1;
  // 16-byte units, at least one full grid-stride round, at most 64 GiB
  bytes = bytes < (64ull << 20) ? (64ull << 20) : (bytes > (64ull << 30) ? (64ull << 30) : bytes);
  bytes &= ~static_cast<uint64_t>(0xFFFFF);
  out->bytes = bytes;
  out->mfma_iters = mfma_iters < 1 ? 1 : (mfma_iters > (1 << 22) ? (1 << 22) : mfma_iters);
  const auto t0 = clk::now();
  auto finish = [&] {
    out->total_us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
    return out->ok ? 0 : 1;
  };
  const int n = mi355x_hsa_probe_init();
  if (n < 0) {
    out->hsa_error = n;
    std::snprintf(out->error, sizeof(out->error), "hsa_init: %.140s", H().loaded ? "runtime init failed" : H().error);
    return 1;
  }
  if (ordinal < 0 || ordinal >= n) {
    std::snprintf(out->error, sizeof(out->error), "no such GPU agent (count=%d)", n);
    return 1;
  }
  if (sweep_still_in_flight(ordinal, out)) return finish();
  const Agent& ag = g_rt.gpus[ordinal];
  uint32_t cus = 0, xcc = 0;
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT), &cus);
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NUM_XCC), &xcc);
  out->cu_count = static_cast<int>(cus);
  out->num_xcc = static_cast<int>(xcc);
  if (cus == 0 || cus > 1024 || !g_rt.has_fine || !g_rt.has_kernarg || !ag.has_coarse) {
    std::snprintf(out->error, sizeof(out->error), "unexpected agent (cus=%u) or missing memory pool", cus);
    return 1;
  }
  const uint32_t fill_wgs = cus * MI355X_HBM_FILL_WGS_PER_CU;
  const uint32_t check_wgs = cus * MI355X_HBM_CHECK_WGS_PER_CU;
  const uint32_t burn_wgs = cus * MI355X_BURN_WGS_PER_CU;
  out->mfma_grid = static_cast<int>(burn_wgs);

  DeviceWork w(ag);
  const char* what = "";
  hsa_status_t s = w.open(ordinal, &what);
  if (s != HSA_STATUS_SUCCESS) {
    set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, what);
    return finish();
  }
  out->kept_queue = w.borrowed() ? 1 : 0;
  KernelSym ks[3];
  const char* names[3] = {"mi355x_hbm_fill.kd", "mi355x_hbm_check.kd", "mi355x_mfma_burn.kd"};
  for (int i = 0; i < 3; ++i)
    if ((s = w.symbol(names[i], &ks[i])) != HSA_STATUS_SUCCESS) {
      set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, "kernel symbol");
      return finish();
    }
  if (ks[0].kseg < sizeof(mi355x_hbm_args) || ks[0].kseg > kKernargBytes || ks[1].kseg < sizeof(mi355x_hbm_args) ||
      ks[1].kseg > kKernargBytes || ks[2].kseg < sizeof(mi355x_burn_args) || ks[2].kseg > kKernargBytes) {
    std::snprintf(out->error, sizeof(out->error), "perf kernarg segments %u/%u/%u: code object / host ABI mismatch",
                  ks[0].kseg, ks[1].kseg, ks[2].kseg);
    return finish();
  }
  uint32_t* buf = nullptr;       // device, `bytes`
  uint32_t* counters = nullptr;  // device, [0] bad words, [2..3] first bad unit
  uint32_t* h_counters = nullptr;
  uint32_t* records = nullptr;   // host-visible, burn_wgs records
  char* kargs = nullptr;         // 3 slots of kKernargBytes
  const size_t rec_bytes = static_cast<size_t>(burn_wgs) * MI355X_PERF_REC_WORDS * sizeof(uint32_t);
  auto free_bufs = [&] {
    if (kargs) H().hsa_amd_memory_pool_free(kargs);
    if (records) H().hsa_amd_memory_pool_free(records);
    if (h_counters) H().hsa_amd_memory_pool_free(h_counters);
    if (counters) H().hsa_amd_memory_pool_free(counters);
    if (buf) H().hsa_amd_memory_pool_free(buf);
  };
  auto abandon = [&](const char* stage) {
    std::snprintf(out->error, sizeof(out->error), "%s did not complete within %.1fs", stage, timeout_s);
    out->hsa_error = -1;
    w.abandon(ordinal, {kargs, buf, counters, h_counters, records}, t0);
    return finish();
  };
#define PERF_CHECK(expr, label)                                                               \
  if ((s = (expr)) != HSA_STATUS_SUCCESS) {                                                   \
    set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, label);                 \
    free_bufs();                                                                              \
    return finish();                                                                          \
  }
  PERF_CHECK(H().hsa_amd_memory_pool_allocate(ag.coarse, bytes, 0, reinterpret_cast<void**>(&buf)), "alloc HBM buffer");
  PERF_CHECK(H().hsa_amd_memory_pool_allocate(ag.coarse, 4096, 0, reinterpret_cast<void**>(&counters)),
             "alloc counters");
  PERF_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.fine, 4096, 0, reinterpret_cast<void**>(&h_counters)),
             "alloc host counters");
  PERF_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.fine, rec_bytes, 0, reinterpret_cast<void**>(&records)),
             "alloc records");
  PERF_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.kernarg, 4 * kKernargBytes, 0, reinterpret_cast<void**>(&kargs)),
             "alloc kernarg");
  PERF_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, h_counters), "allow counters");
  PERF_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, records), "allow records");
  PERF_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, kargs), "allow kernarg");
  // counters: word 0 = 0 (bad words), words 2..3 = all ones (first bad unit)
  PERF_CHECK(H().hsa_amd_memory_fill(counters, 0u, 2), "zero counters");
  PERF_CHECK(H().hsa_amd_memory_fill(counters + 2, 0xFFFFFFFFu, 2), "init first-bad");
  std::memset(h_counters, 0xA5, 16);   // overwritten by the burn kernel's copy
  std::memset(records, 0, rec_bytes);
  std::memset(kargs, 0, 4 * kKernargBytes);
  {
    auto* fa = reinterpret_cast<mi355x_hbm_args*>(kargs);
    auto* ca = reinterpret_cast<mi355x_hbm_args*>(kargs + kKernargBytes);
    auto* ba = reinterpret_cast<mi355x_burn_args*>(kargs + 2 * kKernargBytes);
    auto* c2 = reinterpret_cast<mi355x_hbm_args*>(kargs + 3 * kKernargBytes);
    fa->buf = ca->buf = buf;
    fa->n16 = ca->n16 = bytes / 16;
    fa->bad = ca->bad = counters;
    fa->first_bad = ca->first_bad = reinterpret_cast<uint64_t*>(counters + 2);
    fa->threads = static_cast<uint64_t>(fill_wgs) * MI355X_PERF_THREADS;
    ca->threads = static_cast<uint64_t>(check_wgs) * MI355X_PERF_THREADS;
    fa->poison_unit = g_perf_poison.load(std::memory_order_relaxed);
    ca->poison_unit = ~0ull;
    fa->seed = ca->seed = nonce * 0x01000193u + 0x7F4A7C15u;
    *c2 = *ca;
    c2->bad = counters + 1;  // the second read pass counts on its own
    ba->records = records;
    ba->hbm_counters = counters;
    ba->hbm_counters_host = h_counters;
    ba->nonce = nonce;
    ba->iters = out->mfma_iters;
  }
  w.submit(ks[0], kargs, fill_wgs, MI355X_PERF_THREADS);
  if (!wait_signal(w.sig->s, timeout_s)) return abandon("HBM fill");
  out->fill_us = dispatch_us(ag, w.sig->s);
  w.submit(ks[1], kargs + kKernargBytes, check_wgs, MI355X_PERF_THREADS);
  if (!wait_signal(w.sig->s, timeout_s)) return abandon("HBM check");
  out->check_us = dispatch_us(ag, w.sig->s);
  // a second read pass: steady-state read bandwidth (the first one still
  // competes with the fill's write-back) and a second look at every word
  w.submit(ks[1], kargs + 3 * kKernargBytes, check_wgs, MI355X_PERF_THREADS);
  if (!wait_signal(w.sig->s, timeout_s)) return abandon("HBM check (2nd pass)");
  out->check2_us = dispatch_us(ag, w.sig->s);
  w.submit(ks[2], kargs + 2 * kKernargBytes, burn_wgs, MI355X_PERF_THREADS);
  if (!wait_signal(w.sig->s, timeout_s)) return abandon("MFMA burn");
  out->mfma_us = dispatch_us(ag, w.sig->s);
#undef PERF_CHECK
  {
    out->hbm_bad_words = h_counters[0] > h_counters[1] ? h_counters[0] : h_counters[1];
    out->hbm_bad_words_pass2 = h_counters[1];
    const uint64_t first = (static_cast<uint64_t>(h_counters[3]) << 32) | h_counters[2];
    out->hbm_first_bad = first == ~0ull ? -1 : static_cast<int64_t>(first);
    if (out->fill_us > 0) out->hbm_write_gbps = static_cast<double>(bytes) / (out->fill_us * 1e3);
    const double best_check = out->check2_us > 0 && out->check2_us < out->check_us ? out->check2_us : out->check_us;
    if (best_check > 0) out->hbm_read_gbps = static_cast<double>(bytes) / (best_check * 1e3);
    const double flops = 2.0 * 32 * 32 * 16 * 2.0 * static_cast<double>(out->mfma_iters) *
                         (MI355X_PERF_THREADS / 64) * static_cast<double>(burn_wgs);
    if (out->mfma_us > 0) out->mfma_tflops = flops / (out->mfma_us * 1e6);
    std::vector<double> clocks;
    std::vector<std::vector<double>> per_xcd(16);
    uint32_t ref = 0;
    bool have_ref = false;
    uint32_t xmask = 0;
    for (uint32_t wg = 0; wg < burn_wgs; ++wg) {
      const uint32_t* r = records + static_cast<size_t>(wg) * MI355X_PERF_REC_WORDS;
      if (r[MI355X_PREC_MAGIC] != MI355X_PERF_MAGIC || r[MI355X_PREC_WG] != wg ||
          r[MI355X_PREC_NONCE] != (nonce ^ wg))
        continue;
      ++out->mfma_records_ok;
      for (int v = 0; v < MI355X_PERF_THREADS / 64; ++v) {
        if (!have_ref) {
          ref = r[MI355X_PREC_SUM + v];
          have_ref = true;
        } else if (r[MI355X_PREC_SUM + v] != ref) {
          ++out->mfma_checksum_mismatch;
        }
      }
      const uint64_t rt0 = (static_cast<uint64_t>(r[MI355X_PREC_RT0_HI]) << 32) | r[MI355X_PREC_RT0_LO];
      const uint64_t rt1 = (static_cast<uint64_t>(r[MI355X_PREC_RT1_HI]) << 32) | r[MI355X_PREC_RT1_LO];
      const uint64_t cyc = (static_cast<uint64_t>(r[MI355X_PREC_CYC_HI]) << 32) | r[MI355X_PREC_CYC_LO];
      const uint32_t x = r[MI355X_PREC_XCC] & 0xF;
      xmask |= 1u << x;
      if (rt1 > rt0) {
        const double mhz = static_cast<double>(cyc) / (static_cast<double>(rt1 - rt0) / 100.0);  // ticks per us
        clocks.push_back(mhz);
        per_xcd[x].push_back(mhz);
      }
    }
    out->mfma_xccs = __builtin_popcount(xmask);
    if (!clocks.empty()) {
      out->clock_mhz_min = *std::min_element(clocks.begin(), clocks.end());
      out->clock_mhz_max = *std::max_element(clocks.begin(), clocks.end());
      out->clock_mhz_median = median_of(clocks);
    }
    for (int x = 0; x < 16; ++x) out->xcd_clock_mhz[x] = median_of(per_xcd[x]);
    out->ok = out->hbm_bad_words == 0 && out->mfma_checksum_mismatch == 0 &&
              out->mfma_records_ok == static_cast<int>(burn_wgs) &&
              (out->num_xcc <= 0 || out->mfma_xccs == out->num_xcc);
    if (!out->ok)
      std::snprintf(out->error, sizeof(out->error),
                    "hbm_bad_words=%llu first_bad_unit=%lld mfma records %d/%u checksum mismatches %d, %d/%d XCDs ran",
                    static_cast<unsigned long long>(out->hbm_bad_words), static_cast<long long>(out->hbm_first_bad),
                    out->mfma_records_ok, burn_wgs, out->mfma_checksum_mismatch, out->mfma_xccs, out->num_xcc);
  }
  free_bufs();
  return finish();
}
