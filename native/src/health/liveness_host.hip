// HIP launcher for the MFMA liveness kernel.
//
// Output and meta live in coherent pinned host memory and are poisoned by the
// CPU, so the probe issues exactly ONE GPU dispatch (no memset/blit kernels —
// the first version issued five, see profiles/archive/measurements_r1_r3.md §1).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "liveness_kernel.h"
#include "mi355x/liveness_probe.h"
#include "probe_verify.h"

extern "C" __global__ void mi355x_mfma_liveness(float* out, uint32_t* meta, float* scratch, uint32_t nonce,
                                                int iters);

namespace {

void set_error(mi355x_probe_result* r, hipError_t e, const char* what) {
  if (r->hip_error == 0) r->hip_error = static_cast<int>(e);
  std::snprintf(r->error, sizeof(r->error), "%s: %s", what, hipGetErrorString(e));
}

#define PROBE_CHECK(expr, what)          \
  do {                                   \
    hipError_t _e = (expr);              \
    if (_e != hipSuccess) {              \
      set_error(out, _e, what);          \
      goto done;                         \
    }                                    \
  } while (0)

void fill_identity(int ordinal, mi355x_probe_result* out) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, ordinal) == hipSuccess) {
    std::snprintf(out->arch, sizeof(out->arch), "%s", p.gcnArchName);
    std::snprintf(out->name, sizeof(out->name), "%s", p.name);
    out->pci_domain = p.pciDomainID;
    out->pci_bus = p.pciBusID;
    out->pci_device = p.pciDeviceID;
    out->cu_count = p.multiProcessorCount;
    out->total_mem = p.totalGlobalMem;
    char* u = out->uuid;
    for (int i = 0; i < 16 && i * 2 + 2 < static_cast<int>(sizeof(out->uuid)); ++i)
      std::snprintf(u + 2 * i, 3, "%02x", static_cast<unsigned char>(p.uuid.bytes[i]));
  }
  (void)hipDeviceGetPCIBusId(out->pci_bus_id, sizeof(out->pci_bus_id), ordinal);
  out->kfd_node_id = -1;
  std::snprintf(out->runtime, sizeof(out->runtime), "hip");
}

int g_own_stream = 1;

// What one probe allocated, freed after the verdict (now, or after the JSON
// line with mi355x_probe_defer_release)
struct HipResources {
  float* h_out = nullptr;
  uint32_t* h_meta = nullptr;
  float* d_scratch = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipStream_t stream = nullptr;

  void release() const {
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (h_out) (void)hipHostFree(h_out);
    if (h_meta) (void)hipHostFree(h_meta);
    if (d_scratch) (void)hipFree(d_scratch);
    if (stream) (void)hipStreamDestroy(stream);
  }
};
std::mutex g_deferred_mu;  // probes of several devices run on parallel threads
bool g_defer_release = false;
std::vector<HipResources> g_deferred;

}  // namespace

extern "C" void mi355x_probe_defer_release(int on) {
  std::lock_guard<std::mutex> lk(g_deferred_mu);
  g_defer_release = on != 0;
}

extern "C" void mi355x_probe_release(void) {
  std::vector<HipResources> todo;
  {
    std::lock_guard<std::mutex> lk(g_deferred_mu);
    todo.swap(g_deferred);
  }
  for (const auto& r : todo) r.release();
}

extern "C" void mi355x_probe_set_stream_mode(int own) { g_own_stream = own ? 1 : 0; }

extern "C" int mi355x_probe_device_count(void) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) return -static_cast<int>(e);
  return n;
}

extern "C" int mi355x_probe_identify(int ordinal, mi355x_probe_result* out) {
  std::memset(out, 0, sizeof(*out));
  out->ordinal = ordinal;
  hipError_t e = hipSetDevice(ordinal);
  if (e != hipSuccess) {
    set_error(out, e, "hipSetDevice");
    return 1;
  }
  fill_identity(ordinal, out);
  return 0;
}

extern "C" int mi355x_probe_device(int ordinal, uint32_t nonce, int iters, mi355x_probe_result* out) {
  std::memset(out, 0, sizeof(*out));
  out->ordinal = ordinal;
  out->nonce = nonce;
  out->iters = iters < 1 ? 1 : iters;
  const auto t0 = std::chrono::steady_clock::now();
  auto t_setup = t0;
  float* h_out = nullptr;
  uint32_t* h_meta = nullptr;
  float* d_scratch = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipStream_t stream = nullptr;
  float ms = 0.f;

  // phase_us: [device (hipSetDevice + identity), stream (its hardware queue), buffers (pinned +
  // device memory, events), dispatch_wait (launch -> tile back)], as the HSA path reports them
  auto lap = [&, t = t0]() mutable {
    const auto now = std::chrono::steady_clock::now();
    const double us = std::chrono::duration<double, std::micro>(now - t).count();
    t = now;
    return us;
  };
  PROBE_CHECK(hipSetDevice(ordinal), "hipSetDevice");
  fill_identity(ordinal, out);
  out->phase_us[0] = lap();
  if (g_own_stream) PROBE_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
  out->phase_us[1] = lap();
  PROBE_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_out), MI355X_PROBE_OUT * sizeof(float),
                            hipHostMallocCoherent),
              "hipHostMalloc(out)");
  PROBE_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_meta), MI355X_META_WORDS * sizeof(uint32_t),
                            hipHostMallocCoherent),
              "hipHostMalloc(meta)");
  PROBE_CHECK(hipMalloc(reinterpret_cast<void**>(&d_scratch), MI355X_SCRATCH_FLOATS * sizeof(float)),
              "hipMalloc(scratch)");
  // poison from the CPU so a kernel that never ran cannot pass
  std::memset(h_out, 0xFF, MI355X_PROBE_OUT * sizeof(float));
  std::memset(h_meta, 0, MI355X_META_WORDS * sizeof(uint32_t));
  PROBE_CHECK(hipEventCreate(&ev0), "hipEventCreate");
  PROBE_CHECK(hipEventCreate(&ev1), "hipEventCreate");
  t_setup = std::chrono::steady_clock::now();
  out->phase_us[2] = lap();
  PROBE_CHECK(hipEventRecord(ev0, stream), "hipEventRecord");
  hipLaunchKernelGGL(mi355x_mfma_liveness, dim3(1), dim3(64), 0, stream, h_out, h_meta, d_scratch, nonce,
                     out->iters);
  out->dispatches = 1;
  PROBE_CHECK(hipGetLastError(), "launch");
  PROBE_CHECK(hipEventRecord(ev1, stream), "hipEventRecord");
  PROBE_CHECK(hipStreamSynchronize(stream), "hipStreamSynchronize");
  out->phase_us[3] = lap();
  PROBE_CHECK(hipEventElapsedTime(&ms, ev0, ev1), "hipEventElapsedTime");
  out->kernel_us = ms * 1000.0;
  mi355x::verify_tile(h_out, h_meta, nonce, out->iters, out);

done:
  out->setup_us = std::chrono::duration<double, std::micro>(t_setup - t0).count();
  out->total_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  {
    const HipResources r{h_out, h_meta, d_scratch, ev0, ev1, stream};
    std::unique_lock<std::mutex> lk(g_deferred_mu);
    if (g_defer_release) {
      g_deferred.push_back(r);
    } else {
      lk.unlock();
      r.release();
    }
  }
  return out->ok ? 0 : 1;
}
