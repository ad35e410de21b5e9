// Host launcher + bit-exact verification for the MFMA liveness kernel.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "liveness_kernel.h"
#include "mi355x/liveness_probe.h"

extern "C" __global__ void mi355x_mfma_liveness(float* out, uint32_t* meta, uint32_t nonce, int iters);

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
  hipDeviceGetPCIBusId(out->pci_bus_id, sizeof(out->pci_bus_id), ordinal);
}

}  // namespace

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
  float* d_out = nullptr;
  uint32_t* d_meta = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipStream_t stream = nullptr;
  std::vector<float> h(MI355X_PROBE_OUT, 0.f);
  uint32_t meta[MI355X_META_WORDS] = {0, 0, 0, 0};
  int mism = 0;
  float ms = 0.f;

  PROBE_CHECK(hipSetDevice(ordinal), "hipSetDevice");
  fill_identity(ordinal, out);
  PROBE_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
  PROBE_CHECK(hipMalloc(&d_out, MI355X_PROBE_OUT * sizeof(float)), "hipMalloc(out)");
  PROBE_CHECK(hipMalloc(&d_meta, MI355X_META_WORDS * sizeof(uint32_t)), "hipMalloc(meta)");
  // poison so a kernel that never runs cannot pass
  PROBE_CHECK(hipMemsetAsync(d_out, 0xFF, MI355X_PROBE_OUT * sizeof(float), stream), "hipMemset(out)");
  PROBE_CHECK(hipMemsetAsync(d_meta, 0, MI355X_META_WORDS * sizeof(uint32_t), stream), "hipMemset(meta)");
  PROBE_CHECK(hipEventCreate(&ev0), "hipEventCreate");
  PROBE_CHECK(hipEventCreate(&ev1), "hipEventCreate");
  PROBE_CHECK(hipEventRecord(ev0, stream), "hipEventRecord");
  hipLaunchKernelGGL(mi355x_mfma_liveness, dim3(1), dim3(64), 0, stream, d_out, d_meta, nonce, out->iters);
  PROBE_CHECK(hipGetLastError(), "launch");
  PROBE_CHECK(hipEventRecord(ev1, stream), "hipEventRecord");
  PROBE_CHECK(hipMemcpyAsync(h.data(), d_out, MI355X_PROBE_OUT * sizeof(float), hipMemcpyDeviceToHost, stream),
              "hipMemcpy(out)");
  PROBE_CHECK(hipMemcpyAsync(meta, d_meta, sizeof(meta), hipMemcpyDeviceToHost, stream), "hipMemcpy(meta)");
  PROBE_CHECK(hipStreamSynchronize(stream), "hipStreamSynchronize");
  PROBE_CHECK(hipEventElapsedTime(&ms, ev0, ev1), "hipEventElapsedTime");
  out->kernel_us = ms * 1000.0;

  // host reference: D = C + iters * A·B, exact in f32 for these magnitudes
  for (int i = 0; i < MI355X_PROBE_M; ++i)
    for (int j = 0; j < MI355X_PROBE_N; ++j) {
      float ab = 0.f;
      for (int k = 0; k < MI355X_PROBE_K; ++k) ab += probe_a(i, k, nonce) * probe_b(k, j, nonce);
      float want = probe_c(i, j, nonce) + static_cast<float>(out->iters) * ab;
      if (h[i * MI355X_PROBE_N + j] != want) ++mism;
    }
  out->mismatches = mism;
  out->xcc_id = meta[MI355X_META_XCC];
  out->hw_id = meta[MI355X_META_HWID];
  if (meta[MI355X_META_MAGIC] != MI355X_PROBE_MAGIC || meta[MI355X_META_NONCE] != nonce) {
    std::snprintf(out->error, sizeof(out->error), "meta mismatch: magic=%08x nonce=%u", meta[MI355X_META_MAGIC],
                  meta[MI355X_META_NONCE]);
  } else if (mism) {
    std::snprintf(out->error, sizeof(out->error), "%d/%d MFMA results differ from host reference", mism,
                  MI355X_PROBE_OUT);
  } else {
    out->ok = 1;
  }

done:
  if (ev0) hipEventDestroy(ev0);
  if (ev1) hipEventDestroy(ev1);
  if (d_out) hipFree(d_out);
  if (d_meta) hipFree(d_meta);
  if (stream) hipStreamDestroy(stream);
  out->total_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  return out->ok ? 0 : 1;
}
