// Write shapes for the throughput check's fill pass (tools/archive/experiments/gpurun_hbm_variants.sh):
// 16 B per lane grid-stride (current) vs 64 B contiguous per lane, dword stores, and grid sizes.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ inline uint32_t pat(uint64_t w, uint32_t s) { return (uint32_t)(w ^ (w >> 32)) * 0x9E3779B1u + s; }
__device__ inline u32x4 val(uint64_t i, uint32_t s) {
  u32x4 v; v.x = pat(i * 4, s); v.y = pat(i * 4 + 1, s); v.z = pat(i * 4 + 2, s); v.w = pat(i * 4 + 3, s); return v;
}

// current: one 16-byte unit per lane per iteration, grid-stride
__global__ __launch_bounds__(256) void fill16(u32x4* buf, uint64_t n, uint64_t stride, uint32_t s) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) buf[i] = val(i, s);
}
// a wave writes 4 KiB contiguous per iteration: lane l stores units base+l, base+64+l, base+128+l, base+192+l
__global__ __launch_bounds__(256) void fill_wave4k(u32x4* buf, uint64_t n, uint64_t waves, uint32_t s) {
  const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t base = wave * 256; base < n; base += waves * 256) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t i = base + u * 64 + lane;
      if (i < n) buf[i] = val(i, s);
    }
  }
}
// dword stores: 256 B per wave-instruction
__global__ __launch_bounds__(256) void fill4(uint32_t* buf, uint64_t nw, uint64_t stride, uint32_t s) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += stride) buf[i] = pat(i, s);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  const uint64_t bytes = 8ull << 30, n = bytes / 16;
  u32x4* buf;
  CK(hipMalloc(&buf, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timeit = [&](const char* name, int wpc, auto launch) {
    const uint32_t wgs = cus * wpc;
    std::vector<float> ms;
    for (int r = 0; r < 6; ++r) {
      (void)hipEventRecord(a);
      launch(wgs);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float t;
      (void)hipEventElapsedTime(&t, a, b);
      ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::printf("{\"kernel\":\"%s\",\"wgs_per_cu\":%d,\"tbps_best\":%.2f,\"tbps_median\":%.2f}\n", name, wpc,
                bytes / (ms[0] * 1e9), bytes / (ms[3] * 1e9));
    std::fflush(stdout);
  };
  for (int wpc : {1, 2, 4, 8}) {
    timeit("fill16", wpc, [&](uint32_t g) { fill16<<<g, 256>>>(buf, n, (uint64_t)g * 256, 7); });
    timeit("fill_wave4k", wpc, [&](uint32_t g) { fill_wave4k<<<g, 256>>>(buf, n, (uint64_t)g * 4, 7); });
    timeit("fill4", wpc, [&](uint32_t g) { fill4<<<g, 256>>>((uint32_t*)buf, n * 4, (uint64_t)g * 256, 7); });
  }
  return 0;
}
