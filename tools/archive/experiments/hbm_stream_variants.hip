// Store / load shapes for the throughput check's HBM kernels (tools/archive/gpurun_perfcheck.sh):
// which one reaches the achievable HBM rate on MI355X. hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ inline uint32_t pat(uint64_t w, uint32_t s) { return (uint32_t)(w ^ (w >> 32)) * 0x9E3779B1u + s; }
__device__ inline u32x4 val(uint64_t i, uint32_t s) { u32x4 v; v.x = pat(i*4, s); v.y = pat(i*4+1, s); v.z = pat(i*4+2, s); v.w = pat(i*4+3, s); return v; }

template <int NT, int UNROLL>
__global__ __launch_bounds__(256) void fill(u32x4* buf, uint64_t n, uint64_t stride, uint32_t s) {
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (NT) __builtin_nontemporal_store(val(i + u * stride, s), &buf[i + u * stride]);
      else buf[i + u * stride] = val(i + u * stride, s);
    }
  }
  for (; i < n; i += stride) buf[i] = val(i, s);
}

template <int NT, int UNROLL>
__global__ __launch_bounds__(256) void check(const u32x4* buf, uint64_t n, uint64_t stride, uint32_t s, uint32_t* bad) {
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t b = 0;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = NT ? __builtin_nontemporal_load(&buf[i + u * stride]) : buf[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) { u32x4 e = val(i + u * stride, s); b += (v[u].x != e.x) + (v[u].y != e.y) + (v[u].z != e.z) + (v[u].w != e.w); }
  }
  for (; i < n; i += stride) { u32x4 v = buf[i], e = val(i, s); b += (v.x != e.x) + (v.y != e.y) + (v.z != e.z) + (v.w != e.w); }
  if (b) atomicAdd(bad, b);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  const uint64_t bytes = 8ull << 30, n = bytes / 16;
  u32x4* buf; uint32_t* bad;
  CK(hipMalloc(&buf, bytes)); CK(hipMalloc(&bad, 4)); CK(hipMemset(bad, 0, 4));
  int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto timeit = [&](const char* name, int wpc, auto launch) {
    const uint32_t wgs = cus * wpc; const uint64_t stride = (uint64_t)wgs * 256;
    std::vector<float> ms;
    for (int r = 0; r < 6; ++r) { hipEventRecord(a); launch(wgs, stride); hipEventRecord(b); hipEventSynchronize(b); float t; hipEventElapsedTime(&t, a, b); ms.push_back(t); }
    std::sort(ms.begin(), ms.end());
    std::printf("{\"kernel\":\"%s\",\"wgs_per_cu\":%d,\"ms_best\":%.3f,\"tbps_best\":%.2f,\"tbps_median\":%.2f}\n", name, wpc, ms[0], bytes / (ms[0] * 1e9), bytes / (ms[3] * 1e9));
    std::fflush(stdout);
  };
  for (int wpc : {4, 8, 16}) {
    timeit("fill_nt_u1", wpc, [&](uint32_t g, uint64_t s) { fill<1, 1><<<g, 256>>>(buf, n, s, 7); });
    timeit("fill_nt_u4", wpc, [&](uint32_t g, uint64_t s) { fill<1, 4><<<g, 256>>>(buf, n, s, 7); });
    timeit("fill_plain_u1", wpc, [&](uint32_t g, uint64_t s) { fill<0, 1><<<g, 256>>>(buf, n, s, 7); });
    timeit("fill_plain_u4", wpc, [&](uint32_t g, uint64_t s) { fill<0, 4><<<g, 256>>>(buf, n, s, 7); });
  }
  fill<0, 1><<<cus * 8, 256>>>(buf, n, (uint64_t)cus * 8 * 256, 7);
  for (int wpc : {4, 8, 16}) {
    timeit("check_nt_u4", wpc, [&](uint32_t g, uint64_t s) { check<1, 4><<<g, 256>>>(buf, n, s, 7, bad); });
    timeit("check_nt_u8", wpc, [&](uint32_t g, uint64_t s) { check<1, 8><<<g, 256>>>(buf, n, s, 7, bad); });
    timeit("check_plain_u4", wpc, [&](uint32_t g, uint64_t s) { check<0, 4><<<g, 256>>>(buf, n, s, 7, bad); });
  }
  uint32_t hb = 0; CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  std::printf("{\"bad_words\":%u}\n", hb);
  return hb != 0;
}
