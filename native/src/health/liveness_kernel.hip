// gfx950 (CDNA4) MFMA liveness kernel.
//
// No reference counterpart: the reference's "health" is a sysfs scan that
// marks every device healthy if any kfd GPU node exists
// (internal/pkg/amdgpu/amdgpu.go:865-910). This kernel proves, per HIP/HSA
// device (per partition in CPX), that the command processor dispatches, a
// wave64 executes, the matrix core produces the exact product, and device
// memory round-trips — in ONE dispatch of ONE wave.
//
// Launch: 1 workgroup x 64 lanes. Lane l of v_mfma_f32_32x32x2_f32 holds
// A[l&31][l>>5] and B[l>>5][l&31]; accumulator register r of lane l is
// D[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31] (cdna_hip_programming.md §3).
//
// Data path: accumulators -> device scratch (HBM) -> barrier -> each lane
// reads the OTHER half-wave's slots back -> host-visible tile. A dead
// memory path or a lane that never wrote shows up as a mismatch on the host.
#include <hip/hip_runtime.h>

#include "liveness_kernel.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

// s_getreg_b32 HW_REG_XCC_ID (hwreg 20 on gfx94x/gfx950), bits [3:0].
#define MI355X_HWREG_XCC_ID ((20) | (0 << 6) | ((16 - 1) << 11))
// HW_REG_HW_ID (hwreg 4): wave/simd/cu/se ids, for the record.
#define MI355X_HWREG_HW_ID ((4) | (0 << 6) | ((32 - 1) << 11))

extern "C" __global__ __launch_bounds__(64) void mi355x_mfma_liveness(float* __restrict__ out,
                                                                      uint32_t* __restrict__ meta,
                                                                      float* __restrict__ scratch,
                                                                      uint32_t nonce, int iters) {
  const int lane = threadIdx.x & 63;
  const int row = lane & 31;
  const int kk = lane >> 5;
  const float a = probe_a(row, kk, nonce);
  const float b = probe_b(kk, row, nonce);

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * kk;
    acc[r] = probe_c(i, row, nonce);
  }
  for (int it = 0; it < iters; ++it) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);

  // lane-major slots so each store instruction writes 256 contiguous bytes
#pragma unroll
  for (int r = 0; r < 16; ++r) scratch[r * 64 + lane] = acc[r];
  __threadfence();
  __syncthreads();
  const int peer = lane ^ 32;
  const int pk = peer >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * pk;
    out[i * MI355X_PROBE_N + (peer & 31)] = scratch[r * 64 + peer];
  }
  if (lane == 0) {
    meta[MI355X_META_MAGIC] = MI355X_PROBE_MAGIC;
    meta[MI355X_META_NONCE] = nonce;
    meta[MI355X_META_XCC] = __builtin_amdgcn_s_getreg(MI355X_HWREG_XCC_ID) & 0xF;
    meta[MI355X_META_HWID] = __builtin_amdgcn_s_getreg(MI355X_HWREG_HW_ID);
  }
}

// Full-chip sweep: see liveness_kernel.h. Every path out of the residency wait
// is bounded (wait_ticks), so the grid drains even when some CUs are held by
// other work or disabled; coverage is then reported, not assumed.
extern "C" __global__ __launch_bounds__(MI355X_SWEEP_THREADS) void mi355x_chip_sweep(mi355x_sweep_args args) {
  __shared__ uint32_t lds[MI355X_SWEEP_LDS_WORDS];
  __shared__ uint32_t ctr[16];
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = tid >> 6;
  const int lane = tid & 63;
  const uint32_t wg = blockIdx.x;
  if (tid < 16) ctr[tid] = 0;
  if (tid == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_fetch_add(args.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t seen;
    while ((seen = __hip_atomic_load(args.arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < args.grid) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > args.wait_ticks) break;
      __builtin_amdgcn_s_sleep(4);
    }
    ctr[8] = seen;
    ctr[9] = static_cast<uint32_t>(t0);
    ctr[10] = static_cast<uint32_t>(t0 >> 32);
  }
  __syncthreads();

  // MFMA tile per wave, checked lane by lane against the VALU
  const uint32_t n = sweep_nonce(args.nonce, wg, wave);
  const int row = lane & 31;
  const int kk = lane >> 5;
  const float a = probe_a(row, kk, n);
  const float b = probe_b(kk, row, n);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = probe_c((r & 3) + 8 * (r >> 2) + 4 * kk, row, n);
  for (int it = 0; it < args.iters; ++it) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  uint32_t bad = 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * kk;
    float dot = 0.f;
    for (int k = 0; k < MI355X_PROBE_K; ++k) dot += probe_a(i, k, n) * probe_b(k, row, n);
    const float want = probe_c(i, row, n) + static_cast<float>(args.iters) * dot;
    bad += acc[r] != want;
  }
  if (bad) atomicAdd(&ctr[0], bad);
  if (wave == 0) {
    float* tile = args.tiles + static_cast<size_t>(wg) * MI355X_PROBE_OUT;
#pragma unroll
    for (int r = 0; r < 16; ++r) tile[((r & 3) + 8 * (r >> 2) + 4 * kk) * MI355X_PROBE_N + row] = acc[r];
  }

  // whole-LDS pattern, read back from another wave's writes
  for (uint32_t i = tid; i < MI355X_SWEEP_LDS_WORDS; i += MI355X_SWEEP_THREADS)
    lds[i] = sweep_lds_pattern(i, args.nonce, wg);
  __syncthreads();
  uint32_t lbad = 0;
  const uint32_t other = (tid + 64) & (MI355X_SWEEP_THREADS - 1);
  for (uint32_t i = other; i < MI355X_SWEEP_LDS_WORDS; i += MI355X_SWEEP_THREADS)
    lbad += lds[i] != sweep_lds_pattern(i, args.nonce, wg);
  if (lbad) atomicAdd(&ctr[1], lbad);
  if (lane == 0) ctr[12 + wave] = __builtin_amdgcn_s_getreg(MI355X_HWREG_HW_ID);
  __syncthreads();

  if (tid == 0) {
    uint32_t* rec = args.records + static_cast<size_t>(wg) * MI355X_SWEEP_REC_WORDS;
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    rec[MI355X_REC_NONCE] = args.nonce ^ wg;
    rec[MI355X_REC_XCC] = __builtin_amdgcn_s_getreg(MI355X_HWREG_XCC_ID) & 0xF;
    rec[MI355X_REC_HWID] = ctr[12];
    rec[MI355X_REC_MFMA_BAD] = ctr[0];
    rec[MI355X_REC_LDS_BAD] = ctr[1];
    rec[MI355X_REC_ARRIVED] = ctr[8];
    rec[MI355X_REC_T0_LO] = ctr[9];
    rec[MI355X_REC_T0_HI] = ctr[10];
    rec[MI355X_REC_T1_LO] = static_cast<uint32_t>(t1);
    rec[MI355X_REC_T1_HI] = static_cast<uint32_t>(t1 >> 32);
    rec[MI355X_REC_WG] = wg;
    rec[12] = ctr[13];
    rec[13] = ctr[14];
    rec[14] = ctr[15];
    rec[MI355X_REC_MAGIC] = MI355X_SWEEP_MAGIC;
  }
}

// ---- throughput check: see liveness_kernel.h ---------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Grid-stride over 16-byte units; the check pass keeps 4 nontemporal loads in
// flight per lane (grid shapes: liveness_kernel.h).
extern "C" __global__ __launch_bounds__(MI355X_PERF_THREADS) void mi355x_hbm_fill(mi355x_hbm_args args) {
  u32x4* buf = reinterpret_cast<u32x4*>(args.buf);
  const uint64_t stride = args.threads;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * MI355X_PERF_THREADS + threadIdx.x; i < args.n16;
       i += stride) {
    const uint64_t w = i * 4;
    u32x4 v;
    v.x = hbm_pattern(w, args.seed);
    v.y = hbm_pattern(w + 1, args.seed);
    v.z = hbm_pattern(w + 2, args.seed);
    v.w = hbm_pattern(w + 3, args.seed);
    if (i == args.poison_unit) v.x = ~v.x;
    buf[i] = v;
  }
}

__device__ inline uint32_t hbm_mismatches(const u32x4 v, uint64_t unit, uint32_t seed) {
  const uint64_t w = unit * 4;
  return (v.x != hbm_pattern(w, seed)) + (v.y != hbm_pattern(w + 1, seed)) + (v.z != hbm_pattern(w + 2, seed)) +
         (v.w != hbm_pattern(w + 3, seed));
}

extern "C" __global__ __launch_bounds__(MI355X_PERF_THREADS) void mi355x_hbm_check(mi355x_hbm_args args) {
  const u32x4* buf = reinterpret_cast<const u32x4*>(args.buf);
  const uint64_t stride = args.threads;
  const uint64_t n = args.n16;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * MI355X_PERF_THREADS + threadIdx.x;
  uint32_t bad = 0;
  uint64_t first = ~0ull;
  for (; i + 3 * stride < n; i += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(&buf[i + u * stride]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t m = hbm_mismatches(v[u], i + u * stride, args.seed);
      if (m) {
        bad += m;
        first = first < i + u * stride ? first : i + u * stride;
      }
    }
  }
  for (; i < n; i += stride) {
    const uint32_t m = hbm_mismatches(__builtin_nontemporal_load(&buf[i]), i, args.seed);
    if (m) {
      bad += m;
      first = first < i ? first : i;
    }
  }
  if (bad) {
    atomicAdd(args.bad, bad);
    atomicMin(reinterpret_cast<unsigned long long*>(args.first_bad), static_cast<unsigned long long>(first));
  }
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Register-resident v_mfma_f32_32x32x16_bf16 chains, two per wave, two waves
// per SIMD: the matrix cores' sustained rate at the clock the chip holds under
// this load. Every wave gets the same operands, so every accumulator checksum
// must be bit-identical across waves, CUs and XCDs (the host compares them).
extern "C" __global__ __launch_bounds__(MI355X_PERF_THREADS) void mi355x_mfma_burn(mi355x_burn_args args) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = threadIdx.x >> 6;
  bf16x8 a, b, c, d;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = __builtin_bit_cast(__bf16, burn_bf16_bits(lane, j, args.nonce));
    b[j] = __builtin_bit_cast(__bf16, burn_bf16_bits(lane, j + 8, args.nonce));
    c[j] = __builtin_bit_cast(__bf16, burn_bf16_bits(lane, j + 16, args.nonce));
    d[j] = __builtin_bit_cast(__bf16, burn_bf16_bits(lane, j + 24, args.nonce));
  }
  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
  __syncthreads();
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < args.iters; ++it) {
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c, d, acc1, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += acc0[r] - acc1[r];
  // the wave's checksum: lane sums folded across the wave
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
  uint32_t* rec = args.records + static_cast<size_t>(blockIdx.x) * MI355X_PERF_REC_WORDS;
  if (lane == 0) rec[MI355X_PREC_SUM + wave] = __builtin_bit_cast(uint32_t, s);
  if (blockIdx.x == 0 && threadIdx.x < 4) args.hbm_counters_host[threadIdx.x] = args.hbm_counters[threadIdx.x];
  if (threadIdx.x == 0) {
    const uint64_t cyc = c1 - c0;
    rec[MI355X_PREC_WG] = blockIdx.x;
    rec[MI355X_PREC_XCC] = __builtin_amdgcn_s_getreg(MI355X_HWREG_XCC_ID) & 0xF;
    rec[MI355X_PREC_HWID] = __builtin_amdgcn_s_getreg(MI355X_HWREG_HW_ID);
    rec[MI355X_PREC_RT0_LO] = static_cast<uint32_t>(rt0);
    rec[MI355X_PREC_RT0_HI] = static_cast<uint32_t>(rt0 >> 32);
    rec[MI355X_PREC_RT1_LO] = static_cast<uint32_t>(rt1);
    rec[MI355X_PREC_RT1_HI] = static_cast<uint32_t>(rt1 >> 32);
    rec[MI355X_PREC_CYC_LO] = static_cast<uint32_t>(cyc);
    rec[MI355X_PREC_CYC_HI] = static_cast<uint32_t>(cyc >> 32);
    rec[MI355X_PREC_NONCE] = args.nonce ^ blockIdx.x;
    rec[MI355X_PREC_MAGIC] = MI355X_PERF_MAGIC;
  }
}
