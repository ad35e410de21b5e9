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
