// Shared between the gfx950 liveness kernel, its host launcher and the host
// reference check. One wave64 computes D = iters * (A·B) + C with
// v_mfma_f32_32x32x2_f32 (exact f32: small-integer inputs give bit-exact
// results), so any deviation from the host-computed tile is a hardware/driver
// fault, not rounding.
#pragma once

#include <stdint.h>

#define MI355X_PROBE_M 32
#define MI355X_PROBE_N 32
#define MI355X_PROBE_K 2
#define MI355X_PROBE_OUT (MI355X_PROBE_M * MI355X_PROBE_N)
#define MI355X_PROBE_MAGIC 0x4D464D41u /* "MFMA" */

// meta words written by lane 0
#define MI355X_META_MAGIC 0
#define MI355X_META_NONCE 1
#define MI355X_META_XCC 2
#define MI355X_META_HWID 3
#define MI355X_META_WORDS 4
#define MI355X_SCRATCH_FLOATS (16 * 64)

// explicit kernel arguments, in order (24 + 8 bytes; the kernel uses no hidden args)
struct mi355x_liveness_args {
  float* out;        // host-visible MI355X_PROBE_OUT floats
  uint32_t* meta;    // host-visible MI355X_META_WORDS words
  float* scratch;    // device memory, MI355X_SCRATCH_FLOATS floats
  uint32_t nonce;
  int32_t iters;
};

#if defined(__HIPCC__)
#define MI355X_HD __host__ __device__ inline
#else
#define MI355X_HD static inline
#endif

// Deterministic, asymmetric operands (an A=I / symmetric-B test would not
// catch a transposed store; see cdna_hip_programming.md §3).
MI355X_HD float probe_a(int i, int k, uint32_t nonce) { return (float)((int)((i * 3u + k * 5u + nonce) % 7u) - 3); }
MI355X_HD float probe_b(int k, int j, uint32_t nonce) { return (float)((int)((j * 11u + k * 2u + nonce) % 5u) - 2); }
MI355X_HD float probe_c(int i, int j, uint32_t nonce) { return (float)((int)((i + 2u * j + nonce) % 4u)); }

// ---- full-chip sweep (mi355x_chip_sweep) --------------------------------------
// One 256-lane workgroup per CU: each holds all 160 KiB of its CU's LDS, so no
// two workgroups can share a CU, and they wait (bounded) until the whole grid
// is resident before working — every CU of every XCD runs exactly one. Each of
// the 4 waves runs the MFMA tile (operands vary per workgroup and wave) and
// checks it against a VALU recomputation; the whole LDS is written and read
// back across waves; wave 0's tile also goes to the host for a bit-exact check.
#define MI355X_SWEEP_THREADS 256
#define MI355X_SWEEP_LDS_WORDS (40960 - 16)  // + 16 counter words = 160 KiB
#define MI355X_SWEEP_REC_WORDS 16
#define MI355X_SWEEP_MAGIC 0x43484950u /* "CHIP" */
// record words (one record per workgroup)
#define MI355X_REC_MAGIC 0
#define MI355X_REC_NONCE 1
#define MI355X_REC_XCC 2
#define MI355X_REC_HWID 3        // wave 0; waves 1-3 in 12..14
#define MI355X_REC_MFMA_BAD 4
#define MI355X_REC_LDS_BAD 5
#define MI355X_REC_ARRIVED 6     // workgroups resident when this one started work
#define MI355X_REC_T0_LO 7       // s_memrealtime (100 MHz) at arrival
#define MI355X_REC_T0_HI 8
#define MI355X_REC_T1_LO 9       // at completion
#define MI355X_REC_T1_HI 10
#define MI355X_REC_WG 11

struct mi355x_sweep_args {
  uint32_t* records;   // host-visible, grid * MI355X_SWEEP_REC_WORDS
  float* tiles;        // host-visible, grid * MI355X_PROBE_OUT (wave 0's tile per workgroup)
  uint32_t* arrive;    // device memory, 1 word, zero before launch
  uint32_t nonce;
  int32_t iters;
  uint32_t grid;       // workgroups launched (= CUs of the agent)
  uint32_t wait_ticks; // max residency wait, s_memrealtime ticks
};

MI355X_HD uint32_t sweep_nonce(uint32_t nonce, uint32_t wg, uint32_t wave) { return nonce + wg * 4u + wave; }
MI355X_HD uint32_t sweep_lds_pattern(uint32_t i, uint32_t nonce, uint32_t wg) {
  return (i * 2654435761u) ^ (nonce + wg * 0x9E3779B1u);
}

// ---- throughput check (mi355x_hbm_fill / mi355x_hbm_check / mi355x_mfma_burn) ----
// A GPU can be alive and exact yet slow: a stuck-low clock, an XCD held back,
// an HBM stack running degraded. On an idle GPU the plugin can measure what a
// tenant would get: HBM write and read bandwidth over a patterned buffer (every
// 16-byte unit verified on the read pass) and sustained bf16 MFMA throughput
// with the shader clock of every workgroup (s_memtime over s_memrealtime).
#define MI355X_PERF_THREADS 256
// grid shapes measured on MI355X: plain 16-byte stores peak at 1 workgroup
// per CU (5.8 TB/s vs 5.3-5.4 at 4 per CU; nontemporal stores are slower;
// tools/archive/experiments/hbm_{stream,fill}_variants.hip, 8 GiB). For loads, 16 per CU wins on repeated
// passes over 8 GiB (6.5-6.7 TB/s vs 6.3) but loses on the check's single
// pass right after the fill (1-4 GiB: 3.8-4.8 TB/s vs 5.0-6.1 at 8 per CU,
// tools/archive/gpurun_perfcheck.sh), so the check uses 8.
#define MI355X_HBM_FILL_WGS_PER_CU 1
#define MI355X_HBM_CHECK_WGS_PER_CU 8
#define MI355X_BURN_WGS_PER_CU 2   // 8 waves per CU = 2 per SIMD
#define MI355X_PERF_REC_WORDS 16
#define MI355X_PERF_MAGIC 0x50455246u /* "PERF" */
// mfma_burn record words (one record per workgroup)
#define MI355X_PREC_MAGIC 0
#define MI355X_PREC_WG 1
#define MI355X_PREC_XCC 2
#define MI355X_PREC_HWID 3
#define MI355X_PREC_RT0_LO 4      // s_memrealtime (100 MHz) before the MFMA loop
#define MI355X_PREC_RT0_HI 5
#define MI355X_PREC_RT1_LO 6      // after it
#define MI355X_PREC_RT1_HI 7
#define MI355X_PREC_CYC_LO 8      // s_memtime (shader clock) ticks over the loop
#define MI355X_PREC_CYC_HI 9
#define MI355X_PREC_NONCE 10
#define MI355X_PREC_SUM 12        // 4 words: each wave's accumulator checksum (identical everywhere)

struct mi355x_hbm_args {
  uint32_t* buf;        // device memory, n16 * 16 bytes
  uint64_t n16;         // 16-byte units
  uint32_t* bad;        // device-visible counter of mismatching 32-bit words (check pass)
  uint64_t* first_bad;  // lowest mismatching 16-byte unit (check pass), UINT64_MAX if none
  uint64_t threads;     // lanes in the grid (the grid stride; passed so the kernels need no hidden args)
  uint64_t poison_unit; // fill: write this 16-byte unit's first word inverted (fault injection); UINT64_MAX = off
  uint32_t seed;
  uint32_t pad;
};

struct mi355x_burn_args {
  uint32_t* records;    // host-visible, grid * MI355X_PERF_REC_WORDS
  // the check pass's device counters (4 words), copied by workgroup 0 to the
  // host-visible words after the records: no runtime copy (a device-to-host
  // copy makes ROCr create another queue, +189 MB in the probe server)
  const uint32_t* hbm_counters;
  uint32_t* hbm_counters_host;
  uint32_t nonce;
  int32_t iters;        // MFMA pairs per wave
};

// 32-bit word `word` of the patterned buffer: a bijection of the word index
// (odd multiplier), so a stuck or aliased address bit reads another value
MI355X_HD uint32_t hbm_pattern(uint64_t word, uint32_t seed) {
  return (uint32_t)(word ^ (word >> 32)) * 0x9E3779B1u + seed;
}

// bf16 bit pattern of a pseudo-random operand in +-[2^-7, 2^-1): every MFMA
// input bit toggles (zero or small-integer operands run at a higher clock than
// real data, MI355X_MICROARCH.md "DVFS give-back")
MI355X_HD uint16_t burn_bf16_bits(uint32_t lane, uint32_t j, uint32_t nonce) {
  uint32_t h = (lane * 0x9E3779B1u) ^ (j * 0x85EBCA77u) ^ nonce;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return (uint16_t)((h & 0x807Fu) | ((120u + (h >> 8) % 7u) << 7));
}
