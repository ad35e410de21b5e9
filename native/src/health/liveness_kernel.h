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
