// Bit-exact host check of a liveness tile (shared by the HIP and HSA paths).
#pragma once

#include <cstdio>

#include "liveness_kernel.h"
#include "mi355x/liveness_probe.h"

namespace mi355x {

inline void verify_tile(const float* out, const uint32_t* meta, uint32_t nonce, int iters,
                        mi355x_probe_result* r) {
  int mism = 0;
  for (int i = 0; i < MI355X_PROBE_M; ++i)
    for (int j = 0; j < MI355X_PROBE_N; ++j) {
      float ab = 0.f;
      for (int k = 0; k < MI355X_PROBE_K; ++k) ab += probe_a(i, k, nonce) * probe_b(k, j, nonce);
      const float want = probe_c(i, j, nonce) + static_cast<float>(iters) * ab;
      if (out[i * MI355X_PROBE_N + j] != want) ++mism;
    }
  r->mismatches = mism;
  r->xcc_id = meta[MI355X_META_XCC];
  r->hw_id = meta[MI355X_META_HWID];
  if (meta[MI355X_META_MAGIC] != MI355X_PROBE_MAGIC || meta[MI355X_META_NONCE] != nonce) {
    std::snprintf(r->error, sizeof(r->error), "meta mismatch: magic=%08x nonce=%u (want %u)",
                  meta[MI355X_META_MAGIC], meta[MI355X_META_NONCE], nonce);
  } else if (mism) {
    std::snprintf(r->error, sizeof(r->error), "%d/%d MFMA results differ from host reference", mism,
                  MI355X_PROBE_OUT);
  } else {
    r->ok = 1;
  }
}

}  // namespace mi355x
