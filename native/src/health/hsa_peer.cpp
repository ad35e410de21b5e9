// The xGMI peer copy check (mi355x_hsa_peer_probe, mi355x/liveness_probe.h):
// a verified pattern copied GPU -> peer GPU with the runtime's DMA engines,
// timed, read back through host memory and checked word by word; the kfd
// link type, hop count and NUMA distance of the pair come with it.
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "hsa_runtime.h"

using namespace mi355x::hsa_rt;  // NOLINT(build/namespaces)

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
