// The full-chip sweep (mi355x_hsa_chip_sweep: every CU of every XCD runs the
// MFMA tile and reports where it ran) and the throughput check
// (mi355x_hsa_perf_check: HBM write / read over a verified pattern, sustained
// bf16 MFMA rate, per-XCD clocks), both on the device's kept queue when there
// is one. A dispatch that outlives its deadline is parked in an in-flight
// registry with everything it may still write.
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

#include "hsa_runtime.h"

using namespace mi355x::hsa_rt;  // NOLINT(build/namespaces)

namespace mi355x::hsa_rt {

// A chip sweep whose completion signal did not fire within its deadline: the
// dispatch may still write its records, so none of its resources can be freed
// until it completes. One per device at most (mi355x_hsa_chip_sweep refuses to
// submit another while it is outstanding).
struct SweepInFlight {
  hsa_code_object_reader_t reader{};  // null when the kept queue / executable were borrowed
  hsa_executable_t exe{};
  hsa_queue_t* queue = nullptr;
  std::shared_ptr<SigRef> sig;
  void* bufs[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  std::chrono::steady_clock::time_point since{};

  void release() {
    for (void* b : bufs)
      if (b) H().hsa_amd_memory_pool_free(b);
    if (queue) H().hsa_queue_destroy(queue);
    if (exe.handle) H().hsa_executable_destroy(exe);
    if (reader.handle) H().hsa_code_object_reader_destroy(reader);
    sig.reset();
  }
};
std::mutex g_sweep_mu;
std::vector<std::pair<int, SweepInFlight>> g_sweep_in_flight;

// > 0 (seconds outstanding) when an earlier sweep or throughput check on
// `ordinal` is still running; a completed one is freed here.
double in_flight_for(int ordinal) {
  std::lock_guard<std::mutex> lk(g_sweep_mu);
  for (auto it = g_sweep_in_flight.begin(); it != g_sweep_in_flight.end(); ++it) {
    if (it->first != ordinal) continue;
    if (H().hsa_signal_load_scacquire(it->second.sig->s) < 1) {
      it->second.release();
      g_sweep_in_flight.erase(it);
      return 0;
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - it->second.since).count();
    return s > 0 ? s : 1e-9;
  }
  return 0;
}

template <typename R>
bool sweep_still_in_flight(int ordinal, R* out) {
  const double s = in_flight_for(ordinal);
  if (s <= 0) return false;
  out->in_flight_s = s;
  out->hsa_error = -1;
  std::snprintf(out->error, sizeof(out->error), "earlier chip sweep / check still in flight for %.1fs (not completed)",
                s);
  return true;
}

// runtime shutdown: an outstanding sweep's resources go with the runtime
void forget_in_flight_sweeps() {
  std::lock_guard<std::mutex> lk(g_sweep_mu);
  // a dispatch still running may yet decrement its completion signal: leave
  // the signal to the runtime's own teardown instead of destroying it here
  for (auto& e : g_sweep_in_flight)
    if (e.second.sig && e.second.sig->s.handle && H().hsa_signal_load_scacquire(e.second.sig->s) >= 1)
      e.second.sig->s = hsa_signal_t{};
  g_sweep_in_flight.clear();
}

}  // namespace mi355x::hsa_rt

namespace mi355x::hsa_rt {

// One AQL kernel dispatch (barrier bit, system-scope fences), no wait.
void submit_kernel(hsa_queue_t* queue, uint64_t kobj, uint32_t gseg, uint32_t pseg, void* kargs, uint32_t wgs,
                   uint32_t wg_threads, hsa_signal_t sig) {
  H().hsa_signal_store_screlease(sig, 1);
  const uint64_t idx = H().hsa_queue_add_write_index_screlease(queue, 1);
  auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(queue->base_address) + (idx & (queue->size - 1));
  std::memset(reinterpret_cast<char*>(pkt) + 4, 0, sizeof(*pkt) - 4);
  pkt->workgroup_size_x = static_cast<uint16_t>(wg_threads);
  pkt->workgroup_size_y = 1;
  pkt->workgroup_size_z = 1;
  pkt->grid_size_x = wgs * wg_threads;
  pkt->grid_size_y = 1;
  pkt->grid_size_z = 1;
  pkt->private_segment_size = pseg;
  pkt->group_segment_size = gseg;
  pkt->kernel_object = kobj;
  pkt->kernarg_address = kargs;
  pkt->completion_signal = sig;
  const uint16_t header = static_cast<uint16_t>(
      (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
      (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
      (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), header | (static_cast<uint32_t>(setup) << 16), __ATOMIC_RELEASE);
  H().hsa_signal_store_screlease(queue->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
}

double dispatch_us(const Agent& ag, hsa_signal_t sig) {
  hsa_amd_profiling_dispatch_time_t dt{};
  if (H().hsa_amd_profiling_get_dispatch_time(ag.agent, sig, &dt) != HSA_STATUS_SUCCESS || !g_rt.ts_freq) return 0;
  return static_cast<double>(dt.end - dt.start) * 1e6 / static_cast<double>(g_rt.ts_freq);
}

double median_of(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

struct KernelSym {
  uint64_t kobj = 0;
  uint32_t kseg = 0, gseg = 0, pseg = 0;
};

// The queue and executable a chip sweep or throughput check runs on. With kept
// resources (--serve --keep) the device's kept queue and executable are
// borrowed -- set up here if no probe has yet -- so the check adds no kfd
// queue: no 181 MB context-save area, no HWS runlist update. The slot's mutex
// is held meanwhile, so no probe packet interleaves. Otherwise a private queue
// and executable are created for the check and destroyed after it.
struct DeviceWork {
  explicit DeviceWork(const Agent& a) : ag(a) {}
  DeviceWork(const DeviceWork&) = delete;
  DeviceWork& operator=(const DeviceWork&) = delete;
  ~DeviceWork() {
    if (abandoned || borrowed()) return;
    if (queue) H().hsa_queue_destroy(queue);
    if (exe.handle) H().hsa_executable_destroy(exe);
    if (reader.handle) H().hsa_code_object_reader_destroy(reader);
  }
  bool borrowed() const { return slot != nullptr; }

  hsa_status_t open(int ordinal, const char** what) {
    bool keep;
    {
      std::lock_guard<std::mutex> lk(g_resident_mu);
      keep = g_keep;
    }
    if (keep) {
      Resident* s = resident_slot(ordinal);
      std::unique_lock<std::timed_mutex> lk(s->mu);
      if (!s->ready && !s->pending && !s->blocker) {
        mi355x_probe_result scratch;
        std::memset(&scratch, 0, sizeof(scratch));
        if (setup_resources(ag, s->r, s->k, &scratch))
          s->ready = true;
        else
          s->r.release();
      }
      if (s->ready && !s->pending && !s->blocker) {
        slot = s;
        slot_lk = std::move(lk);
        exe = s->r.exe;
        queue = s->r.queue;
      }
    }
    hsa_status_t st = HSA_STATUS_SUCCESS;
    if (!borrowed()) {
      const size_t co_size = static_cast<size_t>(mi355x_hsaco_end - mi355x_hsaco_start);
      if ((st = H().hsa_code_object_reader_create_from_memory(mi355x_hsaco_start, co_size, &reader)) != 0)
        return *what = "code object", st;
      if ((st = H().hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr,
                                              &exe)) != 0)
        return *what = "executable create", st;
      if ((st = H().hsa_executable_load_agent_code_object(exe, ag.agent, reader, nullptr, nullptr)) != 0)
        return *what = "load code object", st;
      if ((st = H().hsa_executable_freeze(exe, nullptr)) != 0) return *what = "freeze", st;
      if ((st = H().hsa_queue_create(ag.agent, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX,
                                     &queue)) != 0)
        return *what = "queue create", st;
      H().hsa_amd_profiling_set_profiler_enabled(queue, 1);
    }
    if ((st = H().hsa_signal_create(1, 0, nullptr, &sig->s)) != 0) return *what = "signal create", st;
    return st;
  }

  hsa_status_t symbol(const char* name, KernelSym* k) {
    hsa_executable_symbol_t sym{};
    const hsa_status_t st = H().hsa_executable_get_symbol_by_name(exe, name, &ag.agent, &sym);
    if (st != HSA_STATUS_SUCCESS) return st;
    H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->kobj);
    H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->kseg);
    H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->gseg);
    H().hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->pseg);
    return st;
  }

  void submit(const KernelSym& k, void* kargs, uint32_t wgs, uint32_t wg_threads) {
    submit_kernel(queue, k.kobj, k.gseg, k.pseg, kargs, wgs, wg_threads, sig->s);
  }

  // A dispatch did not complete within its deadline: everything it may still
  // write goes to the in-flight registry (at most one per device: later sweeps
  // and checks fail fast until it completes), and a borrowed kept queue blocks
  // probes until then.
  void abandon(int ordinal, std::initializer_list<void*> bufs, std::chrono::steady_clock::time_point since) {
    abandoned = true;
    SweepInFlight f;
    if (!borrowed()) {
      f.reader = reader;
      f.exe = exe;
      f.queue = queue;
    }
    f.sig = sig;
    int i = 0;
    for (void* b : bufs)
      if (i < 6) f.bufs[i++] = b;
    f.since = since;
    {
      std::lock_guard<std::mutex> lk(g_sweep_mu);
      g_sweep_in_flight.emplace_back(ordinal, f);
    }
    if (borrowed()) {
      slot->blocker = sig;
      slot->blocked_since = since;  // when the sweep / check was submitted
    }
  }

  const Agent& ag;
  Resident* slot = nullptr;
  std::unique_lock<std::timed_mutex> slot_lk;
  hsa_code_object_reader_t reader{};
  hsa_executable_t exe{};
  hsa_queue_t* queue = nullptr;
  std::shared_ptr<SigRef> sig = std::make_shared<SigRef>();
  bool abandoned = false;
};

void set_hsa_error(int* err, char* buf, size_t n, hsa_status_t st, const char* what) {
  *err = static_cast<int>(st);
  const char* msg = nullptr;
  H().hsa_status_string(st, &msg);
  std::snprintf(buf, n, "%s: %s", what, msg ? msg : "hsa error");
}

}  // namespace mi355x::hsa_rt

extern "C" int mi355x_hsa_chip_sweep(int ordinal, uint32_t nonce, int iters, double timeout_s,
                                     mi355x_sweep_result* out) {
  using clk = std::chrono::steady_clock;
  std::memset(out, 0, sizeof(*out));
  out->ordinal = ordinal;
  out->nonce = nonce;
  out->iters = iters < 1 ? 1 : (iters > 64 ? 64 : iters);
  const auto t0 = clk::now();
  auto finish = [&] {
    out->total_us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
    return out->ok ? 0 : 1;
  };
  const int n = mi355x_hsa_probe_init();
  if (n < 0) {
    out->hsa_error = n;
    std::snprintf(out->error, sizeof(out->error), "hsa_init: %.140s", H().loaded ? "runtime init failed" : H().error);
    return 1;
  }
  if (ordinal < 0 || ordinal >= n) {
    std::snprintf(out->error, sizeof(out->error), "no such GPU agent (count=%d)", n);
    return 1;
  }
  if (sweep_still_in_flight(ordinal, out)) return finish();
  const Agent& ag = g_rt.gpus[ordinal];
  uint32_t cus = 0, xcc = 0;
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT), &cus);
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NUM_XCC), &xcc);
  out->cu_count = static_cast<int>(cus);
  out->num_xcc = static_cast<int>(xcc);
  if (cus == 0 || cus > 1024 || !g_rt.has_fine || !g_rt.has_kernarg || !ag.has_coarse) {
    std::snprintf(out->error, sizeof(out->error), "unexpected agent (cus=%u) or missing memory pool", cus);
    return 1;
  }
  const uint32_t grid = cus;
  out->grid = static_cast<int>(grid);

  DeviceWork dw(ag);
  const char* what = "";
  hsa_status_t s = dw.open(ordinal, &what);
  if (s != HSA_STATUS_SUCCESS) {
    set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, what);
    return finish();
  }
  out->kept_queue = dw.borrowed() ? 1 : 0;
  KernelSym ksym;
  if ((s = dw.symbol("mi355x_chip_sweep.kd", &ksym)) != HSA_STATUS_SUCCESS) {
    set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, "kernel symbol");
    return finish();
  }
  if (ksym.kseg < sizeof(mi355x_sweep_args) || ksym.kseg > kKernargBytes) {
    std::snprintf(out->error, sizeof(out->error), "sweep kernarg segment %u: code object / host ABI mismatch", ksym.kseg);
    return finish();
  }
  uint32_t* records = nullptr;
  float* tiles = nullptr;
  uint32_t* arrive = nullptr;
  mi355x_sweep_args* kargs = nullptr;
  const size_t rec_bytes = static_cast<size_t>(grid) * MI355X_SWEEP_REC_WORDS * sizeof(uint32_t);
  const size_t tile_bytes = static_cast<size_t>(grid) * MI355X_PROBE_OUT * sizeof(float);
  auto free_bufs = [&] {
    if (kargs) H().hsa_amd_memory_pool_free(kargs);
    if (arrive) H().hsa_amd_memory_pool_free(arrive);
    if (tiles) H().hsa_amd_memory_pool_free(tiles);
    if (records) H().hsa_amd_memory_pool_free(records);
  };
#define SWEEP_CHECK(expr, label)                                                              \
  if ((s = (expr)) != HSA_STATUS_SUCCESS) {                                                   \
    set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, label);                 \
    free_bufs();                                                                              \
    return finish();                                                                          \
  }
  SWEEP_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.fine, rec_bytes, 0, reinterpret_cast<void**>(&records)),
              "alloc records");
  SWEEP_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.fine, tile_bytes, 0, reinterpret_cast<void**>(&tiles)),
              "alloc tiles");
  SWEEP_CHECK(H().hsa_amd_memory_pool_allocate(ag.coarse, 4096, 0, reinterpret_cast<void**>(&arrive)), "alloc arrive");
  SWEEP_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.kernarg, kKernargBytes, 0, reinterpret_cast<void**>(&kargs)),
              "alloc kernarg");
  SWEEP_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, records), "allow records");
  SWEEP_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, tiles), "allow tiles");
  SWEEP_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, kargs), "allow kernarg");
  SWEEP_CHECK(H().hsa_amd_memory_fill(arrive, 0u, 4096 / 4), "zero arrive");
#undef SWEEP_CHECK
  std::memset(records, 0, rec_bytes);
  std::memset(tiles, 0xFF, tile_bytes);
  std::memset(kargs, 0, kKernargBytes);
  kargs->records = records;
  kargs->tiles = tiles;
  kargs->arrive = arrive;
  kargs->nonce = nonce;
  kargs->iters = out->iters;
  kargs->grid = grid;
  kargs->wait_ticks = 2000000;  // 20 ms at the 100 MHz s_memrealtime clock
  dw.submit(ksym, kargs, grid, MI355X_SWEEP_THREADS);
  if (!wait_signal(dw.sig->s, timeout_s)) {
    std::snprintf(out->error, sizeof(out->error), "chip sweep did not complete within %.1fs", timeout_s);
    out->hsa_error = -1;
    dw.abandon(ordinal, {kargs, arrive, tiles, records}, t0);
    return finish();
  }
  out->kernel_us = dispatch_us(ag, dw.sig->s);
  {
    std::vector<uint32_t> keys;
    keys.reserve(grid);
    uint64_t tmin = UINT64_MAX, tmax = 0;
    uint32_t xmask = 0;
    bool all_res = true;
    std::vector<float> want(MI355X_PROBE_OUT);
    for (uint32_t w = 0; w < grid; ++w) {
      const uint32_t* r = records + static_cast<size_t>(w) * MI355X_SWEEP_REC_WORDS;
      const bool present = r[MI355X_REC_MAGIC] == MI355X_SWEEP_MAGIC && r[MI355X_REC_WG] == w &&
                           r[MI355X_REC_NONCE] == (nonce ^ w);
      if (!present) continue;
      out->mfma_bad += r[MI355X_REC_MFMA_BAD];
      out->lds_bad += r[MI355X_REC_LDS_BAD];
      const uint32_t x = r[MI355X_REC_XCC] & 0xF;
      xmask |= 1u << x;
      ++out->wgs_per_xcc[x];
      keys.push_back((x << 16) | ((r[MI355X_REC_HWID] >> 8) & 0xFF));
      all_res = all_res && r[MI355X_REC_ARRIVED] >= grid;
      const uint64_t t = (static_cast<uint64_t>(r[MI355X_REC_T0_HI]) << 32) | r[MI355X_REC_T0_LO];
      tmin = t < tmin ? t : tmin;
      tmax = t > tmax ? t : tmax;
      // wave 0's tile against the host reference
      const uint32_t nw = sweep_nonce(nonce, w, 0);
      uint32_t tb = 0;
      const float* tile = tiles + static_cast<size_t>(w) * MI355X_PROBE_OUT;
      for (int i = 0; i < MI355X_PROBE_M; ++i)
        for (int j = 0; j < MI355X_PROBE_N; ++j) {
          float dot = 0.f;
          for (int k = 0; k < MI355X_PROBE_K; ++k) dot += probe_a(i, k, nw) * probe_b(k, j, nw);
          const float e = probe_c(i, j, nw) + static_cast<float>(out->iters) * dot;
          tb += tile[i * MI355X_PROBE_N + j] != e;
        }
      out->tile_bad += tb;
      if (r[MI355X_REC_MFMA_BAD] == 0 && r[MI355X_REC_LDS_BAD] == 0 && tb == 0) ++out->records_ok;
    }
    std::sort(keys.begin(), keys.end());
    out->cus_covered = static_cast<int>(std::unique(keys.begin(), keys.end()) - keys.begin());
    out->xccs_covered = __builtin_popcount(xmask);
    out->all_resident = all_res && out->records_ok == static_cast<int>(grid);
    if (tmax >= tmin && tmin != UINT64_MAX) out->arrival_spread_us = static_cast<double>(tmax - tmin) / 100.0;
    out->ok = out->records_ok == static_cast<int>(grid) &&
              (out->num_xcc <= 0 || out->xccs_covered == out->num_xcc);
    if (!out->ok)
      std::snprintf(out->error, sizeof(out->error),
                    "%d/%d workgroups correct (mfma_bad=%u lds_bad=%u tile_bad=%u), %d/%d XCDs ran", out->records_ok,
                    grid, out->mfma_bad, out->lds_bad, out->tile_bad, out->xccs_covered, out->num_xcc);
  }
  free_bufs();
  return finish();
}

namespace mi355x::hsa_rt {
std::atomic<uint64_t> g_perf_poison{~0ull};
}  // namespace mi355x::hsa_rt

extern "C" void mi355x_hsa_perf_poison(uint64_t unit) { g_perf_poison.store(unit, std::memory_order_relaxed); }

extern "C" int mi355x_hsa_perf_check(int ordinal, uint32_t nonce, uint64_t bytes, int mfma_iters, double timeout_s,
                                     mi355x_perf_result* out) {
  using clk = std::chrono::steady_clock;
  std::memset(out, 0, sizeof(*out));
  out->ordinal = ordinal;
  out->nonce = nonce;
  out->hbm_first_bad = -1;
  // 16-byte units, at least one full grid-stride round, at most 64 GiB
  bytes = bytes < (64ull << 20) ? (64ull << 20) : (bytes > (64ull << 30) ? (64ull << 30) : bytes);
  bytes &= ~static_cast<uint64_t>(0xFFFFF);
  out->bytes = bytes;
  out->mfma_iters = mfma_iters < 1 ? 1 : (mfma_iters > (1 << 22) ? (1 << 22) : mfma_iters);
  const auto t0 = clk::now();
  auto finish = [&] {
    out->total_us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
    return out->ok ? 0 : 1;
  };
  const int n = mi355x_hsa_probe_init();
  if (n < 0) {
    out->hsa_error = n;
    std::snprintf(out->error, sizeof(out->error), "hsa_init: %.140s", H().loaded ? "runtime init failed" : H().error);
    return 1;
  }
  if (ordinal < 0 || ordinal >= n) {
    std::snprintf(out->error, sizeof(out->error), "no such GPU agent (count=%d)", n);
    return 1;
  }
  if (sweep_still_in_flight(ordinal, out)) return finish();
  const Agent& ag = g_rt.gpus[ordinal];
  uint32_t cus = 0, xcc = 0;
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT), &cus);
  H().hsa_agent_get_info(ag.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NUM_XCC), &xcc);
  out->cu_count = static_cast<int>(cus);
  out->num_xcc = static_cast<int>(xcc);
  if (cus == 0 || cus > 1024 || !g_rt.has_fine || !g_rt.has_kernarg || !ag.has_coarse) {
    std::snprintf(out->error, sizeof(out->error), "unexpected agent (cus=%u) or missing memory pool", cus);
    return 1;
  }
  const uint32_t fill_wgs = cus * MI355X_HBM_FILL_WGS_PER_CU;
  const uint32_t check_wgs = cus * MI355X_HBM_CHECK_WGS_PER_CU;
  const uint32_t burn_wgs = cus * MI355X_BURN_WGS_PER_CU;
  out->mfma_grid = static_cast<int>(burn_wgs);

  DeviceWork w(ag);
  const char* what = "";
  hsa_status_t s = w.open(ordinal, &what);
  if (s != HSA_STATUS_SUCCESS) {
    set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, what);
    return finish();
  }
  out->kept_queue = w.borrowed() ? 1 : 0;
  KernelSym ks[3];
  const char* names[3] = {"mi355x_hbm_fill.kd", "mi355x_hbm_check.kd", "mi355x_mfma_burn.kd"};
  for (int i = 0; i < 3; ++i)
    if ((s = w.symbol(names[i], &ks[i])) != HSA_STATUS_SUCCESS) {
      set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, "kernel symbol");
      return finish();
    }
  if (ks[0].kseg < sizeof(mi355x_hbm_args) || ks[0].kseg > kKernargBytes || ks[1].kseg < sizeof(mi355x_hbm_args) ||
      ks[1].kseg > kKernargBytes || ks[2].kseg < sizeof(mi355x_burn_args) || ks[2].kseg > kKernargBytes) {
    std::snprintf(out->error, sizeof(out->error), "perf kernarg segments %u/%u/%u: code object / host ABI mismatch",
                  ks[0].kseg, ks[1].kseg, ks[2].kseg);
    return finish();
  }
  uint32_t* buf = nullptr;       // device, `bytes`
  uint32_t* counters = nullptr;  // device, [0] bad words, [2..3] first bad unit
  uint32_t* h_counters = nullptr;
  uint32_t* records = nullptr;   // host-visible, burn_wgs records
  char* kargs = nullptr;         // 3 slots of kKernargBytes
  const size_t rec_bytes = static_cast<size_t>(burn_wgs) * MI355X_PERF_REC_WORDS * sizeof(uint32_t);
  auto free_bufs = [&] {
    if (kargs) H().hsa_amd_memory_pool_free(kargs);
    if (records) H().hsa_amd_memory_pool_free(records);
    if (h_counters) H().hsa_amd_memory_pool_free(h_counters);
    if (counters) H().hsa_amd_memory_pool_free(counters);
    if (buf) H().hsa_amd_memory_pool_free(buf);
  };
  auto abandon = [&](const char* stage) {
    std::snprintf(out->error, sizeof(out->error), "%s did not complete within %.1fs", stage, timeout_s);
    out->hsa_error = -1;
    w.abandon(ordinal, {kargs, buf, counters, h_counters, records}, t0);
    return finish();
  };
#define PERF_CHECK(expr, label)                                                               \
  if ((s = (expr)) != HSA_STATUS_SUCCESS) {                                                   \
    set_hsa_error(&out->hsa_error, out->error, sizeof(out->error), s, label);                 \
    free_bufs();                                                                              \
    return finish();                                                                          \
  }
  PERF_CHECK(H().hsa_amd_memory_pool_allocate(ag.coarse, bytes, 0, reinterpret_cast<void**>(&buf)), "alloc HBM buffer");
  PERF_CHECK(H().hsa_amd_memory_pool_allocate(ag.coarse, 4096, 0, reinterpret_cast<void**>(&counters)),
             "alloc counters");
  PERF_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.fine, 4096, 0, reinterpret_cast<void**>(&h_counters)),
             "alloc host counters");
  PERF_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.fine, rec_bytes, 0, reinterpret_cast<void**>(&records)),
             "alloc records");
  PERF_CHECK(H().hsa_amd_memory_pool_allocate(g_rt.kernarg, 4 * kKernargBytes, 0, reinterpret_cast<void**>(&kargs)),
             "alloc kernarg");
  PERF_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, h_counters), "allow counters");
  PERF_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, records), "allow records");
  PERF_CHECK(H().hsa_amd_agents_allow_access(1, &ag.agent, nullptr, kargs), "allow kernarg");
  // counters: word 0 = 0 (bad words), words 2..3 = all ones (first bad unit)
  PERF_CHECK(H().hsa_amd_memory_fill(counters, 0u, 2), "zero counters");
  PERF_CHECK(H().hsa_amd_memory_fill(counters + 2, 0xFFFFFFFFu, 2), "init first-bad");
  std::memset(h_counters, 0xA5, 16);   // overwritten by the burn kernel's copy
  std::memset(records, 0, rec_bytes);
  std::memset(kargs, 0, 4 * kKernargBytes);
  {
    auto* fa = reinterpret_cast<mi355x_hbm_args*>(kargs);
    auto* ca = reinterpret_cast<mi355x_hbm_args*>(kargs + kKernargBytes);
    auto* ba = reinterpret_cast<mi355x_burn_args*>(kargs + 2 * kKernargBytes);
    auto* c2 = reinterpret_cast<mi355x_hbm_args*>(kargs + 3 * kKernargBytes);
    fa->buf = ca->buf = buf;
    fa->n16 = ca->n16 = bytes / 16;
    fa->bad = ca->bad = counters;
    fa->first_bad = ca->first_bad = reinterpret_cast<uint64_t*>(counters + 2);
    fa->threads = static_cast<uint64_t>(fill_wgs) * MI355X_PERF_THREADS;
    ca->threads = static_cast<uint64_t>(check_wgs) * MI355X_PERF_THREADS;
    fa->poison_unit = g_perf_poison.load(std::memory_order_relaxed);
    ca->poison_unit = ~0ull;
    fa->seed = ca->seed = nonce * 0x01000193u + 0x7F4A7C15u;
    *c2 = *ca;
    c2->bad = counters + 1;  // the second read pass counts on its own
    ba->records = records;
    ba->hbm_counters = counters;
    ba->hbm_counters_host = h_counters;
    ba->nonce = nonce;
    ba->iters = out->mfma_iters;
  }
  w.submit(ks[0], kargs, fill_wgs, MI355X_PERF_THREADS);
  if (!wait_signal(w.sig->s, timeout_s)) return abandon("HBM fill");
  out->fill_us = dispatch_us(ag, w.sig->s);
  w.submit(ks[1], kargs + kKernargBytes, check_wgs, MI355X_PERF_THREADS);
  if (!wait_signal(w.sig->s, timeout_s)) return abandon("HBM check");
  out->check_us = dispatch_us(ag, w.sig->s);
  // a second read pass: steady-state read bandwidth (the first one still
  // competes with the fill's write-back) and a second look at every word
  w.submit(ks[1], kargs + 3 * kKernargBytes, check_wgs, MI355X_PERF_THREADS);
  if (!wait_signal(w.sig->s, timeout_s)) return abandon("HBM check (2nd pass)");
  out->check2_us = dispatch_us(ag, w.sig->s);
  w.submit(ks[2], kargs + 2 * kKernargBytes, burn_wgs, MI355X_PERF_THREADS);
  if (!wait_signal(w.sig->s, timeout_s)) return abandon("MFMA burn");
  out->mfma_us = dispatch_us(ag, w.sig->s);
#undef PERF_CHECK
  {
    out->hbm_bad_words = h_counters[0] > h_counters[1] ? h_counters[0] : h_counters[1];
    out->hbm_bad_words_pass2 = h_counters[1];
    const uint64_t first = (static_cast<uint64_t>(h_counters[3]) << 32) | h_counters[2];
    out->hbm_first_bad = first == ~0ull ? -1 : static_cast<int64_t>(first);
    if (out->fill_us > 0) out->hbm_write_gbps = static_cast<double>(bytes) / (out->fill_us * 1e3);
    const double best_check = out->check2_us > 0 && out->check2_us < out->check_us ? out->check2_us : out->check_us;
    if (best_check > 0) out->hbm_read_gbps = static_cast<double>(bytes) / (best_check * 1e3);
    const double flops = 2.0 * 32 * 32 * 16 * 2.0 * static_cast<double>(out->mfma_iters) *
                         (MI355X_PERF_THREADS / 64) * static_cast<double>(burn_wgs);
    if (out->mfma_us > 0) out->mfma_tflops = flops / (out->mfma_us * 1e6);
    std::vector<double> clocks;
    std::vector<std::vector<double>> per_xcd(16);
    uint32_t ref = 0;
    bool have_ref = false;
    uint32_t xmask = 0;
    for (uint32_t wg = 0; wg < burn_wgs; ++wg) {
      const uint32_t* r = records + static_cast<size_t>(wg) * MI355X_PERF_REC_WORDS;
      if (r[MI355X_PREC_MAGIC] != MI355X_PERF_MAGIC || r[MI355X_PREC_WG] != wg ||
          r[MI355X_PREC_NONCE] != (nonce ^ wg))
        continue;
      ++out->mfma_records_ok;
      for (int v = 0; v < MI355X_PERF_THREADS / 64; ++v) {
        if (!have_ref) {
          ref = r[MI355X_PREC_SUM + v];
          have_ref = true;
        } else if (r[MI355X_PREC_SUM + v] != ref) {
          ++out->mfma_checksum_mismatch;
        }
      }
      const uint64_t rt0 = (static_cast<uint64_t>(r[MI355X_PREC_RT0_HI]) << 32) | r[MI355X_PREC_RT0_LO];
      const uint64_t rt1 = (static_cast<uint64_t>(r[MI355X_PREC_RT1_HI]) << 32) | r[MI355X_PREC_RT1_LO];
      const uint64_t cyc = (static_cast<uint64_t>(r[MI355X_PREC_CYC_HI]) << 32) | r[MI355X_PREC_CYC_LO];
      const uint32_t x = r[MI355X_PREC_XCC] & 0xF;
      xmask |= 1u << x;
      if (rt1 > rt0) {
        const double mhz = static_cast<double>(cyc) / (static_cast<double>(rt1 - rt0) / 100.0);  // ticks per us
        clocks.push_back(mhz);
        per_xcd[x].push_back(mhz);
      }
    }
    out->mfma_xccs = __builtin_popcount(xmask);
    if (!clocks.empty()) {
      out->clock_mhz_min = *std::min_element(clocks.begin(), clocks.end());
      out->clock_mhz_max = *std::max_element(clocks.begin(), clocks.end());
      out->clock_mhz_median = median_of(clocks);
    }
    for (int x = 0; x < 16; ++x) out->xcd_clock_mhz[x] = median_of(per_xcd[x]);
    out->ok = out->hbm_bad_words == 0 && out->mfma_checksum_mismatch == 0 &&
              out->mfma_records_ok == static_cast<int>(burn_wgs) &&
              (out->num_xcc <= 0 || out->mfma_xccs == out->num_xcc);
    if (!out->ok)
      std::snprintf(out->error, sizeof(out->error),
                    "hbm_bad_words=%llu first_bad_unit=%lld mfma records %d/%u checksum mismatches %d, %d/%d XCDs ran",
                    static_cast<unsigned long long>(out->hbm_bad_words), static_cast<long long>(out->hbm_first_bad),
                    out->mfma_records_ok, burn_wgs, out->mfma_checksum_mismatch, out->mfma_xccs, out->num_xcc);
  }
  free_bufs();
  return finish();
}
