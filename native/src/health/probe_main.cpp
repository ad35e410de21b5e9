// mi355x-liveness-probe: run the gfx950 MFMA liveness kernel on GPU agents
// and print one JSON document.
//
//   mi355x-liveness-probe [--devices all|0,2,..] [--nonce N] [--iters N] [--identify] [--timeout S]
//   mi355x-liveness-probe --serve [--keep]  (long-lived; requests on stdin, see serve())
//   mi355x-liveness-probe --sweep [--devices ..]   (every CU of every XCD, see mi355x_chip_sweep)
//   mi355x-liveness-probe --perf [--perf-mib M]     (HBM bandwidth + pattern, sustained MFMA rate, clocks)
//   mi355x-liveness-probe --peer [--devices ..] [--peer-bytes B] [--peer-reps R]
//                                      (DMA copy over every GPU pair's link, verified)
//   --corrupt-word K[@O] / $MI355X_PROBE_CORRUPT_FILE: debug fault injection (see refresh_fault_injection)
//
// Built twice from this file: `mi355x-liveness-probe` launches through ROCr
// directly (MI355X_PROBE_HSA; links only libhsa-runtime64, one AQL dispatch),
// `mi355x-liveness-probe-hip` through the HIP runtime.
//
// Exit status: 0 all probed devices live, 1 at least one failed, 2 usage or
// HIP runtime unavailable. The parent (the plugin's health loop, or the
// benchmark's fake container runtime) enforces the deadline by killing us.
#include <signal.h>
#include <sys/prctl.h>
#include <sys/resource.h>
#include <unistd.h>
#include <time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "init_sampler.h"
#include "mi355x/liveness_probe.h"

// defined by the container-emulation builds (native/tools/probe_emu.cpp) only
extern "C" __attribute__((weak)) const char* mi355x_probe_view_json();

namespace {

double cpu_ms(double* user_ms = nullptr) {
  rusage ru;
  getrusage(RUSAGE_SELF, &ru);
  if (user_ms) *user_ms = ru.ru_utime.tv_sec * 1e3 + ru.ru_utime.tv_usec / 1e3;
  return (ru.ru_utime.tv_sec + ru.ru_stime.tv_sec) * 1e3 + (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec) / 1e3;
}

// read syscalls issued so far (/proc/self/io "syscr"): ROCr's start-up is
// dominated by walking the kfd topology in sysfs, this makes that visible.
long long read_syscalls() {
  FILE* f = std::fopen("/proc/self/io", "r");
  if (!f) return -1;
  char line[128];
  long long v = -1;
  while (std::fgets(line, sizeof(line), f))
    if (std::sscanf(line, "syscr: %lld", &v) == 1) break;
  std::fclose(f);
  return v;
}

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<uint64_t>(ts.tv_sec) * 1000000000ull + ts.tv_nsec;
}

std::string json_escape(const char* s) {
  std::string o;
  for (; *s; ++s) {
    char c = *s;
    if (c == '"' || c == '\\') {
      o += '\\';
      o += c;
    } else if (static_cast<unsigned char>(c) < 0x20) {
      char b[8];
      std::snprintf(b, sizeof(b), "\\u%04x", c);
      o += b;
    } else {
      o += c;
    }
  }
  return o;
}

// phase_us of one device: HSA build = code object, queue, buffers, dispatch;
// HIP build = hipSetDevice + identity, the stream's queue, buffers + events, dispatch
#ifdef MI355X_PROBE_HSA
#define PHASE_NAMES "\"code_object\":%.1f,\"queue\":%.1f,\"buffers\":%.1f,\"dispatch_wait\":%.1f"
#else
#define PHASE_NAMES "\"device\":%.1f,\"stream\":%.1f,\"buffers\":%.1f,\"dispatch_wait\":%.1f"
#endif

std::string device_json(const mi355x_probe_result& r) {
  char buf[2048];
  std::snprintf(
      buf, sizeof(buf),
      "{\"ordinal\":%d,\"ok\":%s,\"hip_error\":%d,\"mismatches\":%d,\"nonce\":%u,\"xcc_id\":%u,"
      "\"hw_id\":%u,\"iters\":%d,\"dispatches\":%d,\"kfd_node_id\":%d,\"runtime\":\"%s\","
      "\"kernel_us\":%.3f,\"setup_us\":%.3f,\"total_us\":%.3f,"
      "\"phase_us\":{" PHASE_NAMES "},"
      "\"pci_bus_id\":\"%s\","
      "\"arch\":\"%s\",\"name\":\"%s\",\"uuid\":\"%s\",\"pci_domain\":%d,\"pci_bus\":%d,"
      "\"pci_device\":%d,\"cu_count\":%d,\"total_mem\":%llu,\"late\":%s,\"pending_s\":%.3f,\"error\":\"%s\"}",
      r.ordinal, r.ok ? "true" : "false", r.hip_error, r.mismatches, r.nonce, r.xcc_id, r.hw_id, r.iters,
      r.dispatches, r.kfd_node_id, r.runtime, r.kernel_us, r.setup_us, r.total_us, r.phase_us[0], r.phase_us[1],
      r.phase_us[2], r.phase_us[3], json_escape(r.pci_bus_id).c_str(), json_escape(r.arch).c_str(),
      json_escape(r.name).c_str(), json_escape(r.uuid).c_str(), r.pci_domain, r.pci_bus, r.pci_device,
      r.cu_count, static_cast<unsigned long long>(r.total_mem), r.late ? "true" : "false", r.pending_s,
      json_escape(r.error).c_str());
  return buf;
}

#ifdef MI355X_PROBE_HSA
int device_count() { return mi355x_hsa_probe_init(); }
int probe(int o, uint32_t nonce, int iters, double timeout_s, mi355x_probe_result* r) {
  return mi355x_hsa_probe_device(o, nonce, iters, timeout_s, r);
}
int identify_dev(int o, mi355x_probe_result* r) { return mi355x_hsa_probe_identify(o, r); }
int peer(int a, int b, uint32_t nonce, uint64_t bytes, int reps, double timeout_s, mi355x_peer_result* r) {
  return mi355x_hsa_peer_probe(a, b, nonce, bytes, reps, timeout_s, r);
}
int chip_sweep(int o, uint32_t nonce, int iters, double timeout_s, mi355x_sweep_result* r) {
  return mi355x_hsa_chip_sweep(o, nonce, iters, timeout_s, r);
}
int perf_check(int o, uint32_t nonce, uint64_t bytes, int iters, double timeout_s, mi355x_perf_result* r) {
  return mi355x_hsa_perf_check(o, nonce, bytes, iters, timeout_s, r);
}
void perf_poison(uint64_t unit) { mi355x_hsa_perf_poison(unit); }
void init_phases(double out[5]) { mi355x_hsa_init_phases(out); }
void defer_teardown() { mi355x_hsa_probe_defer_release(1); }
void teardown() { mi355x_hsa_probe_release(); }
void runtime_shutdown() { mi355x_hsa_probe_shutdown(); }
void keep_resources(bool on) { mi355x_hsa_probe_keep(on ? 1 : 0); }
void set_corrupt(int word, int ordinal) { mi355x_hsa_probe_corrupt(word, ordinal); }
void set_stream_mode(bool) {}  // the HSA path has one queue per device
#else
void set_stream_mode(bool own) { mi355x_probe_set_stream_mode(own ? 1 : 0); }
void set_corrupt(int, int) {}
void keep_resources(bool) {}  // the HIP build reuses its runtime's queues anyway
void init_phases(double out[5]) { out[0] = out[1] = out[2] = out[3] = out[4] = 0; }
void defer_teardown() { mi355x_probe_defer_release(1); }
void teardown() { mi355x_probe_release(); }
void runtime_shutdown() {}
int device_count() { return mi355x_probe_device_count(); }
int probe(int o, uint32_t nonce, int iters, double, mi355x_probe_result* r) {
  return mi355x_probe_device(o, nonce, iters, r);
}
int identify_dev(int o, mi355x_probe_result* r) { return mi355x_probe_identify(o, r); }
int chip_sweep(int o, uint32_t nonce, int iters, double, mi355x_sweep_result* r) {
  std::memset(r, 0, sizeof(*r));
  r->ordinal = o;
  r->nonce = nonce;
  r->iters = iters;
  std::snprintf(r->error, sizeof(r->error), "--sweep needs the HSA-direct build (mi355x-liveness-probe)");
  return 1;
}
void perf_poison(uint64_t) {}
int perf_check(int o, uint32_t nonce, uint64_t bytes, int iters, double, mi355x_perf_result* r) {
  std::memset(r, 0, sizeof(*r));
  r->ordinal = o;
  r->nonce = nonce;
  r->bytes = bytes;
  r->mfma_iters = iters;
  std::snprintf(r->error, sizeof(r->error), "--perf needs the HSA-direct build (mi355x-liveness-probe)");
  return 1;
}
int peer(int a, int b, uint32_t, uint64_t bytes, int reps, double, mi355x_peer_result* r) {
  std::memset(r, 0, sizeof(*r));
  r->src = a;
  r->dst = b;
  r->bytes = bytes;
  r->reps = reps;
  std::snprintf(r->error, sizeof(r->error), "--peer needs the HSA-direct build (mi355x-liveness-probe)");
  return 1;
}
#endif

// Debug fault injection for tests of the verdict path on real hardware:
// "K" or "K@O" (flip one bit of output word K, on ordinal O only) from
// --corrupt-word, or from the file named by $MI355X_PROBE_CORRUPT_FILE, which
// is re-read before every request so a test can turn it on and off under a
// running server. Empty / missing = off.
int g_flag_corrupt_word = -1;
int g_flag_corrupt_ordinal = -1;

void parse_corrupt(const char* spec, int* word, int* ordinal) {
  *word = -1;
  *ordinal = -1;
  if (!spec || !*spec) return;
  char* end = nullptr;
  const long w = std::strtol(spec, &end, 0);
  if (end == spec) return;
  *word = static_cast<int>(w);
  if (*end == '@') *ordinal = std::atoi(end + 1);
}

void refresh_fault_injection() {
  int word = g_flag_corrupt_word, ordinal = g_flag_corrupt_ordinal;
  if (const char* path = std::getenv("MI355X_PROBE_CORRUPT_FILE")) {
    char buf[64] = {0};
    if (FILE* f = std::fopen(path, "r")) {
      if (!std::fgets(buf, sizeof(buf), f)) buf[0] = 0;
      std::fclose(f);
    }
    int fw, fo;
    parse_corrupt(buf, &fw, &fo);
    if (fw >= 0) {
      word = fw;
      ordinal = fo;
    }
  }
  set_corrupt(word, ordinal);
}

// Probe (or identify) a set of ordinals, one host thread per GPU so an 8-GPU
// request pays one device setup, not eight. Returns true when all are live.
bool run_batch(const std::vector<int>& ords, const std::vector<uint32_t>& nonces, int iters,
               const std::vector<double>& timeouts, bool identify, int n, std::vector<mi355x_probe_result>& results) {
  results.assign(ords.size(), mi355x_probe_result{});
  std::vector<int> rcs(ords.size(), 1);
  auto run_one = [&](size_t i) {
    if (ords[i] < 0 || ords[i] >= n) {
      results[i].ordinal = ords[i];
      std::snprintf(results[i].error, sizeof(results[i].error), "no such GPU (count=%d)", n);
      return;
    }
    rcs[i] = identify ? identify_dev(ords[i], &results[i]) : probe(ords[i], nonces[i], iters, timeouts[i], &results[i]);
    if (identify && rcs[i] == 0) results[i].ok = 1;
  };
  if (ords.size() > 1) {
    std::vector<std::thread> ths;
    for (size_t i = 0; i < ords.size(); ++i) ths.emplace_back(run_one, i);
    for (auto& t : ths) t.join();
  } else if (!ords.empty()) {
    run_one(0);
  }
  bool all_ok = !ords.empty();
  for (int rc : rcs) all_ok = all_ok && rc == 0;
  return all_ok;
}

std::string peer_json(const mi355x_peer_result& r) {
  char buf[1024];
  std::snprintf(buf, sizeof(buf),
                "{\"src\":%d,\"dst\":%d,\"src_bus_id\":\"%s\",\"dst_bus_id\":\"%s\",\"ok\":%s,\"hsa_error\":%d,"
                "\"access\":%d,\"link_type\":%d,\"hops\":%u,\"numa_distance\":%u,\"link_max_bw_mbps\":%u,"
                "\"bytes\":%llu,\"reps\":%d,\"mismatches\":%llu,\"copy_us_best\":%.2f,\"gbps_best\":%.2f,"
                "\"total_us\":%.1f,\"error\":\"%s\"}",
                r.src, r.dst, json_escape(r.src_bus_id).c_str(), json_escape(r.dst_bus_id).c_str(),
                r.ok ? "true" : "false", r.hsa_error, r.access, r.link_type, r.hops, r.numa_distance,
                r.link_max_bw_mbps, static_cast<unsigned long long>(r.bytes), r.reps,
                static_cast<unsigned long long>(r.mismatches), r.copy_us_best, r.gbps_best, r.total_us,
                json_escape(r.error).c_str());
  return buf;
}

// --peer: every ordered pair of the selected GPUs (or the one GPU with itself),
// one pair at a time so each copy has its link to itself.
int run_peer(const std::vector<int>& ords, uint32_t nonce, uint64_t bytes, int reps, double timeout_s, int n) {
  std::vector<std::pair<int, int>> pairs;
  if (ords.size() == 1) {
    pairs.emplace_back(ords[0], ords[0]);
  } else {
    for (int a : ords)
      for (int b : ords)
        if (a != b) pairs.emplace_back(a, b);
  }
  bool all_ok = !pairs.empty();
  std::string o = "[";
  for (size_t i = 0; i < pairs.size(); ++i) {
    mi355x_peer_result r;
    const int rc = peer(pairs[i].first, pairs[i].second, nonce + static_cast<uint32_t>(i), bytes, reps, timeout_s, &r);
    all_ok = all_ok && rc == 0;
    if (i) o += ",";
    o += peer_json(r);
    if (r.hsa_error == -1) break;  // a copy is still in flight: stop touching the devices
  }
  std::printf("{\"peer\":true,\"ok\":%s,\"hip_device_count\":%d,\"t_ready_ns\":%llu,\"pairs\":%s]}\n",
              all_ok ? "true" : "false", n, static_cast<unsigned long long>(mono_ns()), o.c_str());
  std::fflush(stdout);
  return all_ok ? 0 : 1;
}

std::string sweep_json(const mi355x_sweep_result& r) {
  std::string per = "[";
  for (int i = 0; i < 16 && i < (r.num_xcc > 0 ? r.num_xcc : 8); ++i) {
    if (i) per += ",";
    per += std::to_string(r.wgs_per_xcc[i]);
  }
  per += "]";
  char buf[1024];
  std::snprintf(buf, sizeof(buf),
                "{\"ordinal\":%d,\"ok\":%s,\"hsa_error\":%d,\"nonce\":%u,\"iters\":%d,\"grid\":%d,"
                "\"cu_count\":%d,\"num_xcc\":%d,\"records_ok\":%d,\"mfma_bad\":%u,\"lds_bad\":%u,"
                "\"tile_bad\":%u,\"cus_covered\":%d,\"xccs_covered\":%d,\"all_resident\":%s,"
                "\"wgs_per_xcc\":%s,\"kernel_us\":%.2f,\"arrival_spread_us\":%.2f,\"total_us\":%.1f,"
                "\"in_flight_s\":%.2f,\"kept_queue\":%s,\"error\":\"%s\"}",
                r.ordinal, r.ok ? "true" : "false", r.hsa_error, r.nonce, r.iters, r.grid, r.cu_count, r.num_xcc,
                r.records_ok, r.mfma_bad, r.lds_bad, r.tile_bad, r.cus_covered, r.xccs_covered,
                r.all_resident ? "true" : "false", per.c_str(), r.kernel_us, r.arrival_spread_us, r.total_us,
                r.in_flight_s, r.kept_queue ? "true" : "false", json_escape(r.error).c_str());
  return buf;
}

// --sweep: the full-chip sweep on each selected GPU (parallel host threads).
bool run_sweeps(const std::vector<int>& ords, const std::vector<uint32_t>& nonces, int iters,
                const std::vector<double>& timeouts, int n, std::string& json) {
  std::vector<mi355x_sweep_result> res(ords.size());
  std::vector<int> rcs(ords.size(), 1);
  auto one = [&](size_t i) {
    if (ords[i] < 0 || ords[i] >= n) {
      std::memset(&res[i], 0, sizeof(res[i]));
      res[i].ordinal = ords[i];
      std::snprintf(res[i].error, sizeof(res[i].error), "no such GPU (count=%d)", n);
      return;
    }
    rcs[i] = chip_sweep(ords[i], nonces[i], iters, timeouts[i], &res[i]);
  };
  std::vector<std::thread> ths;
  for (size_t i = 0; i < ords.size(); ++i) ths.emplace_back(one, i);
  for (auto& t : ths) t.join();
  bool ok = !ords.empty();
  json = "[";
  for (size_t i = 0; i < res.size(); ++i) {
    ok = ok && rcs[i] == 0;
    if (i) json += ",";
    json += sweep_json(res[i]);
  }
  json += "]";
  return ok;
}

std::string perf_json(const mi355x_perf_result& r) {
  std::string per = "[";
  for (int i = 0; i < 16 && i < (r.num_xcc > 0 ? r.num_xcc : 8); ++i) {
    char v[32];
    std::snprintf(v, sizeof(v), "%s%.0f", i ? "," : "", r.xcd_clock_mhz[i]);
    per += v;
  }
  per += "]";
  char buf[1536];
  std::snprintf(buf, sizeof(buf),
                "{\"ordinal\":%d,\"ok\":%s,\"hsa_error\":%d,\"nonce\":%u,\"bytes\":%llu,\"cu_count\":%d,"
                "\"num_xcc\":%d,\"fill_us\":%.1f,\"check_us\":%.1f,\"check2_us\":%.1f,\"hbm_write_gbps\":%.1f,"
                "\"hbm_read_gbps\":%.1f,\"hbm_bad_words\":%llu,\"hbm_bad_words_pass2\":%llu,\"hbm_first_bad\":%lld,\"mfma_iters\":%d,\"mfma_grid\":%d,"
                "\"mfma_records_ok\":%d,\"mfma_checksum_mismatch\":%d,\"mfma_xccs\":%d,\"mfma_us\":%.1f,"
                "\"mfma_tflops\":%.1f,\"clock_mhz_min\":%.0f,\"clock_mhz_median\":%.0f,\"clock_mhz_max\":%.0f,"
                "\"xcd_clock_mhz\":%s,\"total_us\":%.1f,\"in_flight_s\":%.2f,\"kept_queue\":%s,\"error\":\"%s\"}",
                r.ordinal, r.ok ? "true" : "false", r.hsa_error, r.nonce, static_cast<unsigned long long>(r.bytes),
                r.cu_count, r.num_xcc, r.fill_us, r.check_us, r.check2_us, r.hbm_write_gbps, r.hbm_read_gbps,
                static_cast<unsigned long long>(r.hbm_bad_words), static_cast<unsigned long long>(r.hbm_bad_words_pass2), static_cast<long long>(r.hbm_first_bad),
                r.mfma_iters, r.mfma_grid, r.mfma_records_ok, r.mfma_checksum_mismatch, r.mfma_xccs, r.mfma_us,
                r.mfma_tflops, r.clock_mhz_min, r.clock_mhz_median, r.clock_mhz_max, per.c_str(), r.total_us,
                r.in_flight_s, r.kept_queue ? "true" : "false", json_escape(r.error).c_str());
  return buf;
}

// --perf: the throughput check on each selected GPU (parallel host threads;
// every GPU has its own HBM and matrix cores).
bool run_perf(const std::vector<int>& ords, const std::vector<uint32_t>& nonces, uint64_t bytes, int iters,
              const std::vector<double>& timeouts, int n, std::string& json) {
  std::vector<mi355x_perf_result> res(ords.size());
  std::vector<int> rcs(ords.size(), 1);
  auto one = [&](size_t i) {
    if (ords[i] < 0 || ords[i] >= n) {
      std::memset(&res[i], 0, sizeof(res[i]));
      res[i].ordinal = ords[i];
      std::snprintf(res[i].error, sizeof(res[i].error), "no such GPU (count=%d)", n);
      return;
    }
    rcs[i] = perf_check(ords[i], nonces[i], bytes, iters, timeouts[i], &res[i]);
  };
  std::vector<std::thread> ths;
  for (size_t i = 0; i < ords.size(); ++i) ths.emplace_back(one, i);
  for (auto& t : ths) t.join();
  bool ok = !ords.empty();
  json = "[";
  for (size_t i = 0; i < res.size(); ++i) {
    ok = ok && rcs[i] == 0;
    if (i) json += ",";
    json += perf_json(res[i]);
  }
  json += "]";
  return ok;
}

std::string devices_json(const std::vector<mi355x_probe_result>& results) {
  std::string o = "[";
  for (size_t i = 0; i < results.size(); ++i) {
    if (i) o += ",";
    o += device_json(results[i]);
  }
  return o + "]";
}

// --serve: a long-lived prober for the plugin's health loop. The runtime is
// initialised once; every request line
//     [@<id> ]probe <iters> <timeout_s> <ordinal>:<nonce>[:<deadline_s>] ...
//     [@<id> ]sweep <iters> <timeout_s> <ordinal>:<nonce>[:<deadline_s>] ...
//     [@<id> ]perf <mfma_iters> <timeout_s> <mib> <ordinal>:<nonce>[:<deadline_s>] ...
// is answered with one JSON line {"id":..,"ok":..,"t_ready_ns":..,"devices":[..]}
// ("id" only for a tagged request). A device's own deadline replaces the
// request's timeout for that device: the plugin gives GPUs that run other
// processes' kernels a short one, since a dispatch queued behind them is
// inconclusive anyway and its verdict is collected by the next request.
// Tagged requests are answered on worker threads, in completion order (the
// HSA build): a PreStartContainer check of one GPU never waits behind a
// health sweep still waiting for another GPU. Requests on the same device
// serialise on its kept queue (each waits no longer than its own deadline).
// "quit" or EOF on stdin ends the server, and so does the parent's death
// (PR_SET_PDEATHSIG). Spawning a fresh probe process per pulse would create
// and tear down a kfd process each time, and a GPU process that starts while
// such a teardown is in flight blocks in open("/dev/kfd") for up to ~150 ms
// (profiles/archive/measurements_r1_r3.md §3c): a pod admitted during a health sweep would pay it.
// With --keep the per-device queue, executable and buffers also stay: a probe
// is then one AQL packet, with no queue creation (an HWS runlist update that
// preempts every queue on that GPU, ~5 ms, profiles/archive/measurements_r1_r3.md §3f) per pulse.
#ifdef MI355X_PROBE_HSA
constexpr bool kConcurrentServe = true;
#else
constexpr bool kConcurrentServe = false;  // the HIP build answers in order
#endif
constexpr int kMaxServeWorkers = 64;  // beyond this a tagged request is answered inline

struct ServeRequest {
  bool tagged = false;
  unsigned long long id = 0;
  std::string kind;  // probe | sweep | perf
  int iters = 0;
  double timeout_s = 0;
  unsigned long long perf_mib = 0;
  std::vector<int> ords;
  std::vector<uint32_t> nonces;
  std::vector<double> timeouts;  // per device
};

bool parse_request(const std::string& line, ServeRequest* r) {
  const char* p = line.c_str();
  if (*p == '@') {
    char* end = nullptr;
    r->id = std::strtoull(p + 1, &end, 10);
    if (end == p + 1 || *end != ' ') return false;
    r->tagged = true;
    p = end + 1;
  }
  int consumed = 0;
  bool parsed = false;
  if (std::strncmp(p, "perf ", 5) == 0) {
    r->kind = "perf";
    parsed = std::sscanf(p, "perf %d %lf %llu %n", &r->iters, &r->timeout_s, &r->perf_mib, &consumed) >= 3;
  } else if (std::strncmp(p, "sweep ", 6) == 0) {
    r->kind = "sweep";
    parsed = std::sscanf(p, "sweep %d %lf %n", &r->iters, &r->timeout_s, &consumed) >= 2;
  } else if (std::strncmp(p, "probe ", 6) == 0) {
    r->kind = "probe";
    parsed = std::sscanf(p, "probe %d %lf %n", &r->iters, &r->timeout_s, &consumed) >= 2;
  }
  if (!parsed || consumed == 0) return false;
  p += consumed;
  while (*p) {
    char* end = nullptr;
    const long o = std::strtol(p, &end, 10);
    if (end == p || *end != ':') break;
    p = end + 1;
    const unsigned long nc = std::strtoul(p, &end, 0);
    if (end == p) break;
    p = end;
    double dl = r->timeout_s;
    if (*p == ':') {
      const double v = std::strtod(p + 1, &end);
      if (end == p + 1) break;
      if (v > 0) dl = v;
      p = end;
    }
    r->ords.push_back(static_cast<int>(o));
    r->nonces.push_back(static_cast<uint32_t>(nc));
    r->timeouts.push_back(dl);
    while (*p == ' ') ++p;
  }
  return true;
}

std::mutex g_out_mu;

void emit_line(const std::string& s) {
  std::lock_guard<std::mutex> lk(g_out_mu);
  std::fputs(s.c_str(), stdout);
  std::fputc('\n', stdout);
  std::fflush(stdout);
}

std::string id_field(const ServeRequest& r) {
  return r.tagged ? "\"id\":" + std::to_string(r.id) + "," : std::string();
}

// One request, start to reply line; then the runtime's deferred frees.
void answer(const ServeRequest& r, int n) {
  refresh_fault_injection();
  defer_teardown();
  std::string body;
  bool ok;
  if (r.kind == "sweep") {
    ok = run_sweeps(r.ords, r.nonces, r.iters, r.timeouts, n, body);
  } else if (r.kind == "perf") {
    ok = run_perf(r.ords, r.nonces, static_cast<uint64_t>(r.perf_mib) << 20, r.iters, r.timeouts, n, body);
  } else {
    std::vector<mi355x_probe_result> results;
    ok = run_batch(r.ords, r.nonces, r.iters, r.timeouts, false, n, results);
    body = devices_json(results);
  }
  char head[256];
  std::snprintf(head, sizeof(head), "{%s\"ok\":%s,\"hip_device_count\":%d,\"sweep\":%s,\"perf\":%s,\"t_ready_ns\":%llu,",
                id_field(r).c_str(), ok ? "true" : "false", n, r.kind == "sweep" ? "true" : "false",
                r.kind == "perf" ? "true" : "false", static_cast<unsigned long long>(mono_ns()));
  emit_line(std::string(head) + "\"devices\":" + body + "}");
  teardown();  // queues/executables go, the runtime (and the kfd process) stays
}

// Tagged requests go to a pool of worker threads that stay for the server's
// life (a thread per request cost its creation on every probe); the pool
// grows while every worker is busy -- a request stuck on a wedged device
// holds its worker, not the others -- up to kMaxServeWorkers, beyond which
// a request is answered inline.
struct ServePool {
  std::mutex mu;
  std::condition_variable cv, done;
  std::deque<ServeRequest> q;
  int workers = 0, idle = 0, busy = 0;
  bool stop = false;
};

void serve_worker(ServePool* pool, int n) {
  while (true) {
    ServeRequest r;
    {
      std::unique_lock<std::mutex> lk(pool->mu);
      pool->idle++;
      pool->cv.wait(lk, [pool] { return pool->stop || !pool->q.empty(); });
      pool->idle--;
      if (pool->q.empty()) return;  // stopping
      r = std::move(pool->q.front());
      pool->q.pop_front();
      pool->busy++;
    }
    answer(r, n);  // no lock held: a request may take its whole deadline
    {
      std::lock_guard<std::mutex> lk(pool->mu);
      pool->busy--;
    }
    pool->done.notify_all();
  }
}

int serve(int n, uint64_t t_start, uint64_t t_runtime) {
  prctl(PR_SET_PDEATHSIG, SIGKILL);
  if (getppid() == 1) return 0;  // parent already gone
  char hello[320];
  std::snprintf(hello, sizeof(hello),
                "{\"serve\":true,\"ok\":%s,\"hip_device_count\":%d,\"concurrent\":%s,\"deadlines\":true,"
                "\"t_start_ns\":%llu,\"t_runtime_ns\":%llu}",
                n >= 0 ? "true" : "false", n < 0 ? 0 : n, kConcurrentServe ? "true" : "false",
                static_cast<unsigned long long>(t_start), static_cast<unsigned long long>(t_runtime));
  emit_line(hello);
  if (n < 0) return 2;
  ServePool pool;
  std::vector<std::thread> threads;
  std::string line;
  char buf[8192];
  while (std::fgets(buf, sizeof(buf), stdin)) {
    line = buf;
    while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.pop_back();
    if (line.empty()) continue;
    if (line == "quit") break;
    ServeRequest r;
    if (!parse_request(line, &r)) {
      emit_line("{" + id_field(r) + "\"ok\":false,\"error\":\"bad request\",\"devices\":[]}");
      continue;
    }
    bool queued = false;
    if (r.tagged && kConcurrentServe) {
      std::lock_guard<std::mutex> lk(pool.mu);
      if (pool.idle > static_cast<int>(pool.q.size()) || pool.workers < kMaxServeWorkers) {
        if (pool.idle <= static_cast<int>(pool.q.size())) {
          pool.workers++;
          threads.emplace_back(serve_worker, &pool, n);
        }
        pool.q.push_back(std::move(r));
        pool.cv.notify_one();
        queued = true;
      }
    }
    if (!queued) answer(r, n);
  }
  {
    // every worker's waits are bounded by its deadlines; one stuck inside the
    // runtime past that keeps the runtime up: exit without shutting it down
    std::unique_lock<std::mutex> lk(pool.mu);
    const bool drained =
        pool.done.wait_for(lk, std::chrono::seconds(60), [&] { return pool.q.empty() && pool.busy == 0; });
    if (!drained) {
      std::fflush(stdout);
      std::_Exit(0);
    }
    pool.stop = true;
    pool.cv.notify_all();
  }
  for (auto& t : threads) t.join();
  runtime_shutdown();
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const uint64_t t_start = mono_ns();
  std::string devices = "all";
  uint32_t nonce = static_cast<uint32_t>(t_start ^ (t_start >> 32));
  int iters = 4;
  double timeout_s = 5.0;
  bool identify = false;
  int sample_us = 0;
  std::string exit_mode = "shutdown";
  bool serve_mode = false;
  bool keep = false;  // --serve --keep: per-device queue/executable/buffers live across requests
  bool peer_mode = false;
  bool sweep_mode = false;
  bool perf_mode = false;
  uint64_t perf_mib = 4096;
  int perf_iters = 1 << 16;
  uint64_t peer_bytes = 64ull << 20;
  int peer_reps = 3;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&](const char* what) -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", what);
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--devices") {
      devices = next("--devices");
    } else if (a == "--nonce") {
      nonce = static_cast<uint32_t>(std::strtoul(next("--nonce"), nullptr, 0));
    } else if (a == "--iters") {
      iters = std::atoi(next("--iters"));
    } else if (a == "--timeout") {
      timeout_s = std::atof(next("--timeout"));
    } else if (a == "--sample-init") {
      sample_us = std::atoi(next("--sample-init"));
    } else if (a == "--exit") {
      exit_mode = next("--exit");
      if (exit_mode != "shutdown" && exit_mode != "release" && exit_mode != "fast") {
        std::fprintf(stderr, "--exit must be shutdown|release|fast\n");
        return 2;
      }
    } else if (a == "--identify") {
      identify = true;
    } else if (a == "--serve") {
      serve_mode = true;
    } else if (a == "--keep") {
      keep = true;
    } else if (a == "--peer") {
      peer_mode = true;
    } else if (a == "--sweep") {
      sweep_mode = true;
    } else if (a == "--perf") {
      perf_mode = true;
    } else if (a == "--perf-mib") {
      perf_mib = std::strtoull(next("--perf-mib"), nullptr, 0);
    } else if (a == "--perf-iters") {
      perf_iters = std::atoi(next("--perf-iters"));
    } else if (a == "--poison-hbm") {
      perf_poison(std::strtoull(next("--poison-hbm"), nullptr, 0));
    } else if (a == "--peer-bytes") {
      peer_bytes = std::strtoull(next("--peer-bytes"), nullptr, 0);
    } else if (a == "--corrupt-word") {
      parse_corrupt(next("--corrupt-word"), &g_flag_corrupt_word, &g_flag_corrupt_ordinal);
    } else if (a == "--hip-stream") {
      const std::string m = next("--hip-stream");
      if (m != "own" && m != "null") {
        std::fprintf(stderr, "--hip-stream must be own|null\n");
        return 2;
      }
      set_stream_mode(m == "own");
    } else if (a == "--peer-reps") {
      peer_reps = std::atoi(next("--peer-reps"));
    } else if (a == "-h" || a == "--help") {
      std::printf("usage: %s [--devices all|0,1,..] [--nonce N] [--iters N] [--identify] [--timeout S] "
                  "[--sample-init PERIOD_US] [--exit shutdown|release|fast] [--serve [--keep]] [--peer [--peer-bytes B] [--peer-reps R]] [--sweep] "
                  "[--perf [--perf-mib M] [--perf-iters N] [--poison-hbm UNIT]] "
                  "[--corrupt-word K[@ORDINAL]] [--hip-stream own|null]\n",
                  argv[0]);
      return 0;
    } else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }

  mi355x::InitSampler sampler(sample_us > 0 ? sample_us : 1);
  if (sample_us > 0) sampler.start();
  const int n = device_count();
  if (sample_us > 0) sampler.stop();
  const std::string init_profile = sample_us > 0 ? sampler.json() : "null";
  const uint64_t t_runtime = mono_ns();  // HIP runtime + ROCr initialised
  double cpu_user_runtime = 0;
  const double cpu_runtime = cpu_ms(&cpu_user_runtime);
  const long long syscr_runtime = read_syscalls();
  // the view's effect on the runtime's start-up walk, read at the same point as syscr
  const std::string view_runtime = mi355x_probe_view_json ? mi355x_probe_view_json() : "";
  double iph[5];
  init_phases(iph);
  if (serve_mode) {
    keep_resources(keep);
    return serve(n, t_start, t_runtime);
  }
  if (n < 0) {
    std::printf("{\"ok\":false,\"hip_device_count\":0,\"error\":\"GPU runtime init failed (%d)\",\"devices\":[],"
                "\"t_start_ns\":%llu,\"t_ready_ns\":0,\"init_profile\":%s}\n",
                -n, static_cast<unsigned long long>(t_start), init_profile.c_str());
    return 2;
  }
  std::vector<int> ords;
  if (devices == "all") {
    for (int i = 0; i < n; ++i) ords.push_back(i);
  } else {
    size_t pos = 0;
    while (pos <= devices.size()) {
      size_t c = devices.find(',', pos);
      if (c == std::string::npos) c = devices.size();
      std::string tok = devices.substr(pos, c - pos);
      if (!tok.empty()) ords.push_back(std::atoi(tok.c_str()));
      pos = c + 1;
    }
  }

  if (peer_mode) return run_peer(ords, nonce, peer_bytes, peer_reps, timeout_s, n);
  std::vector<uint32_t> nonces;
  for (size_t i = 0; i < ords.size(); ++i) nonces.push_back(nonce + static_cast<uint32_t>(i));
  const std::vector<double> timeouts(ords.size(), timeout_s);
  if (perf_mode) {
    std::string body;
    const bool ok = run_perf(ords, nonces, perf_mib << 20, perf_iters, timeouts, n, body);
    std::printf("{\"ok\":%s,\"perf\":true,\"hip_device_count\":%d,\"t_start_ns\":%llu,\"t_runtime_ns\":%llu,"
                "\"t_ready_ns\":%llu,\"devices\":%s}\n",
                ok ? "true" : "false", n, static_cast<unsigned long long>(t_start),
                static_cast<unsigned long long>(t_runtime), static_cast<unsigned long long>(mono_ns()), body.c_str());
    std::fflush(stdout);
    return ok ? 0 : 1;
  }
  if (sweep_mode) {
    std::string body;
    const bool ok = run_sweeps(ords, nonces, iters, timeouts, n, body);
    std::printf("{\"ok\":%s,\"sweep\":true,\"hip_device_count\":%d,\"t_start_ns\":%llu,\"t_runtime_ns\":%llu,"
                "\"t_ready_ns\":%llu,\"devices\":%s}\n",
                ok ? "true" : "false", n, static_cast<unsigned long long>(t_start),
                static_cast<unsigned long long>(t_runtime), static_cast<unsigned long long>(mono_ns()), body.c_str());
    std::fflush(stdout);
    return ok ? 0 : 1;
  }
  std::vector<mi355x_probe_result> results;
  // Queues/executables are torn down after the verdict is printed: the caller
  // (container runtime, health loop) only waits for the JSON line.
  refresh_fault_injection();
  defer_teardown();
  const bool all_ok = run_batch(ords, nonces, iters, timeouts, identify, n, results);
  const uint64_t t_ready = mono_ns();
  const double cpu_ready = cpu_ms();
  std::printf("{\"ok\":%s,\"hip_device_count\":%d,\"identify\":%s,\"t_start_ns\":%llu,\"t_runtime_ns\":%llu,"
              "\"t_ready_ns\":%llu,\"cpu_ms_runtime\":%.2f,\"cpu_user_ms_runtime\":%.2f,\"cpu_ms_ready\":%.2f,\"read_syscalls_runtime\":%lld,"
              "\"init_us\":{\"dlopen\":%.1f,\"kfd_open\":%.1f,\"hsa_init\":%.1f,\"agents\":%.1f,\"pools\":%.1f},\"init_profile\":%s,"
              "\"view\":%s,\"devices\":%s}\n",
              all_ok ? "true" : "false", n, identify ? "true" : "false", static_cast<unsigned long long>(t_start),
              static_cast<unsigned long long>(t_runtime), static_cast<unsigned long long>(t_ready), cpu_runtime,
              cpu_user_runtime, cpu_ready, syscr_runtime, iph[0], iph[1], iph[2], iph[3], iph[4], init_profile.c_str(),
              mi355x_probe_view_json ? view_runtime.c_str() : "null", devices_json(results).c_str());
  std::fflush(stdout);
  // After the verdict. The exit mode was an experiment: the kernel's kfd
  // process teardown after we are gone costs the same either way
  // (profiles/archive/measurements_r1_r3.md §3c).
  const int code = all_ok ? 0 : 1;
  if (exit_mode == "fast") std::_Exit(code);
  teardown();
  if (exit_mode == "shutdown") runtime_shutdown();
  return code;
}
