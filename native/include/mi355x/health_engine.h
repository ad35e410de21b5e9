// Per-device health for the container (KFD) mode, natively: the same sources
// and policy as the Python health monitor (rocm_k8s_device_plugin_amd/health/
// monitor.py, liveness.py), so the interpreter-free daemon runs the north-star
// health path.
//
// Reference: a node-global verdict ("Healthy" if any kfd node is a live GPU)
// copied onto every device and overridden per PCI BDF by the metrics exporter
// (internal/pkg/amdgpu/amdgpu.go:322-345,865-974; internal/pkg/exporter/
// health.go:41-79). Here every device gets its own verdict; it is Healthy only
// if every available source agrees:
//
//   kfd       the device's own kfd node still exists and is a live GPU node
//   exporter  metricssvc.MetricsService/List, per BDF, applied to every
//             partition of that BDF (10 s deadline, never on the control loop)
//   liveness  the gfx950 MFMA probe on that exact ROCr agent, from a persistent
//             `mi355x-liveness-probe --serve [--keep]` child: nonce-checked,
//             identity-checked (the replying agent's PCI location must be the
//             device's), hysteresis (fail / recover thresholds), a busy grace
//             for probes queued behind a tenant's kernel (kfd process list;
//             shorter when it is unreadable) that ends early when amd-smi
//             reports 0% GFX activity, crowded GPUs skipped (the server steps
//             off them), server failures isolated per device in fresh
//             processes, and server-only failures confirmed in a fresh
//             process before they count
//   amd-smi   a rise of the uncorrectable ECC count; a gpu_pre_reset event
//             keeps the device Unhealthy until its gpu_post_reset
//
// and, as a placement input rather than a verdict, xGMI link state
// (-smi_xgmi, health/fabric.py): a link up in the first reading and down
// later degrades that GPU pair (or every xGMI pair of the GPU when amd-smi
// cannot name the peer); the daemon re-initialises its allocators with the
// degraded pairs scoring as the worst link. The devices stay Healthy.
//
// sweep() blocks (probes, exporter, amd-smi) and is meant for a worker
// thread; snapshot() may be called from any thread.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "mi355x/gpu_discovery.h"
#include "mi355x/kfd_topology.h"
#include "mi355x/smi_query.h"

namespace mi355x {
class SmiEventWatcher;
}

namespace mi355x::health {

struct ProbeOutcome {
  bool ok = false;
  bool pending = false;    // the dispatch is still queued (kept slot) or missed its deadline on a busy GPU
  bool interrupted = false;  // shutdown cut the probe short: no verdict either way
  bool queue_lost = false;   // a dispatch timed out on a queue the server cannot free (no kept queues)
  std::string reason;
  double latency_ms = 0;
  int kfd_node_id = -1;    // identity of the agent that answered (-1 / "" = not reported)
  std::string pci_bus_id;  // dddd:bb:dd.f
  // throughput check replies: cu_count, hbm_read_gbps, hbm_write_gbps, hbm_bad_words, mfma_tflops,
  // clock_mhz_median, total_us
  std::map<std::string, double> detail;
  std::vector<double> xcd_clock_mhz;
};

struct ProberConfig {
  std::vector<std::string> argv_prefix;  // e.g. {"python3"} for a scripted stand-in
  std::string exe;                       // mi355x-liveness-probe
  double timeout_s = 10.0;
  // a probe on a GPU other processes have queues on: that long, not timeout_s.
  // A dispatch queued behind a tenant's kernel is inconclusive whenever it
  // ends, and with kept queues its verdict is collected by the next request.
  double busy_deadline_s = 0.05;
  int iters = 4;
  int max_parallel = 8;
  bool persistent = true;                // one --serve child, else a process per device per sweep
  bool keep_queues = true;               // --serve --keep
  std::vector<std::pair<std::string, std::string>> extra_env;
  std::string kfd_proc_dir = "/sys/class/kfd/kfd/proc";
  int perf_mib = 4096;        // throughput check: HBM buffer
  int perf_iters = 1 << 16;   // throughput check: MFMA pairs per wave
};

// The probe processes (LivenessProber in health/liveness.py).
//
// Two kinds of callers share one kept-queue probe server:
//   the health sweep  probe() / probe_ordinal() / set_visible() / close(): one
//                     caller at a time (Engine::sweep); it alone starts,
//                     restarts and stops the server and runs the fallback to
//                     per-device processes.
//   PreStartContainer check(): any thread, at the same time as a sweep. Every
//                     request is tagged and the server answers tagged requests
//                     concurrently, so a check waits for its own GPUs only,
//                     never behind a sweep's wait on another GPU.
class LivenessProber {
 public:
  explicit LivenessProber(ProberConfig cfg);
  ~LivenessProber();
  LivenessProber(const LivenessProber&) = delete;
  LivenessProber& operator=(const LivenessProber&) = delete;

  // host ROCr ordinal -> outcome. `busy`: ordinals whose GPU runs other
  // processes' queues (a pending dispatch there is not re-probed, and with
  // kept queues they get busy_deadline_s).
  std::map<int, ProbeOutcome> probe(const std::vector<int>& ordinals, const std::set<int>& busy = {},
                                    const std::string& kind = "probe");
  // one device in a fresh process (ROCR_VISIBLE_DEVICES=<ordinal>)
  ProbeOutcome probe_ordinal(int ordinal, const std::string& kind = "probe");
  // A PreStartContainer check within `budget_s`, on the running server:
  //   1. every GPU with busy_deadline_s (an idle GPU answers in microseconds);
  //   2. only if some did not pass: `busy_of()` (ordinals other processes
  //      use, a kfd process-list scan). A pending dispatch on a busy GPU is
  //      inconclusive; on an idle one the same dispatch gets until 40% of the
  //      budget;
  //   3. a fresh process for each GPU the server failed or could not answer
  //      for (a pending one only where idle), while at least 1 s is left.
  // Whatever the budget leaves unsettled comes back pending. Never starts,
  // restarts or stops the server; a failure a fresh process does not confirm
  // asks the next sweep to restart it. Leaves the sweep's backoff and counters alone.
  std::map<int, ProbeOutcome> check(const std::vector<int>& ordinals, const std::function<std::set<int>()>& busy_of,
                                    double budget_s);
  // restrict the server to these host ordinals (nullopt = all); a change restarts it
  void set_visible(std::optional<std::vector<int>> ordinals);
  void close();
  bool server_running() const;
  int server_pid() const;  // -1 when none is running
  // the running server's kfd proc entry names (empty while ambiguous / unknown)
  std::set<std::string> own_kfd_entries(const std::set<int64_t>& gpu_ids);
  // a readable fd ends every wait at once (shutdown)
  void set_abort_fd(int fd) { abort_fd_ = fd; }

  // sweep path counters (check() keeps its own)
  std::atomic<int> server_starts{0}, server_restarts{0}, fallbacks{0}, sweeps{0};
  std::atomic<int> checks{0}, check_fresh{0}, check_inconclusive{0};
  const ProberConfig& config() const { return cfg_; }
  enum class Got { kLine, kTimeout, kEof, kAbort };

 private:
  struct Server;
  std::shared_ptr<Server> ensure_server(const std::vector<int>& uniq, std::string* err);
  Got transact(const std::shared_ptr<Server>& s, const std::string& body, double deadline, std::string* reply);
  // one tagged request to `s`; host ordinal -> outcome, or *err
  std::map<int, ProbeOutcome> request(const std::shared_ptr<Server>& s, const std::vector<int>& uniq,
                                      const std::string& kind, const std::map<int, double>& deadlines,
                                      double wait_until, std::string* err);
  std::map<int, ProbeOutcome> probe_server(const std::vector<int>& uniq, const std::set<int>& busy,
                                           const std::string& kind, std::string* err);
  std::map<int, ProbeOutcome> spawn_all(const std::vector<int>& ords, const std::string& kind, double timeout_s);
  double inner_timeout() const;
  ProberConfig cfg_;
  mutable std::mutex mu_;            // server_, visible_, backoff_, issued_, restart_wanted_
  std::shared_ptr<Server> server_;
  int backoff_ = 0;
  bool restart_wanted_ = false;
  // ordinal -> nonces of probe dispatches that may still answer late (kept slot)
  std::map<int, std::vector<uint32_t>> issued_;
  std::optional<std::vector<int>> visible_;
  std::atomic<uint64_t> next_id_{1};
  int abort_fd_ = -1;
};

struct Config {
  std::string sysfs_root = "/sys";
  std::string dev_root = "/dev";
  std::string exporter_socket;           // "" = off
  double exporter_timeout_s = 10.0;
  bool liveness = false;
  ProberConfig prober;
  int fail_threshold = 2;
  int recover_threshold = 1;
  double busy_grace_s = 300.0;
  double unknown_busy_grace_s = 30.0;
  bool corroborate = true;
  int idle_sweeps = 2;
  int crowded_procs = 7;                 // 0 = off
  int crowded_release_sweeps = 5;
  bool smi_ecc = false;
  bool smi_events = false;
  // every N-th sweep (and the first): the full-chip sweep instead of the
  // one-wave probe on GPUs no other process has queues on (0 = off)
  int chip_sweep_every = 0;
  // every N-th sweep (and the first): the throughput check on idle, live GPUs
  // (HBM pattern bandwidth, bf16 MFMA rate, per-XCD clocks); floors per whole
  // MI355X, scaled by the device's CU share; "unhealthy" withdraws degraded GPUs
  int perf_check_every = 0;
  std::string perf_action = "report";
  double perf_min_hbm_read_gbps = 3000.0;
  double perf_min_hbm_write_gbps = 2000.0;
  double perf_min_mfma_tflops = 700.0;
  double perf_min_xcd_clock_ratio = 0.6;
  bool smi_xgmi = false;
  std::string xgmi_file;  // JSON snapshot (smi_xgmi_links' shape) read instead of amd-smi: fault injection
  // kfd proc entries (PIDs) never counted as tenants, besides the probe
  // server's own: e.g. a process embedding the engine that holds GPU queues itself
  std::set<std::string> kfd_exclude;
};

struct Verdict {
  bool healthy = true;
  std::vector<std::string> reasons;
};

class Engine {
 public:
  Engine(std::vector<GpuDevice> devices, const KfdTopology& topo, Config cfg);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  // One sweep; true when any device's health changed. Blocking.
  bool sweep();
  // A liveness check of `ids` now, outside the sweep cadence (a container about
  // to start on them: PreStartContainer), within `budget_s`
  // (LivenessProber::check). Runs beside a sweep, never waiting for it; changes
  // no verdict. id -> outcome; devices without a ROCr ordinal, and devices on
  // GPUs the probe server steps off (crowded with tenant processes), are
  // absent; a reply from another agent than the device's is left to the sweep
  // (pending).
  std::map<std::string, ProbeOutcome> probe_now(const std::vector<std::string>& ids, double budget_s = 5.0);
  std::map<std::string, Verdict> snapshot() const;
  uint64_t version() const;
  void set_abort_fd(int fd);
  void close();

  // device id -> host ROCr ordinal (positional over accessible kfd GPU nodes)
  std::map<std::string, int> ordinals();
  // sources a test (or another collector) can replace
  std::function<std::map<std::string, int>()> activity_source;       // bdf -> GFX activity %, -1 unknown
  std::function<std::map<std::string, bool>()> exporter_source;      // bdf -> healthy
  std::function<SmiXgmiSnapshot()> xgmi_source;                      // instead of amd-smi / xgmi_file

  // xGMI pairs (allocator group keys, ordered) degraded since the first reading
  std::vector<std::pair<std::string, std::string>> degraded_links() const;
  uint64_t fabric_version() const;  // bumped whenever the degraded set changes
  std::map<std::string, int> links_down() const;  // bdf -> links down vs the first reading
  uint64_t xgmi_readings() const;
  std::string xgmi_error() const;

  LivenessProber* prober() { return prober_.get(); }
  uint64_t sweeps() const { return sweeps_; }
  uint64_t identity_remaps() const { return identity_remaps_; }
  uint64_t crowded_skips() const { return crowded_skips_; }
  uint64_t chip_sweeps() const { return chip_sweeps_; }
  uint64_t perf_checks() const { return perf_checks_; }
  // device -> (ok | degraded | failed, reason) of its last throughput check
  std::map<std::string, std::pair<std::string, std::string>> perf_verdicts() const;
  std::map<std::string, ProbeOutcome> perf_last() const;  // device -> its last throughput-check reply
  // why a correct throughput reply counts as degraded ([] if it does not)
  std::vector<std::string> perf_problems(const ProbeOutcome& o) const;
  bool busy_state_known() const { return busy_known_; }
  // kfd gpu_id -> (other processes with queues, their queues) as the last sweep saw it
  std::map<int64_t, std::pair<int, int>> gpu_load() const { return load_; }
  double last_sweep_ms() const { return last_sweep_ms_; }

 private:
  struct Track {
    int fails = 0, oks = 0;
    bool live = true;
    std::string last_reason;
    double pending_since = -1;  // monotonic seconds of the first inconclusive probe
    int idle_pending = 0;
  };
  using Reasons = std::map<std::string, std::vector<std::string>>;  // device -> why it is Unhealthy
  // the phases of sweep()
  void liveness_pass(Reasons* reasons);
  bool ecc_pass(Reasons* reasons);     // false: no amd-smi snapshot this sweep
  bool events_pass(Reasons* reasons);  // false: no event subscription
  bool publish(Reasons reasons);
  // liveness_pass's steps
  std::map<std::string, int> judged_ordinals(const Reasons& reasons);
  bool update_busy_state(const std::map<std::string, int>& ords, std::set<std::string>* busy);
  std::set<std::string> update_crowded(const std::map<std::string, int>& ords);
  std::map<std::string, ProbeOutcome> run_probes(const std::map<std::string, int>& probe_ords,
                                                 const std::set<std::string>& busy, const std::set<std::string>& idle,
                                                 bool known);
  void probe_crowded(const std::set<std::string>& crowded, const std::map<std::string, int>& ords,
                     std::map<std::string, ProbeOutcome>* outcomes);
  void judge_liveness(const std::map<std::string, ProbeOutcome>& outcomes, const std::set<std::string>& busy,
                      Reasons* reasons);
  std::map<std::string, std::string> kfd_verdicts() const;
  std::map<std::string, bool> exporter_health() const;
  std::map<std::string, int> gfx_activity();
  // kfd gpu_id -> (other processes with queues, their queues); false when unreadable
  bool kfd_load(const std::set<std::string>& exclude, std::map<int64_t, std::pair<int, int>>* out) const;
  int64_t gpu_id(const std::string& dev) const;
  std::map<std::string, ProbeOutcome> verify_identity(const std::map<std::string, int>& ords,
                                                      const std::map<std::string, ProbeOutcome>& outcomes);
  bool identity_matches(const GpuDevice& d, const ProbeOutcome& o) const;
  const GpuDevice* dev(const std::string& id) const;
  bool fabric_check();  // false: no xGMI link reading this sweep
  void perf_check(const std::map<std::string, int>& ords);
  SmiXgmiSnapshot read_xgmi();

  std::vector<GpuDevice> devices_;
  std::map<std::string, size_t> by_id_;
  KfdTopology topo_;
  Config cfg_;
  std::unique_ptr<LivenessProber> prober_;
  std::optional<std::map<std::string, int>> ordinals_;
  std::map<std::string, Track> track_;
  std::map<std::string, uint64_t> ecc_;
  std::map<std::string, std::string> resetting_;  // bdf -> pre-reset message
  std::map<std::string, int> crowded_;            // device -> uncrowded sweeps since it got crowded
  std::map<int64_t, std::pair<int, int>> load_;
  std::unique_ptr<mi355x::SmiEventWatcher> events_;
  bool events_started_ = false;
  bool smi_held_ = false;
  bool busy_known_ = true;
  uint64_t sweeps_ = 0, identity_remaps_ = 0, crowded_skips_ = 0, chip_sweeps_ = 0, perf_checks_ = 0;
  std::map<std::string, std::pair<std::string, std::string>> perf_;  // guarded by mu_
  std::map<std::string, ProbeOutcome> perf_last_;                     // guarded by mu_
  uint64_t xgmi_readings_ = 0;
  double last_sweep_ms_ = 0;
  int abort_fd_ = -1;
  // xGMI baseline: bdf -> (links up, -1 unknown; peers seen live)
  std::map<std::string, std::pair<int, std::set<std::string>>> xgmi_base_;
  std::map<std::string, std::string> gpu_by_bdf_;  // lower-case bdf -> allocator group key
  std::string xgmi_error_;

  mutable std::mutex mu_;  // snapshot_ / version_ / degraded_ / fabric_version_ / links_down_
  std::mutex op_mu_;       // the liveness pass of sweep(): one sweep at a time on the prober's sweep path
  mutable std::mutex state_mu_;  // ordinals_ and crowded_, read by probe_now() beside a sweep
  std::set<std::pair<std::string, std::string>> degraded_;
  std::map<std::string, int> links_down_;
  uint64_t fabric_version_ = 0;
  std::map<std::string, Verdict> snapshot_;
  uint64_t version_ = 0;
};

// bdf -> healthy from a metricssvc GPUStateResponse body ({} and *error when malformed)
std::map<std::string, bool> parse_exporter_states(const std::string& body, std::string* error = nullptr);

// bdf -> healthy from metricssvc.MetricsService/List on `socket` ({} when
// unavailable); `abort_fd` ends the wait early.
std::map<std::string, bool> exporter_list(const std::string& socket, double timeout_s, int abort_fd = -1,
                                          std::string* error = nullptr);

// device id -> host ROCr ordinal: position among kfd GPU nodes with a render
// node the process can open (ROCr skips the others), in node-id order.
std::map<std::string, int> hip_ordinals(const std::vector<GpuDevice>& devices, const KfdTopology& topo,
                                        const std::string& dev_root);

}  // namespace mi355x::health
