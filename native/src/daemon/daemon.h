// The native device-plugin daemon: discovery -> resources -> per-resource
// gRPC servers -> registration with kubelet -> the control loop.
//
// Ownership: the Daemon owns the ResourceRegistry (resources, their servers
// and DevicePlugin services, each resource's Registration state), the
// HealthController (health engine + sweep bookkeeping), the worker pool and
// the kubelet-socket watch. Only the control loop (run()) touches them; worker
// threads get self-contained jobs (a Register request by value, a sweep job
// from HealthController::job()) and hand back a Completion.
//
// Control loop (one poll per turn, never blocking on a peer):
//   RPC events        the reference logs every Allocate; metrics, traces
//   kubelet.sock      inotify + 5 s stat poll: a replaced socket restarts the
//                     servers and re-registers (vendored dpm/manager.go:73-84)
//   completions       Register answers (Registration::complete), sweep results
//                     (health -> ListAndWatch lists, xGMI re-weighting)
//   registrations     due Registers go out (backoff, re-register on lost streams)
//   watchdog          Registration::observe: exit 3 when kubelet never lists
//   topology          -topology_watch: a partition switch is re-discovered and
//                     re-advertised, never under a sweep
//   pulse             one sweep per -pulse on a worker thread
#pragma once

#include <signal.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "flags.h"
#include "health_controller.h"
#include "resources.h"
#include "topology_watch.h"
#include "workers.h"
#include "mi355x/dir_watch.h"

namespace mi355x::daemon {

struct Completion {
  enum Kind { kRegister, kSweep } kind = kRegister;
  // kRegister
  size_t resource = 0;
  uint64_t server_gen = 0;   // the server the Register was for
  uint64_t kubelet_gen = 0;  // the kubelet it was sent to
  bool ok = false;
  std::string message;
  // kSweep
  SweepResult sweep;
};

// -prestart_liveness: PreStartContainer's answer from a check of the
// container's devices now (blocking; a gate worker), within what is left of
// `budget_s` since `arrival`. FAILED_PRECONDITION names each device with a
// definite fault; a pending or interrupted probe, a device the probe server
// cannot reach, and a check whose budget ran out do not hold the container
// back (counted in mi355x_dp_prestart_checks_total{result="inconclusive"}).
rpc::Reply prestart_verdict(health::Engine* engine, const std::vector<std::string>& ids, double budget_s,
                            std::chrono::steady_clock::time_point arrival);

// The workers PreStartContainer checks run on, off the RPC thread: a fixed
// pool and a bounded queue. A check that finds the queue full is answered at
// once (`overflow`); one that waited past its budget in the queue runs with
// nothing left and is answered inconclusive.
class GatePool {
 public:
  explicit GatePool(size_t workers = 8, size_t max_queued = 64) : workers_(workers), max_queued_(max_queued) {}
  ~GatePool() { join_all(); }
  // false (and `fn` not run) when the queue is full
  bool submit(std::function<void()> fn);
  // runs what is queued, then stops the workers
  void join_all();
  size_t threads() const;
  size_t max_queued() const { return max_queued_; }

 private:
  void loop();
  const size_t workers_, max_queued_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  std::vector<std::thread> ts_;
  bool stop_ = false;
};

// Register{version=1, endpoint=2, resource_name=3, options=4} on kubelet.sock (blocking; worker thread)
std::string register_with_kubelet(const std::string& name, const std::string& socket, const std::string& options,
                                  const std::string& kubelet_sock, double timeout_s, int abort_fd);

class Daemon {
 public:
  explicit Daemon(Flags f);
  ~Daemon();
  Daemon(const Daemon&) = delete;
  Daemon& operator=(const Daemon&) = delete;

  // Discovery, CDI specs, the first health sweep; -dry_run prints its report.
  // Returns -1 to go on with run(), else the exit code.
  int init();
  // The control loop until `*stop` (set by a signal handler that also writes
  // to `sig_fd`) or the watchdog trips; returns the exit code.
  int run(int sig_fd, const volatile sig_atomic_t* stop);
  // Write end of the pipe that ends every wait of the workers (peer calls,
  // probes, the first sweep in init()): a signal handler writes one byte to it,
  // so a stop during a slow probe is not held until the probe's deadline.
  int stop_fd() const { return stop_pipe_[1]; }

 private:
  std::string write_cdi(const std::set<std::string>& stale);
  void rebuild_health();
  void start_all();
  void try_register(size_t i);
  void on_rpc_events(size_t i);
  void on_kubelet_socket(bool look);
  void on_completions();
  void on_sweep(const SweepResult& r);
  std::string watchdog();
  void topology_tick();
  void reload_topology(const std::string& sig);
  void pulse_tick();
  int poll_timeout_ms(Clock::time_point now) const;
  void shutdown();
  // /healthz: the control loop ran within kLoopStallS; /readyz: every resource
  // is registered with kubelet (a node without GPUs has none and is ready). Both read only the atomics note_tick() sets, on
  // the metrics endpoint's thread.
  void note_tick();
  std::string healthz() const;
  std::string readyz() const;

  Flags f_;
  int dev_limit_ = -1;
  ServeCtx serve_;
  bool impl_ok_ = true;
  Driver driver_ = Driver::Container;
  KfdTopology topo_;
  std::vector<GpuDevice> container_devices_;
  std::vector<std::string> warnings_;
  ResourceRegistry reg_;
  int stop_pipe_[2] = {-1, -1};  // ends every wait of the workers (peer calls, probes)
  std::unique_ptr<HealthController> health_;
  Workers<Completion> workers_;
  // -prestart_liveness: the engine the gate probes with (read on RPC threads)
  std::mutex gate_mu_;
  std::shared_ptr<health::Engine> gate_engine_;
  GatePool gate_pool_;
  // kubelet
  std::string kubelet_sock_;
  DirWatcher watch_;
  uint64_t kubelet_gen_ = 0;  // bumped on every kubelet (re)start: older Register results are stale
  struct SockId {
    bool present = false;
    uint64_t dev = 0, ino = 0;
    int64_t ctime_ns = 0;
    bool operator==(const SockId& o) const {
      return present == o.present && dev == o.dev && ino == o.ino && ctime_ns == o.ctime_ns;
    }
    bool operator!=(const SockId& o) const { return !(*this == o); }
  };
  static SockId sock_id(const std::string& path);
  SockId sock_;
  Clock::time_point next_stat_{};
  // pulse + topology watch
  Clock::time_point next_pulse_{};
  bool topo_watch_ = false;
  std::chrono::milliseconds topo_period_{0};
  TopologyWatch topo_state_;
  Clock::time_point next_topo_{};
  // probe endpoints
  static constexpr double kLoopStallS = 60;  // the loop wakes at least every 5 s (kubelet.sock stat)
  std::atomic<int64_t> loop_tick_ns_{0};
  std::atomic<int> resources_n_{0}, registered_n_{0};
};

}  // namespace mi355x::daemon
