#include "daemon.h"

#include <fcntl.h>
#include <poll.h>
#include <sys/inotify.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>

#include "dry_run.h"
#include "mi355x/cdi.h"
#include "mi355x/constants.h"
#include "mi355x/glog.h"
#include "mi355x/metrics.h"
#include "mi355x/sysfs.h"
#include "mi355x/trace.h"

namespace mi355x::daemon {
namespace pb = mi355x::rpc::pb;

std::string register_with_kubelet(const std::string& name, const std::string& socket, const std::string& options,
                                  const std::string& kubelet_sock, double timeout_s, int abort_fd) {
  rpc::GrpcClient c;
  c.set_abort_fd(abort_fd);
  const std::string err = c.connect(kubelet_sock, timeout_s);
  if (!err.empty()) return "kubelet not reachable at " + kubelet_sock + ": " + err;
  std::string req;
  pb::put_bytes(&req, 1, "v1beta1");
  pb::put_bytes(&req, 2, basename(socket));
  pb::put_bytes(&req, 3, std::string(kResourceNamespace) + "/" + name);
  pb::put_bytes(&req, 4, options);
  const rpc::Reply rep = c.unary("/v1beta1.Registration/Register", req, timeout_s);
  if (rep.status != 0) return "Register failed (" + std::to_string(rep.status) + "): " + rep.message;
  return "";
}

namespace {

RegistrationPolicy policy_of(const Flags& f) {
  RegistrationPolicy p;
  p.watchdog_s = f.grpc_watchdog_s;
  p.reregister_s = f.reregister_s;
  return p;
}

}  // namespace

Daemon::SockId Daemon::sock_id(const std::string& path) {
  SockId s;
  struct stat st {};
  if (::stat(path.c_str(), &st) != 0) return s;
  s.present = true;
  s.dev = st.st_dev;
  s.ino = st.st_ino;
  s.ctime_ns = static_cast<int64_t>(st.st_ctim.tv_sec) * 1000000000 + st.st_ctim.tv_nsec;
  return s;
}

Daemon::Daemon(Flags f) : f_(std::move(f)), reg_(policy_of(f_)) {
  if (::pipe2(stop_pipe_, O_CLOEXEC | O_NONBLOCK) != 0) stop_pipe_[0] = stop_pipe_[1] = -1;
  health_ = std::make_unique<HealthController>(f_, stop_pipe_[0]);
}

Daemon::~Daemon() {
  shutdown();
  for (int fd : stop_pipe_)
    if (fd >= 0) ::close(fd);
}

void Daemon::shutdown() {
  if (stop_pipe_[1] >= 0) {
    const char b = 1;
    if (::write(stop_pipe_[1], &b, 1) < 0) {
    }
  }
  workers_.join_all();  // every wait ends at the stop pipe
  gate_pool_.join_all();
  std::shared_ptr<health::Engine> gate;
  {
    std::lock_guard<std::mutex> lk(gate_mu_);
    gate.swap(gate_engine_);
  }
  gate.reset();  // outside gate_mu_: the last reference closes the probe server
  if (health_) health_->close();
  reg_.stop_all();
}

bool GatePool::submit(std::function<void()> fn) {
  std::lock_guard<std::mutex> lk(mu_);
  if (stop_ || q_.size() >= max_queued_) return false;
  q_.push_back(std::move(fn));
  if (ts_.size() < workers_) ts_.emplace_back([this] { loop(); });  // started on demand
  cv_.notify_one();
  return true;
}

void GatePool::loop() {
  std::unique_lock<std::mutex> lk(mu_);
  while (true) {
    cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
    if (q_.empty()) return;  // stopping, nothing left
    auto fn = std::move(q_.front());
    q_.pop_front();
    lk.unlock();
    fn();
    lk.lock();
  }
}

void GatePool::join_all() {
  std::vector<std::thread> ts;
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
    ts.swap(ts_);
  }
  cv_.notify_all();
  for (auto& t : ts)
    if (t.joinable()) t.join();
}

size_t GatePool::threads() const {
  std::lock_guard<std::mutex> lk(mu_);
  return ts_.size();
}

rpc::Reply prestart_verdict(health::Engine* engine, const std::vector<std::string>& ids, double budget_s,
                            std::chrono::steady_clock::time_point arrival) {
  if (!engine) return rpc::Reply{};
  const auto t0 = std::chrono::steady_clock::now();
  const double queued = std::chrono::duration<double>(t0 - arrival).count();
  std::string bad, unsure;
  for (const auto& [id, o] : engine->probe_now(ids, std::max(0.0, budget_s - queued))) {
    if (!o.ok && !o.pending && !o.interrupted) bad += (bad.empty() ? "" : "; ") + id + ": " + o.reason;
    else if (o.pending) unsure += (unsure.empty() ? "" : "; ") + id + ": " + o.reason;
  }
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - arrival).count();
  auto& m = metrics::global();
  const char* result = !bad.empty() ? "failed" : !unsure.empty() ? "inconclusive" : "ok";
  m.inc("mi355x_dp_prestart_checks_total", {{"result", result}}, 1.0,
        "PreStartContainer liveness checks (-prestart_liveness): ok, failed, inconclusive (busy GPU or budget spent)");
  m.observe_ms("mi355x_dp_prestart_check_seconds", ms, {}, "PreStartContainer liveness check latency (queue wait included)");
  if (!unsure.empty()) MI_VLOG(2, "PreStartContainer: inconclusive, the start goes ahead (%s)", unsure.c_str());
  if (bad.empty()) return rpc::Reply{};
  MI_LOG(kError, "PreStartContainer: MFMA liveness check failed (%s)", bad.c_str());
  return rpc::Reply{rpc::kFailedPrecondition, "MFMA liveness check failed before the container start: " + bad, ""};
}

// ---- CDI specs (-device_list_strategy cdi-*): written before registration,
// since kubelet may hand a CDI name to the runtime as soon as it allocates
std::string Daemon::write_cdi(const std::set<std::string>& stale) {
  if (driver_ != Driver::Container || !f_.lists.cdi()) return "";
  std::vector<std::string> paths;
  const std::string e = cdi::write_specs(f_.cdi_spec_dir, reg_.members(), stale, &paths);
  if (e.empty()) {
    std::string all;
    for (const auto& p : paths) all += (all.empty() ? "" : ", ") + p;
    MI_LOG(kInfo, "CDI specs written: %s", all.c_str());
  }
  return e;
}

void Daemon::rebuild_health() {
  std::shared_ptr<health::Engine> old;
  {
    std::lock_guard<std::mutex> lk(gate_mu_);
    old.swap(gate_engine_);  // no new check starts on the old engine
  }
  health_->rebuild(driver_, container_devices_, topo_, reg_.all());
  {
    std::lock_guard<std::mutex> lk(gate_mu_);
    gate_engine_ = health_->engine();
  }
  // The old engine's probe server is stopped here (its teardown waits for the
  // GPU process), outside gate_mu_, so the RPC thread's PreStartContainer
  // hand-off never waits for it. A check or sweep still holding the engine
  // keeps it until it lets go.
  if (old && old.use_count() == 1) old->close();
}

int Daemon::init() {
  std::string err;
  dev_limit_ = device_count_limit(f_.config, &err);
  if (!err.empty()) {
    MI_LOG(kError, "%s", err.c_str());
    return 1;
  }
  if (f_.topology_view)
    serve_.topo = std::make_shared<views::TopologyViews>(path_join(f_.kubelet_dir, "mi355x-topology"),
                                                         path_join(f_.sysfs_root, "class/kfd/kfd/topology"));
  if (f_.node_view) {  // built at start-up, not inside the first Allocate
    auto nv = std::make_shared<views::NodeView>(path_join(f_.kubelet_dir, "mi355x-node"), f_.sysfs_root,
                                                f_.node_view_alias);
    if (const std::string e = nv->build(); !e.empty()) {
      MI_LOG(kWarning, "node view unavailable: %s", e.c_str());
    } else {
      MI_LOG(kInfo, "node view: %d links, %d per-CPU cache directories left out", nv->links, nv->hidden);
      serve_.node = nv;
    }
  }
  if (f_.prestart_liveness && f_.liveness_mode == "spawn")
    MI_LOG(kWarning, "-prestart_liveness with -liveness_mode=spawn: every container start waits for a fresh probe "
                     "process (GPU runtime start-up) and then for its kfd teardown; -liveness_mode=persistent "
                     "answers from the kept queue in about a millisecond");
  if (f_.prestart_liveness)  // runs on the RPC thread: the check goes to a gate worker
    serve_.prestart = [this](std::vector<std::string> ids, std::function<void(rpc::Reply)> done) {
      const auto arrival = std::chrono::steady_clock::now();
      std::shared_ptr<health::Engine> engine;
      {
        std::lock_guard<std::mutex> lk(gate_mu_);
        engine = gate_engine_;
      }
      auto shared_done = std::make_shared<std::function<void(rpc::Reply)>>(std::move(done));
      const double budget = f_.prestart_budget;
      if (!gate_pool_.submit([engine, ids = std::move(ids), shared_done, budget, arrival] {
            (*shared_done)(prestart_verdict(engine.get(), ids, budget, arrival));
          })) {
        metrics::global().inc("mi355x_dp_prestart_checks_total", {{"result", "overflow"}}, 1.0,
                              "PreStartContainer liveness checks (-prestart_liveness): ok, failed, inconclusive (busy GPU or budget spent)");
        MI_LOG(kWarning, "PreStartContainer: %zu checks already queued; this start goes ahead unchecked",
               gate_pool_.max_queued());
        (*shared_done)(rpc::Reply{});
      }
    };
  // explicit -driver_type: exit 1 when it cannot start (main.go:94-105); else
  // container -> VF -> PF, and with none the manager still starts and idles (main.go:106-119)
  NodeInventory inv;
  if (!f_.driver_type.empty()) {
    const Driver drv = driver_from_name(f_.driver_type);
    const std::string e = init_driver(f_, drv, dev_limit_, serve_, &inv);
    if (!e.empty()) {
      MI_LOG(kError, "Error instantiating driver type %s: %s", f_.driver_type.c_str(), e.c_str());
      return 1;
    }
  } else {
    bool found = false;
    for (Driver drv : {Driver::Container, Driver::Vf, Driver::Pf}) {
      NodeInventory got;
      const std::string e = init_driver(f_, drv, dev_limit_, serve_, &got);
      if (!e.empty()) {
        MI_LOG(kWarning, "%s implementation failed: %s. Trying next...", driver_name(drv), e.c_str());
        continue;
      }
      if (got.resources.empty()) {
        MI_LOG(kWarning, "%s implementation found no devices. Trying next...", driver_name(drv));
        continue;
      }
      inv = std::move(got);
      found = true;
      break;
    }
    impl_ok_ = found;
  }
  driver_ = inv.driver;
  topo_ = std::move(inv.topo);
  container_devices_ = std::move(inv.container_devices);
  warnings_ = std::move(inv.warnings);
  reg_.adopt(std::move(inv.resources));

  if (const std::string e = write_cdi({}); !e.empty()) {
    MI_LOG(kError, "cannot write CDI specs to %s: %s", f_.cdi_spec_dir.c_str(), e.c_str());
    return 1;
  }
  rebuild_health();
  if (f_.pulse > 0 && !reg_.empty()) {
    // one sweep before registering, so the first ListAndWatch already carries
    // real verdicts (the reference advertises everything Healthy until its first pulse)
    const SweepResult first = health_->sweep_now();
    metrics::global().observe_ms("mi355x_dp_health_sweep_seconds", first.sweep_ms, {}, "health sweep latency");
    reg_.apply_health(first.health);
  }
  if (f_.dry_run) {
    const auto eng = health_->engine();
    std::printf("%s\n", dry_run_report(f_, impl_ok_, driver_, reg_.all(), topo_, warnings_, eng.get()).c_str());
    std::fflush(stdout);
    health_->close();
    return 0;
  }
  return -1;
}

void Daemon::try_register(size_t i) {
  Resource& r = reg_.at(i);
  if (!r.server || !r.reg.due(Clock::now()) || !sock_.present) return;
  // the watchdog's baseline: before the request leaves (kubelet may open
  // ListAndWatch before its Register answer reaches us)
  r.reg.begin(kubelet_gen_, r.server->stats());
  workers_.run([name = r.name, socket = r.socket, options = r.options, i, kgen = kubelet_gen_,
                sgen = r.reg.server_gen(), kubelet_sock = kubelet_sock_, timeout = f_.register_timeout_s,
                abort_fd = stop_pipe_[0]] {
    Completion c;
    c.kind = Completion::kRegister;
    c.resource = i;
    c.server_gen = sgen;
    c.kubelet_gen = kgen;
    c.message = register_with_kubelet(name, socket, options, kubelet_sock, timeout, abort_fd);
    c.ok = c.message.empty();
    return c;
  });
}

void Daemon::start_all() {
  kubelet_gen_++;
  const auto now = Clock::now();
  for (size_t i = 0; i < reg_.size(); ++i) {
    if (reg_.at(i).gone) continue;
    if (reg_.start_server(i, now)) try_register(i);
  }
}

void Daemon::on_rpc_events(size_t i) {
  Resource& r = reg_.at(i);
  uint64_t v;
  if (::read(r.service->event_fd(), &v, sizeof(v)) < 0) {
  }
  const auto evs = r.service->drain_events();
  auto& m = metrics::global();
  const metrics::Labels res_l = {{"resource", r.name}};
  if (!evs.empty() && r.server) {
    const auto st = r.server->stats();
    m.set("mi355x_dp_grpc_connections", static_cast<double>(st.connections), res_l, "native gRPC server: connections");
    m.set("mi355x_dp_grpc_calls", static_cast<double>(st.calls), res_l, "native gRPC server: calls");
    m.set("mi355x_dp_grpc_protocol_errors", static_cast<double>(st.protocol_errors), res_l,
          "native gRPC server: protocol errors");
    m.set("mi355x_dp_listandwatch_open_streams", static_cast<double>(st.streams_open), res_l,
          "ListAndWatch streams open on the native server");
  }
  for (const auto& ev : evs) {
    if (trace::global().enabled()) {
      std::string ids;
      for (const auto& id : ev.ids) ids += (ids.empty() ? "" : ",") + id;
      trace::global().complete(ev.rpc, "rpc", ev.t0_ns, ev.dur_ns,
                               {{"resource", r.name}, {"native", ev.native ? "True" : "False"}, {"ids", ids}});
      if (ev.alloc_t0_ns)
        trace::global().complete("allocator.allocate", "alloc", ev.alloc_t0_ns,
                                 static_cast<uint64_t>(ev.alloc_us * 1e3),
                                 {{"candidates", std::to_string(ev.candidates)}, {"native", "True"}});
    }
    m.observe_ms("mi355x_dp_rpc_seconds", ev.dur_ns / 1e6, {{"resource", r.name}, {"rpc", ev.rpc}},
                 "device plugin RPC latency");
    if (ev.rpc == "ListAndWatch")
      m.inc("mi355x_dp_listandwatch_streams_total", res_l, 1.0, "ListAndWatch streams kubelet opened");
    if (ev.status != 0) {
      m.inc("mi355x_dp_rpc_errors_total", {{"resource", r.name}, {"rpc", ev.rpc}}, 1.0, "device plugin RPCs answered with an error");
      MI_LOG(kError, "%s: %s: %s", r.name.c_str(), ev.rpc.c_str(), ev.message.c_str());
    } else if (ev.rpc == "Allocate") {
      std::string ids;
      for (const auto& id : ev.ids) ids += (ids.empty() ? "" : ",") + id;
      MI_LOG(kInfo, "Allocating device IDs: %s", ids.c_str());
    }
    if (glog::vlog_is_on(2, __FILE__)) {
      char ms[32];
      std::snprintf(ms, sizeof(ms), "%.3f", ev.dur_ns / 1e6);
      glog::Fields fl = {{"rpc", ev.rpc}, {"resource", r.name}, {"latency_ms", ms}, {"native", "True"}};
      if (ev.rpc == "GetPreferredAllocation" && ev.candidates >= 0) {
        fl.emplace_back("candidates", std::to_string(ev.candidates));
        fl.emplace_back("short_circuit", ev.short_circuit ? "True" : "False");
      }
      MI_LOG_FIELDS(kInfo, "rpc", (fl));
    }
  }
}

// kubelet restarts: act only when kubelet.sock itself was replaced
void Daemon::on_kubelet_socket(bool look) {
  if (watch_.fd() >= 0 && look) {
    look = false;
    for (const auto& [name, mask] : watch_.read_events()) {
      if (name == "kubelet.sock") look = true;
      if (name.empty() && (mask & (IN_IGNORED | IN_DELETE_SELF | IN_MOVE_SELF))) {
        // the watched directory went away: watch it again once it is back, stat-poll meanwhile
        watch_.close();
        look = true;
      }
    }
  }
  if (watch_.fd() < 0 || Clock::now() >= next_stat_) look = true;
  if (watch_.fd() < 0 && is_dir(f_.kubelet_dir) && watch_.open(f_.kubelet_dir).empty())
    MI_LOG(kInfo, "inotify watch on %s re-established", f_.kubelet_dir.c_str());
  if (!look) return;
  next_stat_ = Clock::now() + std::chrono::seconds(5);
  const SockId cur = sock_id(kubelet_sock_);
  if (cur == sock_) return;
  const bool was = sock_.present;
  sock_ = cur;
  if (cur.present) {
    MI_LOG(kInfo, "kubelet socket (re)created; restarting plugin servers and re-registering");
    start_all();
  } else if (was) {
    MI_LOG(kInfo, "kubelet socket removed; stopping plugin servers");
    kubelet_gen_++;
    reg_.stop_all();
  }
}

void Daemon::on_sweep(const SweepResult& s) {
  const bool current = health_->finished(s);
  metrics::global().observe_ms("mi355x_dp_health_sweep_seconds", s.sweep_ms, {}, "health sweep latency");
  if (!current) return;  // a reload replaced the engine meanwhile: these verdicts are for the old devices
  const auto changed = reg_.apply_health(s.health);
  bool any_changed = false;
  const std::string lw = rpc::DevicePluginService::path("ListAndWatch");
  for (size_t i = 0; i < reg_.size(); ++i) {
    Resource& r = reg_.at(i);
    any_changed = any_changed || changed[i];
    if ((changed[i] || f_.send_every_pulse) && r.server) {
      r.server->broadcast(lw, r.list);
      trace::global().instant("ListAndWatch.send", "rpc",
                              {{"resource", r.name}, {"health_version", std::to_string(s.health_version)},
                               {"streams", std::to_string(r.server->stats().streams_open)}});
    }
  }
  if (any_changed) metrics::global().inc("mi355x_dp_health_changes_total", {}, 1.0, "sweeps that changed some device's health");
  // xGMI link state changed: every allocator re-weighted on the degraded pairs
  if (health_->fabric_changed(s)) {
    reg_.reweight(topo_, f_.allocator_search, s.degraded);
    metrics::global().inc("mi355x_dp_fabric_reweights_total", {}, 1.0,
                          "preferred-allocation re-weightings after an xGMI link state change");
    MI_LOG(kWarning, "xGMI link state changed: preferred allocation re-weighted (%zu degraded GPU pairs)",
           s.degraded.size());
  }
}

void Daemon::on_completions() {
  for (auto& c : workers_.take()) {
    if (c.kind == Completion::kSweep) {
      on_sweep(c.sweep);
      continue;
    }
    if (c.resource >= reg_.size()) continue;
    Resource& r = reg_.at(c.resource);
    switch (r.reg.complete(c.server_gen, c.kubelet_gen, kubelet_gen_, c.ok && r.server != nullptr, Clock::now())) {
      case Registration::Outcome::kRegistered:
        metrics::global().inc("mi355x_dp_registrations_total", {{"resource", r.name}}, 1.0, "Register calls kubelet accepted");
        MI_LOG(kInfo, "%s: Registration for endpoint %s", r.name.c_str(), basename(r.socket).c_str());
        break;
      case Registration::Outcome::kFailed:
        MI_LOG(kError, "%s: %s", r.name.c_str(), c.message.c_str());
        break;
      case Registration::Outcome::kStale:
        break;
    }
  }
  workers_.reap();
}

std::string Daemon::watchdog() {
  const auto now = Clock::now();
  for (auto& r : reg_.all()) {
    if (!r.server) continue;
    const uint64_t before = r.reg.reregistrations();
    const std::string why = r.reg.observe(r.server->stats(), now);
    if (!why.empty()) return r.name + ": " + why;
    if (r.reg.reregistrations() != before) {
      metrics::global().inc("mi355x_dp_reregistrations_total", {{"resource", r.name}}, 1.0,
                            "registrations again after kubelet closed every ListAndWatch stream");
      MI_LOG(kWarning, "%s: kubelet closed every ListAndWatch stream for %gs; registering again", r.name.c_str(),
             f_.reregister_s);
    }
  }
  return "";
}

void Daemon::reload_topology(const std::string& sig) {
  NodeInventory inv;
  const std::string e = init_container(f_, dev_limit_, serve_, &inv);
  topo_state_.applied(sig);
  std::map<std::string, std::string> before, after;  // device id -> partition type
  std::string old_names, new_names;
  std::set<std::string> old_set;
  for (const auto& r : reg_.all())
    if (!r.gone) {
      old_names += (old_names.empty() ? "" : ",") + r.name;
      old_set.insert(r.name);
      for (const auto& d : r.devices) before[d.id] = d.partition_type();
    }
  if (e.empty())
    for (const auto& r : inv.resources) {
      new_names += (new_names.empty() ? "" : ",") + r.name;
      for (const auto& d : r.devices) after[d.id] = d.partition_type();
    }
  if (before == after) return;
  metrics::global().inc("mi355x_dp_topology_reloads_total", {}, 1.0, "GPU topology changes (partition switches) applied");
  MI_LOG(kWarning, "GPU topology changed: %zu -> %zu devices; resources [%s] -> [%s]", before.size(), after.size(),
         old_names.c_str(), new_names.c_str());
  const auto now = Clock::now();
  if (!e.empty()) {
    MI_LOG(kError, "GPU topology changed: %s. Advertising no devices until then.", e.c_str());
    reg_.apply_reload({}, false, now);
    if (const std::string ce = write_cdi(old_set); !ce.empty())
      MI_LOG(kError, "CDI specs not updated after the topology change: %s", ce.c_str());
    container_devices_.clear();
    rebuild_health();
    return;
  }
  topo_ = std::move(inv.topo);
  container_devices_ = std::move(inv.container_devices);
  warnings_ = std::move(inv.warnings);
  const ReloadPlan plan = reg_.apply_reload(std::move(inv.resources), true, now);
  // before any new resource registers: kubelet may hand its CDI names to the runtime at once
  if (const std::string ce = write_cdi(old_set); !ce.empty())
    MI_LOG(kError, "CDI specs not updated after the topology change: %s", ce.c_str());
  for (size_t i : plan.added)
    if (sock_.present && reg_.start_server(i, now)) try_register(i);
  rebuild_health();
  if (f_.pulse > 0) next_pulse_ = now;  // verdicts for the new devices now
}

void Daemon::topology_tick() {
  if (!topo_watch_ || Clock::now() < next_topo_) return;
  next_topo_ = Clock::now() + topo_period_;
  const std::string cur = topology_signature(f_.sysfs_root);
  if (topo_state_.observe(cur, health_->may_reload())) reload_topology(cur);
}

void Daemon::pulse_tick() {
  if (f_.pulse <= 0 || Clock::now() < next_pulse_) return;
  next_pulse_ = Clock::now() + std::chrono::seconds(f_.pulse);
  if (health_->inflight()) {
    MI_LOG(kWarning, "health sweep still running at the next pulse; skipping this pulse");
    return;
  }
  if (reg_.empty()) return;
  health_->started();
  workers_.run([job = health_->job()] {
    Completion c;
    c.kind = Completion::kSweep;
    c.sweep = job();
    return c;
  });
}

int Daemon::poll_timeout_ms(Clock::time_point now) const {
  auto until = [&](Clock::time_point t) -> long long {
    return std::chrono::duration_cast<std::chrono::milliseconds>(t - now).count() + 1;
  };
  long long wait_ms = f_.pulse > 0 ? until(next_pulse_) : 3600 * 1000;
  // inotify is the fast path; the stat poll is the safety net (a dead watch, a replaced directory)
  wait_ms = std::min(wait_ms, watch_.fd() >= 0 ? until(next_stat_) : 1000LL);
  for (const auto& r : reg_.all())
    if (r.server) wait_ms = std::min(wait_ms, until(r.reg.next_event(now)));
  if (topo_watch_) wait_ms = std::min(wait_ms, until(next_topo_));
  return static_cast<int>(std::max(0LL, wait_ms));
}

void Daemon::note_tick() {
  int n = 0, registered = 0;
  for (const auto& r : reg_.all()) {
    n++;
    registered += r.server && r.reg.registered();
  }
  resources_n_.store(n);
  registered_n_.store(registered);
  loop_tick_ns_.store(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count());
}

std::string Daemon::healthz() const {
  const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
  const double age = (now - loop_tick_ns_.load()) * 1e-9;
  if (age <= kLoopStallS) return "";
  char b[128];
  std::snprintf(b, sizeof(b), "control loop stalled: last ran %.0f s ago", age);
  return b;
}

std::string Daemon::readyz() const {
  const int n = resources_n_.load(), registered = registered_n_.load();
  // a node without GPUs idles as the reference's manager does; it is ready, so a
  // DaemonSet rolling update (maxUnavailable) is not held up by CPU-only nodes
  if (registered < n)
    return "registered with kubelet: " + std::to_string(registered) + " of " + std::to_string(n) + " resources";
  return "";
}

int Daemon::run(int sig_fd, const volatile sig_atomic_t* stop) {
  metrics::HttpEndpoint metrics_http;
  note_tick();
  metrics_http.set_checks([this] { return healthz(); }, [this] { return readyz(); });
  if (f_.metrics_port > 0) {
    const std::string merr = metrics_http.start("0.0.0.0", f_.metrics_port);
    if (!merr.empty()) {
      MI_LOG(kError, "cannot serve /metrics: %s", merr.c_str());
      return 1;
    }
    MI_LOG(kInfo, "serving Prometheus /metrics on :%d", metrics_http.port());
  }
  kubelet_sock_ = path_join(f_.kubelet_dir, "kubelet.sock");
  if (const std::string werr = watch_.open(f_.kubelet_dir); !werr.empty())
    MI_LOG(kWarning, "no inotify watch on %s (%s): polling every second", f_.kubelet_dir.c_str(), werr.c_str());
  const auto t0 = Clock::now();
  next_stat_ = t0 + std::chrono::seconds(5);
  next_pulse_ = t0 + std::chrono::seconds(f_.pulse > 0 ? f_.pulse : 3600);
  topo_watch_ = f_.topology_watch_s > 0 && driver_ == Driver::Container;
  topo_period_ = std::chrono::milliseconds(static_cast<long long>(f_.topology_watch_s * 1000));
  topo_state_ = TopologyWatch(topo_watch_ ? topology_signature(f_.sysfs_root) : "");
  next_topo_ = t0 + topo_period_;
  sock_ = sock_id(kubelet_sock_);
  if (sock_.present && !*stop) start_all();  // a signal during init(): straight to shutdown

  int exit_code = 0;
  while (!*stop) {
    std::vector<pollfd> pfd = {{sig_fd, POLLIN, 0}, {workers_.wake_fd(), POLLIN, 0}};
    const bool inotify = watch_.fd() >= 0;
    if (inotify) pfd.push_back({watch_.fd(), POLLIN, 0});
    const size_t ev_base = pfd.size();
    for (const auto& r : reg_.all()) pfd.push_back({r.service->event_fd(), POLLIN, 0});
    ::poll(pfd.data(), pfd.size(), poll_timeout_ms(Clock::now()));
    if (*stop) break;
    for (size_t i = 0; i < reg_.size() && ev_base + i < pfd.size(); ++i)
      if (pfd[ev_base + i].revents & POLLIN) on_rpc_events(i);
    on_kubelet_socket(inotify && (pfd[2].revents & POLLIN));
    on_completions();
    for (size_t i = 0; i < reg_.size(); ++i) try_register(i);  // due ones only (backoff, lost streams)
    if (const std::string why = watchdog(); !why.empty()) {
      MI_LOG(kError, "native gRPC transport watchdog: %s; exiting so the plugin is restarted", why.c_str());
      exit_code = 3;
      break;
    }
    topology_tick();
    pulse_tick();
    note_tick();
  }
  if (*stop) MI_LOG(kInfo, "Received signal, shutting down.");
  shutdown();
  if (const std::string te = trace::global().flush(); !te.empty())
    MI_LOG(kError, "cannot write the trace file: %s", te.c_str());
  return exit_code;
}

}  // namespace mi355x::daemon
