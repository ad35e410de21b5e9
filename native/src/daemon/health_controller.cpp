#include "health_controller.h"

#include <unistd.h>

#include <chrono>

#include "mi355x/glog.h"
#include "mi355x/sysfs.h"

namespace mi355x::daemon {
namespace {

std::string self_dir() {
  char buf[4096];
  const ssize_t n = ::readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return ".";
  buf[n] = 0;
  std::string p = buf;
  return p.substr(0, p.rfind('/'));
}

health::Config engine_config(const Flags& f) {
  health::Config hc;
  hc.sysfs_root = f.sysfs_root;
  hc.dev_root = f.dev_root;
  hc.exporter_socket = f.exporter_socket;
  hc.liveness = f.liveness;
  hc.prober.exe = !f.liveness_probe.empty() ? f.liveness_probe : path_join(self_dir(), "mi355x-liveness-probe");
  hc.prober.timeout_s = f.liveness_timeout;
  hc.prober.busy_deadline_s = f.liveness_busy_deadline;
  hc.prober.iters = f.liveness_iters;
  hc.prober.persistent = f.liveness_mode == "persistent";
  hc.prober.keep_queues = f.liveness_keep_queues;
  hc.fail_threshold = f.liveness_fail_threshold;
  hc.recover_threshold = f.liveness_recover_threshold;
  hc.busy_grace_s = f.liveness_busy_grace;
  hc.unknown_busy_grace_s = f.liveness_unknown_busy_grace;
  hc.corroborate = f.liveness_corroborate;
  hc.idle_sweeps = f.liveness_idle_sweeps;
  hc.crowded_procs = f.liveness_crowded_procs;
  hc.crowded_release_sweeps = f.liveness_crowded_release_sweeps;
  hc.smi_ecc = f.smi_ecc;
  hc.smi_events = f.smi_events;
  hc.smi_xgmi = f.smi_xgmi;
  hc.chip_sweep_every = f.liveness_chip_sweep_every;
  hc.perf_check_every = f.perf_check_every;
  hc.perf_action = f.perf_action;
  hc.perf_min_hbm_read_gbps = f.perf_min_hbm_read_gbps;
  hc.perf_min_mfma_tflops = f.perf_min_mfma_tflops;
  hc.perf_min_xcd_clock_ratio = f.perf_min_xcd_clock_ratio;
  hc.prober.perf_mib = f.perf_mib;
  if (const char* x = std::getenv("MI355X_SMI_XGMI_FILE"); x && *x) hc.xgmi_file = x;  // fault injection
  return hc;
}

}  // namespace

std::map<std::string, bool> passthrough_health(const PassthroughSnapshot& s, int abort_fd) {
  std::map<std::string, bool> out;
  const bool vf = s.driver == Driver::Vf;
  const bool present = is_dir(path_join(s.sysfs_root, vf ? "bus/pci/drivers/gim" : "bus/pci/drivers/vfio-pci"));
  std::map<std::string, bool> exporter;
  if (vf) {
    std::string e;
    exporter = health::exporter_list(s.exporter_socket, 10.0, abort_fd, &e);
    if (!e.empty()) MI_LOG(kError, "Error getting health info svc : %s", e.c_str());
  }
  for (const auto& [g, pfs] : s.groups) {
    bool ok = present;
    if (vf)
      for (const auto& pf : pfs)
        if (auto it = exporter.find(pf); it != exporter.end() && !it->second) ok = false;
    out[g] = ok;
  }
  return out;
}

void HealthController::rebuild(Driver drv, const std::vector<GpuDevice>& devices, const KfdTopology& topo,
                               const std::vector<Resource>& resources) {
  close();
  driver_ = drv;
  gen_++;
  fabric_seen_ = 0;
  pt_ = PassthroughSnapshot{};
  if (drv != Driver::Container) {
    pt_.driver = drv;
    pt_.sysfs_root = f_.sysfs_root;
    pt_.exporter_socket = f_.exporter_socket;
    for (const auto& r : resources)
      for (const auto& g : r.group_ids) {
        std::vector<std::string> pfs;
        for (const auto& fn : r.groups.at(g)) pfs.push_back(fn.pf);
        pt_.groups.emplace_back(g, pfs);
      }
    return;
  }
  if (devices.empty()) return;
  const health::Config hc = engine_config(f_);
  engine_ = std::make_shared<health::Engine>(devices, topo, hc);
  engine_->set_abort_fd(abort_fd_);
  if (f_.liveness) MI_LOG(kInfo, "liveness probe: %s (%s)", hc.prober.exe.c_str(), f_.liveness_mode.c_str());
}

std::function<SweepResult()> HealthController::job() const {
  const uint64_t gen = gen_;
  if (driver_ == Driver::Container) {
    return [engine = engine_, gen] {
      SweepResult r;
      r.engine_gen = gen;
      const auto t0 = std::chrono::steady_clock::now();
      if (engine) {
        engine->sweep();
        for (const auto& [id, v] : engine->snapshot()) r.health[id] = v.healthy;
        r.fabric_version = engine->fabric_version();
        r.degraded = engine->degraded_links();
        r.health_version = engine->version();
      }
      r.sweep_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      return r;
    };
  }
  return [snap = pt_, gen, abort_fd = abort_fd_] {
    SweepResult r;
    r.engine_gen = gen;
    const auto t0 = std::chrono::steady_clock::now();
    r.health = passthrough_health(snap, abort_fd);
    r.sweep_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return r;
  };
}

bool HealthController::finished(const SweepResult& r) {
  inflight_ = false;
  return r.engine_gen == gen_;
}

bool HealthController::fabric_changed(const SweepResult& r) {
  if (r.engine_gen != gen_ || !engine_ || r.fabric_version == fabric_seen_) return false;
  fabric_seen_ = r.fabric_version;
  return true;
}

void HealthController::close() {
  // a sweep still holding the engine closes it when it lets go (~Engine)
  if (engine_ && engine_.use_count() == 1) engine_->close();
  engine_.reset();
}

}  // namespace mi355x::daemon
