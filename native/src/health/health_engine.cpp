// Native per-device health engine (see mi355x/health_engine.h). The policy is
// the Python monitor's (rocm_k8s_device_plugin_amd/health/monitor.py):
// sweep() asks every configured source (kfd, exporter, liveness probes through
// LivenessProber in liveness_prober.cpp, amd-smi ECC / events / xGMI, the
// throughput check) for reasons a device is Unhealthy and publishes verdicts.
#include "mi355x/health_engine.h"

#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "../kube/json.h"
#include "mi355x/dp_service.h"
#include "mi355x/glog.h"
#include "mi355x/metrics.h"
#include "mi355x/trace.h"
#include "mi355x/grpc_server.h"
#include "mi355x/smi_query.h"
#include "mi355x/sysfs.h"

namespace mi355x::health {
namespace {

using Clock = std::chrono::steady_clock;

double mono_s() { return std::chrono::duration<double>(Clock::now().time_since_epoch()).count(); }

}  // namespace

// =============================================================== helpers
// GPUStateResponse{GPUState=1: GPUState{ID=1, UUID=2, Health=3, AssociatedWorkload=4, Device=5}}
// (internal/pkg/exporter/metricssvc/metricssvc.pb.go:95-110,284-291), decoded
// strictly as protobuf does: a malformed message is an error, not a partial map
std::map<std::string, bool> parse_exporter_states(const std::string& body, std::string* error) {
  std::map<std::string, bool> out;
  const bool ok = rpc::pb::scan(
      body.data(), body.size(),
      [&](int f, const char* p, size_t n) {
        if (f != 1) return true;
        std::string health, device;
        const bool inner = rpc::pb::scan(
            p, n,
            [&](int g, const char* q, size_t m) {
              if (g == 3) health.assign(q, m);
              else if (g == 5) device.assign(q, m);
              return true;
            },
            nullptr);
        if (inner && !device.empty()) out[device] = to_lower(trim(health)) == "healthy";
        return inner;
      },
      nullptr);
  if (!ok) {
    if (error) *error = "malformed GPUStateResponse from the metrics exporter";
    return {};
  }
  return out;
}

std::map<std::string, bool> exporter_list(const std::string& socket, double timeout_s, int abort_fd,
                                          std::string* error) {
  std::map<std::string, bool> out;
  if (socket.empty() || !path_exists(socket)) return out;
  rpc::GrpcClient c;
  c.set_abort_fd(abort_fd);
  const std::string cerr = c.connect(socket, timeout_s);
  if (!cerr.empty()) {
    if (error) *error = cerr;
    return out;
  }
  const rpc::Reply rep = c.unary("/metricssvc.MetricsService/List", "", timeout_s);
  if (rep.status != 0) {
    if (error) *error = rep.message;
    return out;
  }
  return parse_exporter_states(rep.body, error);
}

std::map<std::string, int> hip_ordinals(const std::vector<GpuDevice>& devices, const KfdTopology& topo,
                                        const std::string& dev_root) {
  std::map<int, int> pos;  // kfd node id -> ordinal
  const bool check = is_dir(path_join(dev_root, "dri"));
  int n = 0;
  for (const KfdNode* node : topo.gpu_nodes()) {
    const int minor = node->drm_render_minor();
    if (minor <= 0) continue;
    if (check && ::access(path_join(dev_root, "dri/renderD" + std::to_string(minor)).c_str(), R_OK | W_OK) != 0)
      continue;
    pos[node->id] = n++;
  }
  std::map<std::string, int> out;
  for (const auto& d : devices)
    if (auto it = pos.find(d.node_id); it != pos.end()) out[d.id] = it->second;
  return out;
}

// =============================================================== Engine
Engine::Engine(std::vector<GpuDevice> devices, const KfdTopology& topo, Config cfg)
    : devices_(std::move(devices)), topo_(topo), cfg_(std::move(cfg)) {
  for (size_t i = 0; i < devices_.size(); ++i) {
    by_id_[devices_[i].id] = i;
    track_[devices_[i].id] = Track{};
    snapshot_[devices_[i].id] = Verdict{};
    std::string b = devices_[i].bdf;
    for (auto& c : b) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    gpu_by_bdf_.emplace(b, !devices_[i].unique_id.empty() ? devices_[i].unique_id : "bdf:" + devices_[i].bdf);
  }
  if (cfg_.liveness) {
    if (cfg_.prober.kfd_proc_dir.empty() || cfg_.prober.kfd_proc_dir == "/sys/class/kfd/kfd/proc")
      cfg_.prober.kfd_proc_dir = path_join(cfg_.sysfs_root, "class/kfd/kfd/proc");
    prober_ = std::make_unique<LivenessProber>(cfg_.prober);
  }
}

Engine::~Engine() { close(); }

void Engine::set_abort_fd(int fd) {
  abort_fd_ = fd;
  if (prober_) prober_->set_abort_fd(fd);
}

void Engine::close() {
  if (prober_) prober_->close();
  if (events_) events_->stop();
  events_.reset();
  events_started_ = false;
  if (smi_held_) smi_unhold();
  smi_held_ = false;
}

std::map<std::string, Verdict> Engine::snapshot() const {
  std::lock_guard<std::mutex> lk(mu_);
  return snapshot_;
}

uint64_t Engine::version() const {
  std::lock_guard<std::mutex> lk(mu_);
  return version_;
}

const GpuDevice* Engine::dev(const std::string& id) const {
  auto it = by_id_.find(id);
  return it == by_id_.end() ? nullptr : &devices_[it->second];
}

std::map<std::string, int> Engine::ordinals() {
  std::lock_guard<std::mutex> lk(state_mu_);
  if (!ordinals_) ordinals_ = hip_ordinals(devices_, topo_, cfg_.dev_root);
  return *ordinals_;
}

int64_t Engine::gpu_id(const std::string& id) const {
  const GpuDevice* d = dev(id);
  const KfdNode* n = d && d->node_id >= 0 ? topo_.node(d->node_id) : nullptr;
  return n ? n->gpu_id : 0;
}

std::map<std::string, std::string> Engine::kfd_verdicts() const {
  std::map<std::string, std::string> out;
  const std::string nodes = path_join(cfg_.sysfs_root, "class/kfd/kfd/topology/nodes");
  const bool have = is_dir(nodes);
  for (const auto& d : devices_) {
    if (!have) {
      out[d.id] = "kfd topology unavailable";
      continue;
    }
    if (d.node_id < 0) continue;  // no kfd data (cgroup-denied): not evidence of a fault
    const auto kv = parse_kv_file(path_join(nodes, std::to_string(d.node_id) + "/properties"));
    if (!kv) {
      out[d.id] = "kfd node " + std::to_string(d.node_id) + " missing";
      continue;
    }
    const int64_t cores = kv_i64(*kv, "cpu_cores_count", 0), gfx = kv_i64(*kv, "gfx_target_version", 0);
    if (!(cores == 0 && gfx > 0)) out[d.id] = "kfd node " + std::to_string(d.node_id) + " not a live GPU";
  }
  return out;
}

std::map<std::string, bool> Engine::exporter_health() const {
  if (exporter_source) return exporter_source();
  std::string err;
  auto m = exporter_list(cfg_.exporter_socket, cfg_.exporter_timeout_s, abort_fd_, &err);
  if (!err.empty()) MI_LOG(kError, "Error getting health info svc : %s", err.c_str());
  return m;
}

std::map<std::string, int> Engine::gfx_activity() {
  if (activity_source) return activity_source();
  std::map<std::string, int> out;
  if (!smi_available()) return out;
  if (!smi_held_) smi_held_ = smi_hold();
  const SmiSnapshot snap = smi_snapshot();
  if (!snap.ok) return out;
  for (const auto& g : snap.gpus)
    if (g.gfx_activity >= 0) out[g.bdf] = g.gfx_activity;
  return out;
}

bool Engine::kfd_load(const std::set<std::string>& exclude, std::map<int64_t, std::pair<int, int>>* out) const {
  out->clear();
  const std::string root = path_join(cfg_.sysfs_root, "class/kfd/kfd/proc");
  if (!is_dir(root)) return path_exists(root) ? false : true;  // no list at all: no process has queues
  if (::access(root.c_str(), R_OK | X_OK) != 0) return false;
  std::map<int64_t, std::pair<int, int>> load;
  for (const auto& pid : list_dir(root)) {
    if (exclude.count(pid) || cfg_.kfd_exclude.count(pid)) continue;
    const std::string qdir = path_join(path_join(root, pid), "queues");
    if (!is_dir(qdir)) continue;  // exited meanwhile
    if (::access(qdir.c_str(), R_OK | X_OK) != 0) return false;
    std::map<int64_t, int> mine;
    for (const auto& q : list_dir(qdir)) {
      auto g = read_trimmed(path_join(path_join(qdir, q), "gpuid"));
      if (!g) continue;
      const int64_t gid = parse_i64(*g, 0);
      if (gid) mine[gid]++;
    }
    for (const auto& [gid, nq] : mine) {
      load[gid].first += 1;
      load[gid].second += nq;
    }
  }
  *out = std::move(load);
  return true;
}

bool Engine::identity_matches(const GpuDevice& d, const ProbeOutcome& o) const {
  int dom = -1, loc = -1;
  unsigned D = 0, B = 0, Dv = 0, F = 0;
  if (!o.pci_bus_id.empty() && std::sscanf(o.pci_bus_id.c_str(), "%x:%x:%x.%x", &D, &B, &Dv, &F) == 4) {
    dom = static_cast<int>(D);
    loc = static_cast<int>((B << 8) | (Dv << 3) | F);
  }
  if (o.kfd_node_id < 0 && loc < 0) return true;  // the reply names no agent
  // the PCI location (partition index in the function bits) is exact; the
  // agent's node id is the thunk's, renumbered under a device cgroup
  if (loc >= 0 && d.location_id) return dom == d.domain && loc == d.location_id;
  if (o.kfd_node_id >= 0 && d.node_id >= 0) return o.kfd_node_id == d.node_id;
  return true;
}

std::map<std::string, ProbeOutcome> Engine::verify_identity(const std::map<std::string, int>& ords,
                                                            const std::map<std::string, ProbeOutcome>& outcomes) {
  bool bad = false;
  for (const auto& [id, o] : outcomes)
    if (const GpuDevice* d = dev(id); d && !identity_matches(*d, o)) bad = true;
  if (!bad) return outcomes;
  // re-key by identity: every reply names its agent's PCI location
  std::map<std::pair<int, int>, std::pair<int, const ProbeOutcome*>> by_loc;
  std::map<int, std::pair<int, const ProbeOutcome*>> by_node;
  for (const auto& [id, o] : outcomes) {
    unsigned D = 0, B = 0, Dv = 0, F = 0;
    if (!o.pci_bus_id.empty() && std::sscanf(o.pci_bus_id.c_str(), "%x:%x:%x.%x", &D, &B, &Dv, &F) == 4)
      by_loc[{static_cast<int>(D), static_cast<int>((B << 8) | (Dv << 3) | F)}] = {ords.at(id), &o};
    else if (o.kfd_node_id >= 0)
      by_node[o.kfd_node_id] = {ords.at(id), &o};
  }
  std::map<std::string, ProbeOutcome> fixed;
  std::map<std::string, int> new_ords;
  for (const auto& [id, ord] : ords) {
    const GpuDevice* d = dev(id);
    if (!d) continue;
    const std::pair<int, const ProbeOutcome*>* hit = nullptr;
    if (d->location_id)
      if (auto it = by_loc.find({d->domain, d->location_id}); it != by_loc.end()) hit = &it->second;
    if (!hit && d->node_id >= 0)
      if (auto it = by_node.find(d->node_id); it != by_node.end()) hit = &it->second;
    if (hit && identity_matches(*d, *hit->second)) {
      new_ords[id] = hit->first;
      fixed[id] = *hit->second;
      if (hit->first != ord)
        MI_LOG(kError, "probe identity: device %s is ordinal %d, not %d (verdict re-keyed)", id.c_str(), hit->first,
               ord);
    }
  }
  std::string lost;
  for (const auto& [id, ord] : ords)
    if (!new_ords.count(id)) lost += (lost.empty() ? "" : ",") + id;
  if (!lost.empty()) MI_LOG(kError, "probe identity: no probed agent matches %s; they lose their ordinal", lost.c_str());
  std::map<std::string, int> merged;
  for (const auto& [id, o] : ordinals())
    if (!ords.count(id)) merged[id] = o;
  for (const auto& [id, o] : new_ords) merged[id] = o;
  {
    std::lock_guard<std::mutex> lk(state_mu_);
    ordinals_ = merged;
  }
  identity_remaps_++;
  metrics::global().inc("mi355x_dp_probe_identity_mismatch_total", {}, 1.0,
                        "sweeps whose probe replies came from other devices than the positional ordinal map");
  return fixed;
}

// device id -> host ordinal for the devices this sweep judges
std::map<std::string, int> Engine::judged_ordinals(const Reasons& reasons) {
  std::map<std::string, int> ords;
  for (const auto& [id, o] : ordinals())
    if (reasons.count(id)) ords[id] = o;
  return ords;
}

// Busy GPUs (other processes' queues, the probe server's own excluded) into
// *busy; false when the kfd process list is unreadable (then every GPU is busy).
bool Engine::update_busy_state(const std::map<std::string, int>& ords, std::set<std::string>* busy) {
  std::set<int64_t> probed_gids;
  for (const auto& [id, o] : ords) probed_gids.insert(gpu_id(id));
  probed_gids.erase(0);
  const std::set<std::string> own = prober_->own_kfd_entries(probed_gids);
  const bool unresolved = own.empty() && prober_->server_running() && cfg_.prober.keep_queues;
  const bool known = kfd_load(own, &load_);
  if (!known) {
    load_.clear();
    for (const auto& [id, o] : ords) busy->insert(id);
  } else {
    for (const auto& [id, o] : ords)
      if (int64_t g = gpu_id(id); g && load_.count(g)) busy->insert(id);
  }
  const bool now_known = known && !unresolved;
  if (now_known != busy_known_)
    glog::log(now_known ? glog::kInfo : glog::kWarning, __FILE__, __LINE__, "%s",
              now_known ? "busy-GPU state readable again"
                        : "busy-GPU state unknown: every GPU counts as busy, pending probes get the short grace");
  busy_known_ = now_known;
  metrics::global().set("mi355x_dp_busy_state_known", now_known ? 1.0 : 0.0, {},
                        "1 if busy GPUs can be told from idle ones (kfd process list readable)");
  return known;
}

// Crowded GPUs (too many tenant processes or queues): the probe server steps
// off them until they stay uncrowded for crowded_release_sweeps sweeps.
std::set<std::string> Engine::update_crowded(const std::map<std::string, int>& ords) {
  std::set<std::string> crowded;
  std::lock_guard<std::mutex> lk(state_mu_);
  if (cfg_.crowded_procs <= 0) {
    crowded_.clear();
    return crowded;
  }
  for (const auto& [id, o] : ords) {
    const GpuDevice* d = dev(id);
    const KfdNode* node = d && d->node_id >= 0 ? topo_.node(d->node_id) : nullptr;
    const auto ld = load_.count(gpu_id(id)) ? load_.at(gpu_id(id)) : std::make_pair(0, 0);
    const int64_t cp = node ? node->prop("num_cp_queues", 0) : 0;
    const bool is_crowded = ld.first >= cfg_.crowded_procs || (cp > 0 && ld.second + 2 > cp);
    if (is_crowded) {
      if (!crowded_.count(id))
        MI_LOG(kInfo, "GPU of %s is crowded (%d other processes, %d queues): the probe server steps off it",
               id.c_str(), ld.first, ld.second);
      crowded_[id] = 0;
    } else if (crowded_.count(id) && ++crowded_[id] >= cfg_.crowded_release_sweeps) {
      crowded_.erase(id);
      MI_LOG(kInfo, "GPU of %s is no longer crowded: probing it again", id.c_str());
    }
    if (crowded_.count(id)) crowded.insert(id);
  }
  return crowded;
}

// The probe server's round: the full-chip sweep on idle GPUs every
// chip_sweep_every sweeps (never while busy state is unknown), the one-wave
// probe elsewhere; replies are checked against each device's identity.
std::map<std::string, ProbeOutcome> Engine::run_probes(const std::map<std::string, int>& probe_ords,
                                                       const std::set<std::string>& busy,
                                                       const std::set<std::string>& idle, bool known) {
  if (probe_ords.empty()) return {};
  const bool chip = cfg_.chip_sweep_every > 0 && sweeps_ % static_cast<uint64_t>(cfg_.chip_sweep_every) == 0;
  if (chip && !known) MI_LOG(kWarning, "full-chip sweep skipped: busy-GPU state unknown");
  std::map<std::string, ProbeOutcome> raw;
  auto run = [&](const std::map<std::string, int>& sel, const char* kind) {
    std::vector<int> uniq;
    std::set<int> busy_ords;
    for (const auto& [id, o] : sel) {
      uniq.push_back(o);
      if (busy.count(id)) busy_ords.insert(o);
    }
    const auto by_ord = prober_->probe(uniq, busy_ords, kind);
    for (const auto& [id, o] : sel)
      if (auto it = by_ord.find(o); it != by_ord.end()) raw[id] = it->second;
  };
  std::map<std::string, int> swept, rest;
  for (const auto& [id, o] : probe_ords) (chip && idle.count(id) ? swept : rest)[id] = o;
  if (!swept.empty()) {
    run(swept, "sweep");
    chip_sweeps_++;
    metrics::global().inc("mi355x_dp_chip_sweeps_total", {}, 1.0,
                          "full-chip sweeps run (every CU of every XCD on the idle GPUs)");
  }
  if (!rest.empty()) run(rest, "probe");
  return verify_identity(probe_ords, raw);
}

// Crowded GPUs are probed from a fresh process only when amd-smi reports their
// GFX engine idle; otherwise the probe is skipped (and counted).
void Engine::probe_crowded(const std::set<std::string>& crowded, const std::map<std::string, int>& ords,
                           std::map<std::string, ProbeOutcome>* outcomes) {
  if (crowded.empty()) return;
  const auto act = gfx_activity();
  for (const auto& id : crowded) {
    const GpuDevice* d = dev(id);
    auto a = d ? act.find(d->bdf) : act.end();
    if (a != act.end() && a->second == 0) {
      (*outcomes)[id] = prober_->probe_ordinal(ords.at(id));
    } else {
      crowded_skips_++;
      metrics::global().inc("mi355x_dp_liveness_crowded_skips_total", {{"device", id}}, 1.0,
                            "probes skipped on GPUs crowded with tenant processes");
    }
  }
}

// Probe outcomes -> liveness tracks (hysteresis, busy grace, idle corroboration)
// -> a reason for every device whose track is not live.
void Engine::judge_liveness(const std::map<std::string, ProbeOutcome>& outcomes, const std::set<std::string>& busy,
                            Reasons* reasons) {
  const double now = mono_s();
  const double grace = busy_known_ ? cfg_.busy_grace_s : std::min(cfg_.busy_grace_s, cfg_.unknown_busy_grace_s);
  std::set<std::string> idle_wedged;
  std::vector<std::string> waiting;
  for (const auto& [id, o] : outcomes)
    if (o.pending && busy.count(id)) waiting.push_back(id);
  if (!waiting.empty() && cfg_.corroborate) {
    const auto act = gfx_activity();
    for (const auto& id : waiting) {
      const GpuDevice* d = dev(id);
      auto a = d ? act.find(d->bdf) : act.end();
      Track& tr = track_[id];
      tr.idle_pending = a != act.end() && a->second == 0 ? tr.idle_pending + 1 : 0;
      if (tr.idle_pending >= cfg_.idle_sweeps) idle_wedged.insert(id);
    }
  }
  for (const auto& [id, o] : outcomes) {
    Track& tr = track_[id];
    if (o.interrupted) {  // the daemon is stopping: the track keeps its last verdict
      if (!tr.live) (*reasons)[id].push_back("liveness probe: " + tr.last_reason);
      continue;
    }
    metrics::global().set("mi355x_dp_liveness_probe_ms", o.latency_ms, {{"device", id}},
                          "last liveness probe round trip");
    if (!o.pending) tr.idle_pending = 0;
    if (o.ok) {
      tr.fails = 0;
      tr.oks++;
      tr.pending_since = -1;
      if (!tr.live && tr.oks >= cfg_.recover_threshold) tr.live = true;
    } else if (o.pending && busy.count(id) && !idle_wedged.count(id) &&
               now - (tr.pending_since >= 0 ? tr.pending_since : now) < grace) {
      if (tr.pending_since < 0) tr.pending_since = now;  // queued behind a tenant: inconclusive
      metrics::global().inc("mi355x_dp_liveness_inconclusive_total", {{"device", id}}, 1.0,
                            "probes queued behind a busy GPU");
    } else {
      tr.oks = 0;
      tr.fails++;
      tr.last_reason = o.reason;
      if (idle_wedged.count(id)) {
        tr.last_reason += " while the GPU reports 0% GFX activity (" + std::to_string(tr.idle_pending) +
                          " sweeps): no tenant kernel is running";
        metrics::global().inc("mi355x_dp_liveness_idle_pending_total", {{"device", id}}, 1.0,
                              "pending probes on an idle GFX engine");
      }
      if (!o.pending) tr.pending_since = -1;
      if (tr.live && tr.fails >= cfg_.fail_threshold) tr.live = false;
    }
    if (!tr.live) (*reasons)[id].push_back("liveness probe: " + tr.last_reason);
  }
}

void Engine::liveness_pass(Reasons* reasons) {
  std::map<std::string, int> ords = judged_ordinals(*reasons);
  std::set<std::string> busy;
  const bool known = update_busy_state(ords, &busy);
  const std::set<std::string> crowded = update_crowded(ords);
  std::map<std::string, int> probe_ords;
  for (const auto& [id, o] : ords)
    if (!crowded.count(id)) probe_ords[id] = o;
  if (!crowded.empty()) {
    std::vector<int> vis;
    for (const auto& [id, o] : probe_ords) vis.push_back(o);
    prober_->set_visible(vis);
    if (probe_ords.empty() && prober_->server_running()) prober_->close();  // hold nothing on any GPU
  } else {
    prober_->set_visible(std::nullopt);
  }
  // idle GPUs (no other process's queues) for the full-chip sweep and the
  // throughput check; none while busy state is unknown (both hold every CU)
  std::set<std::string> idle;
  if (known)
    for (const auto& [id, o] : probe_ords)
      if (int64_t g = gpu_id(id); g && !load_.count(g)) idle.insert(id);
  std::map<std::string, ProbeOutcome> outcomes = run_probes(probe_ords, busy, idle, known);
  probe_crowded(crowded, ords, &outcomes);
  ords = judged_ordinals(*reasons);  // verify_identity may have remapped the ordinals
  judge_liveness(outcomes, busy, reasons);
  for (auto& [id, rs] : *reasons)
    if (!ords.count(id)) rs.push_back("no HIP device for this ID (render node inaccessible?)");
  if (cfg_.perf_check_every > 0 && sweeps_ % static_cast<uint64_t>(cfg_.perf_check_every) == 0) {
    std::map<std::string, int> cand;
    for (const auto& [id, o] : probe_ords)
      if (idle.count(id) && track_[id].live && ords.count(id)) cand[id] = o;
    if (!cand.empty()) perf_check(cand);
  }
  std::lock_guard<std::mutex> lk(mu_);
  for (const auto& [id, pv] : perf_)
    if (reasons->count(id) && (pv.first == "failed" || (pv.first == "degraded" && cfg_.perf_action == "unhealthy")))
      (*reasons)[id].push_back(pv.second);
}

// amd-smi: a rise of a device's uncorrectable ECC count since the last sweep
bool Engine::ecc_pass(Reasons* reasons) {
  if (!smi_held_) smi_held_ = smi_hold();
  const SmiSnapshot snap = smi_snapshot();
  if (!snap.ok) return false;
  std::map<std::string, const SmiGpu*> by_bdf;
  for (const auto& g : snap.gpus)
    if (g.ecc_ok) by_bdf[g.bdf] = &g;
  for (const auto& d : devices_) {
    auto it = by_bdf.find(d.bdf);
    if (it == by_bdf.end()) continue;
    const uint64_t cur = it->second->ecc_uncorrectable;
    auto prev = ecc_.find(d.id);
    if (prev != ecc_.end() && cur > prev->second)
      (*reasons)[d.id].push_back("uncorrectable ECC errors rose " + std::to_string(prev->second) + "->" +
                                 std::to_string(cur));
    ecc_[d.id] = cur;
  }
  return true;
}

// amd-smi events: counted and logged; a GPU between gpu_pre_reset and
// gpu_post_reset is Unhealthy
bool Engine::events_pass(Reasons* reasons) {
  if (!events_started_) {
    events_started_ = true;
    events_ = std::make_unique<SmiEventWatcher>();
    // vmfault 1, thermal_throttle 2, gpu_pre_reset 3, gpu_post_reset 4, queue_eviction 9
    const uint64_t mask = (1ull << 0) | (1ull << 1) | (1ull << 2) | (1ull << 3) | (1ull << 8);
    const std::string err = events_->start(mask);
    if (!err.empty()) MI_LOG(kWarning, "amd-smi event notification unavailable: %s", err.c_str());
  }
  if (events_ && events_->running()) {
    for (const auto& ev : events_->poll(0)) {
      metrics::global().inc("mi355x_dp_gpu_events_total", {{"bdf", ev.bdf}, {"event", ev.name}}, 1.0,
                            "amd-smi GPU events");
      if (ev.name == "gpu_pre_reset") {
        resetting_[ev.bdf] = ev.message;
        MI_LOG(kWarning, "GPU %s: reset starting (%s)", ev.bdf.c_str(), ev.message.c_str());
      } else if (ev.name == "gpu_post_reset") {
        resetting_.erase(ev.bdf);
        MI_LOG(kWarning, "GPU %s: reset finished", ev.bdf.c_str());
      } else {
        MI_LOG(kInfo, "GPU %s: %s %s", ev.bdf.c_str(), ev.name.c_str(), ev.message.c_str());
      }
    }
  }
  for (const auto& d : devices_)
    if (resetting_.count(d.bdf))
      (*reasons)[d.id].push_back("GPU reset in progress (amd-smi gpu_pre_reset, no post_reset yet)");
  return events_ && events_->running();
}

// reasons -> the published snapshot; true when any device's health changed
bool Engine::publish(Reasons reasons) {
  std::map<std::string, Verdict> next;
  for (auto& [id, rs] : reasons) next[id] = Verdict{rs.empty(), std::move(rs)};
  bool changed = false;
  std::lock_guard<std::mutex> lk(mu_);
  for (const auto& [id, v] : next) {
    auto old = snapshot_.find(id);
    if (old == snapshot_.end() || old->second.healthy != v.healthy) {
      changed = true;
      std::string why;
      for (const auto& r : v.reasons) why += (why.empty() ? "" : "; ") + r;
      MI_LOG(kWarning, "device %s: %s -> %s %s", id.c_str(),
             old == snapshot_.end() ? "?" : (old->second.healthy ? "Healthy" : "Unhealthy"),
             v.healthy ? "Healthy" : "Unhealthy", why.c_str());
    }
  }
  if (changed) version_++;
  snapshot_ = std::move(next);
  for (const auto& [id, v] : snapshot_)
    metrics::global().set("mi355x_dp_device_healthy", v.healthy ? 1.0 : 0.0, {{"device", id}},
                          "1 if the device is advertised Healthy");
  return changed;
}

// PreStartContainer's check: beside any sweep, never behind it.
std::map<std::string, ProbeOutcome> Engine::probe_now(const std::vector<std::string>& ids, double budget_s) {
  if (!cfg_.liveness || !prober_) return {};
  trace::Span span("liveness.prestart", "health", {{"devices", std::to_string(ids.size())}});
  std::map<std::string, int> sel;
  {
    const auto ords = ordinals();
    std::lock_guard<std::mutex> lk(state_mu_);
    for (const auto& id : ids)  // the probe server stays off crowded GPUs here too (update_crowded)
      if (auto it = ords.find(id); it != ords.end() && !crowded_.count(id)) sel[id] = it->second;
  }
  if (sel.empty()) return {};
  std::vector<int> uniq;
  for (const auto& [id, o] : sel) uniq.push_back(o);
  // GPUs with other processes' queues (the probe server's own excluded), as a sweep
  // sees them: a dispatch queued behind their work there is inconclusive and gets
  // no fresh-process confirmation (which the container would wait for). Read only
  // when a probe did not pass at once.
  auto busy_of = [this, &sel] {
    std::set<int64_t> gids;
    for (const auto& [id, o] : sel) gids.insert(gpu_id(id));
    gids.erase(0);
    std::map<int64_t, std::pair<int, int>> load;
    const bool known = kfd_load(prober_->own_kfd_entries(gids), &load);
    std::set<int> busy;
    for (const auto& [id, o] : sel)
      if (!known || load.count(gpu_id(id))) busy.insert(o);
    return busy;
  };
  const auto by_ord = prober_->check(uniq, busy_of, budget_s);
  std::map<std::string, ProbeOutcome> out;
  for (const auto& [id, o] : sel) {
    auto it = by_ord.find(o);
    if (it == by_ord.end()) continue;
    ProbeOutcome r = it->second;
    if (const GpuDevice* d = dev(id); d && !r.interrupted && !identity_matches(*d, r)) {
      // the ordinal map is stale (the sweep re-keys it): no verdict on this device from another agent's reply
      r.ok = false;
      r.pending = true;
      r.reason = "probe reply from agent " + r.pci_bus_id + ", not this device: left to the next sweep";
    }
    out[id] = r;
  }
  return out;
}

// One sweep: every source adds its reasons; a device with none is Healthy.
// one reading of a health source: /metrics shows which sources run and answer
static void source_reading(const char* source, bool ok) {
  metrics::global().inc("mi355x_dp_health_source_readings_total", {{"source", source}, {"result", ok ? "ok" : "error"}},
                        1.0, "readings of each health source per sweep: ok, or error (source unavailable)");
}

bool Engine::sweep() {
  trace::Span span("health.sweep", "health", {{"devices", std::to_string(devices_.size())}});
  const double t0 = mono_s();
  Reasons reasons;
  for (const auto& d : devices_) reasons[d.id];
  const auto kv = kfd_verdicts();
  source_reading("kfd", !(kv.size() == devices_.size() && !devices_.empty() &&
                          kv.begin()->second == "kfd topology unavailable"));
  for (const auto& [id, r] : kv) reasons[id].push_back(r);
  if (!cfg_.exporter_socket.empty() || exporter_source) {
    const auto hmap = exporter_health();
    source_reading("exporter", !hmap.empty());
    for (const auto& d : devices_)
      if (auto it = hmap.find(d.bdf); it != hmap.end() && !it->second)
        reasons[d.id].push_back("exporter reports " + d.bdf + " unhealthy");
  }
  if (cfg_.liveness && prober_) {
    // probe_now() runs beside this pass: it reads the ordinal map and the crowd
    // state under state_mu_ and sends its own tagged request to the probe server
    std::lock_guard<std::mutex> op(op_mu_);
    const uint64_t fb = static_cast<uint64_t>(prober_->fallbacks.load());
    liveness_pass(&reasons);
    source_reading("liveness", static_cast<uint64_t>(prober_->fallbacks.load()) == fb);
  }
  if (cfg_.smi_ecc) {
    const bool ok = smi_available() && ecc_pass(&reasons);
    source_reading("smi_ecc", ok);
  }
  if (cfg_.smi_events) source_reading("smi_events", events_pass(&reasons));
  if (cfg_.smi_xgmi) source_reading("smi_xgmi", fabric_check());
  const bool changed = publish(std::move(reasons));
  sweeps_++;
  last_sweep_ms_ = (mono_s() - t0) * 1e3;
  return changed;
}

// ---- xGMI link state (health/fabric.py FabricWatcher) ----------------------------
namespace {
constexpr int kLinkUp = 1;
constexpr int kLinkTypeXgmi = 2;

std::string lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

// the JSON shape of core().smi_xgmi_links()
SmiXgmiSnapshot xgmi_from_json(const std::string& text) {
  SmiXgmiSnapshot snap;
  std::string err;
  auto doc = json::parse(text, &err);
  if (!doc || doc->kind != json::Value::Object) {
    snap.error = "xgmi snapshot: " + (err.empty() ? std::string("not an object") : err);
    return snap;
  }
  auto flag = [](const json::Value* v) { return v && v->kind == json::Value::Bool && v->b; };
  auto num = [](const json::Value* v, long long dflt) {
    return v && v->kind == json::Value::Number ? std::strtoll(v->s.c_str(), nullptr, 10) : dflt;
  };
  snap.ok = flag(doc->get("ok"));
  snap.error = doc->str("error");
  if (const json::Value* gpus = doc->get("gpus"); gpus && gpus->kind == json::Value::Array)
    for (const auto& g : gpus->arr) {
      SmiXgmiLinks l;
      l.bdf = g.str("bdf");
      l.status_ok = flag(g.get("status_ok"));
      if (const json::Value* st = g.get("status"); st && st->kind == json::Value::Array)
        for (const auto& x : st->arr) l.status.push_back(static_cast<int>(num(&x, -1)));
      l.metrics_ok = flag(g.get("metrics_ok"));
      if (const json::Value* ps = g.get("peers"); ps && ps->kind == json::Value::Array)
        for (const auto& p : ps->arr) {
          SmiLinkPeer q;
          q.peer_bdf = p.str("peer_bdf");
          q.link_type = static_cast<int>(num(p.get("link_type"), -1));
          q.bit_rate_gbps = static_cast<uint32_t>(num(p.get("bit_rate_gbps"), 1));
          l.peers.push_back(q);
        }
      snap.gpus.push_back(std::move(l));
    }
  return snap;
}
}  // namespace

SmiXgmiSnapshot Engine::read_xgmi() {
  if (xgmi_source) return xgmi_source();
  if (!cfg_.xgmi_file.empty()) {
    auto text = read_file(cfg_.xgmi_file);
    if (!text) {
      SmiXgmiSnapshot s;
      s.error = "xgmi snapshot " + cfg_.xgmi_file + " unreadable";
      return s;
    }
    return xgmi_from_json(*text);
  }
  return smi_xgmi_links();
}

bool Engine::fabric_check() {
  const SmiXgmiSnapshot snap = read_xgmi();
  if (!snap.ok) {
    if (snap.error != xgmi_error_) MI_LOG(kWarning, "xGMI link state unavailable: %s", snap.error.c_str());
    xgmi_error_ = snap.error;
    return false;
  }
  xgmi_error_.clear();
  xgmi_readings_++;
  std::set<std::pair<std::string, std::string>> degraded;
  std::map<std::string, int> down;
  auto pair = [](const std::string& a, const std::string& b) { return a <= b ? std::make_pair(a, b) : std::make_pair(b, a); };
  for (const auto& g : snap.gpus) {
    const std::string bdf = lower(g.bdf);
    auto me_it = gpu_by_bdf_.find(bdf);
    if (me_it == gpu_by_bdf_.end()) continue;  // a GPU this plugin does not advertise
    const std::string& me = me_it->second;
    int up = -1;
    if (g.status_ok) up = static_cast<int>(std::count(g.status.begin(), g.status.end(), kLinkUp));
    std::set<std::string> live;
    if (g.metrics_ok)
      for (const auto& p : g.peers) {
        const std::string pb = lower(p.peer_bdf);
        if (p.link_type == kLinkTypeXgmi && gpu_by_bdf_.count(pb) && p.bit_rate_gbps > 0) live.insert(pb);
      }
    auto base = xgmi_base_.find(bdf);
    if (base == xgmi_base_.end()) {
      xgmi_base_[bdf] = {up, live};
      continue;
    }
    std::vector<std::string> lost_peers;
    for (const auto& pb : base->second.second)
      if (!live.count(pb)) lost_peers.push_back(pb);
    const int lost_links = base->second.first >= 0 && up >= 0 ? base->second.first - up : 0;
    if (!lost_peers.empty()) {
      for (const auto& pb : lost_peers) degraded.insert(pair(me, gpu_by_bdf_.at(pb)));
    } else if (lost_links > 0) {
      // no peer can be named: every xGMI pair of this GPU
      std::set<std::string> peers = base->second.second;
      if (peers.empty())
        for (const auto& [b, k] : gpu_by_bdf_)
          if (b != bdf) peers.insert(b);
      for (const auto& pb : peers) {
        auto o = gpu_by_bdf_.find(pb);
        if (o != gpu_by_bdf_.end() && o->second != me) degraded.insert(pair(me, o->second));
      }
    }
    if (lost_links > 0 || !lost_peers.empty())
      down[bdf] = std::max(lost_links, static_cast<int>(lost_peers.size()));
  }
  int total = 0;
  for (const auto& [b, n] : down) total += n;
  std::lock_guard<std::mutex> lk(mu_);
  links_down_ = down;
  if (degraded == degraded_) return true;
  for (const auto& p : degraded)
    if (!degraded_.count(p))
      MI_LOG(kWarning, "xGMI link between GPUs %s and %s is down: multi-GPU placement avoids the pair",
             p.first.c_str(), p.second.c_str());
  for (const auto& p : degraded_)
    if (!degraded.count(p))
      MI_LOG(kWarning, "xGMI link between GPUs %s and %s is back up", p.first.c_str(), p.second.c_str());
  degraded_ = std::move(degraded);
  fabric_version_++;
  metrics::global().set("mi355x_dp_xgmi_links_down", total, {}, "xGMI links down vs the first reading");
  return true;
}

std::vector<std::pair<std::string, std::string>> Engine::degraded_links() const {
  std::lock_guard<std::mutex> lk(mu_);
  return {degraded_.begin(), degraded_.end()};
}

uint64_t Engine::fabric_version() const {
  std::lock_guard<std::mutex> lk(mu_);
  return fabric_version_;
}

std::map<std::string, int> Engine::links_down() const {
  std::lock_guard<std::mutex> lk(mu_);
  return links_down_;
}

// ---- throughput check (health/monitor.py _perf_check) ----------------------------
std::vector<std::string> Engine::perf_problems(const ProbeOutcome& o) const {
  auto get = [&](const char* k) {
    auto it = o.detail.find(k);
    return it == o.detail.end() ? 0.0 : it->second;
  };
  const double cus = get("cu_count");
  const double share = cus > 0 ? std::min(1.0, cus / 256.0) : 1.0;  // a CPX partition has 1/8 of the CUs
  std::vector<std::string> out;
  struct Floor {
    const char* key;
    double floor;
    const char* what;
    const char* unit;
  };
  for (const Floor& f : {Floor{"hbm_read_gbps", cfg_.perf_min_hbm_read_gbps, "HBM read", "GB/s"},
                         Floor{"hbm_write_gbps", cfg_.perf_min_hbm_write_gbps, "HBM write", "GB/s"},
                         Floor{"mfma_tflops", cfg_.perf_min_mfma_tflops, "bf16 MFMA", "TFLOP/s"}}) {
    const double v = get(f.key);
    if (f.floor > 0 && v < f.floor * share) {
      char b[128];
      std::snprintf(b, sizeof(b), "%s %.0f %s < %.0f", f.what, v, f.unit, f.floor * share);
      out.push_back(b);
    }
  }
  std::vector<double> clocks;
  for (double c : o.xcd_clock_mhz)
    if (c > 0) clocks.push_back(c);
  if (clocks.size() >= 2 && cfg_.perf_min_xcd_clock_ratio > 0) {
    std::vector<double> sorted = clocks;
    std::sort(sorted.begin(), sorted.end());
    const double med = sorted[sorted.size() / 2];
    const size_t i = static_cast<size_t>(std::min_element(clocks.begin(), clocks.end()) - clocks.begin());
    if (clocks[i] < cfg_.perf_min_xcd_clock_ratio * med) {
      char b[128];
      std::snprintf(b, sizeof(b), "XCD %zu at %.0f MHz vs median %.0f MHz under MFMA load", i, clocks[i], med);
      out.push_back(b);
    }
  }
  return out;
}

void Engine::perf_check(const std::map<std::string, int>& ords) {
  trace::Span span("health.perf_check", "health", {{"devices", std::to_string(ords.size())}});
  std::vector<int> uniq;
  for (const auto& [id, o] : ords) uniq.push_back(o);
  const auto by_ord = prober_->probe(uniq, {}, "perf");
  perf_checks_++;
  auto& m = metrics::global();
  m.inc("mi355x_dp_perf_checks_total", {}, 1.0, "throughput checks run (HBM pattern + MFMA + clocks)");
  static const std::map<std::string, double> kState = {{"ok", 0.0}, {"degraded", 1.0}, {"failed", 2.0}};
  for (const auto& [id, ord] : ords) {
    auto it = by_ord.find(ord);
    if (it == by_ord.end()) continue;
    const ProbeOutcome& o = it->second;
    if (o.interrupted) continue;  // stopped by the shutdown, not failed: the last result stands
    std::string state = "ok", why;
    if (!o.ok) {
      state = "failed";
      why = "throughput check: " + o.reason;
    } else if (const auto probs = perf_problems(o); !probs.empty()) {
      state = "degraded";
      why = "throughput check: ";
      for (size_t i = 0; i < probs.size(); ++i) why += (i ? "; " : "") + probs[i];
    }
    std::string prev = "ok";
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (auto p = perf_.find(id); p != perf_.end()) prev = p->second.first;
      perf_[id] = {state, why};
      perf_last_[id] = o;
    }
    if (state != prev)
      glog::log(state == "ok" ? glog::kInfo : glog::kWarning, __FILE__, __LINE__, "device %s: throughput check %s -> %s %s",
                id.c_str(), prev.c_str(), state.c_str(), why.c_str());
    auto get = [&](const char* k) {
      auto d = o.detail.find(k);
      return d == o.detail.end() ? 0.0 : d->second;
    };
    if (o.ok)
      MI_VLOG(2, "device %s: throughput HBM write %.0f / read %.0f GB/s, bf16 MFMA %.0f TFLOP/s at %.0f MHz", id.c_str(),
              get("hbm_write_gbps"), get("hbm_read_gbps"), get("mfma_tflops"), get("clock_mhz_median"));
    const metrics::Labels dev = {{"device", id}};
    m.set("mi355x_dp_perf_state", kState.at(state), dev,
          "last throughput check: 0 ok, 1 degraded (rates under the floors), 2 failed");
    if (o.ok) {
      m.set("mi355x_dp_perf_hbm_read_gbps", get("hbm_read_gbps"), dev, "last throughput check: HBM read bandwidth");
      m.set("mi355x_dp_perf_hbm_write_gbps", get("hbm_write_gbps"), dev, "last throughput check: HBM write bandwidth");
      m.set("mi355x_dp_perf_mfma_tflops", get("mfma_tflops"), dev,
            "last throughput check: sustained dense bf16 MFMA rate");
      m.set("mi355x_dp_perf_clock_mhz", get("clock_mhz_median"), dev,
            "last throughput check: median workgroup shader clock under MFMA load");
      for (size_t x = 0; x < o.xcd_clock_mhz.size(); ++x)
        m.set("mi355x_dp_perf_xcd_clock_mhz", o.xcd_clock_mhz[x], {{"device", id}, {"xcd", std::to_string(x)}},
              "last throughput check: median shader clock per XCD");
    }
  }
}

std::map<std::string, ProbeOutcome> Engine::perf_last() const {
  std::lock_guard<std::mutex> lk(mu_);
  return perf_last_;
}

uint64_t Engine::xgmi_readings() const { return xgmi_readings_; }
std::string Engine::xgmi_error() const { return xgmi_error_; }

std::map<std::string, std::pair<std::string, std::string>> Engine::perf_verdicts() const {
  std::lock_guard<std::mutex> lk(mu_);
  return perf_;
}

}  // namespace mi355x::health
