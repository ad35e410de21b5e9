// pybind11 bindings of the native health engine (mi355x/health_engine.h): the
// policy the native daemon runs, driven from the tests with the same stub
// probes and fixtures as the Python monitor's tests.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "mi355x/gpu_discovery.h"
#include "mi355x/health_engine.h"
#include "mi355x/metrics.h"
#include "mi355x/kfd_topology.h"

namespace py = pybind11;
using namespace mi355x;

namespace {

class PyHealthEngine {
 public:
  PyHealthEngine(const std::string& sysfs_root, const py::dict& opts) {
    health::Config c;
    c.sysfs_root = sysfs_root;
    auto get = [&](const char* k) -> py::object {
      if (opts.contains(k)) return py::object(opts[k]);
      return py::none();
    };
    auto s = [&](const char* k, std::string* out) {
      if (auto v = get(k); !v.is_none()) *out = v.cast<std::string>();
    };
    auto d = [&](const char* k, double* out) {
      if (auto v = get(k); !v.is_none()) *out = v.cast<double>();
    };
    auto i = [&](const char* k, int* out) {
      if (auto v = get(k); !v.is_none()) *out = v.cast<int>();
    };
    auto b = [&](const char* k, bool* out) {
      if (auto v = get(k); !v.is_none()) *out = v.cast<bool>();
    };
    s("dev_root", &c.dev_root);
    s("exporter_socket", &c.exporter_socket);
    d("exporter_timeout_s", &c.exporter_timeout_s);
    b("liveness", &c.liveness);
    i("fail_threshold", &c.fail_threshold);
    i("recover_threshold", &c.recover_threshold);
    d("busy_grace_s", &c.busy_grace_s);
    d("unknown_busy_grace_s", &c.unknown_busy_grace_s);
    b("corroborate", &c.corroborate);
    i("idle_sweeps", &c.idle_sweeps);
    i("crowded_procs", &c.crowded_procs);
    i("crowded_release_sweeps", &c.crowded_release_sweeps);
    b("smi_ecc", &c.smi_ecc);
    b("smi_events", &c.smi_events);
    b("smi_xgmi", &c.smi_xgmi);
    i("chip_sweep_every", &c.chip_sweep_every);
    i("perf_check_every", &c.perf_check_every);
    s("perf_action", &c.perf_action);
    d("perf_min_hbm_read_gbps", &c.perf_min_hbm_read_gbps);
    d("perf_min_hbm_write_gbps", &c.perf_min_hbm_write_gbps);
    d("perf_min_mfma_tflops", &c.perf_min_mfma_tflops);
    d("perf_min_xcd_clock_ratio", &c.perf_min_xcd_clock_ratio);
    i("perf_mib", &c.prober.perf_mib);
    i("perf_iters", &c.prober.perf_iters);
    s("xgmi_file", &c.xgmi_file);
    s("probe_exe", &c.prober.exe);
    d("probe_timeout_s", &c.prober.timeout_s);
    d("busy_deadline_s", &c.prober.busy_deadline_s);
    i("probe_iters", &c.prober.iters);
    i("probe_max_parallel", &c.prober.max_parallel);
    b("persistent", &c.prober.persistent);
    b("keep_queues", &c.prober.keep_queues);
    s("kfd_proc_dir", &c.prober.kfd_proc_dir);
    if (auto v = get("argv_prefix"); !v.is_none()) c.prober.argv_prefix = v.cast<std::vector<std::string>>();
    if (auto v = get("extra_env"); !v.is_none())
      for (auto& [k, val] : v.cast<std::map<std::string, std::string>>()) c.prober.extra_env.emplace_back(k, val);
    if (auto v = get("kfd_exclude"); !v.is_none())
      for (const auto& pid : v.cast<std::vector<std::string>>()) c.kfd_exclude.insert(pid);
    const KfdTopology topo = KfdTopology::load_sysfs(sysfs_root);
    DiscoveryResult res = discover_gpus(sysfs_root, topo);
    if (auto v = get("device_ids"); !v.is_none()) {  // judge only these (as the daemon's -device_ids)
      const auto ids = v.cast<std::vector<std::string>>();
      const std::set<std::string> keep(ids.begin(), ids.end());
      std::vector<GpuDevice> sel;
      for (auto& d : res.devices)
        if (keep.count(d.id)) sel.push_back(std::move(d));
      res.devices = std::move(sel);
    }
    eng_ = std::make_unique<health::Engine>(std::move(res.devices), topo, c);
  }

  bool sweep() {
    py::gil_scoped_release nogil;
    return eng_->sweep();
  }
  py::dict snapshot() const {
    py::dict out;
    for (const auto& [id, v] : eng_->snapshot()) out[py::str(id)] = py::make_tuple(v.healthy, v.reasons);
    return out;
  }
  py::dict stats() {
    py::dict d;
    d["sweeps"] = eng_->sweeps();
    d["identity_remaps"] = eng_->identity_remaps();
    d["crowded_skips"] = eng_->crowded_skips();
    d["busy_state_known"] = eng_->busy_state_known();
    d["last_sweep_ms"] = eng_->last_sweep_ms();
    d["version"] = eng_->version();
    d["chip_sweeps"] = eng_->chip_sweeps();
    d["perf_checks"] = eng_->perf_checks();
    if (auto* p = eng_->prober()) {
      d["server_starts"] = p->server_starts.load();
      d["server_restarts"] = p->server_restarts.load();
      d["fallbacks"] = p->fallbacks.load();
      d["prober_sweeps"] = p->sweeps.load();
      d["checks"] = p->checks.load();
      d["check_fresh"] = p->check_fresh.load();
      d["check_inconclusive"] = p->check_inconclusive.load();
      d["server_running"] = p->server_running();
      d["server_pid"] = p->server_pid();
    }
    d["xgmi_readings"] = eng_->xgmi_readings();
    d["xgmi_error"] = eng_->xgmi_error();
    return d;
  }
  std::vector<std::pair<std::string, std::string>> degraded_links() const { return eng_->degraded_links(); }
  uint64_t fabric_version() const { return eng_->fabric_version(); }
  std::map<std::string, std::pair<std::string, std::string>> perf_verdicts() const { return eng_->perf_verdicts(); }
  std::vector<std::string> perf_problems(const py::dict& d) const {
    health::ProbeOutcome o;
    for (auto [k, v] : d) {
      const std::string key = k.cast<std::string>();
      if (key == "xcd_clock_mhz") o.xcd_clock_mhz = v.cast<std::vector<double>>();
      else o.detail[key] = v.cast<double>();
    }
    return eng_->perf_problems(o);
  }
  std::map<std::string, int> links_down() const { return eng_->links_down(); }
  void set_activity(std::optional<std::map<std::string, int>> a) {
    if (!a) eng_->activity_source = nullptr;
    else eng_->activity_source = [a] { return *a; };
  }
  void set_exporter(std::optional<std::map<std::string, bool>> h) {
    if (!h) eng_->exporter_source = nullptr;
    else eng_->exporter_source = [h] { return *h; };
  }
  std::map<std::string, int> ordinals() { return eng_->ordinals(); }
  // kfd gpu_id -> (other processes with queues, their queues) as the last sweep saw it
  std::map<int64_t, std::pair<int, int>> gpu_load() const { return eng_->gpu_load(); }
  // the running probe server's kfd proc entries covering these kfd gpu ids
  std::set<std::string> own_kfd_entries(const std::set<int64_t>& gpu_ids) {
    auto* p = eng_->prober();
    return p ? p->own_kfd_entries(gpu_ids) : std::set<std::string>{};
  }
  // PreStartContainer's check (Engine::probe_now): device id -> outcome dict
  py::dict check(const std::vector<std::string>& ids, double budget_s) {
    std::map<std::string, health::ProbeOutcome> res;
    {
      py::gil_scoped_release nogil;
      res = eng_->probe_now(ids, budget_s);
    }
    py::dict out;
    for (const auto& [id, o] : res) {
      py::dict d;
      d["ok"] = o.ok;
      d["pending"] = o.pending;
      d["interrupted"] = o.interrupted;
      d["reason"] = o.reason;
      d["latency_ms"] = o.latency_ms;
      out[py::str(id)] = d;
    }
    return out;
  }
  void close() {
    py::gil_scoped_release nogil;
    eng_->close();
  }

 private:
  std::unique_ptr<health::Engine> eng_;
};

}  // namespace

void bind_health(py::module_& m) {
  py::class_<PyHealthEngine>(m, "HealthEngine",
                             "native per-device health engine (the native daemon's); options as health::Config")
      .def(py::init<const std::string&, const py::dict&>(), py::arg("sysfs_root"), py::arg("options") = py::dict())
      .def("sweep", &PyHealthEngine::sweep, "one sweep; True when a verdict changed")
      .def("snapshot", &PyHealthEngine::snapshot, "device id -> (healthy, reasons)")
      .def("stats", &PyHealthEngine::stats)
      .def("ordinals", &PyHealthEngine::ordinals)
      .def("gpu_load", &PyHealthEngine::gpu_load)
      .def("own_kfd_entries", &PyHealthEngine::own_kfd_entries, py::arg("gpu_ids"))
      .def("check", &PyHealthEngine::check, py::arg("ids"), py::arg("budget_s") = 5.0,
           "PreStartContainer's check of these devices now (beside any sweep)")
      .def("set_activity", &PyHealthEngine::set_activity, py::arg("activity"),
           "bdf -> GFX activity % used instead of amd-smi (None = amd-smi)")
      .def("set_exporter", &PyHealthEngine::set_exporter, py::arg("health"),
           "bdf -> healthy used instead of the exporter socket (None = socket)")
      .def("degraded_links", &PyHealthEngine::degraded_links, "xGMI pairs (allocator group keys) degraded")
      .def("fabric_version", &PyHealthEngine::fabric_version)
      .def("perf_verdicts", &PyHealthEngine::perf_verdicts, "device -> (ok | degraded | failed, reason)")
      .def("perf_problems", &PyHealthEngine::perf_problems, py::arg("detail"))
      .def("links_down", &PyHealthEngine::links_down)
      .def("close", &PyHealthEngine::close);
  // a private registry (the process-wide one is metrics::global(), see `metrics_render`)
  py::class_<metrics::Registry>(m, "MetricsRegistry", "Prometheus registry of the native daemon (mi355x/metrics.h)")
      .def(py::init<>())
      .def("inc", [](metrics::Registry& r, const std::string& name, double v, const std::string& help,
                     const std::map<std::string, std::string>& labels) {
             r.inc(name, metrics::Labels(labels.begin(), labels.end()), v, help);
           }, py::arg("name"), py::arg("v") = 1.0, py::arg("help") = "", py::arg("labels") = std::map<std::string, std::string>())
      .def("set", [](metrics::Registry& r, const std::string& name, double v, const std::string& help,
                     const std::map<std::string, std::string>& labels) {
             r.set(name, v, metrics::Labels(labels.begin(), labels.end()), help);
           }, py::arg("name"), py::arg("v"), py::arg("help") = "", py::arg("labels") = std::map<std::string, std::string>())
      .def("observe_ms", [](metrics::Registry& r, const std::string& name, double ms, const std::string& help,
                            const std::map<std::string, std::string>& labels) {
             r.observe_ms(name, ms, metrics::Labels(labels.begin(), labels.end()), help);
           }, py::arg("name"), py::arg("ms"), py::arg("help") = "", py::arg("labels") = std::map<std::string, std::string>())
      .def("render", &metrics::Registry::render);
  m.def("metrics_render", [] { return metrics::global().render(); }, "the process-wide native registry");
  m.def("exporter_list", [](const std::string& socket, double timeout_s) {
    std::string err;
    std::map<std::string, bool> h;
    {
      py::gil_scoped_release nogil;
      h = health::exporter_list(socket, timeout_s, -1, &err);
    }
    return py::make_tuple(h, err);
  });
}
