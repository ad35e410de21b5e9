#include "flags.h"

#include <cstdlib>
#include <map>
#include <set>

#include "mi355x/goflag.h"

namespace mi355x::daemon {

std::string usage(const std::string& argv0) {
  return "usage: " + argv0 +
         " [-pulse N] [-driver_type container|vf-passthrough|pf-passthrough] "
         "[-resource_naming_strategy single|mixed] [-kubelet_dir DIR] [-sysfs_root DIR] [-dev_root DIR] "
         "[-exporter_socket PATH] [-send_every_pulse] [-allocator_search auto|reference|extended] "
         "[-allocator_extended_search] [-grpc_watchdog S] [-reregister S] [-register_timeout S] [-config FILE] "
         "[-metrics_port N] [-topology_watch S] "
         "[-device_list_strategy device-specs|cdi-cri|cdi-annotations[,...]] [-cdi_spec_dir DIR] "
         "[-liveness [-liveness_mode persistent|spawn] [-liveness_keep_queues] [-prestart_liveness [-prestart_budget S]] [-liveness_timeout S] [-liveness_busy_deadline S] "
         "[-liveness_fail_threshold N] [-liveness_busy_grace S] [-liveness_unknown_busy_grace S] "
         "[-liveness_corroborate] [-liveness_crowded_procs N] [-liveness_probe PATH] [-liveness_chip_sweep_every N] "
         "[-perf_check_every N [-perf_mib N] [-perf_action report|unhealthy] [-perf_min_hbm_read_gbps X] "
         "[-perf_min_mfma_tflops X] [-perf_min_xcd_clock_ratio X]]] [-smi_ecc] [-smi_events] [-smi_xgmi] "
         "[-dry_run] [-trace_file PATH] [-node_view [-node_view_alias PATH]] [-topology_view] [-device_ids ID,...] "
         "[-log_format glog|json] [-v N] [-logtostderr] [-alsologtostderr] [-stderrthreshold SEV] [-log_dir DIR] "
         "[-vmodule P=N] [-log_backtrace_at FILE:N]\n";
}

bool parse_flags(int argc, char** argv, Flags* f, std::string* err, bool* help, bool* syntax) {
  *help = false;
  err->clear();
  bool syntax_scratch = false;
  if (!syntax) syntax = &syntax_scratch;
  *syntax = false;
  std::map<std::string, bool*> bools = {
      {"send_every_pulse", &f->send_every_pulse}, {"allocator_extended_search", &f->allocator_extended_search},
      {"liveness", &f->liveness}, {"liveness_keep_queues", &f->liveness_keep_queues},
      {"prestart_liveness", &f->prestart_liveness},
      {"liveness_corroborate", &f->liveness_corroborate}, {"smi_ecc", &f->smi_ecc}, {"smi_events", &f->smi_events},
      {"smi_xgmi", &f->smi_xgmi}, {"dry_run", &f->dry_run}, {"node_view", &f->node_view},
      {"topology_view", &f->topology_view}};
  std::map<std::string, int*> ints = {
      {"pulse", &f->pulse}, {"liveness_iters", &f->liveness_iters},
      {"liveness_fail_threshold", &f->liveness_fail_threshold},
      {"liveness_recover_threshold", &f->liveness_recover_threshold},
      {"liveness_idle_sweeps", &f->liveness_idle_sweeps}, {"liveness_crowded_procs", &f->liveness_crowded_procs},
      {"liveness_crowded_release_sweeps", &f->liveness_crowded_release_sweeps}, {"metrics_port", &f->metrics_port},
      {"liveness_chip_sweep_every", &f->liveness_chip_sweep_every}, {"perf_check_every", &f->perf_check_every},
      {"perf_mib", &f->perf_mib}};
  std::map<std::string, double*> floats = {
      {"liveness_timeout", &f->liveness_timeout}, {"liveness_busy_grace", &f->liveness_busy_grace},
      {"prestart_budget", &f->prestart_budget}, {"liveness_busy_deadline", &f->liveness_busy_deadline},
      {"liveness_unknown_busy_grace", &f->liveness_unknown_busy_grace}, {"grpc_watchdog", &f->grpc_watchdog_s},
      {"register_timeout", &f->register_timeout_s}, {"topology_watch", &f->topology_watch_s},
      {"reregister", &f->reregister_s},
      {"perf_min_hbm_read_gbps", &f->perf_min_hbm_read_gbps}, {"perf_min_mfma_tflops", &f->perf_min_mfma_tflops},
      {"perf_min_xcd_clock_ratio", &f->perf_min_xcd_clock_ratio}};
  std::map<std::string, std::string*> strs = {
      {"driver_type", &f->driver_type}, {"resource_naming_strategy", &f->naming},
      {"kubelet_dir", &f->kubelet_dir}, {"sysfs_root", &f->sysfs_root}, {"dev_root", &f->dev_root},
      {"exporter_socket", &f->exporter_socket}, {"liveness_mode", &f->liveness_mode},
      {"liveness_probe", &f->liveness_probe}, {"config", &f->config}, {"allocator_search", &f->allocator_search},
      {"device_list_strategy", &f->device_list_strategy}, {"cdi_spec_dir", &f->cdi_spec_dir},
      {"perf_action", &f->perf_action}, {"trace_file", &f->trace_file}, {"node_view_alias", &f->node_view_alias},
      {"device_ids", &f->device_ids}};
  if (const char* c = std::getenv("CONFIG_FILE_PATH")) f->config = c;
  static std::string ignored;
  strs["kubelet-url"] = &ignored;  // accepted for compatibility (docs promise it; registration uses the UDS)
  // the flag package's own errors (exit 2 in main)
  auto bad = [&](std::string msg) {
    *err = std::move(msg);
    *syntax = true;
    return false;
  };
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--") break;                            // terminator, consumed
    if (a.size() < 2 || a[0] != '-') break;          // first non-flag argument: parsing stops
    a = a.substr(a[1] == '-' ? 2 : 1);
    if (a.empty() || a[0] == '-' || a[0] == '=') return bad("bad flag syntax: " + std::string(argv[i]));
    std::string name = a, value;
    bool has_value = false;
    const size_t eq = a.find('=');
    if (eq != std::string::npos) {
      name = a.substr(0, eq);
      value = a.substr(eq + 1);
      has_value = true;
    }
    if (name == "h" || name == "help") return *help = true, true;
    if (!bools.count(name) && !ints.count(name) && !floats.count(name) && !strs.count(name) && !glog::is_flag(name))
      return bad("flag provided but not defined: -" + name);
    if (bools.count(name) || glog::is_bool_flag(name)) {
      if (glog::is_bool_flag(name)) {
        glog::parse_flag(name, value, has_value, &f->log, err);
        if (!err->empty()) return bad(*err);
      } else if (!has_value) {
        *bools[name] = true;                          // -flag alone sets a boolean
      } else if (!goflag::parse_bool(value, bools[name])) {
        return bad("invalid boolean value \"" + value + "\" for -" + name);
      }
      continue;
    }
    if (!has_value) {
      if (i + 1 >= argc) return bad("flag needs an argument: -" + name);
      value = argv[++i];
    }
    if (glog::parse_flag(name, value, true, &f->log, err)) {
      if (!err->empty()) return bad(*err);
    } else if (ints.count(name)) {
      if (!goflag::parse_int_flag(value, ints[name])) return bad("invalid value \"" + value + "\" for flag -" + name);
    } else if (floats.count(name)) {
      if (!goflag::parse_float(value, floats[name])) return bad("invalid value \"" + value + "\" for flag -" + name);
    } else {
      *strs[name] = value;
    }
  }
  // validateFlags (main.go:59-75)
  if (f->pulse < 0) return *err = "pulse must be a non-negative integer", false;
  if (f->metrics_port < 0 || f->metrics_port > 65535) return *err = "metrics_port must be in 0..65535", false;
  if (!f->driver_type.empty() && f->driver_type != "container" && f->driver_type != "vf-passthrough" &&
      f->driver_type != "pf-passthrough")
    return *err = "invalid driver_type provided: " + f->driver_type +
                  ", supported values are container, vf-passthrough, or pf-passthrough",
           false;
  if (f->naming != "single" && f->naming != "mixed")
    return *err = "invalid resource_naming_strategy provided: " + f->naming + ", supported values are single or mixed",
           false;
  if (f->liveness_mode != "persistent" && f->liveness_mode != "spawn")
    return *err = "invalid liveness_mode provided: " + f->liveness_mode + ", supported values are persistent or spawn",
           false;
  if (f->grpc_watchdog_s < 0) return *err = "grpc_watchdog must be >= 0", false;
  if (f->reregister_s < 0) return *err = "reregister must be >= 0", false;
  if (f->topology_watch_s < 0) return *err = "topology_watch must be >= 0", false;
  if (!cdi::parse_strategies(f->device_list_strategy, &f->lists, err)) return false;
  if (f->allocator_search != "auto" && f->allocator_search != "reference" && f->allocator_search != "extended")
    return *err = "invalid allocator_search provided: " + f->allocator_search +
                  ", supported values are auto, reference, extended",
           false;
  if (f->allocator_extended_search) f->allocator_search = "extended";
  if (f->liveness && f->pulse == 0) return *err = "-liveness needs -pulse > 0 (the probe runs once per pulse)", false;
  if (f->prestart_liveness && !f->liveness)
    return *err = "prestart_liveness needs -liveness (the check runs in the probe server)", false;
  if (!(f->prestart_budget > 0 && f->prestart_budget < 30))
    return *err = "prestart_budget must be in (0, 30) seconds (kubelet's PreStartContainer deadline is 30 s)", false;
  if (!(f->liveness_busy_deadline > 0)) return *err = "liveness_busy_deadline must be > 0", false;
  if (f->perf_action != "report" && f->perf_action != "unhealthy")
    return *err = "invalid perf_action provided: " + f->perf_action + ", supported values are report or unhealthy",
           false;
  if (f->perf_check_every > 0 && !f->liveness)
    return *err = "perf_check_every needs -liveness (the throughput check runs in the probe server)", false;
  return true;
}

}  // namespace mi355x::daemon
