// Command line of mi355x-device-plugin: the reference's flags
// (cmd/k8s-device-plugin/main.go:50-75), glog's (mi355x/glog.h) and this
// build's health / allocation / observability flags.
#pragma once

#include <string>

#include "mi355x/cdi.h"
#include "mi355x/glog.h"
#include "mi355x/views.h"

namespace mi355x::daemon {

struct Flags {
  int pulse = 0;
  std::string driver_type;
  std::string naming = "single";
  std::string kubelet_dir = "/var/lib/kubelet/device-plugins";
  std::string sysfs_root = "/sys";
  std::string dev_root = "/dev";
  std::string exporter_socket = "/var/lib/amd-metrics-exporter/amdgpu_device_metrics_exporter_grpc.socket";
  bool send_every_pulse = false;
  double register_timeout_s = 10.0;
  double grpc_watchdog_s = 10.0;
  // kubelet ended every ListAndWatch stream of a registered resource while its
  // socket stayed the same: register again after this long (0 = never)
  double reregister_s = 2.0;
  bool allocator_extended_search = false;  // forces "extended"
  std::string allocator_search = "auto";   // auto | reference | extended
  // health (same names and defaults as the Python CLI)
  bool liveness = false;
  std::string liveness_mode = "persistent";
  bool liveness_keep_queues = true;
  // PreStartContainer probes the container's GPUs (through the probe server) and
  // fails the start on a definite fault; needs -liveness
  bool prestart_liveness = false;
  // the check's whole budget, kubelet's 30 s PreStartContainer deadline in
  // mind (v1beta1/constants.go:44): what it cannot settle in time is let through
  double prestart_budget = 5.0;
  double liveness_timeout = 10.0;
  // probe deadline on a GPU other processes have queues on (kept queues): a
  // dispatch queued behind a tenant's kernel is inconclusive however long it waits
  double liveness_busy_deadline = 0.05;
  int liveness_iters = 4;
  int liveness_fail_threshold = 2;
  int liveness_recover_threshold = 1;
  double liveness_busy_grace = 300.0;
  double liveness_unknown_busy_grace = 30.0;
  bool liveness_corroborate = true;
  int liveness_idle_sweeps = 2;
  int liveness_crowded_procs = 7;
  int liveness_crowded_release_sweeps = 5;
  std::string liveness_probe;  // default: mi355x-liveness-probe next to this binary
  bool smi_ecc = false;
  bool smi_events = false;
  bool smi_xgmi = false;  // xGMI link state re-weights preferred allocation
  int liveness_chip_sweep_every = 0;
  int perf_check_every = 0;
  int perf_mib = 4096;
  std::string perf_action = "report";
  double perf_min_hbm_read_gbps = 3000.0;
  double perf_min_mfma_tflops = 700.0;
  double perf_min_xcd_clock_ratio = 0.6;
  std::string config;  // YAML config file (gpu.device_count), default $CONFIG_FILE_PATH
  bool dry_run = false;  // print the node report (what kubelet would be told) and exit
  std::string trace_file;  // Chrome-trace spans, written at shutdown
  bool node_view = false;      // experimental: NUMA-node sysfs view without per-CPU cache descriptors
  bool topology_view = false;  // experimental: per-allocation filtered kfd topology
  std::string node_view_alias = views::kNodeAlias;  // where the real node directory is mounted in the container
  std::string device_ids;  // advertise only these device IDs (comma-separated; default: every discovered one)
  int metrics_port = 0;  // Prometheus /metrics (0 = off)
  double topology_watch_s = 5.0;  // re-discovery check period (partition switches); 0 = off
  std::string device_list_strategy = "device-specs";
  std::string cdi_spec_dir = "/var/run/cdi";
  cdi::Strategies lists;  // parsed -device_list_strategy
  glog::Options log;
};

// Go flag syntax (-name=value, -name value, --name, bare booleans; parsing
// stops at the first non-flag argument or after "--") plus validateFlags
// (main.go:59-75). false and *err on a bad command line, with *syntax set when
// the flag package itself would have refused it (an undefined flag, a missing
// or unparsable value: Go prints the error and the usage and exits 2) rather
// than validateFlags (logged, exit 1). -h / -help set *help and return true.
bool parse_flags(int argc, char** argv, Flags* f, std::string* err, bool* help, bool* syntax = nullptr);

// the flag synopsis printed by -h (after the version banner)
std::string usage(const std::string& argv0);

}  // namespace mi355x::daemon
