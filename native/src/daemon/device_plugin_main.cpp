// mi355x-device-plugin: the kubelet device plugin as one native process — the
// primary entrypoint of this framework (docs/architecture.md).
//
// The reference ships its plugin as a single compiled binary
// (cmd/k8s-device-plugin/main.go). This is the same thing built from the
// framework's C++ core, with no interpreter in the process:
//
//   flags          -pulse, -driver_type, -resource_naming_strategy (main.go:50-75),
//                  glog's -v / -logtostderr / -alsologtostderr / -stderrthreshold /
//                  -log_dir / -vmodule / -log_backtrace_at (mi355x/glog.h),
//                  -kubelet_dir / -sysfs_root / -dev_root / -exporter_socket /
//                  -send_every_pulse, the health flags of the Python CLI
//                  (-liveness*, -smi_ecc, -smi_events), -allocator_extended_search,
//                  -grpc_watchdog, -metrics_port, -topology_watch
//   discovery      discover_gpus over the kfd topology (gpu_discovery.cpp)
//   resources      single -> "gpu"; mixed -> "<compute>_<memory>"; heterogeneous
//                  partitions with single is an error (amdgpu.go:68-88,122-162)
//   per resource   the native gRPC server on <kubelet_dir>/amd.com_<resource>
//                  with the DevicePlugin service: hive-aware
//                  GetPreferredAllocation (HiveAllocator), Allocate = /dev/kfd +
//                  card + renderD per device (amdgpu.go:255-319), ListAndWatch
//   registration   Register on kubelet.sock through the native client, on a
//                  worker thread; again whenever kubelet.sock is replaced
//                  (inotify on the plugin directory, as the vendored dpm does with
//                  fsnotify; a 5 s stat poll as a safety net)
//   health         every -pulse on a worker thread (health_engine.h): kfd node,
//                  metrics exporter per BDF, the gfx950 MFMA liveness probe server
//                  with hysteresis, busy grace, identity check and crowded
//                  step-off, amd-smi ECC and reset events; the list is pushed when
//                  a verdict changes (or every pulse with -send_every_pulse)
//   watchdog       Register acknowledged but no ListAndWatch within
//                  -grpc_watchdog s, or HTTP/2 protocol errors on the plugin
//                  socket: exit 3 so the DaemonSet restarts the plugin instead of
//                  leaving it registered and invisible
//   topology       -topology_watch: a partition switch is re-discovered and
//                  re-advertised (resources stop, change or appear)
//   metrics        -metrics_port: Prometheus /metrics on a thread of its own,
//                  the Python CLI's series (mi355x/metrics.h)
//   signals        SIGTERM / SIGINT / SIGQUIT stop the servers, the probe server
//                  and the workers, and remove the sockets
//   passthrough    -driver_type vf-passthrough / pf-passthrough (amdgpu_sriov.go,
//                  amdgpu_pf.go): one device per IOMMU group, Allocate =
//                  /dev/vfio/<group> + /dev/vfio/vfio (mrw) and
//                  PCI_RESOURCE_AMD_COM_<RES> = the BDFs of every requested group;
//                  health = driver present (+ exporter PF verdicts for VFs);
//                  without -driver_type: container -> VF -> PF (main.go:106-115)
//
// The control loop never blocks on a peer: Register and every health source
// run on worker threads with their own deadlines, and results come back
// through a pipe the loop polls.
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/inotify.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "mi355x/allocator.h"
#include "mi355x/cdi.h"
#include "mi355x/constants.h"
#include "mi355x/dir_watch.h"
#include "mi355x/dp_service.h"
#include "mi355x/glog.h"
#include "mi355x/gpu_discovery.h"
#include "mi355x/grpc_server.h"
#include "mi355x/health_engine.h"
#include "mi355x/kfd_topology.h"
#include "mi355x/metrics.h"
#include "mi355x/trace.h"
#include "mi355x/views.h"
#include "mi355x/pci_scan.h"
#include "mi355x/sysfs.h"
#include "../kube/json.h"
#include "../kube/yaml.h"

namespace {

using namespace mi355x;
namespace pb = mi355x::rpc::pb;
using Clock = std::chrono::steady_clock;

// ---- flags ------------------------------------------------------------------
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
  bool allocator_extended_search = false;  // forces "extended"
  std::string allocator_search = "auto";   // auto | reference | extended
  // health (same names and defaults as the Python CLI)
  bool liveness = false;
  std::string liveness_mode = "persistent";
  bool liveness_keep_queues = true;
  double liveness_timeout = 10.0;
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

// Flags only the Python CLI implements (k8s-device-plugin): refused with a pointer to it.
const std::set<std::string> kPythonOnly = {"grpc_server"};

bool parse_bool(const std::string& v, bool* out) {
  if (v.empty() || v == "1" || v == "true" || v == "True" || v == "TRUE" || v == "t" || v == "T") return *out = true, true;
  if (v == "0" || v == "false" || v == "False" || v == "FALSE" || v == "f" || v == "F") return *out = false, true;
  return false;
}

// Go flag syntax: -name=value, -name value, --name, bare booleans.
bool parse_flags(int argc, char** argv, Flags* f, std::string* err) {
  std::map<std::string, bool*> bools = {
      {"send_every_pulse", &f->send_every_pulse}, {"allocator_extended_search", &f->allocator_extended_search},
      {"liveness", &f->liveness}, {"liveness_keep_queues", &f->liveness_keep_queues},
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
      {"liveness_unknown_busy_grace", &f->liveness_unknown_busy_grace}, {"grpc_watchdog", &f->grpc_watchdog_s},
      {"register_timeout", &f->register_timeout_s}, {"topology_watch", &f->topology_watch_s},
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
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a.size() < 2 || a[0] != '-') return *err = "unexpected argument " + a, false;
    a = a.substr(a[1] == '-' ? 2 : 1);
    std::string name = a, value;
    bool has_value = false;
    const size_t eq = a.find('=');
    if (eq != std::string::npos) {
      name = a.substr(0, eq);
      value = a.substr(eq + 1);
      has_value = true;
    }
    if (name == "h" || name == "help") {
      std::printf(
          "usage: %s [-pulse N] [-driver_type container|vf-passthrough|pf-passthrough] "
          "[-resource_naming_strategy single|mixed] [-kubelet_dir DIR] [-sysfs_root DIR] [-dev_root DIR] "
          "[-exporter_socket PATH] [-send_every_pulse] [-allocator_search auto|reference|extended] "
          "[-allocator_extended_search] [-grpc_watchdog S] [-config FILE] [-metrics_port N] [-topology_watch S] "
          "[-device_list_strategy device-specs|cdi-cri|cdi-annotations[,...]] [-cdi_spec_dir DIR] "
          "[-liveness [-liveness_mode persistent|spawn] [-liveness_keep_queues] [-liveness_timeout S] "
          "[-liveness_fail_threshold N] [-liveness_busy_grace S] [-liveness_unknown_busy_grace S] "
          "[-liveness_corroborate] [-liveness_crowded_procs N] [-liveness_probe PATH] [-liveness_chip_sweep_every N] "
          "[-perf_check_every N [-perf_mib N] [-perf_action report|unhealthy] [-perf_min_hbm_read_gbps X] "
          "[-perf_min_mfma_tflops X] [-perf_min_xcd_clock_ratio X]]] [-smi_ecc] [-smi_events] [-smi_xgmi] "
          "[-dry_run] [-trace_file PATH] [-node_view [-node_view_alias PATH]] [-topology_view] [-device_ids ID,...] [-log_format glog|json] [-v N] [-logtostderr] [-alsologtostderr] [-stderrthreshold SEV] [-log_dir DIR] [-vmodule P=N] "
          "[-log_backtrace_at FILE:N]\n",
          argv[0]);
      std::exit(0);
    }
    if (bools.count(name) || glog::is_bool_flag(name)) {
      if (glog::is_bool_flag(name)) {
        glog::parse_flag(name, value, has_value, &f->log, err);
        if (!err->empty()) return false;
      } else if (!parse_bool(has_value ? value : "", bools[name])) {
        return *err = "invalid boolean value \"" + value + "\" for -" + name, false;
      }
      continue;
    }
    if (kPythonOnly.count(name))
      return *err = "-" + name + " is implemented by the Python entrypoint (k8s-device-plugin), not by the native "
                    "daemon",
             false;
    if (!has_value) {
      if (i + 1 >= argc) return *err = "flag needs an argument: -" + name, false;
      value = argv[++i];
    }
    if (glog::parse_flag(name, value, true, &f->log, err)) {
      if (!err->empty()) return false;
    } else if (ints.count(name)) {
      char* end = nullptr;
      const long v = std::strtol(value.c_str(), &end, 10);
      if (value.empty() || *end) return *err = "invalid value \"" + value + "\" for flag -" + name, false;
      *ints[name] = static_cast<int>(v);
    } else if (floats.count(name)) {
      char* end = nullptr;
      const double v = std::strtod(value.c_str(), &end);
      if (value.empty() || *end) return *err = "invalid value \"" + value + "\" for flag -" + name, false;
      *floats[name] = v;
    } else if (strs.count(name)) {
      *strs[name] = value;
    } else {
      return *err = "flag provided but not defined: -" + name, false;
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
  if (f->topology_watch_s < 0) return *err = "topology_watch must be >= 0", false;
  if (!cdi::parse_strategies(f->device_list_strategy, &f->lists, err)) return false;
  if (f->allocator_search != "auto" && f->allocator_search != "reference" && f->allocator_search != "extended")
    return *err = "invalid allocator_search provided: " + f->allocator_search +
                  ", supported values are auto, reference, extended",
           false;
  if (f->allocator_extended_search) f->allocator_search = "extended";
  if (f->liveness && f->pulse == 0) return *err = "-liveness needs -pulse > 0 (the probe runs once per pulse)", false;
  if (f->perf_action != "report" && f->perf_action != "unhealthy")
    return *err = "invalid perf_action provided: " + f->perf_action + ", supported values are report or unhealthy",
           false;
  if (f->perf_check_every > 0 && !f->liveness)
    return *err = "perf_check_every needs -liveness (the throughput check runs in the probe server)", false;
  return true;
}

// ---- protobuf messages (v1beta1 field numbers, api.proto) -------------------
// DeviceSpec{container_path=1, host_path=2, permissions=3}
std::string device_spec(const std::string& path, const char* perms = "rw") {
  std::string s;
  pb::put_bytes(&s, 1, path);
  pb::put_bytes(&s, 2, path);
  pb::put_bytes(&s, 3, perms);
  return s;
}

std::string device_msg(const GpuDevice& d, bool healthy) {  // Device{ID=1, health=2, topology=3{nodes=1{ID=1}}}
  std::string m;
  pb::put_bytes(&m, 1, d.id);
  pb::put_bytes(&m, 2, healthy ? "Healthy" : "Unhealthy");
  if (d.numa_node >= 0) {
    std::string node, topo;
    pb::put_tag(&node, 1, 0);
    pb::put_varint(&node, static_cast<uint64_t>(d.numa_node));
    pb::put_bytes(&topo, 1, node);
    pb::put_bytes(&m, 3, topo);
  }
  return m;
}

// ---- one advertised resource ------------------------------------------------
enum class Driver { Container, Vf, Pf };

struct Resource {
  std::string name;  // "gpu", "cpx_nps1", "gpu_vf", ...
  Driver driver = Driver::Container;
  std::vector<GpuDevice> devices;          // container driver
  std::vector<std::string> group_ids;      // passthrough: IOMMU groups, numeric order
  IommuMap groups;                         // group -> PCI functions
  std::string socket;  // <kubelet_dir>/amd.com_<name>
  std::string options;
  rpc::AllocateTemplate tmpl;
  bool gone = false;  // removed by a topology change: no server, no devices (the slot keeps indices stable)
  std::unique_ptr<rpc::GrpcServer> server;
  std::unique_ptr<rpc::DevicePluginService> service;
  std::shared_ptr<const HiveAllocator> allocator;
  std::map<std::string, bool> health;  // device id -> healthy
  std::string list;                    // serialized ListAndWatchResponse
  // registration (worker thread) and the transport watchdog
  bool registered = false;
  bool register_inflight = false;
  uint64_t server_gen = 0;             // bumped on every (re)start of the server
  Clock::time_point next_register{};
  int retry_ms = 100;  // kubelet.sock appears (bind) just before kubelet listens: retry soon, then back off to 3 s
  Clock::time_point registered_at{};
  uint64_t streams_at_register = 0, perr_at_register = 0;
  bool list_seen = false;
};

std::string list_bytes(const Resource& r) {
  std::string out;
  for (const auto& g : r.group_ids) {  // passthrough: Device{ID=group, health}, no topology
    auto it = r.health.find(g);
    std::string m;
    pb::put_bytes(&m, 1, g);
    pb::put_bytes(&m, 2, it == r.health.end() || it->second ? "Healthy" : "Unhealthy");
    pb::put_bytes(&out, 1, m);
  }
  for (const auto& d : r.devices) {
    auto it = r.health.find(d.id);
    pb::put_bytes(&out, 1, device_msg(d, it == r.health.end() || it->second));
  }
  return out;
}

std::string group_key(const GpuDevice& d) { return !d.unique_id.empty() ? d.unique_id : "bdf:" + d.bdf; }

// BestEffortPolicy.init over `devs`; `degraded`: xGMI pairs (group keys) scored as the worst link
std::shared_ptr<const HiveAllocator> build_allocator(const std::vector<GpuDevice>& devs, const KfdTopology& topo,
                                                     const std::string& search,
                                                     const std::vector<std::pair<std::string, std::string>>& degraded,
                                                     std::string* err) {
  std::vector<AllocDevice> ad;
  for (const auto& d : devs) {
    AllocDevice a;
    a.id = d.id;
    a.node_id = d.node_id;
    a.numa_node = d.numa_node;
    a.unique_id = group_key(d);
    a.hive_id = d.hive_id;
    a.inferred_links = d.node_id < 0 && d.identity == "sysfs";
    ad.push_back(a);
  }
  AllocatorOptions opt;
  opt.extended_search = search == "extended";
  opt.extended_search_auto = search == "auto";  // extended on partitioned nodes
  opt.degraded_links = degraded;
  auto alloc = std::make_shared<HiveAllocator>();
  *err = alloc->init(ad, topo, opt);
  return alloc;
}

// the opt-in container start-up views (mi355x/views.h)
struct ViewCtx {
  std::shared_ptr<views::NodeView> node;
  std::shared_ptr<views::TopologyViews> topo;
};

// Mount{container_path=1, host_path=2, read_only=3}, as ContainerAllocateResponse.mounts (2)
std::string mount_field(const std::string& host, const std::string& ctr) {
  std::string m, out;
  pb::put_bytes(&m, 1, ctr);
  pb::put_bytes(&m, 2, host);
  pb::put_bool(&m, 3, true);
  pb::put_bytes(&out, 2, m);
  return out;
}

void prepare(Resource& r, const KfdTopology& topo, const std::set<std::string>& unresolved,
             const std::string& search, const cdi::Strategies& lists, const ViewCtx& vc) {
  // allocator (BestEffortPolicy.init); on failure kubelet allocates by itself
  bool alloc_ok = true;
  for (const auto& d : r.devices)
    if (unresolved.count(d.id)) alloc_ok = false;
  if (!alloc_ok) {
    MI_LOG(kError, "allocator disabled for plugin %s: no physical-GPU identity for some devices. Falling back to "
                   "kubelet default allocation.", r.name.c_str());
  } else {
    std::string err;
    auto alloc = build_allocator(r.devices, topo, search, {}, &err);
    if (!err.empty()) {
      MI_LOG(kError, "allocator init failed for plugin %s. Falling back to kubelet default allocation. Error %s",
             r.name.c_str(), err.c_str());
      alloc_ok = false;
    } else {
      r.allocator = alloc;
    }
  }
  r.options.clear();
  if (alloc_ok) pb::put_bool(&r.options, 2, true);  // get_preferred_allocation_available
  // ContainerAllocateResponse{devices=3 (DeviceSpec), annotations=4, cdi_devices=5 (CDIDevice{name=1})}
  rpc::AllocateTemplate t;
  t.resource = r.name;
  if (lists.specs) pb::put_bytes(&t.container_prefix, 3, device_spec("/dev/kfd"));
  if (lists.annotations) t.annotation_key = cdi::annotation_key(r.name);
  for (const auto& d : r.devices) {
    std::string car;
    if (lists.specs) {
      if (d.card >= 0) pb::put_bytes(&car, 3, device_spec("/dev/dri/card" + std::to_string(d.card)));
      if (d.render_minor >= 0)
        pb::put_bytes(&car, 3, device_spec("/dev/dri/renderD" + std::to_string(d.render_minor)));
    }
    if (lists.cri) {
      std::string dev;
      pb::put_bytes(&dev, 1, cdi::qualified_name(r.name, d.id));
      pb::put_bytes(&car, 5, dev);
    }
    if (lists.annotations) t.annotation_names[d.id] = cdi::qualified_name(r.name, d.id);
    t.per_device[d.id] = car;
  }
  if (vc.topo) {  // one filtered topology per distinct allocated node set, built on first use
    std::map<std::string, int> node_of;
    for (const auto& d : r.devices) node_of[d.id] = d.node_id;
    t.container_extra = [views = vc.topo, node_of](const std::vector<std::string>& ids) -> std::string {
      std::vector<int> nodes;
      for (const auto& id : ids) {
        auto it = node_of.find(id);
        if (it == node_of.end() || it->second < 0) return "";
        nodes.push_back(it->second);
      }
      std::string err;
      const std::string path = views->get(nodes, &err);
      if (path.empty()) {  // never fail an admission over an optimisation
        MI_LOG(kWarning, "topology view unavailable: %s", err.c_str());
        return "";
      }
      return mount_field(path, views::kKfdTopologyContainerPath);
    };
  }
  if (vc.node)
    for (const auto& [host, ctr] : vc.node->mounts()) t.container_nonempty += mount_field(host, ctr);
  r.service = std::make_unique<rpc::DevicePluginService>();
  r.service->set_fallback([name = r.name](const std::string& method, const std::string&) {
    // everything the native daemon serves has prepared state; a method without it is not implemented
    return rpc::Reply{rpc::kUnimplemented, "not served by the native daemon: " + method + " (" + name + ")", ""};
  });
  r.service->set_options(r.options);
  if (r.allocator) r.service->set_allocator(r.allocator);
  r.service->set_allocate_template(t);
  r.tmpl = t;
  r.list = list_bytes(r);
  r.service->set_device_list(r.list);
}

// passthrough resources: no preferred allocation, vfio Allocate template
void prepare_passthrough(Resource& r) {
  r.options.clear();
  rpc::AllocateTemplate t;
  t.resource = r.name;
  std::string up = r.name;
  for (auto& c : up) c = static_cast<char>(std::toupper(static_cast<unsigned char>(c)));
  t.env_key = "PCI_RESOURCE_AMD_COM_" + up;
  pb::put_bytes(&t.container_nonempty, 3, device_spec("/dev/vfio/vfio", "mrw"));
  for (const auto& g : r.group_ids) {
    std::string car;
    pb::put_bytes(&car, 3, device_spec("/dev/vfio/" + g, "mrw"));
    t.per_device[g] = car;
    std::string bdfs;
    for (const auto& fn : r.groups.at(g)) {
      if (!bdfs.empty()) bdfs += ",";
      bdfs += r.driver == Driver::Vf ? fn.vf : fn.pf;
    }
    t.env_values[g] = bdfs;
  }
  r.service = std::make_unique<rpc::DevicePluginService>();
  r.service->set_fallback([name = r.name](const std::string& method, const std::string&) {
    // kubelet only asks when get_preferred_allocation_available is set; answer empty as the reference does
    if (method == "GetPreferredAllocation") return rpc::Reply{rpc::kOk, "", ""};
    return rpc::Reply{rpc::kUnimplemented, "not served by the native daemon: " + method + " (" + name + ")", ""};
  });
  r.service->set_options(r.options);
  r.service->set_allocate_template(t);
  r.list = list_bytes(r);
  r.service->set_device_list(r.list);
}

bool start_server(Resource& r) {
  r.server = std::make_unique<rpc::GrpcServer>();
  r.service->attach(*r.server);
  const std::string err = r.server->start(r.socket);
  if (!err.empty()) {
    MI_LOG(kError, "%s: could not serve on %s: %s", r.name.c_str(), r.socket.c_str(), err.c_str());
    r.server.reset();
    return false;
  }
  static uint64_t seq = 0;
  r.server_gen = ++seq;  // unique across slots: a Register answer names the server it was for
  MI_LOG(kInfo, "%s: serving on %s", r.name.c_str(), r.socket.c_str());
  return true;
}

void stop_server(Resource& r) {
  if (r.server) {
    r.server->stop(0.5);
    r.server.reset();
    ::unlink(r.socket.c_str());
  }
  r.registered = false;
  r.list_seen = false;
}

// ---- worker threads -----------------------------------------------------------
// Jobs run on their own threads; completions are queued here and the control
// loop is woken through a pipe.
struct Completion {
  enum Kind { kRegister, kSweep } kind;
  size_t resource = 0;
  uint64_t gen = 0;
  bool ok = false;
  std::string message;
  std::map<std::string, bool> health;  // kSweep: device id -> healthy (every resource's devices)
  double sweep_ms = 0;
  uint64_t server_gen = 0;              // kRegister: the server the Register was for
};

class Workers {
 public:
  Workers() {
    if (::pipe2(wake_, O_CLOEXEC | O_NONBLOCK) != 0) wake_[0] = wake_[1] = -1;
  }
  ~Workers() { close(); }
  int wake_fd() const { return wake_[0]; }
  void run(std::function<Completion()> job) {
    auto done = std::make_shared<std::atomic<bool>>(false);
    std::lock_guard<std::mutex> lk(mu_);
    threads_.emplace_back(std::thread([this, done, job = std::move(job)] {
                            Completion c = job();
                            {
                              std::lock_guard<std::mutex> lk2(mu_);
                              done_.push_back(std::move(c));
                            }
                            done->store(true);
                            const char b = 1;
                            if (::write(wake_[1], &b, 1) < 0) {
                            }
                          }),
                          done);
  }
  std::vector<Completion> take() {
    char buf[256];
    while (::read(wake_[0], buf, sizeof(buf)) > 0) {
    }
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<Completion> out;
    out.swap(done_);
    return out;
  }
  // joins the threads that have finished
  void reap() {
    std::vector<std::thread> finished;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto it = threads_.begin(); it != threads_.end();) {
        if (it->second->load()) {
          finished.push_back(std::move(it->first));
          it = threads_.erase(it);
        } else {
          ++it;
        }
      }
    }
    for (auto& t : finished) t.join();
  }
  void join_all() {
    std::vector<std::pair<std::thread, std::shared_ptr<std::atomic<bool>>>> ts;
    {
      std::lock_guard<std::mutex> lk(mu_);
      ts.swap(threads_);
    }
    for (auto& t : ts)
      if (t.first.joinable()) t.first.join();
  }
  void close() {
    join_all();
    if (wake_[0] >= 0) ::close(wake_[0]);
    if (wake_[1] >= 0) ::close(wake_[1]);
    wake_[0] = wake_[1] = -1;
  }

 private:
  std::mutex mu_;
  std::vector<std::pair<std::thread, std::shared_ptr<std::atomic<bool>>>> threads_;
  std::vector<Completion> done_;
  int wake_[2] = {-1, -1};
};

// Register{version=1, endpoint=2, resource_name=3, options=4} on kubelet.sock (blocking; worker thread)
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

volatile sig_atomic_t g_stop = 0;
int g_sig_pipe[2] = {-1, -1};

void on_signal(int) {
  g_stop = 1;
  const char b = 1;
  if (g_sig_pipe[1] >= 0 && ::write(g_sig_pipe[1], &b, 1) < 0) {
  }
}

// identity of kubelet.sock: a restart replaces the file (new inode / ctime)
struct SockId {
  bool present = false;
  dev_t dev = 0;
  ino_t ino = 0;
  int64_t ctime_ns = 0;
  bool operator==(const SockId& o) const {
    return present == o.present && dev == o.dev && ino == o.ino && ctime_ns == o.ctime_ns;
  }
  bool operator!=(const SockId& o) const { return !(*this == o); }
};

SockId sock_id(const std::string& path) {
  SockId s;
  struct stat st {};
  if (::stat(path.c_str(), &st) != 0) return s;
  s.present = true;
  s.dev = st.st_dev;
  s.ino = st.st_ino;
  s.ctime_ns = static_cast<int64_t>(st.st_ctim.tv_sec) * 1000000000 + st.st_ctim.tv_nsec;
  return s;
}

// AMD_GPU_DEVICE_COUNT, else gpu.device_count of the -config file: advertise
// the devices of the first N physical GPUs (documented by the reference,
// docs/user-guide/configuration.md:11,45-91, never implemented there; the
// Python CLI's topology.device_count_limit_from_env)
int device_count_limit(const std::string& config, std::string* err) {
  if (const char* e = std::getenv("AMD_GPU_DEVICE_COUNT"); e && *e) {
    char* end = nullptr;
    const long n = std::strtol(e, &end, 10);
    if (!*end && n >= 0) return static_cast<int>(n);
  }
  if (config.empty()) return -1;
  auto text = read_file(config);
  if (!text) return *err = "config file " + config + " is unreadable", -1;
  std::string perr;
  auto doc = yaml::parse(*text, &perr);
  if (!doc) return *err = "config file " + config + ": " + perr, -1;
  const json::Value* gpu = doc->get("gpu");
  const json::Value* dc = gpu ? gpu->get("device_count") : nullptr;
  if (!dc || dc->kind == json::Value::Null) return -1;
  char* end = nullptr;
  const long n = std::strtol(dc->s.c_str(), &end, 10);
  if (dc->s.empty() || *end || n < 0) return *err = "config file " + config + ": bad gpu.device_count", -1;
  return static_cast<int>(n);
}

std::vector<GpuDevice> limit_physical(const std::vector<GpuDevice>& devs, int limit) {
  if (limit < 0) return devs;
  std::vector<std::string> seen;
  for (const auto& d : devs) {
    const std::string k = !d.unique_id.empty() ? d.unique_id : d.bdf;
    if (std::find(seen.begin(), seen.end(), k) == seen.end()) seen.push_back(k);
  }
  if (seen.size() > static_cast<size_t>(limit)) seen.resize(static_cast<size_t>(limit));
  std::vector<GpuDevice> out;
  for (const auto& d : devs)
    if (std::find(seen.begin(), seen.end(), !d.unique_id.empty() ? d.unique_id : d.bdf) != seen.end()) out.push_back(d);
  return out;
}

std::string self_dir() {
  char buf[4096];
  const ssize_t n = ::readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return ".";
  buf[n] = 0;
  std::string p = buf;
  return p.substr(0, p.rfind('/'));
}

// ---- -dry_run: the node report (cli/device_plugin.py dry_run_report) ----------
json::Value jnum(double v) {
  json::Value x;
  x.kind = json::Value::Number;
  char b[64];
  if (v == static_cast<double>(static_cast<long long>(v)) && std::fabs(v) < 1e15)
    std::snprintf(b, sizeof(b), "%lld", static_cast<long long>(v));
  else
    std::snprintf(b, sizeof(b), "%.17g", v);
  x.s = b;
  return x;
}
json::Value jbool(bool v) {
  json::Value x;
  x.kind = json::Value::Bool;
  x.b = v;
  return x;
}
json::Value jarr() {
  json::Value x;
  x.kind = json::Value::Array;
  return x;
}
json::Value jnull() { return json::Value{}; }

// xGMI fabric of an allocated set (parallel/fabric.py Fabric.report): whether it
// is one hive, and the ring all-reduce bound its links imply (GB/s)
struct FabricReport {
  bool one_hive = false;
  bool has_bound = false;
  double bound_gbs = 0;
};

int model_xgmi_link_mbps(int device_id, int gfx) {  // models/gpu.py xgmi_link_mbps
  switch (device_id) {
    case 0x75a3: case 0x75b3: return 76000;  // MI355X (measured)
    case 0x74a1: case 0x74a2: return 64000;  // MI300X / MI308X
    case 0x740f: return 50000;               // MI210
  }
  switch (gfx) {
    case 90500: return 76000;
    case 90402: return 64000;
    case 90010: return 50000;
  }
  return 0;
}

FabricReport fabric_report(const std::vector<const GpuDevice*>& devs, const KfdTopology& topo) {
  std::map<std::pair<int, int>, std::pair<int, int64_t>> links;  // io_links win over p2p_links
  for (const KfdNode* n : topo.gpu_nodes()) {
    for (const auto& l : n->p2p_links) links[{l.node_from, l.node_to}] = {l.type, l.max_bandwidth};
    for (const auto& l : n->io_links) links[{l.node_from, l.node_to}] = {l.type, l.max_bandwidth};
  }
  auto link = [&](const GpuDevice* a, const GpuDevice* b) -> std::pair<std::string, int64_t> {
    if (!a->unique_id.empty() && a->unique_id == b->unique_id) return {"same_gpu", 0};
    auto it = links.find({a->node_id, b->node_id});
    if (it == links.end()) it = links.find({b->node_id, a->node_id});
    if (it == links.end()) return {"unknown", 0};
    int64_t bw = it->second.second;
    if (it->second.first == kLinkXgmi) {
      if (bw <= 0) bw = model_xgmi_link_mbps(a->pci_device_id, a->gfx_target_version);
      return {"xgmi", bw};
    }
    if (it->second.first == kLinkPcie) return {"pcie", bw};
    return {"unknown", bw};
  };
  FabricReport rep;
  std::vector<const GpuDevice*> reps;
  std::set<std::string> seen;
  std::set<uint64_t> hives;
  for (const GpuDevice* d : devs) {
    hives.insert(d->hive_id);
    if (seen.insert(!d->unique_id.empty() ? d->unique_id : d->bdf).second) reps.push_back(d);
  }
  rep.one_hive = hives.size() == 1 && !hives.count(0);
  if (reps.size() <= 1) return rep;
  int64_t egress_min = -1;
  std::vector<std::pair<std::string, int64_t>> slow;
  for (const GpuDevice* a : reps) {
    int64_t eg = 0;
    for (const GpuDevice* b : reps) {
      if (a == b) continue;
      const auto [cls, bw] = link(a, b);
      if (cls == "xgmi") eg += bw;
      else slow.emplace_back(cls, bw);
    }
    egress_min = egress_min < 0 ? eg : std::min(egress_min, eg);
  }
  if (slow.empty() && egress_min > 0) {
    rep.has_bound = true;
    rep.bound_gbs = static_cast<double>(egress_min) / 1000.0;
  } else if (std::any_of(slow.begin(), slow.end(), [](const auto& x) { return x.first == "unknown"; })) {
    // no bound without kfd links
  } else if (!slow.empty()) {
    int64_t mn = -1;
    for (const auto& [c, bw] : slow)
      if (bw > 0) mn = mn < 0 ? bw : std::min(mn, bw);
    if (mn > 0) {
      rep.has_bound = true;
      rep.bound_gbs = static_cast<double>(mn) / 1000.0;
    }
  }
  return rep;
}

}  // namespace

int main(int argc, char** argv) {
  Flags f;
  std::string err;
  if (!parse_flags(argc, argv, &f, &err)) {
    glog::init(f.log);
    MI_LOG(kError, "%s", err.c_str());
    return 1;
  }
  if (f.log.program.empty()) f.log.program = "k8s-device-plugin";
  err = glog::init(f.log);
  if (!err.empty()) {
    glog::Options o;
    glog::init(o);
    MI_LOG(kError, "%s", err.c_str());
    return 1;
  }
  MI_LOG(kInfo, "AMD GPU device plugin for Kubernetes (MI355X-native, native daemon)");
  trace::global().configure(f.trace_file);
  if (::pipe2(g_sig_pipe, O_CLOEXEC | O_NONBLOCK) != 0) return 1;
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGQUIT, &sa, nullptr);
  signal(SIGPIPE, SIG_IGN);

  const int dev_limit = device_count_limit(f.config, &err);
  if (!err.empty()) {
    MI_LOG(kError, "%s", err.c_str());
    return 1;
  }
  std::vector<Resource> resources;
  KfdTopology topo;
  std::vector<GpuDevice> container_devices;  // every advertised container-mode device (health engine)
  std::vector<std::string> discovery_warnings;
  ViewCtx view_ctx;
  if (f.topology_view)
    view_ctx.topo = std::make_shared<views::TopologyViews>(path_join(f.kubelet_dir, "mi355x-topology"),
                                                           path_join(f.sysfs_root, "class/kfd/kfd/topology"));
  if (f.node_view) {  // built at start-up, not inside the first Allocate
    auto nv = std::make_shared<views::NodeView>(path_join(f.kubelet_dir, "mi355x-node"), f.sysfs_root,
                                                f.node_view_alias);
    if (const std::string e = nv->build(); !e.empty()) {
      MI_LOG(kWarning, "node view unavailable: %s", e.c_str());
    } else {
      MI_LOG(kInfo, "node view: %d links, %d per-CPU cache directories left out", nv->links, nv->hidden);
      view_ctx.node = nv;
    }
  }
  bool impl_ok = true;  // a driver initialised (auto mode: container -> VF -> PF)
  Driver driver = Driver::Container;
  // one driver's resources; "" on success (an empty list = no devices), else the init error
  auto init_container = [&](std::vector<Resource>* out) -> std::string {
    if (!is_dir(path_join(f.sysfs_root, "class/kfd"))) return "No kfd found (" + f.sysfs_root + "/class/kfd)";
    topo = KfdTopology::load_sysfs(f.sysfs_root);
    DiscoveryResult res = discover_gpus(f.sysfs_root, topo);
    res.devices = limit_physical(res.devices, dev_limit);
    if (!f.device_ids.empty()) {  // -device_ids: a node shared between plugin instances, or GPUs held back
      std::set<std::string> want;
      for (size_t a = 0; a <= f.device_ids.size();) {
        size_t b = f.device_ids.find(',', a);
        if (b == std::string::npos) b = f.device_ids.size();
        if (b > a) want.insert(f.device_ids.substr(a, b - a));
        a = b + 1;
      }
      std::vector<GpuDevice> kept;
      for (const auto& d : res.devices)
        if (want.erase(d.id)) kept.push_back(d);
      for (const auto& id : want) MI_LOG(kWarning, "-device_ids: %s is not a discovered device", id.c_str());
      res.devices = std::move(kept);
    }
    for (const auto& w : res.warnings) MI_LOG(kWarning, "%s", w.c_str());
    discovery_warnings = res.warnings;
    MI_LOG(kInfo, "Found %zu AMDGPUs", res.devices.size());
    auto& m = metrics::global();
    m.set("mi355x_dp_kfd_unreadable_nodes", static_cast<double>(res.kfd_unreadable_nodes.size()), {},
          "kfd topology nodes whose properties the plugin cannot read (EPERM)");
    m.set("mi355x_dp_devices_identity_from_sysfs", res.recovered_devices, {},
          "devices identified from PCI sysfs because their kfd node is unreadable");
    m.set("mi355x_dp_devices_identity_unknown", static_cast<double>(res.unresolved.size()), {},
          "devices without a known physical GPU / xGMI hive (placement not topology-aware)");
    const bool homogeneous = is_homogeneous(res.devices);
    if (!homogeneous && f.naming == "single")
      return "Partitions of different styles across GPUs in a node is not supported with single strategy. "
             "Please start device plugin with mixed strategy";
    const auto counts = partition_config_count(res.devices);
    std::vector<std::string> names;
    if (!res.devices.empty()) {
      if (homogeneous && (f.naming == "single" || counts.empty()))
        names.push_back(kDeviceTypeGpu);
      else
        for (const auto& [t, c] : counts)
          if (c > 0) names.push_back(t);
    }
    const std::set<std::string> unresolved(res.unresolved.begin(), res.unresolved.end());
    container_devices.clear();
    for (const auto& name : names) {
      Resource r;
      r.name = name;
      for (const auto& d : res.devices)
        if (homogeneous || d.partition_type() == name) {
          r.devices.push_back(d);
          container_devices.push_back(d);
        }
      r.socket = path_join(f.kubelet_dir, std::string(kResourceNamespace) + "_" + name);
      prepare(r, topo, unresolved, f.allocator_search, f.lists, view_ctx);
      out->push_back(std::move(r));
    }
    return "";
  };
  auto init_passthrough = [&](Driver drv, std::vector<Resource>* out) -> std::string {
    const bool vf = drv == Driver::Vf;
    if (!is_dir(path_join(f.sysfs_root, vf ? "bus/pci/drivers/gim" : "bus/pci/drivers/vfio-pci")))
      return vf ? "No amd gim driver loaded" : "No vfio-pci driver loaded";
    const PciScanResult scan = vf ? scan_vf_mapping(f.sysfs_root) : scan_pf_mapping(f.sysfs_root);
    if (!scan.ok) return std::string("Failed to generate ") + (vf ? "vf" : "pf") + " map: " + scan.error;
    MI_LOG(kInfo, "Found %zu %s IOMMU groups", scan.groups.size(), vf ? "vf-passthrough" : "pf-passthrough");
    if (scan.groups.empty()) return "";
    Resource r;
    r.driver = drv;
    r.name = f.naming == "mixed" ? (vf ? "gpu_vf" : "gpu_pf") : kDeviceTypeGpu;
    r.groups = scan.groups;
    for (const auto& [g, fns] : scan.groups) r.group_ids.push_back(g);
    std::sort(r.group_ids.begin(), r.group_ids.end(), [](const std::string& x, const std::string& y) {
      const bool dx = is_all_digits(x), dy = is_all_digits(y);
      if (dx != dy) return dx;
      if (dx && x.size() != y.size()) return x.size() < y.size();  // numeric order
      return x < y;
    });
    r.socket = path_join(f.kubelet_dir, std::string(kResourceNamespace) + "_" + r.name);
    prepare_passthrough(r);
    out->push_back(std::move(r));
    return "";
  };
  auto init_driver = [&](const std::string& type, std::vector<Resource>* out) {
    if (type == "container") return init_container(out);
    return init_passthrough(type == "vf-passthrough" ? Driver::Vf : Driver::Pf, out);
  };
  if (!f.driver_type.empty()) {
    const std::string e = init_driver(f.driver_type, &resources);
    if (!e.empty()) {
      MI_LOG(kError, "Error instantiating driver type %s: %s", f.driver_type.c_str(), e.c_str());
      return 1;
    }
    driver = f.driver_type == "container" ? Driver::Container
             : f.driver_type == "vf-passthrough" ? Driver::Vf : Driver::Pf;
  } else {
    // container -> VF -> PF; the reference starts its manager even when none initialised, and idles
    bool impl_found = false;
    for (const char* type : {"container", "vf-passthrough", "pf-passthrough"}) {
      std::vector<Resource> got;
      const std::string e = init_driver(type, &got);
      if (!e.empty()) {
        MI_LOG(kWarning, "%s implementation failed: %s. Trying next...", type, e.c_str());
        continue;
      }
      if (got.empty()) {
        MI_LOG(kWarning, "%s implementation found no devices. Trying next...", type);
        continue;
      }
      resources = std::move(got);
      impl_found = true;
      driver = std::string(type) == "container" ? Driver::Container
               : std::string(type) == "vf-passthrough" ? Driver::Vf : Driver::Pf;
      break;
    }
    impl_ok = impl_found;
  }

  // ---- CDI specs (-device_list_strategy cdi-*): written before registration,
  // since kubelet may hand a CDI name to the runtime as soon as it allocates
  auto write_cdi = [&](const std::set<std::string>& stale) -> std::string {
    if (driver != Driver::Container || !f.lists.cdi()) return "";
    std::map<std::string, std::vector<GpuDevice>> members;
    for (const auto& r : resources)
      if (!r.gone) members[r.name] = r.devices;
    std::vector<std::string> paths;
    const std::string e = cdi::write_specs(f.cdi_spec_dir, members, stale, &paths);
    if (e.empty()) {
      std::string all;
      for (const auto& p : paths) all += (all.empty() ? "" : ", ") + p;
      MI_LOG(kInfo, "CDI specs written: %s", all.c_str());
    }
    return e;
  };
  if (const std::string e = write_cdi({}); !e.empty()) {
    MI_LOG(kError, "cannot write CDI specs to %s: %s", f.cdi_spec_dir.c_str(), e.c_str());
    return 1;
  }

  // ---- health ---------------------------------------------------------------
  // The shutdown pipe ends every wait of the workers (peer calls, probes).
  int stop_pipe[2] = {-1, -1};
  if (::pipe2(stop_pipe, O_CLOEXEC | O_NONBLOCK) != 0) return 1;
  std::unique_ptr<health::Engine> engine;
  uint64_t fabric_seen = 0;  // engine->fabric_version() the allocators were built for
  auto make_engine = [&] {
    engine.reset();
    if (driver != Driver::Container || container_devices.empty()) return;
    health::Config hc;
    hc.sysfs_root = f.sysfs_root;
    hc.dev_root = f.dev_root;
    hc.exporter_socket = f.exporter_socket;
    hc.liveness = f.liveness;
    hc.prober.exe = !f.liveness_probe.empty() ? f.liveness_probe : path_join(self_dir(), "mi355x-liveness-probe");
    hc.prober.timeout_s = f.liveness_timeout;
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
    engine = std::make_unique<health::Engine>(container_devices, topo, hc);
    fabric_seen = 0;
    engine->set_abort_fd(stop_pipe[0]);
    if (f.liveness) MI_LOG(kInfo, "liveness probe: %s (%s)", hc.prober.exe.c_str(), f.liveness_mode.c_str());
  };
  make_engine();
  // one health pass (blocking; worker thread): device id -> healthy for every resource
  auto health_pass = [&]() -> std::map<std::string, bool> {
    std::map<std::string, bool> out;
    if (driver == Driver::Container) {
      if (engine) {
        engine->sweep();
        for (const auto& [id, v] : engine->snapshot()) out[id] = v.healthy;
      }
      return out;
    }
    const bool vf = driver == Driver::Vf;
    // gim gone -> every group Unhealthy; else a group is Unhealthy if any parent PF is (amdgpu_sriov.go:217-308)
    // vfio-pci present -> Healthy (amdgpu_pf.go:210-229)
    const bool present = is_dir(path_join(f.sysfs_root, vf ? "bus/pci/drivers/gim" : "bus/pci/drivers/vfio-pci"));
    std::map<std::string, bool> exporter;
    if (vf) {
      std::string e;
      exporter = health::exporter_list(f.exporter_socket, 10.0, stop_pipe[0], &e);
      if (!e.empty()) MI_LOG(kError, "Error getting health info svc : %s", e.c_str());
    }
    for (const auto& r : resources)
      for (const auto& g : r.group_ids) {
        bool ok = present;
        if (vf)
          for (const auto& fn : r.groups.at(g))
            if (auto it = exporter.find(fn.pf); it != exporter.end() && !it->second) ok = false;
        out[g] = ok;
      }
    return out;
  };
  // applies verdicts; true when a resource's list changed
  auto apply_health = [&](Resource& r, const std::map<std::string, bool>& h) {
    bool changed = false;
    auto set = [&](const std::string& id) {
      auto it = h.find(id);
      if (it == h.end()) return;
      auto cur = r.health.find(id);
      const bool prev = cur == r.health.end() || cur->second;
      if (prev != it->second) changed = true;
      r.health[id] = it->second;
    };
    for (const auto& d : r.devices) set(d.id);
    for (const auto& g : r.group_ids) set(g);
    if (changed) {
      r.list = list_bytes(r);
      r.service->set_device_list(r.list);
    }
    return changed;
  };
  if (f.pulse > 0 && !resources.empty()) {
    // one sweep before registering, so the first ListAndWatch already carries
    // real verdicts (the reference advertises everything Healthy until its first pulse)
    const auto h = health_pass();
    for (auto& r : resources) apply_health(r, h);
  }

  if (f.dry_run) {
    json::Value out = json::Value::object();
    const char* impl_name = driver == Driver::Container ? "container" : driver == Driver::Vf ? "vf-passthrough"
                                                                                            : "pf-passthrough";
    out.set("implementation", impl_ok ? json::Value::string(impl_name) : jnull());
    json::Value res = json::Value::object();
    for (const auto& r : resources) {
      json::Value rv = json::Value::object();
      json::Value devs = jarr();
      std::vector<std::string> ids;
      auto health_of = [&](const std::string& id) {
        auto it = r.health.find(id);
        return json::Value::string(it == r.health.end() || it->second ? "Healthy" : "Unhealthy");
      };
      for (const auto& g : r.group_ids) {
        json::Value d = json::Value::object();
        d.set("id", json::Value::string(g));
        d.set("health", health_of(g));
        d.set("numa", jarr());
        devs.arr.push_back(d);
        ids.push_back(g);
      }
      std::map<std::string, const GpuDevice*> by_id;
      for (const auto& gd : r.devices) {
        json::Value d = json::Value::object();
        d.set("id", json::Value::string(gd.id));
        d.set("health", health_of(gd.id));
        json::Value numa = jarr();
        if (gd.numa_node >= 0) numa.arr.push_back(jnum(gd.numa_node));
        d.set("numa", numa);
        devs.arr.push_back(d);
        ids.push_back(gd.id);
        by_id[gd.id] = &gd;
      }
      rv.set("devices", devs);
      rv.set("preferred_allocation", jbool(r.allocator != nullptr));
      if (r.allocator && !ids.empty()) {
        json::Value prefs = json::Value::object();
        std::set<int> ks = {1, 2, 4, 8, static_cast<int>(ids.size())};
        for (int k : ks) {
          if (k < 1 || k > static_cast<int>(ids.size())) continue;
          const AllocResult a = r.allocator->allocate(ids, {}, k);
          json::Value pv = json::Value::object();
          json::Value chosen = jarr();
          std::vector<const GpuDevice*> set;
          for (const auto& id : a.ids) {
            chosen.arr.push_back(json::Value::string(id));
            if (by_id.count(id)) set.push_back(by_id[id]);
          }
          pv.set("ids", chosen);
          if (driver == Driver::Container) {
            const FabricReport fr = fabric_report(set, topo);
            pv.set("one_hive", jbool(fr.one_hive));
            pv.set("allreduce_bound_gbs", fr.has_bound ? jnum(fr.bound_gbs) : jnull());
          }
          prefs.set(std::to_string(k), pv);
        }
        rv.set("allocations", prefs);
      }
      res.set(std::string(kResourceNamespace) + "/" + r.name, rv);
    }
    out.set("resources", res);
    if (driver == Driver::Container && impl_ok) {
      json::Value w = jarr();
      for (const auto& x : discovery_warnings) w.arr.push_back(json::Value::string(x));
      out.set("warnings", w);
      json::Value ls = jarr();
      for (const auto& x : f.lists.order) ls.arr.push_back(json::Value::string(x));
      out.set("device_list_strategy", ls);
      if (f.lists.cdi()) out.set("cdi_spec_dir", json::Value::string(f.cdi_spec_dir));
    }
    if (engine && f.smi_xgmi) {
      json::Value x = json::Value::object();
      x.set("readings", jnum(static_cast<double>(engine->xgmi_readings())));
      x.set("error", json::Value::string(engine->xgmi_error()));
      json::Value pairs = jarr();
      for (const auto& [a, b] : engine->degraded_links()) {
        json::Value pr = jarr();
        pr.arr.push_back(json::Value::string(a));
        pr.arr.push_back(json::Value::string(b));
        pairs.arr.push_back(pr);
      }
      x.set("degraded_pairs", pairs);
      json::Value down = json::Value::object();
      for (const auto& [bdf, n] : engine->links_down()) down.set(bdf, jnum(n));
      x.set("links_down", down);
      out.set("xgmi", x);
    }
    if (engine && !engine->perf_last().empty()) {
      const auto verdicts = engine->perf_verdicts();
      json::Value thr = json::Value::object();
      for (const auto& [dev, o] : engine->perf_last()) {
        json::Value t = json::Value::object();
        auto v = verdicts.find(dev);
        t.set("state", json::Value::string(v == verdicts.end() ? "ok" : v->second.first));
        t.set("reason", json::Value::string(v == verdicts.end() ? "" : v->second.second));
        for (const char* k : {"hbm_write_gbps", "hbm_read_gbps", "hbm_bad_words", "mfma_tflops", "clock_mhz_median"})
          if (auto d = o.detail.find(k); d != o.detail.end()) t.set(k, jnum(d->second));
        if (!o.xcd_clock_mhz.empty()) {
          json::Value xs = jarr();
          for (double c : o.xcd_clock_mhz) xs.arr.push_back(jnum(c));
          t.set("xcd_clock_mhz", xs);
        }
        if (auto d = o.detail.find("total_us"); d != o.detail.end()) t.set("total_us", jnum(d->second));
        thr.set(dev, t);
      }
      out.set("throughput", thr);
    }
    std::printf("%s\n", json::serialize(out).c_str());
    std::fflush(stdout);
    if (engine) engine->close();
    return 0;
  }

  metrics::HttpEndpoint metrics_http;
  if (f.metrics_port > 0) {
    const std::string merr = metrics_http.start("0.0.0.0", f.metrics_port);
    if (!merr.empty()) {
      MI_LOG(kError, "cannot serve /metrics: %s", merr.c_str());
      return 1;
    }
    MI_LOG(kInfo, "serving Prometheus /metrics on :%d", metrics_http.port());
  }

  const std::string kubelet_sock = path_join(f.kubelet_dir, "kubelet.sock");
  DirWatcher watch;
  std::string werr = watch.open(f.kubelet_dir);
  if (!werr.empty()) MI_LOG(kWarning, "no inotify watch on %s (%s): polling every second", f.kubelet_dir.c_str(),
                            werr.c_str());
  Workers workers;
  uint64_t kubelet_gen = 0;  // bumped on every kubelet (re)start: older Register results are stale
  auto try_register = [&](size_t i) {
    Resource& r = resources[i];
    if (r.register_inflight || !r.server) return;
    r.register_inflight = true;
    const uint64_t gen = kubelet_gen;
    workers.run([&f, &kubelet_sock, name = r.name, socket = r.socket, options = r.options, i, gen,
                 sgen = r.server_gen, abort_fd = stop_pipe[0]] {
      Completion c{Completion::kRegister, i, gen, false, "", {}, 0, sgen};
      c.message = register_with_kubelet(name, socket, options, kubelet_sock, f.register_timeout_s, abort_fd);
      c.ok = c.message.empty();
      return c;
    });
  };
  auto start_all = [&] {
    kubelet_gen++;
    for (size_t i = 0; i < resources.size(); ++i) {
      Resource& r = resources[i];
      stop_server(r);
      r.retry_ms = 100;
      r.next_register = Clock::now();
      if (start_server(r)) {
        r.register_inflight = false;  // a Register of the previous kubelet completes as stale
        try_register(i);
      }
    }
  };
  SockId sock = sock_id(kubelet_sock);
  if (sock.present) start_all();

  bool sweep_inflight = false;
  auto next_pulse = Clock::now() + std::chrono::seconds(f.pulse > 0 ? f.pulse : 3600);

  // ---- topology watch (container driver): an amd-smi partition switch changes
  // the devices; vanished resources stop serving (kubelet drops them when the
  // stream ends), kept ones get the new devices, allocator and list, new ones
  // register; the health engine is rebuilt (a probe server's agents were
  // enumerated at its start). The Python CLI's reload_topology (plugin/container.py).
  const bool topo_watch = f.topology_watch_s > 0 && driver == Driver::Container;
  const auto topo_period = std::chrono::milliseconds(static_cast<long long>(f.topology_watch_s * 1000));
  std::string topo_sig = topo_watch ? topology_signature(f.sysfs_root) : "", topo_seen = topo_sig;
  auto next_topo = Clock::now() + topo_period;
  auto reload_topology = [&](const std::string& sig) {
    std::vector<Resource> fresh;
    const std::string e = init_container(&fresh);  // re-reads topo and container_devices
    topo_sig = sig;
    std::map<std::string, std::string> before, after;  // device id -> partition type
    std::string old_names, new_names;
    for (const auto& r : resources)
      if (!r.gone) {
        old_names += (old_names.empty() ? "" : ",") + r.name;
        for (const auto& d : r.devices) before[d.id] = d.partition_type();
      }
    if (e.empty())
      for (const auto& r : fresh) {
        new_names += (new_names.empty() ? "" : ",") + r.name;
        for (const auto& d : r.devices) after[d.id] = d.partition_type();
      }
    if (before == after) return;
    std::set<std::string> old_set;
    for (const auto& r : resources)
      if (!r.gone) old_set.insert(r.name);
    metrics::global().inc("mi355x_dp_topology_reloads_total");
    MI_LOG(kWarning, "GPU topology changed: %zu -> %zu devices; resources [%s] -> [%s]", before.size(), after.size(),
           old_names.c_str(), new_names.c_str());
    const std::string lw = rpc::DevicePluginService::path("ListAndWatch");
    if (!e.empty()) {
      MI_LOG(kError, "GPU topology changed: %s. Advertising no devices until then.", e.c_str());
      for (auto& r : resources) {
        if (r.gone) continue;
        r.devices.clear();
        r.health.clear();
        r.allocator.reset();
        r.service->set_allocator(nullptr);
        r.list = list_bytes(r);
        r.service->set_device_list(r.list);
        if (r.server) r.server->broadcast(lw, r.list);
      }
      if (const std::string ce = write_cdi(old_set); !ce.empty())
        MI_LOG(kError, "CDI specs not updated after the topology change: %s", ce.c_str());
      container_devices.clear();
      make_engine();
      return;
    }
    std::set<std::string> names;
    for (const auto& fr : fresh) names.insert(fr.name);
    for (auto& r : resources)
      if (!r.gone && !names.count(r.name)) {
        MI_LOG(kWarning, "resource %s no longer exists: stopping its plugin server", r.name.c_str());
        stop_server(r);
        r.gone = true;
        r.devices.clear();
        r.health.clear();
      }
    std::vector<size_t> to_start;  // new resources: served and registered once their CDI specs exist
    for (auto& fr : fresh) {
      auto it = std::find_if(resources.begin(), resources.end(), [&](const Resource& r) { return r.name == fr.name; });
      if (it != resources.end() && !it->gone) {
        Resource& r = *it;
        const bool opts_changed = r.options != fr.options;
        std::map<std::string, bool> kept;
        for (const auto& d : fr.devices)
          if (auto h = r.health.find(d.id); h != r.health.end()) kept[d.id] = h->second;
        r.devices = std::move(fr.devices);
        r.health = std::move(kept);
        r.allocator = fr.allocator;
        r.options = fr.options;
        r.tmpl = fr.tmpl;
        r.service->set_options(r.options);
        r.service->set_allocator(r.allocator);
        r.service->set_allocate_template(r.tmpl);
        r.list = list_bytes(r);
        r.service->set_device_list(r.list);
        if (r.server) r.server->broadcast(lw, r.list);
        if (opts_changed && r.server) {  // kubelet reads the options at registration
          r.registered = false;
          r.next_register = Clock::now();
        }
        continue;
      }
      size_t i;
      if (it != resources.end()) {
        *it = std::move(fr);
        i = static_cast<size_t>(it - resources.begin());
      } else {
        resources.push_back(std::move(fr));
        i = resources.size() - 1;
      }
      MI_LOG(kInfo, "new resource %s (%zu devices)", resources[i].name.c_str(), resources[i].devices.size());
      to_start.push_back(i);
    }
    // before any new resource registers: kubelet may hand its CDI names to the runtime at once
    if (const std::string ce = write_cdi(old_set); !ce.empty())
      MI_LOG(kError, "CDI specs not updated after the topology change: %s", ce.c_str());
    for (size_t i : to_start)
      if (sock.present && start_server(resources[i])) try_register(i);
    make_engine();
    if (f.pulse > 0) next_pulse = Clock::now();  // verdicts for the new devices now
  };
  auto next_stat = Clock::now() + std::chrono::seconds(5);
  int exit_code = 0;
  while (!g_stop) {
    std::vector<pollfd> pfd = {{g_sig_pipe[0], POLLIN, 0}, {workers.wake_fd(), POLLIN, 0}};
    const bool inotify = watch.fd() >= 0;
    if (inotify) pfd.push_back({watch.fd(), POLLIN, 0});
    const size_t ev_base = pfd.size();
    for (const auto& r : resources) pfd.push_back({r.service->event_fd(), POLLIN, 0});
    const auto now = Clock::now();
    auto until = [&](Clock::time_point t) -> long long {
      return std::chrono::duration_cast<std::chrono::milliseconds>(t - now).count() + 1;
    };
    long long wait_ms = f.pulse > 0 ? until(next_pulse) : 3600 * 1000;
    // inotify is the fast path; the stat poll is the safety net (a dead watch, a replaced directory)
    wait_ms = std::min(wait_ms, inotify ? until(next_stat) : 1000LL);
    for (const auto& r : resources) {
      if (r.server && !r.registered && !r.register_inflight) wait_ms = std::min(wait_ms, until(r.next_register));
      if (r.registered && !r.list_seen && f.grpc_watchdog_s > 0) wait_ms = std::min(wait_ms, 250LL);
    }
    if (f.grpc_watchdog_s > 0) wait_ms = std::min(wait_ms, 1000LL);
    if (topo_watch) wait_ms = std::min(wait_ms, until(next_topo));
    ::poll(pfd.data(), pfd.size(), static_cast<int>(std::max(0LL, wait_ms)));
    if (g_stop) break;
    // ---- RPC events: the reference logs every Allocate
    for (size_t i = 0; i < resources.size(); ++i)
      if (pfd[ev_base + i].revents & POLLIN) {
        uint64_t v;
        if (::read(resources[i].service->event_fd(), &v, sizeof(v)) < 0) {
        }
        const auto evs = resources[i].service->drain_events();
        auto& m = metrics::global();
        const metrics::Labels res_l = {{"resource", resources[i].name}};
        if (!evs.empty() && resources[i].server) {
          const auto st = resources[i].server->stats();
          m.set("mi355x_dp_grpc_connections", static_cast<double>(st.connections), res_l,
                "native gRPC server: connections");
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
                                     {{"resource", resources[i].name}, {"native", ev.native ? "True" : "False"},
                                      {"ids", ids}});
            if (ev.alloc_t0_ns)
              trace::global().complete("allocator.allocate", "alloc", ev.alloc_t0_ns,
                                       static_cast<uint64_t>(ev.alloc_us * 1e3),
                                       {{"candidates", std::to_string(ev.candidates)}, {"native", "True"}});
          }
          m.observe_ms("mi355x_dp_rpc_seconds", ev.dur_ns / 1e6, {{"resource", resources[i].name}, {"rpc", ev.rpc}},
                       "device plugin RPC latency");
          if (ev.rpc == "ListAndWatch") m.inc("mi355x_dp_listandwatch_streams_total", res_l);
          if (ev.status != 0) {
            m.inc("mi355x_dp_rpc_errors_total", {{"resource", resources[i].name}, {"rpc", ev.rpc}});
            MI_LOG(kError, "%s: %s: %s", resources[i].name.c_str(), ev.rpc.c_str(), ev.message.c_str());
          } else if (ev.rpc == "Allocate") {
            std::string ids;
            for (const auto& id : ev.ids) ids += (ids.empty() ? "" : ",") + id;
            MI_LOG(kInfo, "Allocating device IDs: %s", ids.c_str());
          }
          if (glog::vlog_is_on(2, __FILE__)) {
            char ms[32];
            std::snprintf(ms, sizeof(ms), "%.3f", ev.dur_ns / 1e6);
            glog::Fields fl = {{"rpc", ev.rpc}, {"resource", resources[i].name}, {"latency_ms", ms}, {"native", "True"}};
            if (ev.rpc == "GetPreferredAllocation" && ev.candidates >= 0) {
              fl.emplace_back("candidates", std::to_string(ev.candidates));
              fl.emplace_back("short_circuit", ev.short_circuit ? "True" : "False");
            }
            MI_LOG_FIELDS(kInfo, "rpc", (fl));
          }
        }
      }
    // ---- kubelet restarts: act only when kubelet.sock itself was replaced
    bool look = !inotify || Clock::now() >= next_stat;
    if (inotify && (pfd[2].revents & POLLIN)) {
      for (const auto& [name, mask] : watch.read_events()) {
        if (name == "kubelet.sock") look = true;
        if (name.empty() && (mask & (IN_IGNORED | IN_DELETE_SELF | IN_MOVE_SELF))) {
          // the watched directory went away: watch it again once it is back, stat-poll meanwhile
          watch.close();
          look = true;
        }
      }
    }
    if (watch.fd() < 0 && is_dir(f.kubelet_dir) && watch.open(f.kubelet_dir).empty())
      MI_LOG(kInfo, "inotify watch on %s re-established", f.kubelet_dir.c_str());
    if (look) {
      next_stat = Clock::now() + std::chrono::seconds(5);
      const SockId cur = sock_id(kubelet_sock);
      if (cur != sock) {
        if (cur.present) {
          MI_LOG(kInfo, "kubelet socket (re)created; restarting plugin servers and re-registering");
          start_all();
        } else if (sock.present) {
          MI_LOG(kInfo, "kubelet socket removed; stopping plugin servers");
          kubelet_gen++;
          for (auto& r : resources) stop_server(r);
        }
        sock = cur;
      }
    }
    // ---- worker completions
    for (auto& c : workers.take()) {
      if (c.kind == Completion::kRegister) {
        Resource& r = resources[c.resource];
        if (c.server_gen != r.server_gen) continue;  // an earlier server's answer (restart, topology change)
        r.register_inflight = false;
        if (c.gen != kubelet_gen || !r.server) continue;  // a previous kubelet's answer
        if (c.ok) {
          r.registered = true;
          r.retry_ms = 100;
          r.registered_at = Clock::now();
          const auto st = r.server->stats();
          r.streams_at_register = st.streams_opened;
          r.perr_at_register = st.protocol_errors;
          r.list_seen = false;
          metrics::global().inc("mi355x_dp_registrations_total", {{"resource", r.name}});
          MI_LOG(kInfo, "%s: Registration for endpoint %s", r.name.c_str(), basename(r.socket).c_str());
        } else {
          MI_LOG(kError, "%s: %s", r.name.c_str(), c.message.c_str());
          r.next_register = Clock::now() + std::chrono::milliseconds(r.retry_ms);
          r.retry_ms = std::min(2 * r.retry_ms, 3000);
        }
      } else {
        sweep_inflight = false;
        metrics::global().observe_ms("mi355x_dp_health_sweep_seconds", c.sweep_ms, {}, "health sweep latency");
        bool any_changed = false;
        for (auto& r : resources) {
          const bool changed = apply_health(r, c.health);
          any_changed = any_changed || changed;
          if ((changed || f.send_every_pulse) && r.server) {
            r.server->broadcast(rpc::DevicePluginService::path("ListAndWatch"), r.list);
            trace::global().instant("ListAndWatch.send", "rpc",
                                    {{"resource", r.name}, {"health_version", std::to_string(engine ? engine->version() : 0)},
                                     {"streams", std::to_string(r.server->stats().streams_open)}});
          }
        }
        if (any_changed) metrics::global().inc("mi355x_dp_health_changes_total");
        // xGMI link state changed: every allocator re-weighted on the degraded pairs
        if (engine && engine->fabric_version() != fabric_seen) {
          fabric_seen = engine->fabric_version();
          const auto degraded = engine->degraded_links();
          for (auto& r : resources) {
            if (r.gone || !r.allocator) continue;
            std::string aerr;
            auto a = build_allocator(r.devices, topo, f.allocator_search, degraded, &aerr);
            if (!aerr.empty()) {
              MI_LOG(kError, "%s: allocator re-weighting failed: %s", r.name.c_str(), aerr.c_str());
              continue;
            }
            r.allocator = a;
            r.service->set_allocator(a);
          }
          metrics::global().inc("mi355x_dp_fabric_reweights_total");
          MI_LOG(kWarning, "xGMI link state changed: preferred allocation re-weighted (%zu degraded GPU pairs)",
                 degraded.size());
        }
      }
    }
    workers.reap();
    // ---- registrations that failed (kubelet not serving yet): retry, rate-limited
    for (size_t i = 0; i < resources.size(); ++i) {
      Resource& r = resources[i];
      if (r.server && !r.registered && !r.register_inflight && sock.present && Clock::now() >= r.next_register)
        try_register(i);
    }
    // ---- transport watchdog
    if (f.grpc_watchdog_s > 0) {
      std::string why;
      for (auto& r : resources) {
        if (!r.registered || !r.server) continue;
        const auto st = r.server->stats();
        if (st.streams_opened > r.streams_at_register) r.list_seen = true;
        if (st.protocol_errors > r.perr_at_register) {
          why = r.name + ": " + std::to_string(st.protocol_errors - r.perr_at_register) +
                " HTTP/2 protocol error(s) on the plugin socket";
        } else if (!r.list_seen && std::chrono::duration<double>(Clock::now() - r.registered_at).count() >
                                       f.grpc_watchdog_s) {
          char b[96];
          std::snprintf(b, sizeof(b), "no ListAndWatch stream within %gs of Register", f.grpc_watchdog_s);
          why = r.name + ": " + b;
        }
        if (!why.empty()) break;
      }
      if (!why.empty()) {
        MI_LOG(kError, "native gRPC transport watchdog: %s; exiting so the plugin is restarted", why.c_str());
        exit_code = 3;
        break;
      }
    }
    // ---- topology watch: a new signature must hold for one interval (a partition
    // switch passes through states with devices half gone); never under a sweep
    if (topo_watch && Clock::now() >= next_topo) {
      next_topo = Clock::now() + topo_period;
      const std::string cur = topology_signature(f.sysfs_root);
      if (cur != topo_seen) {
        topo_seen = cur;
      } else if (cur != topo_sig && !sweep_inflight) {
        reload_topology(cur);
      }
    }
    // ---- health pulse (worker thread; a sweep still running skips this pulse)
    if (f.pulse > 0 && Clock::now() >= next_pulse) {
      next_pulse = Clock::now() + std::chrono::seconds(f.pulse);
      if (sweep_inflight) {
        MI_LOG(kWarning, "health sweep still running at the next pulse; skipping this pulse");
      } else if (!resources.empty()) {
        sweep_inflight = true;
        workers.run([&health_pass] {
          Completion c{Completion::kSweep, 0, 0, true, "", {}, 0, 0};
          const auto t0 = Clock::now();
          c.health = health_pass();
          c.sweep_ms = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
          return c;
        });
      }
    }
  }
  if (g_stop) MI_LOG(kInfo, "Received signal, shutting down.");
  const char b = 1;
  if (::write(stop_pipe[1], &b, 1) < 0) {
  }
  workers.join_all();  // every wait ends at the stop pipe
  if (engine) engine->close();
  for (auto& r : resources) stop_server(r);
  if (const std::string te = trace::global().flush(); !te.empty())
    MI_LOG(kError, "cannot write the trace file: %s", te.c_str());
  return exit_code;
}
