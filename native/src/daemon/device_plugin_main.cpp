// mi355x-device-plugin: the kubelet device plugin as one native process.
//
// The reference ships its plugin as a single compiled binary
// (cmd/k8s-device-plugin/main.go). This is the same thing built from the
// framework's C++ core, with no interpreter in the process:
//
//   flags          -pulse, -driver_type, -resource_naming_strategy (main.go:50-75),
//                  glog flags accepted; -kubelet_dir / -sysfs_root / -dev_root /
//                  -exporter_socket / -send_every_pulse as in the Python CLI
//   discovery      discover_gpus over the kfd topology (gpu_discovery.cpp)
//   resources      single -> "gpu"; mixed -> "<compute>_<memory>"; heterogeneous
//                  partitions with single is an error (amdgpu.go:68-88,122-162)
//   per resource   the native gRPC server on <kubelet_dir>/amd.com_<resource>
//                  with the DevicePlugin service: hive-aware
//                  GetPreferredAllocation (HiveAllocator), Allocate = /dev/kfd +
//                  card + renderD per device (amdgpu.go:255-319), ListAndWatch
//   registration   Register on kubelet.sock through the native client; again
//                  whenever kubelet.sock is re-created (inotify on the plugin
//                  directory, as the vendored dpm does with fsnotify)
//   health         every -pulse: the device's kfd node is a live GPU, and the
//                  metrics exporter's per-BDF verdict when its socket exists
//                  (amdgpu.go:322-345, exporter/health.go:41-79); the list is
//                  pushed when a verdict changes (or every pulse with
//                  -send_every_pulse, the reference's behaviour)
//   signals        SIGTERM / SIGINT stop the servers and remove the sockets
//   passthrough    -driver_type vf-passthrough / pf-passthrough (amdgpu_sriov.go,
//                  amdgpu_pf.go): one device per IOMMU group, Allocate =
//                  /dev/vfio/<group> + /dev/vfio/vfio (mrw) and
//                  PCI_RESOURCE_AMD_COM_<RES> = the BDFs of every requested group;
//                  health = driver present (+ exporter PF verdicts for VFs);
//                  without -driver_type: container -> VF -> PF (main.go:106-115)
//
// The Python CLI (scripts/k8s-device-plugin) is the full-featured entrypoint:
// the MFMA liveness probes and throughput checks, amd-smi, CDI, container
// views, topology reloads, metrics and tracing. This binary is for nodes that
// want the reference's feature set without Python.
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/inotify.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "mi355x/allocator.h"
#include "mi355x/constants.h"
#include "mi355x/dir_watch.h"
#include "mi355x/dp_service.h"
#include "mi355x/gpu_discovery.h"
#include "mi355x/grpc_server.h"
#include "mi355x/kfd_topology.h"
#include "mi355x/pci_scan.h"
#include "mi355x/sysfs.h"

namespace {

using namespace mi355x;
namespace pb = mi355x::rpc::pb;

// ---- logging (glog line format) --------------------------------------------
void logf(char sev, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void logf(char sev, const char* fmt, ...) {
  timespec ts{};
  clock_gettime(CLOCK_REALTIME, &ts);
  tm t{};
  localtime_r(&ts.tv_sec, &t);
  char msg[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(msg, sizeof(msg), fmt, ap);
  va_end(ap);
  std::fprintf(stderr, "%c%02d%02d %02d:%02d:%02d.%06ld %7d device_plugin_main.cpp] %s\n", sev, t.tm_mon + 1,
               t.tm_mday, t.tm_hour, t.tm_min, t.tm_sec, ts.tv_nsec / 1000, static_cast<int>(getpid()), msg);
}

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
};

bool parse_bool(const std::string& v) { return v.empty() || v == "1" || v == "true" || v == "True" || v == "t"; }

// Go flag syntax: -name=value, -name value, --name, bare booleans.
bool parse_flags(int argc, char** argv, Flags* f, std::string* err) {
  static const std::set<std::string> kBool = {"send_every_pulse", "logtostderr", "alsologtostderr", "h", "help"};
  static const std::set<std::string> kIgnoredValue = {"v", "stderrthreshold", "log_dir", "vmodule",
                                                      "log_backtrace_at", "kubelet-url"};
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
      std::printf("usage: %s [-pulse N] [-driver_type container|vf-passthrough|pf-passthrough] [-resource_naming_strategy single|mixed] "
                  "[-kubelet_dir DIR] [-sysfs_root DIR] [-dev_root DIR] [-exporter_socket PATH] "
                  "[-send_every_pulse] (glog flags accepted)\n", argv[0]);
      std::exit(0);
    }
    if (kBool.count(name)) {
      if (name == "send_every_pulse") f->send_every_pulse = parse_bool(value);
      continue;
    }
    if (!has_value) {
      if (i + 1 >= argc) return *err = "flag needs an argument: -" + name, false;
      value = argv[++i];
    }
    if (name == "pulse") {
      char* end = nullptr;
      const long v = std::strtol(value.c_str(), &end, 10);
      if (end == value.c_str() || *end) return *err = "invalid value \"" + value + "\" for flag -pulse", false;
      f->pulse = static_cast<int>(v);
    } else if (name == "driver_type") {
      f->driver_type = value;
    } else if (name == "resource_naming_strategy") {
      f->naming = value;
    } else if (name == "kubelet_dir") {
      f->kubelet_dir = value;
    } else if (name == "sysfs_root") {
      f->sysfs_root = value;
    } else if (name == "dev_root") {
      f->dev_root = value;
    } else if (name == "exporter_socket") {
      f->exporter_socket = value;
    } else if (!kIgnoredValue.count(name)) {
      return *err = "flag provided but not defined: -" + name, false;
    }
  }
  // validateFlags (main.go:59-75)
  if (f->pulse < 0) return *err = "pulse must be a non-negative integer", false;
  if (!f->driver_type.empty() && f->driver_type != "container" && f->driver_type != "vf-passthrough" &&
      f->driver_type != "pf-passthrough")
    return *err = "invalid driver_type provided: " + f->driver_type +
                  ", supported values are container, vf-passthrough, or pf-passthrough",
           false;
  if (f->naming != "single" && f->naming != "mixed")
    return *err = "invalid resource_naming_strategy provided: " + f->naming + ", supported values are single or mixed",
           false;
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
  std::unique_ptr<rpc::GrpcServer> server;
  std::unique_ptr<rpc::DevicePluginService> service;
  std::shared_ptr<const HiveAllocator> allocator;
  std::map<std::string, bool> health;  // device id -> healthy
  std::string list;                    // serialized ListAndWatchResponse
  bool registered = false;
  std::chrono::steady_clock::time_point next_register{};
  int retry_ms = 100;  // kubelet.sock appears (bind) just before kubelet listens: retry soon, then back off to 3 s
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

void prepare(Resource& r, const KfdTopology& topo, const std::set<std::string>& unresolved) {
  // allocator (BestEffortPolicy.init); on failure kubelet allocates by itself
  bool alloc_ok = true;
  for (const auto& d : r.devices)
    if (unresolved.count(d.id)) alloc_ok = false;
  if (!alloc_ok) {
    logf('E', "allocator disabled for plugin %s: no physical-GPU identity for some devices. Falling back to "
              "kubelet default allocation.", r.name.c_str());
  } else {
    std::vector<AllocDevice> ad;
    for (const auto& d : r.devices) {
      AllocDevice a;
      a.id = d.id;
      a.node_id = d.node_id;
      a.numa_node = d.numa_node;
      a.unique_id = group_key(d);
      a.hive_id = d.hive_id;
      a.inferred_links = d.node_id < 0 && d.identity == "sysfs";
      ad.push_back(a);
    }
    auto alloc = std::make_shared<HiveAllocator>();
    const std::string err = alloc->init(ad, topo);
    if (!err.empty()) {
      logf('E', "allocator init failed for plugin %s. Falling back to kubelet default allocation. Error %s",
           r.name.c_str(), err.c_str());
      alloc_ok = false;
    } else {
      r.allocator = alloc;
    }
  }
  r.options.clear();
  if (alloc_ok) pb::put_bool(&r.options, 2, true);  // get_preferred_allocation_available
  rpc::AllocateTemplate t;
  t.resource = r.name;
  pb::put_bytes(&t.container_prefix, 3, device_spec("/dev/kfd"));
  for (const auto& d : r.devices) {
    std::string car;
    if (d.card >= 0) pb::put_bytes(&car, 3, device_spec("/dev/dri/card" + std::to_string(d.card)));
    if (d.render_minor >= 0) pb::put_bytes(&car, 3, device_spec("/dev/dri/renderD" + std::to_string(d.render_minor)));
    t.per_device[d.id] = car;
  }
  r.service = std::make_unique<rpc::DevicePluginService>();
  r.service->set_fallback([name = r.name](const std::string& method, const std::string&) {
    // everything the native daemon serves has prepared state; a method without it is not implemented
    return rpc::Reply{rpc::kUnimplemented, "not served by the native daemon: " + method + " (" + name + ")", ""};
  });
  r.service->set_options(r.options);
  if (r.allocator) r.service->set_allocator(r.allocator);
  r.service->set_allocate_template(t);
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
    logf('E', "%s: could not serve on %s: %s", r.name.c_str(), r.socket.c_str(), err.c_str());
    r.server.reset();
    return false;
  }
  logf('I', "%s: serving on %s", r.name.c_str(), r.socket.c_str());
  return true;
}

void stop_server(Resource& r) {
  if (r.server) {
    r.server->stop(0.5);
    r.server.reset();
    ::unlink(r.socket.c_str());
  }
  r.registered = false;
}

// Register{version=1, endpoint=2, resource_name=3, options=4} on kubelet.sock
bool register_with_kubelet(Resource& r, const std::string& kubelet_sock, double timeout_s) {
  rpc::GrpcClient c;
  const std::string err = c.connect(kubelet_sock);
  if (!err.empty()) {
    logf('W', "%s: kubelet not reachable at %s: %s", r.name.c_str(), kubelet_sock.c_str(), err.c_str());
    return false;
  }
  std::string req;
  pb::put_bytes(&req, 1, "v1beta1");
  pb::put_bytes(&req, 2, basename(r.socket));
  pb::put_bytes(&req, 3, std::string(kResourceNamespace) + "/" + r.name);
  pb::put_bytes(&req, 4, r.options);
  const rpc::Reply rep = c.unary("/v1beta1.Registration/Register", req, timeout_s);
  if (rep.status != 0) {
    logf('E', "%s: Register failed (%d): %s", r.name.c_str(), rep.status, rep.message.c_str());
    return false;
  }
  logf('I', "%s: Registration for endpoint %s", r.name.c_str(), basename(r.socket).c_str());
  return true;
}

// ---- health -------------------------------------------------------------------
// The device's kfd node still describes a live GPU (ContainerImpl's kfd verdict).
bool kfd_node_live(const std::string& sysfs_root, const GpuDevice& d) {
  if (d.node_id < 0) return true;  // no kfd data for this device (cgroup-denied): not evidence of a fault
  const auto kv = parse_kv_file(path_join(sysfs_root, "class/kfd/kfd/topology/nodes/" + std::to_string(d.node_id) +
                                                          "/properties"));
  if (!kv) return false;
  const auto cores = kv->find("cpu_cores_count");
  const auto gfx = kv->find("gfx_target_version");
  return cores != kv->end() && gfx != kv->end() && parse_i64(cores->second, 1) == 0 &&
         parse_i64(gfx->second, 0) > 0;
}

// metricssvc.MetricsService/List -> BDF -> healthy; empty when unavailable
std::map<std::string, bool> exporter_health(const std::string& socket) {
  std::map<std::string, bool> out;
  if (socket.empty() || !path_exists(socket)) return out;
  rpc::GrpcClient c;
  if (!c.connect(socket).empty()) return out;
  const rpc::Reply rep = c.unary("/metricssvc.MetricsService/List", "", 10.0);
  if (rep.status != 0) {
    logf('E', "Error getting health info svc : %s", rep.message.c_str());
    return out;
  }
  // GPUStateResponse{GPUState=1: GPUState{ID=1, UUID=2, Health=3, AssociatedWorkload=4, Device=5}}
  pb::scan(
      rep.body.data(), rep.body.size(),
      [&](int field, const char* p, size_t n) {
        if (field != 1) return true;
        std::string health, device;
        pb::scan(
            p, n,
            [&](int f, const char* q, size_t m) {
              if (f == 3) health.assign(q, m);
              if (f == 5) device.assign(q, m);
              return true;
            },
            [](int, uint64_t) { return true; });
        if (!device.empty()) out[device] = to_lower(trim(health)) == "healthy";
        return true;
      },
      [](int, uint64_t) { return true; });
  return out;
}

bool set_health(Resource& r, const std::string& id, bool ok) {
  auto it = r.health.find(id);
  const bool prev = it == r.health.end() || it->second;
  r.health[id] = ok;
  if (prev == ok) return false;
  logf('W', "device %s: %s -> %s", id.c_str(), prev ? "Healthy" : "Unhealthy", ok ? "Healthy" : "Unhealthy");
  return true;
}

// one health pass; true when a verdict changed
bool refresh_health(Resource& r, const Flags& f, const std::map<std::string, bool>& exporter) {
  bool changed = false;
  if (r.driver == Driver::Vf) {
    // gim gone -> every group Unhealthy; else a group is Unhealthy if any parent PF is (amdgpu_sriov.go:217-308)
    const bool gim = is_dir(path_join(f.sysfs_root, "bus/pci/drivers/gim"));
    for (const auto& g : r.group_ids) {
      bool ok = gim;
      for (const auto& fn : r.groups.at(g)) {
        auto e = exporter.find(fn.pf);
        if (e != exporter.end() && !e->second) ok = false;
      }
      changed |= set_health(r, g, ok);
    }
    return changed;
  }
  if (r.driver == Driver::Pf) {  // vfio-pci present -> Healthy (amdgpu_pf.go:210-229)
    const bool vfio = is_dir(path_join(f.sysfs_root, "bus/pci/drivers/vfio-pci"));
    for (const auto& g : r.group_ids) changed |= set_health(r, g, vfio);
    return changed;
  }
  for (const auto& d : r.devices) {
    bool ok = kfd_node_live(f.sysfs_root, d);
    auto e = exporter.find(d.bdf);
    if (e != exporter.end() && !e->second) ok = false;
    auto it = r.health.find(d.id);
    const bool prev = it == r.health.end() || it->second;
    if (prev != ok) {
      logf('W', "device %s: %s -> %s", d.id.c_str(), prev ? "Healthy" : "Unhealthy", ok ? "Healthy" : "Unhealthy");
      changed = true;
    }
    r.health[d.id] = ok;
  }
  return changed;
}

volatile sig_atomic_t g_stop = 0;
int g_sig_pipe[2] = {-1, -1};

void on_signal(int) {
  g_stop = 1;
  const char b = 1;
  if (g_sig_pipe[1] >= 0 && ::write(g_sig_pipe[1], &b, 1) < 0) {
  }
}

}  // namespace

int main(int argc, char** argv) {
  Flags f;
  std::string err;
  if (!parse_flags(argc, argv, &f, &err)) {
    logf('E', "%s", err.c_str());
    return 1;
  }
  logf('I', "AMD GPU device plugin for Kubernetes (MI355X-native, native daemon)");
  if (::pipe(g_sig_pipe) != 0) return 1;
  ::fcntl(g_sig_pipe[0], F_SETFL, O_NONBLOCK);
  ::fcntl(g_sig_pipe[1], F_SETFL, O_NONBLOCK);
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGQUIT, &sa, nullptr);
  signal(SIGPIPE, SIG_IGN);

  std::vector<Resource> resources;
  KfdTopology topo;
  // one driver's resources; "" on success (an empty list = no devices), else the init error
  auto init_container = [&](std::vector<Resource>* out) -> std::string {
    if (!is_dir(path_join(f.sysfs_root, "class/kfd"))) return "No kfd found (" + f.sysfs_root + "/class/kfd)";
    topo = KfdTopology::load_sysfs(f.sysfs_root);
    const DiscoveryResult res = discover_gpus(f.sysfs_root, topo);
    for (const auto& w : res.warnings) logf('W', "%s", w.c_str());
    logf('I', "Found %zu AMDGPUs", res.devices.size());
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
    const auto exporter = exporter_health(f.exporter_socket);
    for (const auto& name : names) {
      Resource r;
      r.name = name;
      for (const auto& d : res.devices)
        if (homogeneous || d.partition_type() == name) r.devices.push_back(d);
      r.socket = path_join(f.kubelet_dir, std::string(kResourceNamespace) + "_" + name);
      refresh_health(r, f, exporter);
      prepare(r, topo, unresolved);
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
    logf('I', "Found %zu %s IOMMU groups", scan.groups.size(), vf ? "vf-passthrough" : "pf-passthrough");
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
    refresh_health(r, f, exporter_health(vf ? f.exporter_socket : ""));
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
      logf('E', "Error instantiating driver type %s: %s", f.driver_type.c_str(), e.c_str());
      return 1;
    }
  } else {
    // container -> VF -> PF; the reference starts its manager even when none initialised, and idles
    for (const char* type : {"container", "vf-passthrough", "pf-passthrough"}) {
      std::vector<Resource> got;
      const std::string e = init_driver(type, &got);
      if (!e.empty()) {
        logf('W', "%s implementation failed: %s. Trying next...", type, e.c_str());
        continue;
      }
      if (got.empty()) {
        logf('W', "%s implementation found no devices. Trying next...", type);
        continue;
      }
      resources = std::move(got);
      break;
    }
  }

  const std::string kubelet_sock = path_join(f.kubelet_dir, "kubelet.sock");
  DirWatcher watch;
  const std::string werr = watch.open(f.kubelet_dir);
  if (!werr.empty()) logf('W', "no inotify watch on %s (%s): polling every second", f.kubelet_dir.c_str(), werr.c_str());
  auto try_register = [&](Resource& r) {
    r.registered = register_with_kubelet(r, kubelet_sock, f.register_timeout_s);
    r.next_register = std::chrono::steady_clock::now() + std::chrono::milliseconds(r.retry_ms);
    r.retry_ms = r.registered ? 100 : std::min(2 * r.retry_ms, 3000);
  };
  auto start_all = [&] {
    for (auto& r : resources) {
      stop_server(r);
      r.retry_ms = 100;
      if (start_server(r)) try_register(r);
    }
  };
  if (path_exists(kubelet_sock)) start_all();

  using clk = std::chrono::steady_clock;
  auto next_pulse = clk::now() + std::chrono::seconds(f.pulse > 0 ? f.pulse : 3600);
  bool sock_present = path_exists(kubelet_sock);
  while (!g_stop) {
    pollfd pfd[2] = {{g_sig_pipe[0], POLLIN, 0}, {watch.fd(), POLLIN, 0}};
    const int nfd = watch.fd() >= 0 ? 2 : 1;
    auto wait_ms = std::chrono::duration_cast<std::chrono::milliseconds>(next_pulse - clk::now()).count();
    if (watch.fd() < 0) wait_ms = std::min<long long>(wait_ms, 1000);
    for (const auto& r : resources)
      if (r.server && !r.registered)
        wait_ms = std::min<long long>(
            wait_ms, std::chrono::duration_cast<std::chrono::milliseconds>(r.next_register - clk::now()).count() + 1);
    ::poll(pfd, nfd, static_cast<int>(std::max<long long>(0, wait_ms)));
    if (g_stop) break;
    bool kubelet_event = false;
    if (nfd == 2 && (pfd[1].revents & POLLIN)) {
      for (const auto& [name, mask] : watch.read_events())
        if (name == "kubelet.sock" || name.empty()) kubelet_event = true;
    }
    const bool present = path_exists(kubelet_sock);
    if (kubelet_event || present != sock_present) {
      if (present) {
        logf('I', "kubelet socket (re)created; restarting plugin servers and re-registering");
        start_all();
      } else if (sock_present) {
        logf('I', "kubelet socket removed; stopping plugin servers");
        for (auto& r : resources) stop_server(r);
      }
      sock_present = present;
    }
    // registrations that failed (kubelet not serving yet): retry, rate-limited
    for (auto& r : resources)
      if (r.server && !r.registered && present && clk::now() >= r.next_register) try_register(r);
    if (f.pulse > 0 && clk::now() >= next_pulse) {
      next_pulse = clk::now() + std::chrono::seconds(f.pulse);
      const auto exporter = exporter_health(f.exporter_socket);
      for (auto& r : resources) {
        const bool changed = refresh_health(r, f, exporter);
        if (changed || f.send_every_pulse) {
          r.list = list_bytes(r);
          r.service->set_device_list(r.list);
          if (r.server) r.server->broadcast(rpc::DevicePluginService::path("ListAndWatch"), r.list);
        }
      }
    }
  }
  logf('I', "Received signal, shutting down.");
  for (auto& r : resources) stop_server(r);
  return 0;
}
