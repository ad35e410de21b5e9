#include "resources.h"

#include <unistd.h>

#include <algorithm>
#include <cctype>

#include "mi355x/cdi.h"
#include "mi355x/constants.h"
#include "mi355x/glog.h"
#include "mi355x/metrics.h"
#include "mi355x/sysfs.h"
#include "../kube/json.h"
#include "../kube/yaml.h"

namespace mi355x::daemon {
namespace pb = mi355x::rpc::pb;

const char* driver_name(Driver d) {
  return d == Driver::Container ? "container" : d == Driver::Vf ? "vf-passthrough" : "pf-passthrough";
}

Driver driver_from_name(const std::string& n) {
  return n == "vf-passthrough" ? Driver::Vf : n == "pf-passthrough" ? Driver::Pf : Driver::Container;
}

namespace {

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

// Mount{container_path=1, host_path=2, read_only=3}, as ContainerAllocateResponse.mounts (2)
std::string mount_field(const std::string& host, const std::string& ctr) {
  std::string m, out;
  pb::put_bytes(&m, 1, ctr);
  pb::put_bytes(&m, 2, host);
  pb::put_bool(&m, 3, true);
  pb::put_bytes(&out, 2, m);
  return out;
}

// the container DeviceImpl's Start/GetOptions/Allocate state (amdgpu.go:90-119,165-177,255-297)
void prepare(Resource& r, const KfdTopology& topo, const std::set<std::string>& unresolved, const std::string& search,
             const cdi::Strategies& lists, const ServeCtx& vc) {
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
  if (vc.prestart) pb::put_bool(&r.options, 1, true);  // pre_start_required
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
  r.service->set_prestart_gate(vc.prestart);
  if (r.allocator) r.service->set_allocator(r.allocator);
  r.service->set_allocate_template(t);
  r.tmpl = t;
  r.list = list_bytes(r);
  r.service->set_device_list(r.list);
}

// passthrough resources: no preferred allocation, vfio Allocate template (amdgpu_sriov.go:150-204, amdgpu_pf.go:146-197)
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

std::set<std::string> split_ids(const std::string& csv) {
  std::set<std::string> out;
  for (size_t a = 0; a <= csv.size();) {
    size_t b = csv.find(',', a);
    if (b == std::string::npos) b = csv.size();
    if (b > a) out.insert(csv.substr(a, b - a));
    a = b + 1;
  }
  return out;
}

}  // namespace

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

// AMD_GPU_DEVICE_COUNT, else gpu.device_count of the -config file: advertise
// the devices of the first N physical GPUs (documented by the reference,
// docs/user-guide/configuration.md:11,45-91, never implemented there; the
// Python CLI's topology.device_count_limit_from_env)
int device_count_limit(const std::string& config, std::string* err) {
  if (const char* e = std::getenv("AMD_GPU_DEVICE_COUNT"); e && *e) {  // surrounding blanks ignored
    char* end = nullptr;
    const long n = std::strtol(e, &end, 10);
    while (std::isspace(static_cast<unsigned char>(*end))) ++end;
    if (end != e && !*end && n >= 0) return static_cast<int>(n);
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

// NewGPUKFDImpl + Init + GetResourceNames (amdgpu.go:56-162)
std::string init_container(const Flags& f, int dev_limit, const ServeCtx& vc, NodeInventory* out) {
  out->driver = Driver::Container;
  if (!is_dir(path_join(f.sysfs_root, "class/kfd"))) return "No kfd found (" + f.sysfs_root + "/class/kfd)";
  out->topo = KfdTopology::load_sysfs(f.sysfs_root);
  DiscoveryResult res = discover_gpus(f.sysfs_root, out->topo);
  res.devices = limit_physical(res.devices, dev_limit);
  if (!f.device_ids.empty()) {  // -device_ids: a node shared between plugin instances, or GPUs held back
    std::set<std::string> want = split_ids(f.device_ids);
    std::vector<GpuDevice> kept;
    for (const auto& d : res.devices)
      if (want.erase(d.id)) kept.push_back(d);
    for (const auto& id : want) MI_LOG(kWarning, "-device_ids: %s is not a discovered device", id.c_str());
    res.devices = std::move(kept);
  }
  for (const auto& w : res.warnings) MI_LOG(kWarning, "%s", w.c_str());
  out->warnings = res.warnings;
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
  out->container_devices.clear();
  for (const auto& name : names) {
    Resource r;
    r.name = name;
    for (const auto& d : res.devices)
      if (homogeneous || d.partition_type() == name) {
        r.devices.push_back(d);
        out->container_devices.push_back(d);
      }
    r.socket = path_join(f.kubelet_dir, std::string(kResourceNamespace) + "_" + name);
    prepare(r, out->topo, unresolved, f.allocator_search, f.lists, vc);
    out->resources.push_back(std::move(r));
  }
  return "";
}

// NewGPUVFImpl / NewGPUPFImpl + Init + GetResourceNames (amdgpu_sriov.go:71-110, amdgpu_pf.go:67-106)
std::string init_passthrough(const Flags& f, Driver drv, NodeInventory* out) {
  out->driver = drv;
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
  out->resources.push_back(std::move(r));
  return "";
}

std::string init_driver(const Flags& f, Driver drv, int dev_limit, const ServeCtx& vc, NodeInventory* out) {
  if (drv == Driver::Container) return init_container(f, dev_limit, vc, out);
  return init_passthrough(f, drv, out);
}

// ---- ResourceRegistry ----------------------------------------------------------
void ResourceRegistry::adopt(std::vector<Resource> rs) {
  rs_ = std::move(rs);
  for (auto& r : rs_) r.reg = Registration(policy_);
}

bool ResourceRegistry::start_server(size_t i, Clock::time_point now) {
  Resource& r = rs_.at(i);
  stop_server(i);
  r.server = std::make_unique<rpc::GrpcServer>();
  r.service->attach(*r.server);
  const std::string err = r.server->start(r.socket);
  if (!err.empty()) {
    MI_LOG(kError, "%s: could not serve on %s: %s", r.name.c_str(), r.socket.c_str(), err.c_str());
    r.server.reset();
    return false;
  }
  r.reg.server_started(++server_seq_, now);
  MI_LOG(kInfo, "%s: serving on %s", r.name.c_str(), r.socket.c_str());
  return true;
}

void ResourceRegistry::stop_server(size_t i) {
  Resource& r = rs_.at(i);
  if (r.server) {
    if (r.service) r.service->detach();  // a PreStartContainer answer still on its way is dropped
    r.server->stop(0.5);
    r.server.reset();
    ::unlink(r.socket.c_str());
  }
  r.reg.server_stopped();
}

void ResourceRegistry::stop_all() {
  for (size_t i = 0; i < rs_.size(); ++i) stop_server(i);
}

std::vector<bool> ResourceRegistry::apply_health(const std::map<std::string, bool>& h) {
  std::vector<bool> changed(rs_.size(), false);
  for (size_t i = 0; i < rs_.size(); ++i) {
    Resource& r = rs_[i];
    auto set = [&](const std::string& id) {
      auto it = h.find(id);
      if (it == h.end()) return;
      auto cur = r.health.find(id);
      const bool prev = cur == r.health.end() || cur->second;
      if (prev != it->second) changed[i] = true;
      r.health[id] = it->second;
    };
    for (const auto& d : r.devices) set(d.id);
    for (const auto& g : r.group_ids) set(g);
    if (changed[i]) {
      r.list = list_bytes(r);
      r.service->set_device_list(r.list);
    }
  }
  return changed;
}

void ResourceRegistry::reweight(const KfdTopology& topo, const std::string& search,
                                const std::vector<std::pair<std::string, std::string>>& degraded) {
  for (auto& r : rs_) {
    if (r.gone || !r.allocator) continue;
    std::string aerr;
    auto a = build_allocator(r.devices, topo, search, degraded, &aerr);
    if (!aerr.empty()) {
      MI_LOG(kError, "%s: allocator re-weighting failed: %s", r.name.c_str(), aerr.c_str());
      continue;
    }
    r.allocator = a;
    r.service->set_allocator(a);
  }
}

ReloadPlan ResourceRegistry::apply_reload(std::vector<Resource> fresh, bool ok, Clock::time_point now) {
  ReloadPlan plan;
  const std::string lw = rpc::DevicePluginService::path("ListAndWatch");
  if (!ok) {  // discovery failed: advertise nothing until it works again
    for (size_t i = 0; i < rs_.size(); ++i) {
      Resource& r = rs_[i];
      if (r.gone) continue;
      r.devices.clear();
      r.health.clear();
      r.allocator.reset();
      r.service->set_allocator(nullptr);
      r.list = list_bytes(r);
      r.service->set_device_list(r.list);
      if (r.server) r.server->broadcast(lw, r.list);
      plan.updated.push_back(i);
    }
    return plan;
  }
  std::set<std::string> names;
  for (const auto& fr : fresh) names.insert(fr.name);
  for (size_t i = 0; i < rs_.size(); ++i) {
    Resource& r = rs_[i];
    if (!r.gone && !names.count(r.name)) {
      MI_LOG(kWarning, "resource %s no longer exists: stopping its plugin server", r.name.c_str());
      stop_server(i);
      r.gone = true;
      r.devices.clear();
      r.health.clear();
      plan.stopped.push_back(i);
    }
  }
  for (auto& fr : fresh) {
    auto it = std::find_if(rs_.begin(), rs_.end(), [&](const Resource& r) { return r.name == fr.name; });
    if (it != rs_.end() && !it->gone) {
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
      if (opts_changed && r.server) r.reg.force(now);  // kubelet reads the options at registration
      plan.updated.push_back(static_cast<size_t>(it - rs_.begin()));
      continue;
    }
    size_t i;
    fr.reg = Registration(policy_);
    if (it != rs_.end()) {
      *it = std::move(fr);
      i = static_cast<size_t>(it - rs_.begin());
    } else {
      rs_.push_back(std::move(fr));
      i = rs_.size() - 1;
    }
    MI_LOG(kInfo, "new resource %s (%zu devices)", rs_[i].name.c_str(), rs_[i].devices.size());
    plan.added.push_back(i);
  }
  return plan;
}

std::map<std::string, std::vector<GpuDevice>> ResourceRegistry::members() const {
  std::map<std::string, std::vector<GpuDevice>> out;
  for (const auto& r : rs_)
    if (!r.gone) out[r.name] = r.devices;
  return out;
}

}  // namespace mi355x::daemon
