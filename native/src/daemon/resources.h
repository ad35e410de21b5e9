// What the daemon advertises: one Resource per kubelet resource name, built
// from discovery (container driver: kfd topology + PCI sysfs; passthrough:
// IOMMU groups) and owned by the ResourceRegistry, which also owns each
// resource's gRPC server and DevicePlugin service.
//
// Reference: the container DeviceImpl (internal/pkg/amdgpu/amdgpu.go:68-345:
// Init, GetResourceNames, Enumerate, Allocate, GetPreferredAllocation), the VF
// and PF impls (amdgpu_sriov.go, amdgpu_pf.go) and the per-resource dpm server
// (vendored dpm/plugin.go:51-123).
#pragma once

#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "flags.h"
#include "registration.h"
#include "mi355x/allocator.h"
#include "mi355x/dp_service.h"
#include "mi355x/gpu_discovery.h"
#include "mi355x/grpc_server.h"
#include "mi355x/kfd_topology.h"
#include "mi355x/pci_scan.h"
#include "mi355x/views.h"

namespace mi355x::daemon {

enum class Driver { Container, Vf, Pf };
const char* driver_name(Driver d);
Driver driver_from_name(const std::string& name);  // container | vf-passthrough | pf-passthrough

// the opt-in container start-up views (mi355x/views.h)
// What a container resource's service gets from the daemon besides its devices:
// the start-up views its Allocate returns as mounts, and the PreStartContainer
// check (-prestart_liveness; set: the options ask kubelet for PreStartContainer)
struct ServeCtx {
  std::shared_ptr<views::NodeView> node;
  std::shared_ptr<views::TopologyViews> topo;
  rpc::DevicePluginService::PreStartGate prestart;
};

struct Resource {
  std::string name;  // "gpu", "cpx_nps1", "gpu_vf", ...
  Driver driver = Driver::Container;
  std::vector<GpuDevice> devices;          // container driver
  std::vector<std::string> group_ids;      // passthrough: IOMMU groups, numeric order
  IommuMap groups;                         // group -> PCI functions
  std::string socket;  // <kubelet_dir>/amd.com_<name>
  std::string options;  // serialized DevicePluginOptions
  rpc::AllocateTemplate tmpl;
  std::shared_ptr<const HiveAllocator> allocator;
  std::map<std::string, bool> health;  // device id -> healthy
  std::string list;                    // serialized ListAndWatchResponse
  bool gone = false;  // removed by a topology change: no server, no devices (the slot keeps indices stable)
  // serving state (ResourceRegistry)
  std::unique_ptr<rpc::GrpcServer> server;
  std::unique_ptr<rpc::DevicePluginService> service;
  Registration reg;
};

// ListAndWatchResponse{devices=1: Device{ID=1, health=2, topology=3}} from the resource's current health
std::string list_bytes(const Resource& r);
// the allocator's physical-GPU key of a device
std::string group_key(const GpuDevice& d);

// BestEffortPolicy.init over `devs`; `degraded`: xGMI pairs (group keys) scored as the worst link
std::shared_ptr<const HiveAllocator> build_allocator(const std::vector<GpuDevice>& devs, const KfdTopology& topo,
                                                     const std::string& search,
                                                     const std::vector<std::pair<std::string, std::string>>& degraded,
                                                     std::string* err);

// What discovery found for one driver.
struct NodeInventory {
  Driver driver = Driver::Container;
  std::vector<Resource> resources;
  KfdTopology topo;                           // container driver
  std::vector<GpuDevice> container_devices;   // every advertised container-mode device (health engine)
  std::vector<std::string> warnings;
};

// AMD_GPU_DEVICE_COUNT, else gpu.device_count of the -config file; -1 = no limit
int device_count_limit(const std::string& config, std::string* err);
std::vector<GpuDevice> limit_physical(const std::vector<GpuDevice>& devs, int limit);

// One driver's resources: "" on success (no resources = no devices), else the init error.
std::string init_container(const Flags& f, int dev_limit, const ServeCtx& vc, NodeInventory* out);
std::string init_passthrough(const Flags& f, Driver drv, NodeInventory* out);
std::string init_driver(const Flags& f, Driver drv, int dev_limit, const ServeCtx& vc, NodeInventory* out);

// What a topology reload changed (ResourceRegistry::apply_reload).
struct ReloadPlan {
  std::vector<size_t> stopped;   // resources that no longer exist (servers stopped, slots marked gone)
  std::vector<size_t> updated;   // kept resources with new devices / allocator / list
  std::vector<size_t> added;     // new resources: serve and register once their CDI specs exist
};

class ResourceRegistry {
 public:
  explicit ResourceRegistry(RegistrationPolicy p = {}) : policy_(p) {}

  std::vector<Resource>& all() { return rs_; }
  const std::vector<Resource>& all() const { return rs_; }
  size_t size() const { return rs_.size(); }
  Resource& at(size_t i) { return rs_.at(i); }
  bool empty() const { return rs_.empty(); }

  void adopt(std::vector<Resource> rs);
  // (re)start resource i's server on its socket; false (logged) when it cannot listen
  bool start_server(size_t i, Clock::time_point now);
  void stop_server(size_t i);
  void stop_all();

  // verdicts (device id -> healthy) into every resource; true for each resource whose list changed
  std::vector<bool> apply_health(const std::map<std::string, bool>& h);
  // every live resource's allocator re-weighted over `degraded`
  void reweight(const KfdTopology& topo, const std::string& search,
                const std::vector<std::pair<std::string, std::string>>& degraded);
  // the devices of a reload (fresh = init_container's resources): stops vanished
  // resources, updates kept ones in place (health kept per device), appends new
  // ones (not served yet); `ok` false = discovery failed: every resource
  // advertises no devices
  ReloadPlan apply_reload(std::vector<Resource> fresh, bool ok, Clock::time_point now);
  // resource name -> devices, for the CDI specs
  std::map<std::string, std::vector<GpuDevice>> members() const;

 private:
  RegistrationPolicy policy_;
  std::vector<Resource> rs_;
  uint64_t server_seq_ = 0;  // unique across slots: a Register answer names the server it was for
};

}  // namespace mi355x::daemon
