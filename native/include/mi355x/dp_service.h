// v1beta1.DevicePlugin on the native gRPC server.
//
// Reference semantics: AMDGPUPlugin (internal/pkg/plugin/plugin.go:132-186),
// the container DeviceImpl's Allocate / GetPreferredAllocation
// (internal/pkg/amdgpu/amdgpu.go:255-319) and the wire contract
// (vendor/k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto). Error
// strings match the reference's (GetPreferredAllocation:
// "unable to get preferred allocation list. Error:...", amdgpu.go:310-311).
//
// The kubelet's admission RPCs are answered without entering Python:
//   GetPreferredAllocation  protobuf decode -> HiveAllocator -> encode
//   Allocate                per-device response fragments prepared by the
//                           plugin (DeviceSpecs, CDI devices, annotation names)
//   GetDevicePluginOptions  bytes prepared by the plugin
//   ListAndWatch            first message = the current list (prepared bytes),
//                           later lists pushed by the plugin on health changes
//   PreStartContainer       empty response, or (with a gate) the answer of a
//                           check of the devices that runs off the I/O thread
// Whatever has no prepared state (allocator disabled, Allocate mounts that
// are created per request, tracing) goes to a fallback: the Python servicer.
// Every call leaves an event (timing, allocator outcome, allocated IDs) in a
// queue signalled through an eventfd, so logs and metrics stay in Python, off
// the RPC path.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <unordered_map>
#include <vector>

#include "mi355x/allocator.h"
#include "mi355x/grpc_server.h"

namespace mi355x::rpc {

// Allocate fast path: every ContainerAllocateResponse is
//   container_prefix + per_device[id] for each requested id (request order)
//   + (at least one id) container_extra(ids)   (per-request fields, e.g. a topology-view mount)
//   + (at least one id) container_nonempty
//   + (annotation_key set) annotations{annotation_key: join(annotation_names[id], ",")}
//   + (env_key set, at least one id) envs{env_key: join(env_values[id], ",")}
//     (passthrough: PCI_RESOURCE_AMD_COM_<RES> = the BDFs of every requested group)
// as raw protobuf field bytes; an unknown ID is an INVALID_ARGUMENT error.
struct AllocateTemplate {
  std::string resource;  // for error messages
  std::string container_prefix;
  std::unordered_map<std::string, std::string> per_device;
  std::function<std::string(const std::vector<std::string>& ids)> container_extra;  // optional; runs on the server thread
  std::string container_nonempty;  // e.g. the node-view mounts of a container that got devices
  std::string annotation_key;
  std::unordered_map<std::string, std::string> annotation_names;
  std::string env_key;
  std::unordered_map<std::string, std::string> env_values;
};

struct RpcEvent {
  std::string rpc;
  int status = 0;
  std::string message;
  uint64_t t0_ns = 0;   // CLOCK_MONOTONIC
  uint64_t dur_ns = 0;
  bool native = true;   // false: served by the fallback
  // GetPreferredAllocation (last container request) / Allocate
  int candidates = -1;
  bool short_circuit = false;
  int weight = -1;
  double alloc_us = 0;
  uint64_t alloc_t0_ns = 0;
  std::vector<std::string> ids;  // chosen (preferred) / allocated IDs, all containers
};

class DevicePluginService {
 public:
  using Fallback = std::function<Reply(const std::string& method, const std::string& request)>;
  // PreStartContainer(devices_ids): called on the I/O thread; must hand the
  // check to another thread and call done(reply) from there exactly once
  using PreStartGate = std::function<void(std::vector<std::string> ids, std::function<void(Reply)> done)>;

  DevicePluginService();
  ~DevicePluginService();

  // Routes /v1beta1.DevicePlugin/* on `srv` (before srv.start()).
  void attach(GrpcServer& srv);
  // Before `srv` stops: a gate answer that arrives later is dropped (the
  // server has answered the call UNAVAILABLE) instead of reaching another server.
  void detach();
  // nullptr (default): PreStartContainer answers at once, as the reference's no-op
  void set_prestart_gate(PreStartGate g);

  // The fallback is fixed before the server starts.
  void set_fallback(Fallback f);
  void set_options(std::optional<std::string> bytes);
  void set_allocator(std::shared_ptr<const HiveAllocator> a);
  void set_allocate_template(std::optional<AllocateTemplate> t);
  void set_device_list(std::optional<std::string> bytes);
  // route everything to the fallback (e.g. while tracing)
  void set_native_enabled(bool on);

  std::vector<RpcEvent> drain_events();
  int event_fd() const { return evfd_; }
  static const char* path(const char* method);

 private:
  Reply preferred(const std::string& req, RpcEvent* ev);
  Reply allocate(const std::string& req, RpcEvent* ev);
  Reply fallback(const char* method, const std::string& req, RpcEvent* ev);
  void record(RpcEvent ev);
  void notify();  // eventfd, if events were recorded since the last call (I/O thread, after the writes)

  // where a deferred PreStartContainer answer goes: the server attached when
  // the call arrived (a new sink per attach; detach() / the destructor clear it)
  struct Sink {
    std::mutex mu;
    GrpcServer* srv = nullptr;
  };
  std::optional<Reply> prestart(uint64_t call_id, const std::string& req);

  mutable std::mutex mu_;
  std::shared_ptr<Sink> sink_;
  std::shared_ptr<const PreStartGate> gate_;
  std::shared_ptr<const Fallback> fallback_;
  std::shared_ptr<const std::string> options_;
  std::shared_ptr<const HiveAllocator> alloc_;
  std::shared_ptr<const AllocateTemplate> tmpl_;
  std::shared_ptr<const std::string> list_;
  bool native_ = true;

  std::mutex ev_mu_;
  std::vector<RpcEvent> events_;
  std::atomic<bool> notify_pending_{false};
  int evfd_ = -1;
};

// ---- minimal protobuf wire format (device-plugin messages) ----------------
namespace pb {
void put_varint(std::string* out, uint64_t v);
void put_tag(std::string* out, int field, int wire);
void put_bytes(std::string* out, int field, const std::string& v);
void put_bool(std::string* out, int field, bool v);
// Parses a message's length-delimited / varint fields in order: calls
// on_bytes(field, data, len) and on_varint(field, value). false = malformed.
bool scan(const char* p, size_t n, const std::function<bool(int, const char*, size_t)>& on_bytes,
          const std::function<bool(int, uint64_t)>& on_varint);
}  // namespace pb

}  // namespace mi355x::rpc
