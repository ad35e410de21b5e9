// The device-plugin server as the native daemon runs it, for the server-side
// fuzz targets: devices discovered from a generated MI355X sysfs tree
// ($MI355X_FUZZ_SYSFS, CPX: 64 devices in 8 physical GPUs), the hive
// allocator over its kfd topology, Allocate fragments per device, options and
// the ListAndWatch list, on a Unix socket in the scratch directory.
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "fuzz_common.h"
#include "mi355x/allocator.h"
#include "mi355x/dp_service.h"
#include "mi355x/gpu_discovery.h"
#include "mi355x/grpc_server.h"
#include "mi355x/kfd_topology.h"

namespace mi355x::fuzz {

struct DpServer {
  std::string sock;
  std::vector<std::string> ids;
  std::unique_ptr<rpc::GrpcServer> server;
  std::unique_ptr<rpc::DevicePluginService> service;
};

inline std::string device_spec(const std::string& path) {
  std::string s;
  rpc::pb::put_bytes(&s, 1, path);
  rpc::pb::put_bytes(&s, 2, path);
  rpc::pb::put_bytes(&s, 3, "rw");
  return s;
}

inline DpServer& dp_server() {
  static DpServer* srv = [] {
    auto* d = new DpServer;
    const std::string root = env_or_die("MI355X_FUZZ_SYSFS");
    const KfdTopology topo = KfdTopology::load_sysfs(root);
    const DiscoveryResult res = discover_gpus(root, topo);
    if (res.devices.empty()) fail("no devices under", root);
    std::vector<AllocDevice> ad;
    rpc::AllocateTemplate t;
    t.resource = "gpu";
    rpc::pb::put_bytes(&t.container_prefix, 3, device_spec("/dev/kfd"));
    std::string list;
    for (const auto& g : res.devices) {
      d->ids.push_back(g.id);
      AllocDevice a;
      a.id = g.id;
      a.node_id = g.node_id;
      a.numa_node = g.numa_node;
      a.unique_id = !g.unique_id.empty() ? g.unique_id : "bdf:" + g.bdf;
      a.hive_id = g.hive_id;
      ad.push_back(a);
      std::string frag;
      rpc::pb::put_bytes(&frag, 3, device_spec("/dev/dri/card" + std::to_string(g.card)));
      rpc::pb::put_bytes(&frag, 3, device_spec("/dev/dri/renderD" + std::to_string(g.render_minor)));
      t.per_device[g.id] = frag;
      std::string dev;
      rpc::pb::put_bytes(&dev, 1, g.id);
      rpc::pb::put_bytes(&dev, 2, "Healthy");
      rpc::pb::put_bytes(&list, 1, dev);
    }
    // a per-request field as the topology view adds (runs on the server thread)
    t.container_extra = [](const std::vector<std::string>& ids) {
      std::string m;
      rpc::pb::put_bytes(&m, 1, "/sys/class/kfd/kfd/topology");
      rpc::pb::put_bytes(&m, 2, "/view/" + std::to_string(ids.size()));
      std::string out;
      rpc::pb::put_bytes(&out, 2, m);
      return out;
    };
    AllocatorOptions opt;
    opt.extended_search_auto = true;
    opt.extended_node_limit = 200000;  // bounded per input, as the daemon's search is
    auto alloc = std::make_shared<HiveAllocator>();
    if (const std::string e = alloc->init(ad, topo, opt); !e.empty()) fail("allocator init", e);
    d->service = std::make_unique<rpc::DevicePluginService>();
    d->server = std::make_unique<rpc::GrpcServer>();
    std::string options;
    rpc::pb::put_bool(&options, 2, true);
    d->service->set_options(options);
    d->service->set_allocator(alloc);
    d->service->set_allocate_template(t);
    d->service->set_device_list(list);
    // PreStartContainer through a gate, as -prestart_liveness runs it: every other
    // check answers at once on the I/O thread, the rest from a thread of their own
    d->service->set_prestart_gate([](std::vector<std::string>, std::function<void(rpc::Reply)> done) {
      static std::atomic<uint64_t> n{0};
      if (n++ % 2 == 0) return done(rpc::Reply{});
      std::thread([done = std::move(done)] { done(rpc::Reply{}); }).detach();
    });
    d->service->attach(*d->server);
    d->sock = scratch_dir() + "/amd.com_gpu";
    if (const std::string e = d->server->start(d->sock); !e.empty()) fail("server start", e);
    return d;
  }();
  return *srv;
}

// one well-formed call on a fresh connection: the server must still serve
inline void check_server_alive(const char* after) {
  rpc::GrpcClient c;
  if (const std::string e = c.connect(dp_server().sock, 5.0); !e.empty()) fail("server unreachable after", after);
  const rpc::Reply r = c.unary(rpc::DevicePluginService::path("GetDevicePluginOptions"), "", 5.0);
  if (r.status != 0) fail("GetDevicePluginOptions failed after", std::string(after) + ": " + r.message);
  std::string want;
  rpc::pb::put_bool(&want, 2, true);
  if (r.body != want) fail("GetDevicePluginOptions body changed after", after);
}

}  // namespace mi355x::fuzz
