// C++ unit tests for the native core (ctest). Built plain and under
// -fsanitize=address,undefined / thread (MI355X_SANITIZE) — the reference has
// no race or sanitizer coverage at all.
//
//   test_core <repo testdata dir> [<reference testdata dir>]
//
// Reference fixtures are optional: missing => those cases are skipped.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#ifdef MI355X_TEST_HTTP
#include "../src/kube/http.h"
#endif
#include "../src/kube/labels.h"
#include "../src/rpc/hpack.h"
#include "flags.h"
#include "health_controller.h"
#include "registration.h"
#include "topology_watch.h"
#include "workers.h"
#include "mi355x/allocator.h"
#include "mi355x/cdi.h"
#include "mi355x/dp_service.h"
#include "mi355x/gpu_discovery.h"
#include "mi355x/grpc_server.h"
#include "mi355x/kfd_topology.h"
#include "mi355x/metrics.h"
#include "mi355x/pci_scan.h"
#include "mi355x/sysfs.h"

using namespace mi355x;

static int g_fail = 0, g_pass = 0, g_skip = 0;
#define CHECK(cond)                                                   \
  do {                                                                \
    if (cond) {                                                       \
      ++g_pass;                                                       \
    } else {                                                          \
      ++g_fail;                                                       \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                 \
  } while (0)

static std::vector<AllocDevice> synthetic_devices(int dev_count, int parts, int numa_count, int start, int end) {
  // mirrors the reference test-device generator semantics (device_test.go:43-67):
  // first partition of GPU i is "test<i+1>", the rest "amdgpu_xcp_<8i+j>"
  std::vector<AllocDevice> out;
  int node = start;
  for (int i = 0; i < dev_count; ++i) {
    int per_numa = dev_count / numa_count;
    for (int j = 0; j < parts; ++j) {
      if (node > end) break;
      std::string id = j == 0 ? "test" + std::to_string(i + 1) : "amdgpu_xcp_" + std::to_string(i * 8 + j);
      out.push_back(AllocDevice{id, node, i / per_numa, std::to_string(i), 0});
      ++node;
    }
  }
  return out;
}

static std::vector<std::string> ids_of(const std::vector<AllocDevice>& d) {
  std::vector<std::string> o;
  for (auto& x : d) o.push_back(x.id);
  return o;
}

static std::set<std::string> as_set(const std::vector<std::string>& v) { return {v.begin(), v.end()}; }

static void test_parsers(const std::string& ref) {
  auto kv = parse_kv_file(ref + "/topology-parsing/topology/nodes/2/properties");
  if (!kv) {
    ++g_skip;
    return;
  }
  CHECK(kv_i64(*kv, "simd_count", 0) == 256);
  CHECK(kv_i64(*kv, "simd_id_base", 0) == 2147487744LL);
  CHECK(kv->find("asdf") == kv->end());
  auto mb = parse_kv_file(ref + "/topology-parsing/topology/nodes/1/mem_banks/0/properties");
  CHECK(mb && kv_u64(*mb, "size_in_bytes", 0) == 17163091968ULL);
  auto t = KfdTopology::load(ref + "/topology-parsing/topology/nodes");
  CHECK(t.count_gpu_nodes() == 2);
  auto fw = parse_debugfs_firmware_info(ref + "/debugfs-parsing/amdgpu_firmware_info");
  CHECK(fw.feature.size() == 14 && fw.firmware.size() == 14);
  CHECK(fw.firmware["VCE"] == 0x352d0400u && fw.feature["MEC2"] == 33u);
  auto m = KfdTopology::load(ref + "/topology-parsing-mi308/topology/nodes");
  auto r2u = m.render_to_unique_id();
  CHECK(r2u.size() == 32);
  CHECK(r2u[128] == "598046273873802902" && r2u[187] == "6576958293045616595");
}

static void test_allocator_reference_contract(const std::string& ref) {
  auto topo = KfdTopology::load(ref + "/topo-mi300-cpx/topology/nodes");
  if (topo.nodes().empty()) {
    ++g_skip;
    return;
  }
  auto devs = synthetic_devices(8, 8, 2, 2, 64);
  HiveAllocator a;
  CHECK(a.init(devs, topo).empty());
  auto all = ids_of(devs);
  auto r = a.allocate(all, {}, 1);
  CHECK(r.error.empty() && r.ids == std::vector<std::string>{"test8"});
  r = a.allocate(all, {}, 8);
  CHECK(as_set(r.ids) == as_set({"test1", "amdgpu_xcp_1", "amdgpu_xcp_2", "amdgpu_xcp_3", "amdgpu_xcp_4",
                                 "amdgpu_xcp_5", "amdgpu_xcp_6", "amdgpu_xcp_7"}));
  r = a.allocate({"test3", "test4", "test5", "test6", "test7", "test8"}, {"test5"}, 3);
  CHECK(as_set(r.ids) == as_set({"test5", "test6", "test7"}));
  // exact search and the ordered BFS agree on every size
  for (int k = 1; k <= 40; k += 3) {
    auto e = a.allocate(all, {}, k);
    auto b = a.reference_allocate(all, {}, k);
    CHECK(e.error.empty() && b.error.empty());
    CHECK(e.weight == b.weight);
    CHECK(e.ids == b.ids);
  }
  // reentrancy: concurrent allocate() on a shared const allocator
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&] {
      for (int i = 0; i < 50; ++i)
        if (a.allocate(all, {}, 10).ids.size() != 10) ++bad;
    });
  for (auto& x : th) x.join();
  CHECK(bad == 0);
  // extended search: never heavier than the reference family, valid sets, concurrent-safe
  AllocatorOptions ext;
  ext.extended_search = true;
  HiveAllocator x;
  CHECK(x.init(devs, topo, ext).empty());
  for (int k = 1; k <= 62; k += 5) {
    auto e = x.allocate(all, {}, k);
    auto b = a.allocate(all, {}, k);
    CHECK(e.error.empty() && e.ids.size() == static_cast<size_t>(k) && e.weight <= b.weight);
  }
  std::vector<std::thread> th2;
  for (int t = 0; t < 4; ++t)
    th2.emplace_back([&] {
      for (int i = 0; i < 20; ++i)
        if (x.allocate(all, {"test2"}, 12).ids.size() != 12) ++bad;
    });
  for (auto& t : th2) t.join();
  CHECK(bad == 0);
}

static void test_errors() {
  KfdTopology empty;
  HiveAllocator a;
  CHECK(!a.init({}, empty).empty());
  CHECK(a.allocate({"a", "b"}, {}, 1).error == "Init method must be called before Allocate");
  auto devs = synthetic_devices(4, 1, 1, 2, 5);
  CHECK(a.init(devs, empty).empty());
  CHECK(a.allocate({"test1"}, {}, 0).error == "allocation size can not be negative");
  CHECK(a.allocate({"test1"}, {}, 2).error == "available devices count less than allocation size");
  CHECK(a.allocate({"test1", "test2"}, {"test1", "test2", "test3"}, 2).error ==
        "must_include devices size is more than allocation size");
  CHECK(a.allocate({"test1", "test2", "test3"}, {"test4"}, 2).error ==
        "No candidate subset found with matching criteria");
  auto r = a.allocate({"test1", "test2"}, {}, 2);
  CHECK(r.short_circuit && r.ids.size() == 2);
}

// xGMI link down at run time (AllocatorOptions::degraded_links): the pair
// scores as the worst link, so packing avoids it; the search and the
// reference BFS still agree on the re-weighted matrix.
static void test_degraded_links(const std::string& ref) {
  auto topo = KfdTopology::load(ref + "/topo-mi210-xgmi-pcie/nodes");
  if (topo.nodes().empty()) {
    ++g_skip;
    return;
  }
  auto devs = synthetic_devices(8, 1, 2, 1, 8);
  HiveAllocator a;
  CHECK(a.init(devs, topo).empty());
  auto all = ids_of(devs);
  auto before = a.allocate(all, {}, 2);
  CHECK(before.error.empty() && before.ids.size() == 2);
  // degrade the chosen pair (physical GPU keys = unique_id = GPU index here)
  AllocatorOptions opt;
  std::string ka, kb;
  for (auto& d : devs) {
    if (d.id == before.ids[0]) ka = d.unique_id;
    if (d.id == before.ids[1]) kb = d.unique_id;
  }
  opt.degraded_links = {{kb, ka}};  // order does not matter
  CHECK(a.init(devs, topo, opt).empty());
  auto after = a.allocate(all, {}, 2);
  CHECK(after.error.empty() && as_set(after.ids) != as_set(before.ids));
  CHECK(after.weight <= before.weight);  // another same-hive pair is as good
  auto forced = a.allocate(before.ids, {}, 2);  // only the degraded pair available
  CHECK(forced.short_circuit && as_set(forced.ids) == as_set(before.ids));
  for (int k = 2; k <= 7; ++k) {
    auto e = a.allocate(all, {}, k);
    auto b = a.reference_allocate(all, {}, k);
    CHECK(e.weight == b.weight);
  }
}

static std::string unhex(const char* h) {
  std::string o;
  for (size_t i = 0; h[i] && h[i + 1]; i += 2) o.push_back(static_cast<char>(std::stoi(std::string(h + i, 2), nullptr, 16)));
  return o;
}

static void test_hpack() {
  using namespace mi355x::rpc;
  CHECK(huffman_kraft_sum() == (1ull << 30));  // complete prefix code
  const char* vec[][2] = {{"www.example.com", "f1e3c2e5f23a6ba0ab90f4ff"},
                          {"no-cache", "a8eb10649cbf"},
                          {"custom-key", "25a849e95ba97d7f"},
                          {"custom-value", "25a849e95bb8e8b4bf"},
                          {"Mon, 21 Oct 2013 20:13:21 GMT", "d07abe941054d444a8200595040b8166e082a62d1bff"}};
  for (auto& v : vec) {
    std::string enc, dec;
    huffman_encode(v[0], &enc);
    CHECK(enc == unhex(v[1]));
    const std::string raw = unhex(v[1]);
    CHECK(huffman_decode(reinterpret_cast<const uint8_t*>(raw.data()), raw.size(), &dec) && dec == v[0]);
  }
  std::string junk;
  const uint8_t eos_pad[] = {0xff, 0xff, 0xff, 0xff};  // EOS in the string: invalid
  CHECK(!huffman_decode(eos_pad, sizeof(eos_pad), &junk));
  // RFC 7541 C.4: three requests sharing one dynamic table
  HpackDecoder dec;
  HeaderList hl;
  const std::string r1 = unhex("828684418cf1e3c2e5f23a6ba0ab90f4ff");
  CHECK(dec.decode(reinterpret_cast<const uint8_t*>(r1.data()), r1.size(), &hl));
  CHECK(hl.size() == 4 && hl[3].first == ":authority" && hl[3].second == "www.example.com");
  CHECK(dec.table_bytes() == 57);
  hl.clear();
  const std::string r2 = unhex("828684be5886a8eb10649cbf");
  CHECK(dec.decode(reinterpret_cast<const uint8_t*>(r2.data()), r2.size(), &hl));
  CHECK(hl.size() == 5 && hl[3].second == "www.example.com" && hl[4].first == "cache-control" &&
        hl[4].second == "no-cache");
  CHECK(dec.table_bytes() == 110);
  hl.clear();
  const std::string r3 = unhex("828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf");
  CHECK(dec.decode(reinterpret_cast<const uint8_t*>(r3.data()), r3.size(), &hl));
  CHECK(hl.size() == 5 && hl[2].second == "/index.html" && hl[4].first == "custom-key" &&
        hl[4].second == "custom-value");
  CHECK(dec.table_bytes() == 164);
  hl.clear();
  const std::string bad = unhex("8286bf");  // index 63 does not exist in a fresh table
  HpackDecoder fresh;
  CHECK(!fresh.decode(reinterpret_cast<const uint8_t*>(bad.data()), bad.size(), &hl));
}

// ---- raw HTTP/2 client for the native gRPC server --------------------------
namespace h2t {
std::string frame(uint8_t type, uint8_t flags, uint32_t sid, const std::string& p) {
  std::string f;
  f.push_back(static_cast<char>(p.size() >> 16));
  f.push_back(static_cast<char>(p.size() >> 8));
  f.push_back(static_cast<char>(p.size()));
  f.push_back(static_cast<char>(type));
  f.push_back(static_cast<char>(flags));
  for (int i = 3; i >= 0; --i) f.push_back(static_cast<char>(sid >> (8 * i)));
  return f + p;
}
std::string request(uint32_t sid, const std::string& path, const std::string& msg) {
  std::string h;
  mi355x::rpc::hpack_put_indexed(&h, 3);  // :method POST
  mi355x::rpc::hpack_put_indexed(&h, 6);  // :scheme http
  mi355x::rpc::hpack_put_literal(&h, 4, path);
  mi355x::rpc::hpack_put_literal(&h, 31, "application/grpc");
  mi355x::rpc::hpack_put_literal(&h, "te", "trailers");
  std::string body;
  body.push_back(0);
  for (int i = 3; i >= 0; --i) body.push_back(static_cast<char>(msg.size() >> (8 * i)));
  body += msg;
  return frame(1, 4, sid, h) + frame(0, 1, sid, body);
}
struct Result {
  int grpc_status = -1;
  std::string grpc_message;
  std::vector<std::string> messages;
};
// reads frames until END_STREAM on `sid`
bool read_call(int fd, uint32_t sid, Result* r, mi355x::rpc::HpackDecoder* dec, size_t max_messages = 100) {
  std::string buf, data;
  char tmp[4096];
  while (true) {
    while (buf.size() >= 9) {
      const auto* h = reinterpret_cast<const uint8_t*>(buf.data());
      const size_t len = (size_t(h[0]) << 16) | (size_t(h[1]) << 8) | h[2];
      if (buf.size() < 9 + len) break;
      const uint8_t type = h[3], flags = h[4];
      const uint32_t s = ((h[5] & 0x7f) << 24) | (h[6] << 16) | (h[7] << 8) | h[8];
      std::string p = buf.substr(9, len);
      buf.erase(0, 9 + len);
      if (s != sid) continue;
      if (type == 3) {  // RST_STREAM
        r->grpc_status = -2;
        return true;
      }
      if (type == 1) {
        mi355x::rpc::HeaderList hl;
        if (!dec->decode(reinterpret_cast<const uint8_t*>(p.data()), p.size(), &hl)) return false;
        for (auto& [k, v] : hl) {
          if (k == "grpc-status") r->grpc_status = std::atoi(v.c_str());
          if (k == "grpc-message") r->grpc_message = v;
        }
      } else if (type == 0) {
        data += p;
        while (data.size() >= 5) {
          const size_t n = (size_t(uint8_t(data[1])) << 24) | (size_t(uint8_t(data[2])) << 16) |
                           (size_t(uint8_t(data[3])) << 8) | uint8_t(data[4]);
          if (data.size() < 5 + n) break;
          r->messages.push_back(data.substr(5, n));
          data.erase(0, 5 + n);
          if (r->messages.size() >= max_messages) return true;
        }
      }
      if (flags & 1) return true;
    }
    const ssize_t n = ::read(fd, tmp, sizeof(tmp));
    if (n <= 0) return false;
    buf.append(tmp, static_cast<size_t>(n));
  }
}
int connect_unix(const std::string& path) {
  const int fd = ::socket(AF_UNIX, SOCK_STREAM, 0);
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  std::snprintf(a.sun_path, sizeof(a.sun_path), "%s", path.c_str());
  if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
    ::close(fd);
    return -1;
  }
  std::string pre = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n" + frame(4, 0, 0, "");
  if (::write(fd, pre.data(), pre.size()) != static_cast<ssize_t>(pre.size())) return -1;
  return fd;
}
}  // namespace h2t

static void test_grpc_server() {
  using namespace mi355x::rpc;
  char tmpl[] = "/tmp/mi355x-rpc-XXXXXX";
  const char* dir = ::mkdtemp(tmpl);
  if (!dir) {
    ++g_skip;
    return;
  }
  const std::string sock = std::string(dir) + "/dp.sock";
  GrpcServer srv;
  DevicePluginService svc;
  svc.attach(srv);
  svc.set_options(std::string("\x10\x01", 2));  // get_preferred_allocation_available
  AllocateTemplate t;
  t.resource = "gpu";
  t.per_device["a"] = "A";
  svc.set_allocate_template(t);
  svc.set_device_list(std::string("L0"));
  CHECK(srv.start(sock).empty());
  const int fd = h2t::connect_unix(sock);
  CHECK(fd >= 0);
  if (fd < 0) return;
  HpackDecoder dec;
  auto call = [&](uint32_t sid, const char* method, const std::string& msg, h2t::Result* r) {
    const std::string req = h2t::request(sid, std::string("/v1beta1.DevicePlugin/") + method, msg);
    return ::write(fd, req.data(), req.size()) == static_cast<ssize_t>(req.size()) && h2t::read_call(fd, sid, r, &dec);
  };
  h2t::Result r1;
  CHECK(call(1, "GetDevicePluginOptions", "", &r1) && r1.grpc_status == 0 && r1.messages.size() == 1 &&
        r1.messages[0] == std::string("\x10\x01", 2));
  std::string areq;  // AllocateRequest{container_requests{devices_ids: "a"}}
  {
    std::string c;
    pb::put_bytes(&c, 1, "a");
    pb::put_bytes(&areq, 1, c);
  }
  h2t::Result r2;
  CHECK(call(3, "Allocate", areq, &r2) && r2.grpc_status == 0 && r2.messages.size() == 1);
  if (r2.messages.size() == 1) CHECK(r2.messages[0] == std::string("\x0a\x01" "A", 3));
  std::string bad;
  {
    std::string c;
    pb::put_bytes(&c, 1, "zz");
    pb::put_bytes(&bad, 1, c);
  }
  h2t::Result r3;
  CHECK(call(5, "Allocate", bad, &r3) && r3.grpc_status == kInvalidArgument);
  h2t::Result r4;
  CHECK(call(7, "Nope", "", &r4) && r4.grpc_status == kUnimplemented);
  // ListAndWatch: the list, then broadcasts from another thread
  const std::string lw = h2t::request(9, DevicePluginService::path("ListAndWatch"), "");
  CHECK(::write(fd, lw.data(), lw.size()) == static_cast<ssize_t>(lw.size()));
  h2t::Result r5;
  CHECK(h2t::read_call(fd, 9, &r5, &dec, 1) && r5.messages.size() == 1 && r5.messages[0] == "L0");
  std::thread pusher([&] {
    for (int i = 1; i <= 20; ++i) {
      while (srv.broadcast(DevicePluginService::path("ListAndWatch"), "L" + std::to_string(i)) == 0)
        std::this_thread::yield();
    }
  });
  h2t::Result r6;
  CHECK(h2t::read_call(fd, 9, &r6, &dec, 20) && r6.messages.size() == 20 && r6.messages.back() == "L20");
  pusher.join();
  srv.stop(0.5);  // the open stream ends with OK trailers
  h2t::Result r7;
  CHECK(h2t::read_call(fd, 9, &r7, &dec) && r7.grpc_status == 0);
  CHECK(svc.drain_events().size() == 4);  // options, 2x Allocate, ListAndWatch (unknown methods are not service calls)
  ::close(fd);
  ::unlink(sock.c_str());
  ::rmdir(dir);
}

// PreStartContainer with a gate: the answer comes from another thread later;
// calls on the same connection are answered meanwhile; a stopping server
// answers a check still running UNAVAILABLE and drops its late answer.
static void test_grpc_deferred_prestart() {
  using namespace mi355x::rpc;
  char tmpl[] = "/tmp/mi355x-rpc-XXXXXX";
  const char* dir = ::mkdtemp(tmpl);
  if (!dir) {
    ++g_skip;
    return;
  }
  const std::string sock = std::string(dir) + "/dp.sock";
  GrpcServer srv;
  DevicePluginService svc;
  svc.attach(srv);
  svc.set_options(std::string("\x08\x01", 2));  // pre_start_required
  std::vector<std::thread> gates;
  std::mutex held_mu;
  std::vector<std::function<void(Reply)>> held;  // checks that finish only when the test says
  svc.set_prestart_gate([&](std::vector<std::string> ids, std::function<void(Reply)> done) {
    if (ids.size() == 1 && ids[0] == "hold") {
      std::lock_guard<std::mutex> lk(held_mu);
      held.push_back(std::move(done));
      return;
    }
    gates.emplace_back([ids, done = std::move(done)] {
      std::this_thread::sleep_for(std::chrono::milliseconds(200));
      done(ids[0] == "bad" ? Reply{kFailedPrecondition, "bad GPU", ""} : Reply{});
    });
  });
  CHECK(srv.start(sock).empty());
  const int fd = h2t::connect_unix(sock);
  CHECK(fd >= 0);
  if (fd < 0) return;
  HpackDecoder dec;
  auto req = [](const std::string& id) {
    std::string r;
    pb::put_bytes(&r, 1, id);
    return r;
  };
  auto send = [&](uint32_t sid, const char* method, const std::string& msg) {
    const std::string q = h2t::request(sid, DevicePluginService::path(method), msg);
    return ::write(fd, q.data(), q.size()) == static_cast<ssize_t>(q.size());
  };
  // a check in flight, and GetDevicePluginOptions on the next stream answered first
  CHECK(send(1, "PreStartContainer", req("a")) && send(3, "GetDevicePluginOptions", ""));
  std::vector<uint32_t> order;  // streams in the order they ended
  std::map<uint32_t, int> status;
  {
    std::string buf;
    char tmp[4096];
    while (order.size() < 2) {
      while (buf.size() >= 9) {
        const auto* f = reinterpret_cast<const uint8_t*>(buf.data());
        const size_t len = (size_t(f[0]) << 16) | (size_t(f[1]) << 8) | f[2];
        if (buf.size() < 9 + len) break;
        const uint32_t sid = ((f[5] & 0x7f) << 24) | (f[6] << 16) | (f[7] << 8) | f[8];
        if (f[3] == 1) {  // HEADERS: every block decoded in order
          HeaderList hl;
          CHECK(dec.decode(f + 9, len, &hl));
          for (auto& [k, v] : hl)
            if (k == "grpc-status") status[sid] = std::atoi(v.c_str());
        }
        if ((f[3] == 0 || f[3] == 1) && (f[4] & 1)) order.push_back(sid);
        buf.erase(0, 9 + len);
      }
      if (order.size() >= 2) break;
      const ssize_t n = ::read(fd, tmp, sizeof(tmp));
      if (n <= 0) break;
      buf.append(tmp, static_cast<size_t>(n));
    }
  }
  CHECK(order == (std::vector<uint32_t>{3, 1}) && status[3] == 0 && status[1] == 0);
  CHECK(send(5, "PreStartContainer", req("bad")));
  h2t::Result b;
  CHECK(h2t::read_call(fd, 5, &b, &dec) && b.grpc_status == kFailedPrecondition && b.grpc_message == "bad GPU");
  // a check that outlives the server: UNAVAILABLE at stop; its late answer goes nowhere
  CHECK(send(7, "PreStartContainer", req("hold")));
  for (int i = 0; i < 200; ++i) {
    {
      std::lock_guard<std::mutex> lk(held_mu);
      if (!held.empty()) break;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  svc.detach();
  srv.stop(0.5);
  h2t::Result h;
  CHECK(h2t::read_call(fd, 7, &h, &dec) && h.grpc_status == kUnavailable);
  {
    std::lock_guard<std::mutex> lk(held_mu);
    CHECK(held.size() == 1);
    for (auto& d : held) d(Reply{});  // after detach: dropped, nothing touches the stopped server
  }
  for (auto& t : gates) t.join();
  ::close(fd);
  ::unlink(sock.c_str());
  ::rmdir(dir);
}

// Random and mutated input for the HPACK decoder and the HTTP/2 frame parser:
// nothing may crash or hang (run under ASan/UBSan by the sanitizer ctest), and
// the server must keep answering a well-formed client afterwards.
static void test_fuzz_rpc(const std::string& ref) {
  using namespace mi355x::rpc;
  uint64_t x = 0x9E3779B97F4A7C15ull;
  auto rnd = [&x]() {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
  };
  const std::string valid[] = {unhex("828684418cf1e3c2e5f23a6ba0ab90f4ff"), unhex("828684be5886a8eb10649cbf"),
                               unhex("828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf")};
  int decoded = 0;
  for (int i = 0; i < 20000; ++i) {
    std::string b;
    if (i % 2) {
      b = valid[i % 3];
      for (int m = 0; m < 1 + static_cast<int>(rnd() % 4); ++m) b[rnd() % b.size()] = static_cast<char>(rnd());
    } else {
      b.resize(rnd() % 64);
      for (auto& c : b) c = static_cast<char>(rnd());
    }
    HpackDecoder dec(static_cast<size_t>(rnd() % 5000));
    HeaderList hl;
    decoded += dec.decode(reinterpret_cast<const uint8_t*>(b.data()), b.size(), &hl);
    std::string h;
    huffman_decode(reinterpret_cast<const uint8_t*>(b.data()), b.size(), &h);
  }
  CHECK(decoded > 0);

  char tmpl[] = "/tmp/mi355x-fuzz-XXXXXX";
  const char* dir = ::mkdtemp(tmpl);
  if (!dir) {
    ++g_skip;
    return;
  }
  const std::string sock = std::string(dir) + "/f.sock";
  GrpcServer srv;
  DevicePluginService svc;
  svc.attach(srv);
  svc.set_options(std::string("\x10\x01", 2));
  CHECK(srv.start(sock).empty());
  for (int i = 0; i < 300; ++i) {
    const int fd = h2t::connect_unix(sock);
    if (fd < 0) continue;
    std::string junk;
    // random frames after a valid preface: random type / flags / stream / payload
    for (int f = 0; f < 1 + static_cast<int>(rnd() % 6); ++f) {
      std::string p(rnd() % 80, '\0');
      for (auto& c : p) c = static_cast<char>(rnd());
      junk += h2t::frame(static_cast<uint8_t>(rnd() % 11), static_cast<uint8_t>(rnd()),
                         static_cast<uint32_t>(rnd() % 16), p);
    }
    if (::write(fd, junk.data(), junk.size()) < 0) {
    }
    ::shutdown(fd, SHUT_WR);
    char buf[4096];
    while (::read(fd, buf, sizeof(buf)) > 0) {
    }
    ::close(fd);
  }
  const int fd = h2t::connect_unix(sock);
  HpackDecoder dec;
  h2t::Result r;
  const std::string req = h2t::request(1, "/v1beta1.DevicePlugin/GetDevicePluginOptions", "");
  CHECK(fd >= 0 && ::write(fd, req.data(), req.size()) == static_cast<ssize_t>(req.size()) &&
        h2t::read_call(fd, 1, &r, &dec) && r.grpc_status == 0 && r.messages.size() == 1);
  // well-formed calls with random / mutated protobuf bodies: every one gets a
  // gRPC status (the allocator on the reference's MI300X CPX capture when present)
  auto topo = KfdTopology::load(ref + "/topo-mi300-cpx/topology/nodes");
  const auto devs = synthetic_devices(8, 8, 2, 2, 64);
  if (!topo.nodes().empty()) {
    auto a = std::make_shared<HiveAllocator>();
    CHECK(a->init(devs, topo).empty());
    svc.set_allocator(a);
  }
  AllocateTemplate t;
  t.resource = "gpu";
  for (const auto& d : devs) t.per_device[d.id] = "spec-" + d.id;
  svc.set_allocate_template(t);
  std::string pref_ok, alloc_ok;
  {
    std::string c;
    for (int i = 0; i < 12; ++i) pb::put_bytes(&c, 1, devs[i].id);
    pb::put_bytes(&c, 2, devs[3].id);
    pb::put_varint(&c, (3 << 3) | 0);
    pb::put_varint(&c, 4);
    pb::put_bytes(&pref_ok, 1, c);
    std::string ac;
    pb::put_bytes(&ac, 1, devs[0].id);
    pb::put_bytes(&ac, 1, devs[9].id);
    pb::put_bytes(&alloc_ok, 1, ac);
  }
  const char* methods[] = {"GetPreferredAllocation", "Allocate", "PreStartContainer", "GetDevicePluginOptions"};
  int answered = 0, ok_calls = 0;
  uint32_t sid = 3;
  for (int i = 0; i < 3000 && fd >= 0; ++i, sid += 2) {
    const int m = static_cast<int>(rnd() % 4);
    std::string body = m == 0 ? pref_ok : alloc_ok;
    switch (rnd() % 4) {
      case 0:
        break;  // valid
      case 1:   // a few random bytes changed
        for (int k = 0; k < 1 + static_cast<int>(rnd() % 3); ++k) body[rnd() % body.size()] = static_cast<char>(rnd());
        break;
      case 2:   // truncated
        body.resize(rnd() % body.size());
        break;
      default:  // random bytes
        body.assign(rnd() % 48, '\0');
        for (auto& ch : body) ch = static_cast<char>(rnd());
    }
    h2t::Result rr;
    const std::string q = h2t::request(sid, std::string("/v1beta1.DevicePlugin/") + methods[m], body);
    if (::write(fd, q.data(), q.size()) != static_cast<ssize_t>(q.size()) || !h2t::read_call(fd, sid, &rr, &dec)) break;
    answered += rr.grpc_status >= 0;
    ok_calls += rr.grpc_status == 0;
  }
  CHECK(answered == 3000);
  CHECK(ok_calls > 300);
  svc.drain_events();
  if (fd >= 0) ::close(fd);
  srv.stop(0.1);
  ::unlink(sock.c_str());
  ::rmdir(dir);
}


// ---- daemon parts (native/src/daemon): registration rules, watchdog, topology watch, sweeps
static rpc::ServerStats stats(uint64_t opened, uint64_t open, uint64_t perr, uint64_t caller_perr) {
  rpc::ServerStats st;
  st.streams_opened = opened;
  st.streams_open = open;
  st.protocol_errors = perr;
  st.caller_protocol_errors = caller_perr;
  return st;
}

static void test_registration_generations() {
  using daemon::Registration;
  using Outcome = daemon::Registration::Outcome;
  const auto t0 = daemon::Clock::now();
  auto ms = [&](int n) { return t0 + std::chrono::milliseconds(n); };
  daemon::RegistrationPolicy pol;
  pol.watchdog_s = 1.0;
  pol.reregister_s = 0.5;
  Registration r(pol);
  CHECK(!r.due(t0));                       // no server yet
  r.server_started(7, t0);
  CHECK(r.due(t0) && r.server_gen() == 7);
  r.begin(/*kubelet_gen=*/1, stats(0, 0, 0, 0));
  CHECK(r.inflight() && !r.due(t0));
  // an answer for an earlier server: ignored outright (stays in flight)
  CHECK(r.complete(6, 1, 1, true, ms(5)) == Outcome::kStale && r.inflight() && !r.registered());
  // an answer from the previous kubelet: in-flight ends, nothing registered, due again
  CHECK(r.complete(7, 1, 2, true, ms(5)) == Outcome::kStale && !r.inflight() && !r.registered() && r.due(ms(5)));
  // failures back off: 100 ms, doubling, capped at 3 s
  r.begin(2, stats(0, 0, 0, 0));
  CHECK(r.complete(7, 2, 2, false, ms(10)) == Outcome::kFailed);
  CHECK(!r.due(ms(100)) && r.due(ms(110)));
  int expect = 200;
  for (int i = 0; i < 8; ++i) {
    r.begin(2, stats(0, 0, 0, 0));
    r.complete(7, 2, 2, false, ms(10));
    CHECK(r.retry_ms() == std::min(expect * 2, 3000) || r.retry_ms() == 3000);
    expect = std::min(expect * 2, 3000);
  }
  // success resets the backoff
  r.begin(2, stats(0, 0, 0, 0));
  CHECK(r.complete(7, 2, 2, true, ms(20)) == Outcome::kRegistered && r.registered() && r.retry_ms() == 100);
  CHECK(r.registrations() == 1);
  // a server restart (new generation) makes the old answer stale and registers again
  r.server_started(8, ms(30));
  CHECK(!r.registered() && r.due(ms(30)));
  CHECK(r.complete(7, 2, 2, true, ms(31)) == Outcome::kStale);
  r.server_stopped();
  CHECK(!r.due(ms(40)));
}

static void test_registration_watchdog() {
  using daemon::Registration;
  const auto t0 = daemon::Clock::now();
  auto ms = [&](int n) { return t0 + std::chrono::milliseconds(n); };
  daemon::RegistrationPolicy pol;
  pol.watchdog_s = 1.0;
  pol.reregister_s = 0.5;
  {  // kubelet never lists: trips after watchdog_s, not before
    Registration r(pol);
    r.server_started(1, t0);
    r.begin(1, stats(3, 0, 0, 0));
    r.complete(1, 1, 1, true, ms(10));
    CHECK(r.armed() && r.observe(stats(3, 0, 0, 0), ms(900)).empty());
    CHECK(r.observe(stats(3, 0, 0, 0), ms(1100)).find("no ListAndWatch stream within 1s") != std::string::npos);
  }
  {  // kubelet opens ListAndWatch before its Register answer reaches us: counted (baseline at begin())
    Registration r(pol);
    r.server_started(1, t0);
    r.begin(1, stats(0, 0, 0, 0));
    CHECK(r.observe(stats(1, 1, 0, 0), ms(5)).empty() && r.list_seen());  // stream opened while in flight
    r.complete(1, 1, 1, true, ms(10));
    CHECK(r.observe(stats(1, 1, 0, 0), ms(5000)).empty() && !r.armed());
  }
  {  // stray clients (errors on connections without a call) never trip it; kubelet's connection does
    Registration r(pol);
    r.server_started(1, t0);
    r.begin(1, stats(0, 0, 5, 1));
    r.complete(1, 1, 1, true, ms(10));
    CHECK(r.observe(stats(0, 0, 9, 1), ms(100)).empty());
    CHECK(r.observe(stats(0, 0, 9, 2), ms(200)).find("kubelet's connection") != std::string::npos);
  }
  {  // after ListAndWatch: disarmed for good, even for errors on kubelet's connection
    Registration r(pol);
    r.server_started(1, t0);
    r.begin(1, stats(0, 0, 0, 0));
    r.complete(1, 1, 1, true, ms(10));
    CHECK(r.observe(stats(1, 1, 0, 0), ms(20)).empty() && r.list_seen());
    CHECK(r.observe(stats(1, 1, 4, 4), ms(30)).empty() && r.observe(stats(1, 1, 4, 4), ms(60000)).empty());
    // every stream closed for reregister_s: register again (once)
    CHECK(r.observe(stats(1, 0, 4, 4), ms(100)).empty() && r.registered());
    CHECK(r.observe(stats(1, 0, 4, 4), ms(400)).empty() && r.registered());
    CHECK(r.observe(stats(1, 0, 4, 4), ms(700)).empty() && !r.registered() && r.due(ms(700)));
    CHECK(r.reregistrations() == 1);
    // the new registration is watched again from its own baseline
    r.begin(1, stats(1, 0, 4, 4));
    r.complete(1, 1, 1, true, ms(710));
    CHECK(r.armed() && r.observe(stats(2, 1, 4, 4), ms(720)).empty() && r.list_seen());
  }
  {  // a stream that comes back in time cancels the re-registration
    Registration r(pol);
    r.server_started(1, t0);
    r.begin(1, stats(0, 0, 0, 0));
    r.complete(1, 1, 1, true, ms(10));
    r.observe(stats(1, 1, 0, 0), ms(20));
    r.observe(stats(1, 0, 0, 0), ms(100));
    r.observe(stats(2, 1, 0, 0), ms(300));
    CHECK(r.observe(stats(2, 1, 0, 0), ms(900)).empty() && r.registered() && r.reregistrations() == 0);
  }
  {  // -grpc_watchdog 0: never trips; poll deadlines stay sane
    daemon::RegistrationPolicy off = pol;
    off.watchdog_s = 0;
    Registration r(off);
    r.server_started(1, t0);
    r.begin(1, stats(0, 0, 0, 0));
    r.complete(1, 1, 1, true, ms(10));
    CHECK(r.observe(stats(0, 0, 3, 3), ms(100000)).empty() && !r.armed());
    CHECK(r.next_event(ms(10)) >= ms(10));
  }
}


// random event sequences against Registration: its invariants hold in every state
static void test_registration_random_sequences() {
  using daemon::Registration;
  daemon::RegistrationPolicy pol;
  pol.watchdog_s = 0.5;
  pol.reregister_s = 0.2;
  uint64_t seed = 0x9e3779b97f4a7c15ull;
  auto rnd = [&](uint64_t n) {
    seed ^= seed << 13;
    seed ^= seed >> 7;
    seed ^= seed << 17;
    return seed % n;
  };
  int bad = 0;
  for (int run = 0; run < 200; ++run) {
    Registration r(pol);
    auto now = daemon::Clock::now();
    uint64_t sgen = 0, kgen = 1, opened = 0, open = 0, caller = 0;
    bool tripped = false;
    std::vector<std::pair<uint64_t, uint64_t>> pending;  // (server gen, kubelet gen) of Registers in flight
    for (int step = 0; step < 300 && !tripped; ++step) {
      now += std::chrono::milliseconds(rnd(120));
      switch (rnd(9)) {
        case 0: r.server_started(++sgen, now); open = 0; break;
        case 1: r.server_stopped(); open = 0; break;
        case 2: ++kgen; break;
        case 3:
          if (r.due(now)) {
            r.begin(kgen, stats(opened, open, 0, caller));
            pending.emplace_back(sgen, kgen);
          }
          break;
        case 4:
          if (!pending.empty()) {
            const size_t k = rnd(pending.size());
            r.complete(pending[k].first, pending[k].second, kgen, rnd(4) != 0, now);
            pending.erase(pending.begin() + static_cast<long>(k));
          }
          break;
        case 5: ++opened; ++open; break;                 // kubelet opens a stream
        case 6: if (open) --open; break;                 // a stream ends
        case 7: if (rnd(8) == 0) ++caller; break;        // a protocol error on a calling connection
        case 8: r.force(now); break;
      }
      const bool was_seen = r.list_seen();
      const std::string why = r.observe(stats(opened, open, 0, caller), now);
      if (!why.empty()) {
        tripped = true;
        if (was_seen) ++bad;                              // never after ListAndWatch was seen
      }
      if (r.registered() && !r.serving()) ++bad;
      if (r.due(now) && (r.registered() || r.inflight() || !r.serving())) ++bad;
      if (r.armed() && r.list_seen()) ++bad;
      if (r.next_event(now) < now) ++bad;
    }
  }
  CHECK(bad == 0);
}

static void test_topology_watch() {
  daemon::TopologyWatch w("a");
  CHECK(!w.observe("a", true));
  CHECK(!w.observe("b", true));   // first sight of a new signature: wait one period
  CHECK(!w.observe("b", false));  // held, but a sweep is running: not now
  CHECK(w.observe("b", true));
  w.applied("b");
  CHECK(!w.observe("b", true) && w.current() == "b");
  CHECK(!w.observe("c", true) && !w.observe("d", true));  // still changing: nothing
  CHECK(w.observe("d", true));
}

// Go's flag package: syntax errors (exit 2) vs validateFlags (exit 1), the
// first non-flag argument or "--" ends parsing, an undefined flag is refused
// before it can take the next argument as its value
static void test_flags_go_semantics() {
  auto parse = [](std::vector<std::string> args, bool* syntax, std::string* err, daemon::Flags* out = nullptr) {
    args.insert(args.begin(), "k8s-device-plugin");
    std::vector<char*> argv;
    for (auto& a : args) argv.push_back(a.data());
    daemon::Flags f;
    bool help = false;
    const bool ok = daemon::parse_flags(static_cast<int>(argv.size()), argv.data(), &f, err, &help, syntax);
    if (out) *out = f;
    return ok;
  };
  bool syn = false;
  std::string err;
  daemon::Flags f;
  CHECK(parse({"-pulse=30", "--driver_type", "container", "-v=5", "-logtostderr"}, &syn, &err, &f) && f.pulse == 30 &&
        f.driver_type == "container" && f.log.v == 5);
  CHECK(!parse({"-nope", "-pulse=3"}, &syn, &err) && syn && err == "flag provided but not defined: -nope");
  CHECK(!parse({"-pulse", "x"}, &syn, &err) && syn && err.find("invalid value") == 0);
  CHECK(!parse({"-pulse"}, &syn, &err) && syn && err == "flag needs an argument: -pulse");
  CHECK(!parse({"-liveness=maybe"}, &syn, &err) && syn);
  CHECK(!parse({"---pulse=1"}, &syn, &err) && syn && err.find("bad flag syntax") == 0);
  CHECK(!parse({"-pulse=-1"}, &syn, &err) && !syn && err == "pulse must be a non-negative integer");
  CHECK(!parse({"-driver_type", "gim"}, &syn, &err) && !syn);
  CHECK(parse({"-pulse=2", "extra", "-nope"}, &syn, &err, &f) && f.pulse == 2);  // stops at "extra"
  CHECK(parse({"-pulse=2", "--", "-nope"}, &syn, &err, &f) && f.pulse == 2);
  CHECK(parse({"-pulse=2", "-", "-nope"}, &syn, &err, &f) && f.pulse == 2);      // "-" is an argument
  // strconv.ParseBool: an empty value is an error, not true
  CHECK(!parse({"-liveness="}, &syn, &err) && syn && err == "invalid boolean value \"\" for -liveness");
  CHECK(!parse({"-logtostderr="}, &syn, &err) && syn);
  CHECK(parse({"-liveness", "-pulse=1"}, &syn, &err, &f) && f.liveness);
  CHECK(parse({"-liveness=F", "-pulse=1"}, &syn, &err, &f) && !f.liveness);
  // strconv.ParseInt(s, 0, 64): base prefixes, leading-0 octal, '_' between digits, range
  CHECK(parse({"-pulse=0x1e"}, &syn, &err, &f) && f.pulse == 30);
  CHECK(parse({"-pulse=0o17"}, &syn, &err, &f) && f.pulse == 15);
  CHECK(parse({"-pulse=017"}, &syn, &err, &f) && f.pulse == 15);
  CHECK(parse({"-pulse=0b101"}, &syn, &err, &f) && f.pulse == 5);
  CHECK(parse({"-pulse=1_000"}, &syn, &err, &f) && f.pulse == 1000);
  CHECK(parse({"-pulse=+7"}, &syn, &err, &f) && f.pulse == 7);
  CHECK(parse({"-pulse=0"}, &syn, &err, &f) && f.pulse == 0);
  for (const char* badv : {"-pulse=08", "-pulse=1__0", "-pulse=_1", "-pulse=1_", "-pulse=0x", "-pulse=1.5",
                           "-pulse= 3", "-pulse=99999999999", "-pulse=9223372036854775808"})
    CHECK(!parse({badv}, &syn, &err) && syn && err.find("invalid value") == 0);
  // glog's -v: strconv.Atoi (64-bit) stored as an int32 (Level.Set, glog_flags.go:115-130), so
  // leading zeros are decimal, prefixes are refused, and 2^32 + 3 is level 3
  CHECK(parse({"-v=05"}, &syn, &err, &f) && f.log.v == 5);
  CHECK(!parse({"-v=0x5"}, &syn, &err) && syn);
  CHECK(parse({"-v=4294967299"}, &syn, &err, &f) && f.log.v == 3);
  CHECK(!parse({"-v=9223372036854775808"}, &syn, &err) && syn);
  // strconv.ParseFloat
  CHECK(parse({"-liveness_timeout=2.5e1"}, &syn, &err, &f) && f.liveness_timeout == 25.0);
  CHECK(!parse({"-liveness_timeout= 2"}, &syn, &err) && syn);
  CHECK(!parse({"-liveness_timeout=1e999"}, &syn, &err) && syn);
  // '_' right after a base prefix is Go literal syntax too (0x_1e); not before the prefix's digits end
  CHECK(parse({"-pulse=0x_1e"}, &syn, &err, &f) && f.pulse == 30);
  CHECK(parse({"-pulse=0b1_01"}, &syn, &err, &f) && f.pulse == 5);
  CHECK(parse({"-pulse=0o_1_7"}, &syn, &err, &f) && f.pulse == 15);
  CHECK(parse({"-pulse=-0x_1"}, &syn, &err) == false && !syn);  // parses (-1), then validateFlags refuses it
  CHECK(!parse({"-pulse=0x1e_"}, &syn, &err) && syn);
  // validateFlags: enumerated string flags
  CHECK(!parse({"-allocator_search=fastest"}, &syn, &err) && !syn &&
        err.find("invalid allocator_search provided: fastest") == 0);
}

// the CDI spec's strings, byte-for-byte as the Python oracle's json.dumps(os.fsdecode(...)) (expected
// values generated by Python): UTF-8 as \\uXXXX (surrogate pairs above U+FFFF), other bytes as \\udcXX
static void test_cdi_json_strings() {
  CHECK(cdi::json_str(std::string("\xc3\xa9", 2)) == "\"\\u00e9\"");
  CHECK(cdi::json_str(std::string("\xf0\x9f\x98\x80", 4)) == "\"\\ud83d\\ude00\"");
  CHECK(cdi::json_str(std::string("\xff", 1)) == "\"\\udcff\"");
  CHECK(cdi::json_str(std::string("\xe0\x80\x80", 3)) == "\"\\udce0\\udc80\\udc80\"");
  CHECK(cdi::json_str(std::string("\x61\x22\x62\x5c", 4)) == "\"a\\\"b\\\\\"");
  CHECK(cdi::json_str(std::string("\x01\x7f", 2)) == "\"\\u0001\\u007f\"");
  CHECK(cdi::json_str(std::string("\xc3", 1)) == "\"\\udcc3\"");
  CHECK(cdi::json_str(std::string("\xed\xa0\x80", 3)) == "\"\\udced\\udca0\\udc80\"");
  CHECK(cdi::json_str(std::string("\xf4\x90\x80\x80", 4)) == "\"\\udcf4\\udc90\\udc80\\udc80\"");
  CHECK(cdi::json_str(std::string("\x2f\x64\x65\x76\x2f\x64\x72\x69\x2f\x72\x65\x6e\x64\x65\x72\x44\x31\x32\x38", 19)) == "\"/dev/dri/renderD128\"");
}

// amd-smi's driver version of an in-tree amdgpu is the kernel banner (spaces removed on the
// MI355X host): the label takes the release, as labels.py's re.match(r"^Linux\s*version\s*([0-9][^\s(]*)")
static void test_driver_version_value() {
  using labeller::driver_version_value;
  CHECK(driver_version_value("Linuxversion6.18.54-ant.1(nixbld@localhost)(gcc(GCC)15.3.0)#1") == "6.18.54-ant.1");
  CHECK(driver_version_value("Linux version 6.8.0-45-generic (buildd@lcy02) #45") == "6.8.0-45-generic");
  CHECK(driver_version_value("Linux  version\t6.1(x)") == "6.1");
  for (const char* same : {"6.12.12", "Linux version abc", "Linuxversion", "linux version 6.1", "", "Linux"})
    CHECK(driver_version_value(same) == same);
}

#ifdef MI355X_TEST_HTTP
// $NO_PROXY / $HTTPS_PROXY as Go's golang.org/x/net/http/httpproxy reads them
static void test_proxy_environment() {
  using http::no_proxy_match;
  CHECK(no_proxy_match("*", "anything.example", 443));
  CHECK(no_proxy_match("foo.com", "foo.com", 443) && no_proxy_match("foo.com", "bar.foo.com", 443));
  CHECK(!no_proxy_match("foo.com", "barfoo.com", 443));
  CHECK(!no_proxy_match(".foo.com", "foo.com", 443) && no_proxy_match(".foo.com", "bar.foo.com", 443));
  CHECK(!no_proxy_match("*.foo.com", "foo.com", 443) && no_proxy_match("*.foo.com", "a.b.foo.com", 443));
  CHECK(no_proxy_match("10.0.0.0/8", "10.1.2.3", 443) && !no_proxy_match("10.0.0.0/8", "11.0.0.1", 443));
  CHECK(!no_proxy_match("10.0.0.0/8", "ten.example", 443));
  CHECK(no_proxy_match("fd00::/8", "fd12::1", 443) && !no_proxy_match("fd00::/8", "fe80::1", 443));
  CHECK(no_proxy_match("192.168.1.1", "192.168.1.1", 6443) && !no_proxy_match("192.168.1.1", "192.168.1.2", 6443));
  CHECK(no_proxy_match("2001:db8::1", "2001:db8:0::1", 443));
  CHECK(no_proxy_match("[2001:db8::2]:443", "2001:db8::2", 443) && !no_proxy_match("[2001:db8::2]:443", "2001:db8::2", 80));
  CHECK(no_proxy_match("foo.com:8443", "foo.com", 8443) && !no_proxy_match("foo.com:8443", "foo.com", 443));
  CHECK(no_proxy_match(" bar.com , FOO.com ", "api.foo.COM", 443));
  CHECK(!no_proxy_match("", "foo.com", 443) && !no_proxy_match(",,", "foo.com", 443));
  ::setenv("HTTPS_PROXY", "proxy.example:3128", 1);
  ::setenv("NO_PROXY", ".svc,10.96.0.0/12", 1);
  ::setenv("HTTP_PROXY", "", 1);
  ::setenv("http_proxy", "http://lower.example:8080", 1);
  CHECK(http::env_proxy(true, "api.example", 6443) == "http://proxy.example:3128");
  CHECK(http::env_proxy(true, "kubernetes.default.svc", 443).empty());
  CHECK(http::env_proxy(true, "10.96.0.1", 443).empty() && http::env_proxy(true, "10.112.0.1", 443) != "");
  CHECK(http::env_proxy(true, "localhost", 443).empty() && http::env_proxy(true, "127.0.0.1", 443).empty() &&
        http::env_proxy(true, "::1", 443).empty());
  CHECK(http::env_proxy(false, "api.example", 80) == "http://lower.example:8080");  // an empty HTTP_PROXY falls back
  for (const char* v : {"HTTPS_PROXY", "NO_PROXY", "HTTP_PROXY", "http_proxy"}) ::unsetenv(v);
  CHECK(http::env_proxy(true, "api.example", 6443).empty());
}
#endif

static void test_metrics_registry() {
  metrics::Registry r;
  r.inc("mi355x_x_total", {{"b", "2"}, {"a", "1"}}, 1.0, "things");
  r.inc("mi355x_x_total", {{"a", "1"}, {"b", "2"}}, 2.0);  // label order does not make a new series
  r.set("mi355x_g", 3.5);
  r.set("mi355x_g", 1.25);
  r.observe_ms("mi355x_h_seconds", 0.2, {{"rpc", "Allocate"}});
  r.observe_ms("mi355x_h_seconds", 7000, {{"rpc", "Allocate"}});
  CHECK(r.value("mi355x_x_total", {{"a", "1"}, {"b", "2"}}) == 3.0);
  CHECK(r.value("mi355x_g") == 1.25 && r.value("mi355x_absent") == 0.0);
  CHECK(r.count("mi355x_h_seconds", {{"rpc", "Allocate"}}) == 2 && r.count("mi355x_h_seconds") == 0);
  const std::string t = r.render();
  CHECK(t.find("# HELP mi355x_x_total things\n# TYPE mi355x_x_total counter\n") != std::string::npos);
  CHECK(t.find("mi355x_x_total{a=\"1\",b=\"2\"} 3.0\n") != std::string::npos);
  CHECK(t.find("# TYPE mi355x_g gauge\nmi355x_g 1.25\n") != std::string::npos);
  CHECK(t.find("mi355x_h_seconds_bucket{rpc=\"Allocate\",le=\"+Inf\"} 2\n") != std::string::npos);
  CHECK(t.find("mi355x_h_seconds_count{rpc=\"Allocate\"} 2\n") != std::string::npos);
  CHECK(t.find("mi355x_h_seconds_sum{rpc=\"Allocate\"} 7.0002\n") != std::string::npos);
  // buckets (rendered in seconds) are cumulative: 0.2 ms lands in le=0.00025 and every bucket above it
  CHECK(t.find("mi355x_h_seconds_bucket{rpc=\"Allocate\",le=\"0.0001\"} 0\n") != std::string::npos);
  CHECK(t.find("mi355x_h_seconds_bucket{rpc=\"Allocate\",le=\"0.00025\"} 1\n") != std::string::npos);
  r.clear();
  CHECK(r.render().empty() && r.value("mi355x_g") == 0.0 && r.count("mi355x_h_seconds", {{"rpc", "Allocate"}}) == 0);
}

// one GET over loopback: the status line
static std::string http_status(int port, const char* path) {
  const int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return "";
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  std::string got;
  if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0) {
    const std::string req = std::string("GET ") + path + " HTTP/1.0\r\n\r\n";
    if (::write(fd, req.data(), req.size()) == static_cast<ssize_t>(req.size())) {
      char b[512];
      ssize_t n;
      while ((n = ::read(fd, b, sizeof(b))) > 0) got.append(b, static_cast<size_t>(n));
    }
  }
  ::close(fd);
  return got;
}

static void test_http_endpoint_checks() {
  // /healthz and /readyz answer 200 "ok" or 503 with the check's reason; the
  // checks run on the endpoint's thread at every request
  metrics::Registry reg;
  metrics::HttpEndpoint ep(reg);
  std::atomic<bool> live{true}, ready{false};
  ep.set_checks([&] { return live ? std::string() : std::string("control loop stalled"); },
                [&] { return ready ? std::string() : std::string("registered with kubelet: 0 of 1 resources"); });
  CHECK(ep.start("127.0.0.1", 0).empty());
  const int port = ep.port();
  CHECK(http_status(port, "/healthz").rfind("HTTP/1.0 200 OK\r\n", 0) == 0);
  std::string r = http_status(port, "/readyz");
  CHECK(r.rfind("HTTP/1.0 503 Service Unavailable\r\n", 0) == 0);
  CHECK(r.find("\r\n\r\nregistered with kubelet: 0 of 1 resources\n") != std::string::npos);
  ready = true;
  live = false;
  CHECK(http_status(port, "/readyz").find("\r\n\r\nok\n") != std::string::npos);
  CHECK(http_status(port, "/healthz").rfind("HTTP/1.0 503 ", 0) == 0);
  CHECK(http_status(port, "/other").rfind("HTTP/1.0 404 ", 0) == 0);
  ep.stop();
  // no checks set: both always ok
  metrics::HttpEndpoint plain(reg);
  CHECK(plain.start("127.0.0.1", 0).empty());
  CHECK(http_status(plain.port(), "/readyz").find("\r\n\r\nok\n") != std::string::npos);
  plain.stop();
}

static void test_health_controller_generations(const std::string& tmp) {
  // passthrough sweeps on worker threads against a reload on the control thread
  // (run under TSan in CI: the job shares nothing with the controller)
  daemon::Flags f;
  f.sysfs_root = tmp + "/no-such-sysfs";
  f.exporter_socket = "";
  daemon::HealthController hc(f, -1);
  std::vector<daemon::Resource> rs(1);
  rs[0].group_ids = {"3", "4"};
  rs[0].groups["3"] = {PciFunctionInfo{}};
  rs[0].groups["4"] = {PciFunctionInfo{}};
  hc.rebuild(daemon::Driver::Pf, {}, KfdTopology{}, rs);
  daemon::Workers<daemon::SweepResult> w;
  hc.started();
  w.run(hc.job());
  CHECK(hc.inflight() && !hc.may_reload());
  std::vector<daemon::SweepResult> got;
  for (int i = 0; i < 500 && got.empty(); ++i) {
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
    got = w.take();
  }
  CHECK(got.size() == 1 && hc.finished(got[0]) && hc.may_reload());
  CHECK(got.size() == 1 && got[0].health.size() == 2 && !got[0].health.at("3"));  // vfio-pci absent: Unhealthy
  // a reload while a sweep runs: the old sweep's result is dropped
  hc.started();
  w.run(hc.job());
  rs[0].group_ids = {"5"};
  rs[0].groups["5"] = {PciFunctionInfo{}};
  hc.rebuild(daemon::Driver::Pf, {}, KfdTopology{}, rs);
  w.join_all();
  got = w.take();
  CHECK(got.size() == 1 && !hc.finished(got[0]));
  hc.started();
  w.run(hc.job());
  w.join_all();
  got = w.take();
  CHECK(got.size() == 1 && hc.finished(got[0]) && got[0].health.count("5") == 1);
}

int main(int argc, char** argv) {
  std::string repo = argc > 1 ? argv[1] : "testdata";
  std::string ref = argc > 2 ? argv[2] : "/root/reference/testdata";
  (void)repo;
  test_parsers(ref);
  test_allocator_reference_contract(ref);
  test_errors();
  test_degraded_links(ref);
  test_hpack();
  test_grpc_server();
  test_grpc_deferred_prestart();
  test_fuzz_rpc(ref);
  test_registration_generations();
  test_registration_watchdog();
  test_registration_random_sequences();
  test_topology_watch();
  test_flags_go_semantics();
  test_metrics_registry();
  test_http_endpoint_checks();
  test_driver_version_value();
  test_cdi_json_strings();
#ifdef MI355X_TEST_HTTP
  test_proxy_environment();
#endif
  {
    char dir[] = "/tmp/mi355x-test-core-XXXXXX";
    if (::mkdtemp(dir)) {
      test_health_controller_generations(dir);
      ::rmdir(dir);
    }
  }
  std::printf("test_core: %d passed, %d failed, %d skipped\n", g_pass, g_fail, g_skip);
  return g_fail ? 1 : 0;
}
