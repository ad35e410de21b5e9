// DevicePlugin RPC bodies (src/rpc/dp_service.cpp + the hive allocator) over
// well-formed gRPC calls: the protobuf a kubelet sends, mutated. Byte 0 picks
// the method, the rest is the request message. Invariants:
//   * every call gets a gRPC status (never a transport failure);
//   * GetPreferredAllocation OK -> one answer per container request; for a
//     request kubelet can send (no repeated IDs, must_include within available)
//     exactly allocation_size distinct IDs, all available, every must_include
//     ID among them;
//   * Allocate OK -> one ContainerAllocateResponse per container request with
//     /dev/kfd plus the card and render node of every requested ID, in order;
//     an unknown ID is INVALID_ARGUMENT.
#include <set>
#include <string>
#include <vector>

#include "dp_fixture.h"

using namespace mi355x::fuzz;
namespace rpc = mi355x::rpc;
namespace pb = mi355x::rpc::pb;

namespace {

struct Container {
  std::vector<std::string> a, b;  // available / must (GPA), ids (Allocate)
  int64_t size = 0;
};

bool parse_requests(const std::string& body, bool gpa, std::vector<Container>* out) {
  return pb::scan(
      body.data(), body.size(),
      [&](int f, const char* p, size_t n) {
        if (f != 1) return true;
        Container c;
        const bool ok = pb::scan(
            p, n,
            [&](int g, const char* q, size_t m) {
              if (g == 1) c.a.emplace_back(q, m);
              else if (g == 2 && gpa) c.b.emplace_back(q, m);
              return true;
            },
            [&](int g, uint64_t v) {
              if (g == 3 && gpa) c.size = static_cast<int32_t>(static_cast<uint32_t>(v));
              return true;
            });
        out->push_back(std::move(c));
        return ok;
      },
      nullptr);
}

std::vector<std::vector<std::string>> repeated_strings(const std::string& body, int outer, int inner) {
  std::vector<std::vector<std::string>> out;
  const bool ok = pb::scan(
      body.data(), body.size(),
      [&](int f, const char* p, size_t n) {
        if (f != outer) return true;
        std::vector<std::string> v;
        pb::scan(
            p, n,
            [&](int g, const char* q, size_t m) {
              if (g == inner) v.emplace_back(q, m);
              return true;
            },
            nullptr);
        out.push_back(std::move(v));
        return true;
      },
      nullptr);
  if (!ok) fail("server sent a malformed response body");
  return out;
}

rpc::GrpcClient& client() {
  static rpc::GrpcClient c;
  if (!c.connected() || c.going_away()) {
    c.close();
    if (const std::string e = c.connect(dp_server().sock, 5.0); !e.empty()) fail("connect", e);
  }
  return c;
}

}  // namespace

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  dp_server();
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size == 0 || size > 256 * 1024) return 0;
  static const char* kMethods[] = {"GetPreferredAllocation", "Allocate", "GetDevicePluginOptions",
                                   "PreStartContainer"};
  const unsigned sel = data[0] % 5;
  const std::string body(reinterpret_cast<const char*>(data) + 1, size - 1);
  const std::string path = sel < 4 ? rpc::DevicePluginService::path(kMethods[sel]) : "/v1beta1.DevicePlugin/Nope";
  const rpc::Reply r = client().unary(path, body, 10.0);
  dp_server().service->drain_events();
  if (r.status < 0) fail("transport failure on a well-formed call", r.message);
  if (sel == 4) {
    if (r.status != rpc::kUnimplemented) fail("unknown method not UNIMPLEMENTED");
    return 0;
  }
  if (sel == 3) {  // PreStartContainer through the gate: OK unless the request does not parse
    const bool wellformed = rpc::pb::scan(body.data(), body.size(), nullptr, nullptr);
    if (wellformed ? r.status != 0 : r.status != rpc::kInternal) fail("PreStart answer", r.message);
    return 0;
  }
  if (sel == 2) {
    if (r.status != 0) fail("Options failed", r.message);
    return 0;
  }
  std::vector<Container> req;
  const bool parsed = parse_requests(body, sel == 0, &req);
  if (!parsed) {
    if (r.status == 0) fail("malformed request accepted");
    return 0;
  }
  const std::set<std::string> known(dp_server().ids.begin(), dp_server().ids.end());
  if (sel == 0) {
    if (r.status != 0) {
      if (r.status != rpc::kUnknown) fail("GetPreferredAllocation error with an unexpected code", r.message);
      return 0;
    }
    const auto got = repeated_strings(r.body, 1, 1);
    if (got.size() != req.size()) fail("GetPreferredAllocation: answers != container requests");
    for (size_t i = 0; i < req.size(); ++i) {
      const std::set<std::string> avail(req[i].a.begin(), req[i].a.end());
      const std::set<std::string> must(req[i].b.begin(), req[i].b.end());
      const std::set<std::string> chosen(got[i].begin(), got[i].end());
      const bool dup_free = avail.size() == req[i].a.size() && must.size() == req[i].b.size();
      if (!dup_free) continue;  // kubelet never repeats an ID; the reference returns such lists as given
      // kubelet's must-include IDs are a subset of the available ones; the reference's
      // short-circuits (|available| == size -> available, |must| == size -> must) return
      // other requests' lists unchanged (besteffort_policy.go:110-116), and so does this one
      bool must_in_avail = true;
      for (const auto& id : must) must_in_avail = must_in_avail && avail.count(id);
      if (!must_in_avail) continue;
      if (static_cast<int64_t>(got[i].size()) != req[i].size || chosen.size() != got[i].size())
        fail("GetPreferredAllocation: wrong number of distinct IDs");
      for (const auto& id : chosen)
        if (!avail.count(id)) fail("GetPreferredAllocation: chose an unavailable ID", id);
      for (const auto& id : must)
        if (!chosen.count(id)) fail("GetPreferredAllocation: dropped a must-include ID", id);
    }
    return 0;
  }
  // Allocate
  bool unknown = false;
  for (const auto& c : req)
    for (const auto& id : c.a)
      if (!known.count(id)) unknown = true;
  if (unknown) {
    if (r.status != rpc::kInvalidArgument) fail("Allocate of an unknown ID not INVALID_ARGUMENT");
    return 0;
  }
  if (r.status != 0) fail("Allocate of known IDs failed", r.message);
  const auto specs = repeated_strings(r.body, 1, 3);
  if (specs.size() != req.size()) fail("Allocate: responses != container requests");
  for (size_t i = 0; i < req.size(); ++i) {
    const size_t want = 1 + 2 * req[i].a.size();
    if (specs[i].size() != want) fail("Allocate: wrong number of DeviceSpecs");
  }
  return 0;
}
