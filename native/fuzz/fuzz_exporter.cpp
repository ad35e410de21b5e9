// metricssvc GPUStateResponse decoding (parse_exporter_states,
// src/health/health_engine.cpp): the metrics exporter's List reply, read by
// the native daemon every health pulse. Invariants: a body that decodes
// yields a map that, encoded again, decodes to the same map; a malformed body
// yields an error and no verdicts (protobuf's strictness, as the reference's
// generated client has).
#include <map>
#include <string>

#include "fuzz_common.h"
#include "mi355x/dp_service.h"
#include "mi355x/health_engine.h"

using mi355x::fuzz::fail;
namespace pb = mi355x::rpc::pb;

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  const std::string body(reinterpret_cast<const char*>(data), size);
  std::string err;
  const auto m = mi355x::health::parse_exporter_states(body, &err);
  if (!err.empty()) {
    if (!m.empty()) fail("verdicts returned with an error");
    return 0;
  }
  std::string again;
  for (const auto& [bdf, healthy] : m) {
    std::string st;
    pb::put_bytes(&st, 1, "0");
    pb::put_bytes(&st, 3, healthy ? "healthy" : "unhealthy");
    pb::put_bytes(&st, 5, bdf);
    pb::put_bytes(&again, 1, st);
  }
  std::string err2;
  if (mi355x::health::parse_exporter_states(again, &err2) != m || !err2.empty()) fail("re-encoded states differ");
  return 0;
}
