// YAML reader (src/kube/yaml.cpp) behind -kubeconfig and the device plugin's
// -config file. Invariants: whatever parses is a JSON tree that serialises to
// valid JSON, and that JSON read back through the YAML reader (JSON documents
// are read as JSON) gives the same tree.
#include <string>

#include "../src/kube/json.h"
#include "../src/kube/yaml.h"
#include "fuzz_common.h"

using mi355x::fuzz::fail;
namespace json = mi355x::json;
namespace yaml = mi355x::yaml;

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size > 64 * 1024) return 0;
  const std::string text(reinterpret_cast<const char*>(data), size);
  std::string err;
  auto v = yaml::parse(text, &err);
  if (!v) {
    if (err.empty()) fail("parse failed without an error message");
    return 0;
  }
  const std::string s1 = json::serialize(*v);
  std::string e2;
  auto j = json::parse(s1, &e2);
  if (!j) fail("YAML tree does not serialise to JSON", e2 + " in " + s1.substr(0, 200));
  auto y = yaml::parse(s1, &e2);
  if (!y) fail("JSON text of a YAML tree does not parse as YAML", e2 + " in " + s1.substr(0, 200));
  if (json::serialize(*y) != s1) fail("YAML -> JSON -> YAML changed the tree", s1.substr(0, 200));
  return 0;
}
