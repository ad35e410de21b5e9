// JSON reader / writer of the native labeller (src/kube/json.cpp): Node objects
// and watch events come from the apiserver. Invariants: whatever parses
// serialises to text that parses again to the same serialisation (a GET + PUT
// round trip never rewrites a Node), and the label view agrees with the tree.
#include <string>

#include "../src/kube/json.h"
#include "fuzz_common.h"

using mi355x::fuzz::fail;
namespace json = mi355x::json;

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  const std::string text(reinterpret_cast<const char*>(data), size);
  std::string err;
  auto v = json::parse(text, &err);
  if (!v) {
    if (err.empty()) fail("parse failed without an error message");
    return 0;
  }
  const std::string s1 = json::serialize(*v);
  std::string err2;
  auto v2 = json::parse(s1, &err2);
  if (!v2) fail("serialised document does not parse", err2 + " in " + s1.substr(0, 200));
  const std::string s2 = json::serialize(*v2);
  if (s1 != s2) fail("serialisation is not a fixed point", s1.substr(0, 200) + " vs " + s2.substr(0, 200));
  const auto labels = json::node_labels(*v);
  if (labels != json::node_labels(*v2)) fail("labels changed over a round trip");
  // the PATCH / PUT paths edit labels in place and serialise again
  json::Value edited = *v;
  if (edited.kind == json::Value::Object) {
    json::Value* md = edited.get("metadata");
    if (!md) md = &edited.set("metadata", json::Value::object());
    if (md->kind == json::Value::Object) {
      json::Value* lb = md->get("labels");
      if (!lb || lb->kind != json::Value::Object) lb = &md->set("labels", json::Value::object());
      lb->set("amd.com/gpu.fuzz", json::Value::string(text.substr(0, 16)));
      auto back = json::parse(json::serialize(edited), &err2);
      if (!back) fail("edited document does not parse", err2);
      if (json::node_labels(*back).count("amd.com/gpu.fuzz") != 1) fail("label edit lost");
    }
  }
  for (const char* k : {"type", "object", "metadata"}) (void)v->str(k, "");
  return 0;
}
