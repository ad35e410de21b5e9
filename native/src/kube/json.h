// Minimal JSON value for the native node labeller: parse a Node object or a
// watch event, edit metadata.labels, serialise it back. Numbers keep their
// source text, so a GET + Update round trip does not reformat a Node.
#pragma once

#include <map>
#include <memory>
#include <optional>
#include <string>
#include <utility>
#include <vector>

namespace mi355x::json {

struct Value {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  std::string s;  // String: decoded text; Number: source text
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;  // insertion order kept

  const Value* get(const std::string& key) const;  // Object member or nullptr
  Value* get(const std::string& key);
  Value& set(const std::string& key, Value v);     // replace or append
  std::string str(const std::string& key, const std::string& fallback = "") const;

  static Value string(std::string v) {
    Value x;
    x.kind = String;
    x.s = std::move(v);
    return x;
  }
  static Value object() {
    Value x;
    x.kind = Object;
    return x;
  }
};

// Parses one JSON document; error text (with the byte offset) on failure.
std::optional<Value> parse(const std::string& text, std::string* error = nullptr);
std::string serialize(const Value& v);
std::string quote(const std::string& s);  // JSON string literal (ASCII-safe, \uXXXX escapes)

// metadata.labels of a Node (empty when absent)
std::map<std::string, std::string> node_labels(const Value& node);

}  // namespace mi355x::json
