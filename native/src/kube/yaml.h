// A YAML reader for configuration files (kubeconfig, the device plugin's
// -config file): block and flow mappings / sequences, plain and quoted
// scalars, literal / folded block scalars and comments, into a JSON value.
// JSON documents are read as JSON. Anchors, tags and multi-document streams
// are not supported (no kubeconfig or plugin config uses them).
#pragma once

#include <optional>
#include <string>

#include "json.h"

namespace mi355x::yaml {

std::optional<json::Value> parse(const std::string& text, std::string* error);

}  // namespace mi355x::yaml
