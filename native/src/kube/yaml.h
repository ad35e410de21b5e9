// A YAML reader for configuration files (kubeconfig, the device plugin's
// -config file): block and flow mappings / sequences (compact nested ones
// too), plain and quoted scalars over several lines with YAML's line folding
// and escaped line breaks, literal / folded block scalars with chomping and
// indentation indicators, the standard !!str / !!null / !!bool / !!int /
// !!float tags, anchors / aliases / merge keys (aliases copy the anchored
// node, at most 2^20 nodes per document), one document with its --- / ...
// markers and % directives, and comments, into a JSON value. Plain scalars
// other than booleans and null stay text. JSON documents are read as JSON.
// Custom tags, complex (`?`) keys and a second document are refused (no
// kubeconfig or plugin config uses them). Checked against PyYAML on generated
// documents (tests/test_native_yaml.py).
#pragma once

#include <optional>
#include <string>

#include "json.h"

namespace mi355x::yaml {

std::optional<json::Value> parse(const std::string& text, std::string* error);

}  // namespace mi355x::yaml
