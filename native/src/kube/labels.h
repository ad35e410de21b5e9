// Label generation of the native node labeller (the 13 generators of the
// reference labeller, cmd/k8s-node-labeller/main.go:85-505, plus the opt-in
// gfx-target / xgmi-hive-count / xgmi-links-down), over the C++ core: kfd
// topology, sysfs, libdrm and amd-smi. Output equals
// rocm_k8s_device_plugin_amd/labeller/labels.py (tests/test_native_labeller.py).
// A library of its own so the fuzz target (native/fuzz/fuzz_labels.cpp) runs
// the same code as mi355x-node-labeller.
#pragma once

#include <map>
#include <string>
#include <vector>

namespace mi355x::labeller {

using Labels = std::map<std::string, std::string>;

struct LabelOptions {
  std::map<std::string, bool> enabled;  // label kind -> on (missing = off)
  std::string driver_type;              // "" = container -> VF -> PF
  std::string sysfs_root = "/sys";
  std::string dev_root = "/dev";
};

// every label kind, constants.go:21 order, then the opt-in additions
const std::vector<std::string>& label_kinds();
// "amd.com/gpu.<kind>" or "beta.amd.com/gpu.<kind>"
std::string prefix_of(const std::string& kind, bool experimental);

// apimachinery IsValidLabelValue / IsQualifiedName (a DNS-subdomain prefix, a
// name of <= 63 characters): the apiserver rejects a whole patch with one bad
// label, which would leave the node with none
bool valid_label_value(const std::string& v);
bool valid_label_key(const std::string& k);
std::string sanitize_label_value(const std::string& v);
// values sanitised; a label whose key is invalid (a value that went into the
// key: product name, firmware name) is dropped with a warning
Labels clean_labels(const Labels& in);
// amd-smi's driver string of an in-tree amdgpu -> the kernel release
std::string driver_version_value(const std::string& raw);

// generateLabels (main.go:389-408): explicit mode, else container -> VF -> PF
Labels generate_labels(const LabelOptions& opt);

}  // namespace mi355x::labeller
