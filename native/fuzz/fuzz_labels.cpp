// Node labels (src/kube/labels.cpp, the native labeller's generators) over a
// generated MI355X sysfs tree whose files the input rewrites or removes
// (sysfs_mutator.h): product names, device ids, driver versions, kfd
// properties and partition modes as a driver or firmware could report them.
// Invariants: every label key is a valid qualified name and every value a
// valid label value (one bad label makes the apiserver reject the whole
// patch), and the same tree gives the same labels. Every label kind is on
// except xgmi-links-down (an amd-smi reading, not sysfs).
#include <memory>
#include <string>

#include "../src/kube/labels.h"
#include "mi355x/glog.h"
#include "sysfs_mutator.h"

using namespace mi355x;
using mi355x::fuzz::fail;

namespace {
std::unique_ptr<fuzz::SysfsMutator> g_tree;
labeller::LabelOptions g_opt;
}  // namespace

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  glog::Options quiet;  // the generators log every libdrm / sysfs miss: gigabytes over a campaign
  quiet.discard = true;
  glog::init(quiet);
  g_tree = std::make_unique<fuzz::SysfsMutator>(fuzz::env_or_die("MI355X_FUZZ_SYSFS_MUT"));
  g_opt.sysfs_root = g_tree->root();
  g_opt.dev_root = fuzz::scratch_dir() + "/dev";  // no /dev/dri nodes: libdrm queries fail fast
  for (const auto& k : labeller::label_kinds()) g_opt.enabled[k] = k != "xgmi-links-down";
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size > 64 * 1024) return 0;
  g_tree->apply(data, size);
  // auto mode (container -> VF -> PF), as the DaemonSet runs it; discovery dominates the cost
  const labeller::Labels a = labeller::generate_labels(g_opt);
  for (const auto& [k, v] : a) {
    if (!labeller::valid_label_key(k)) fail("invalid label key", k);
    if (!labeller::valid_label_value(v)) fail("invalid label value", k + "=" + v);
  }
  if (labeller::generate_labels(g_opt) != a) fail("labels differ for the same tree");
  g_tree->restore();
  return 0;
}
