// Container-entrypoint build of the liveness probe for the fake CRI runtime
// (container_runtime.py): probe_main + the HSA-direct path with path
// interposition, so the whole entrypoint (ROCr init, code object, queue, MFMA
// dispatch, verify) runs against the container's view without root: its /dev
// as the Allocate DeviceSpecs build it (MI355X_DEV_ALLOW) and the Allocate
// mounts (MI355X_INITPROF_REDIRECT), see path_interpose.h. Not shipped in the
// plugin image.
#include "path_interpose.h"

namespace {
struct Configure {
  Configure() { path_interpose_configure(); }
} configure_at_start;
std::string g_view_json;
}  // namespace

// probe_main.cpp prints this as the reply's "view" field when it is linked in:
// what the emulated view did to the runtime's file walk (paths seen, per-CPU
// cache descriptors opened under the NUMA-node tree, redirected, refused)
extern "C" const char* mi355x_probe_view_json() {
  g_view_json = path_interpose_view_json();
  return g_view_json.c_str();
}
