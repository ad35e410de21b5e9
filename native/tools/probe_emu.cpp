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
}  // namespace
