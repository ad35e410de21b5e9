// Measurement build of the liveness probe: probe_main + the HSA-direct path
// with path interposition, so the whole container entrypoint (ROCr init, code
// object, queue, MFMA dispatch, verify) can run against an emulated container
// sysfs view (MI355X_INITPROF_REDIRECT, see path_interpose.h). Not shipped.
#include "path_interpose.h"

namespace {
struct Configure {
  Configure() { path_interpose_configure(); }
} configure_at_start;
}  // namespace
