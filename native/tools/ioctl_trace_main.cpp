// Link into any entrypoint (with -rdynamic) to get its kfd/drm ioctl wall
// times on stderr at exit: "IOCTL_TRACE {...}" (measurement builds only).
#include <cstdio>

#include "ioctl_trace.h"

namespace {
__attribute__((destructor)) void dump_ioctls() {
  std::fprintf(stderr, "IOCTL_TRACE %s\n", ioctl_trace_json(0).c_str());
}
}  // namespace
