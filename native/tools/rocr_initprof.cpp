// mi355x-rocr-initprof: which files does ROCr's hsa_init() walk, and what does
// hiding or redirecting some of them save? (measurement tool, not shipped)
//
//   [MI355X_INITPROF_HIDE=...] [MI355X_INITPROF_REDIRECT=...] mi355x-rocr-initprof  -> one JSON line
#include <hsa/hsa.h>

#include "path_interpose.h"

namespace {
double now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}
}  // namespace

int main(int argc, char** argv) {
  path_interpose_configure();
  const double t0 = now_ms();
  void* lib = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) lib = dlopen("/opt/rocm/lib/libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) {
    std::printf("{\"ok\":false,\"error\":\"dlopen: %s\"}\n", dlerror());
    return 2;
  }
  auto init = reinterpret_cast<hsa_status_t (*)()>(dlsym(lib, "hsa_init"));
  auto iterate = reinterpret_cast<hsa_status_t (*)(hsa_status_t (*)(hsa_agent_t, void*), void*)>(
      dlsym(lib, "hsa_iterate_agents"));
  const double t1 = now_ms();
  const hsa_status_t s = init();
  const double t2 = now_ms();
  int agents = 0;
  if (s == HSA_STATUS_SUCCESS)
    iterate([](hsa_agent_t, void* n) { ++*static_cast<int*>(n); return HSA_STATUS_SUCCESS; }, &agents);
  std::printf("{\"ok\":%s,\"hsa_status\":%d,\"agents\":%d,\"dlopen_ms\":%.2f,\"hsa_init_ms\":%.2f,\"walk\":%s}\n",
              s == HSA_STATUS_SUCCESS ? "true" : "false", static_cast<int>(s), agents, t1 - t0, t2 - t1,
              path_interpose_json().c_str());
  (void)argc;
  (void)argv;
  return s == HSA_STATUS_SUCCESS ? 0 : 1;
}
