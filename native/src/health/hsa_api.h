// ROCr entry points used by the HSA-direct probe, resolved at run time.
//
// libhsa-runtime64's static constructors cost ~8.7 ms per process (measured:
// dlopen 10.3 ms vs 0.1 ms of relocation, profiles/archive/measurements_r1_r3.md §3d). Linked
// normally, that cost is paid before main() and nothing can overlap it.
// Loaded with dlopen() from main(), it runs while another thread opens
// /dev/kfd — the kernel-side kfd process creation, the other fixed cost of a
// GPU process' start-up — so the two overlap. hsa_init's own open() then finds
// the process already created.
#pragma once

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#define MI355X_HSA_FUNCS(X)                  \
  X(hsa_init)                                \
  X(hsa_shut_down)                           \
  X(hsa_status_string)                       \
  X(hsa_system_get_info)                     \
  X(hsa_iterate_agents)                      \
  X(hsa_agent_get_info)                      \
  X(hsa_amd_agent_iterate_memory_pools)      \
  X(hsa_amd_memory_pool_get_info)            \
  X(hsa_amd_memory_pool_allocate)            \
  X(hsa_amd_memory_pool_free)                \
  X(hsa_amd_agents_allow_access)             \
  X(hsa_code_object_reader_create_from_memory) \
  X(hsa_code_object_reader_destroy)          \
  X(hsa_executable_create_alt)               \
  X(hsa_executable_load_agent_code_object)   \
  X(hsa_executable_freeze)                   \
  X(hsa_executable_get_symbol_by_name)       \
  X(hsa_executable_symbol_get_info)          \
  X(hsa_executable_destroy)                  \
  X(hsa_queue_create)                        \
  X(hsa_queue_destroy)                       \
  X(hsa_queue_add_write_index_screlease)     \
  X(hsa_signal_create)                       \
  X(hsa_signal_destroy)                      \
  X(hsa_signal_store_screlease)              \
  X(hsa_signal_wait_scacquire)               \
  X(hsa_signal_load_scacquire)               \
  X(hsa_amd_profiling_set_profiler_enabled)  \
  X(hsa_amd_profiling_get_dispatch_time)     \
  X(hsa_amd_agent_memory_pool_get_info)      \
  X(hsa_amd_memory_async_copy)               \
  X(hsa_amd_memory_fill)

namespace mi355x {

struct HsaApi {
#define MI355X_HSA_PTR(name) decltype(&::name) name = nullptr;
  MI355X_HSA_FUNCS(MI355X_HSA_PTR)
#undef MI355X_HSA_PTR
  bool loaded = false;
  double load_us = 0;   // dlopen (library constructors) + symbol lookup
  char error[160] = {0};
};

// Loads libhsa-runtime64 once (thread-safe); check .loaded / .error.
const HsaApi& hsa_api();

}  // namespace mi355x
