// ROCr state shared by the HSA-direct probe's translation units:
// hsa_probe.cpp (runtime start-up, the liveness probe, kept per-device
// queues), hsa_peer.cpp (the xGMI peer copy check) and hsa_chip.cpp (the
// full-chip sweep and the throughput check). Internal to src/health.
#pragma once

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>
#include <vector>

#include "hsa_api.h"
#include "liveness_kernel.h"
#include "mi355x/liveness_probe.h"

// The gfx950 code object, embedded in hsa_probe.cpp at build time.
extern "C" const unsigned char mi355x_hsaco_start[];
extern "C" const unsigned char mi355x_hsaco_end[];

namespace mi355x::hsa_rt {

inline const HsaApi& H() { return hsa_api(); }

struct Agent {
  hsa_agent_t agent{};
  hsa_amd_memory_pool_t coarse{};  // device HBM
  bool has_coarse = false;
};

struct Runtime {
  std::mutex mu;
  bool inited = false;
  hsa_status_t init_status = HSA_STATUS_SUCCESS;
  std::vector<Agent> gpus;
  hsa_agent_t cpu{};
  hsa_amd_memory_pool_t kernarg{};
  hsa_amd_memory_pool_t fine{};
  bool has_kernarg = false, has_fine = false;
  uint64_t ts_freq = 0;
  // dlopen(ROCr), pre-open of /dev/kfd (overlapped with dlopen), hsa_init,
  // agent enumeration, pool discovery
  double init_us[5] = {0, 0, 0, 0, 0};
  int kfd_fd = -1;
};

// A completion signal shared by whoever may still need it: a chip sweep or
// throughput check whose dispatch outlived its deadline is referenced both by
// the in-flight registry and by the kept queue it was submitted on.
struct SigRef {
  hsa_signal_t s{};
  SigRef() = default;
  SigRef(const SigRef&) = delete;
  SigRef& operator=(const SigRef&) = delete;
  ~SigRef() {
    if (s.handle) H().hsa_signal_destroy(s);
  }
};

// Everything one probe allocates. Released right after the verdict, or — for
// the container entrypoint, which reports "ready" as soon as the verdict is
// known — after the JSON line is out (mi355x_hsa_probe_defer_release).
struct ProbeResources {
  hsa_code_object_reader_t reader{};
  hsa_executable_t exe{};
  hsa_queue_t* queue = nullptr;
  hsa_signal_t sig{};
  float* h_out = nullptr;
  uint32_t* h_meta = nullptr;
  float* d_scratch = nullptr;
  mi355x_liveness_args* kargs = nullptr;

  void release() {
    if (kargs) H().hsa_amd_memory_pool_free(kargs);
    if (d_scratch) H().hsa_amd_memory_pool_free(d_scratch);
    if (h_meta) H().hsa_amd_memory_pool_free(h_meta);
    if (h_out) H().hsa_amd_memory_pool_free(h_out);
    if (sig.handle) H().hsa_signal_destroy(sig);
    if (queue) H().hsa_queue_destroy(queue);
    if (exe.handle) H().hsa_executable_destroy(exe);
    if (reader.handle) H().hsa_code_object_reader_destroy(reader);
    *this = ProbeResources{};
  }
};

// kernarg buffer size; the code object's segment size is checked against it
constexpr uint32_t kKernargBytes = 256;

struct KernelInfo {
  uint64_t kobj = 0;
  uint32_t kseg = 0, gseg = 0, pseg = 0;
};

// Kept ("resident") per-device resources for mi355x_hsa_probe_keep(1).
struct Resident {
  std::timed_mutex mu;  // one probe at a time per device (a waiter gives up at its deadline)
  bool ready = false;
  ProbeResources r;
  KernelInfo k;
  // a dispatch that has not completed yet (a tenant's long kernel holds every
  // CU, or the device hangs): the next probe waits for it instead of
  // submitting another or abandoning the queue with its 181 MB save area
  bool pending = false;
  uint32_t pending_nonce = 0;
  int pending_iters = 1;
  std::chrono::steady_clock::time_point pending_since{};
  // a chip sweep / throughput check submitted on this kept queue that did not
  // complete within its deadline: probes report pending until it has
  std::shared_ptr<SigRef> blocker;
  std::chrono::steady_clock::time_point blocked_since{};
};

extern Runtime g_rt;                 // the process' ROCr view (hsa_probe.cpp)
extern std::mutex g_resident_mu;     // guards g_keep and the kept-slot list
extern bool g_keep;                  // mi355x_hsa_probe_keep(1): per-device queues stay

// identity / error helpers
void set_status(mi355x_probe_result* r, hsa_status_t s, const char* what);
void fill_identity(const Agent& ag, int ordinal, mi355x_probe_result* out);
void bus_id(const Agent& ag, char* out, size_t n);
// bounded wait for a completion signal (value 1 -> 0)
bool wait_signal(hsa_signal_t sig, double timeout_s);

// queue + buffers and the liveness executable for `ag`; false with out->error
bool setup_resources(const Agent& ag, ProbeResources& r, KernelInfo& k, mi355x_probe_result* out);
// the kept slot of `ordinal` (created on first use); every kept slot freed
Resident* resident_slot(int ordinal);
void release_residents();

// chip sweeps / throughput checks that outlived their deadline (hsa_chip.cpp):
// seconds the one on `ordinal` has been outstanding (0 = none; a completed
// one is freed), and forgetting them all at runtime shutdown
double in_flight_for(int ordinal);
void forget_in_flight_sweeps();

}  // namespace mi355x::hsa_rt
