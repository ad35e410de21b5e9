// Host side of the per-device MFMA liveness probe.
//
// Used three ways:
//   * `mi355x-liveness-probe` executable — what the device plugin's health
//     loop runs in a child process per sweep, under a hard deadline, so a
//     wedged GPU can never block ListAndWatch and no HIP context is held on
//     devices that pods own;
//   * the same executable is the "container entrypoint" of the
//     Allocate->ContainerReady benchmark;
//   * the `_hip` Python extension, for in-process GPU tests and smoke().
#pragma once

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int ordinal;            // HIP device ordinal probed
  int ok;                 // 1 = tile bit-exact, nonce echoed, no HIP error
  int hip_error;          // first hipError_t seen (0 = none)
  int mismatches;         // elements differing from the host reference
  uint32_t nonce;
  uint32_t xcc_id;        // HW_REG_XCC_ID of the wave that ran
  uint32_t hw_id;
  int iters;
  double kernel_us;       // hipEvent-timed dispatch
  double total_us;        // set-device + alloc + launch + copy-back + verify
  char pci_bus_id[32];    // hipDeviceGetPCIBusId
  char arch[64];          // gcnArchName, e.g. "gfx950:sramecc+:xnack-"
  char name[128];
  char uuid[40];          // hex of hipDeviceProp_t.uuid
  int pci_domain, pci_bus, pci_device;
  int cu_count;
  uint64_t total_mem;
  char error[160];
} mi355x_probe_result;

// Number of HIP devices, or -hipError on failure.
int mi355x_probe_device_count(void);
// Probe one device. Returns 0 if the device is live, non-zero otherwise
// (details in *out).
int mi355x_probe_device(int ordinal, uint32_t nonce, int iters, mi355x_probe_result* out);
// Fill only the identity fields (bus id, uuid, arch) without launching.
int mi355x_probe_identify(int ordinal, mi355x_probe_result* out);

#ifdef __cplusplus
}
#endif
