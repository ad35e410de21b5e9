// Host side of the per-device MFMA liveness probe.
//
// Two launch paths for the same gfx950 code object:
//   * HSA-direct (mi355x_hsa_*): ROCr only, code object loaded from the
//     embedded .hsaco, one AQL kernel-dispatch packet on a private queue,
//     output in fine-grained host memory — exactly one dispatch per probe and
//     no HIP runtime start-up cost. This is what the plugin's health loop and
//     the benchmark's container entrypoint run by default.
//   * HIP (mi355x_probe_*): the same kernel through the HIP runtime, for the
//     in-process `_hip` extension and as a cross-check.
#pragma once

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int ordinal;            // HIP / HSA GPU agent ordinal probed
  int ok;                 // 1 = tile bit-exact, nonce echoed, no runtime error
  int hip_error;          // first hipError_t / hsa_status_t seen (0 = none)
  int mismatches;         // elements differing from the host reference
  uint32_t nonce;
  uint32_t xcc_id;        // HW_REG_XCC_ID of the wave that ran
  uint32_t hw_id;
  int iters;
  int dispatches;         // GPU dispatches issued by this probe
  int kfd_node_id;        // kfd topology node of the agent (-1 if unknown)
  double kernel_us;       // dispatch start->end (HSA profiling) or hipEvent time
  double setup_us;        // code object load + queue/stream + buffers
  double total_us;        // everything for this device, including verify
  // HSA path phases (us): 0 code object load+freeze, 1 queue+signal+buffers
  // (on a helper thread, overlapped with 0), 2 unused, 3 doorbell -> completion
  // signal observed on the host
  double phase_us[4];
  char runtime[8];        // "hsa" | "hip"
  char pci_bus_id[32];    // dddd:bb:dd.f
  char arch[64];          // e.g. "gfx950" / "gfx950:sramecc+:xnack-"
  char name[128];
  char uuid[40];
  int pci_domain, pci_bus, pci_device;
  int cu_count;
  uint64_t total_mem;
  // kept-queue path: the verdict belongs to a dispatch submitted by an earlier
  // probe (1), and how long the current outstanding dispatch has been pending
  int late;
  double pending_s;
  char error[160];
} mi355x_probe_result;

// ---- HIP path -------------------------------------------------------------
int mi355x_probe_device_count(void);
int mi355x_probe_device(int ordinal, uint32_t nonce, int iters, mi355x_probe_result* out);
int mi355x_probe_identify(int ordinal, mi355x_probe_result* out);
// 1 (default): the probe creates its own non-blocking stream; 0: it uses the
// null stream (measurement of what the stream's queue costs a HIP program)
void mi355x_probe_set_stream_mode(int own);
// 1: a probe's stream, events and buffers are kept until mi355x_probe_release()
// instead of freed before it returns -- the container entrypoint reports
// "ready" at the verified tile and tears down after its JSON line is out, as
// the HSA path does (mi355x_hsa_probe_defer_release)
void mi355x_probe_defer_release(int on);
void mi355x_probe_release(void);

// ---- HSA-direct path ------------------------------------------------------
// hsa_init + GPU agent enumeration; returns the number of GPU agents or
// -hsa_status_t. Idempotent.
int mi355x_hsa_probe_init(void);
int mi355x_hsa_probe_device(int ordinal, uint32_t nonce, int iters, double timeout_s, mi355x_probe_result* out);
int mi355x_hsa_probe_identify(int ordinal, mi355x_probe_result* out);
void mi355x_hsa_probe_shutdown(void);
// With defer on, probe resources (queue, executable, buffers) outlive the
// verdict until mi355x_hsa_probe_release(): a caller that reports readiness
// takes teardown off its critical path.
void mi355x_hsa_probe_defer_release(int on);
void mi355x_hsa_probe_release(void);
// With keep on, each device's queue, executable and buffers are created by its
// first probe and reused by every later one (released by shutdown, or dropped
// after a failed probe). A kept probe is one AQL packet: no kfd ioctl, so no
// HWS runlist update that would preempt the queues of the pods on that GPU.
void mi355x_hsa_probe_keep(int on);
// Debug fault injection: flip one bit of output word `word` (0..1023; -1 = off)
// of every later probe on `ordinal` (-1 = all devices) before verification.
// The verdict path (tile compare, JSON, plugin health) sees a wrong MFMA result.
void mi355x_hsa_probe_corrupt(int word, int ordinal);
// Runtime start-up split of the last mi355x_hsa_probe_init (us): dlopen of
// ROCr (its constructors), pre-open of /dev/kfd (on a second thread,
// overlapped with the dlopen), hsa_init, agent enumeration, pool discovery.
void mi355x_hsa_init_phases(double out_us[5]);

// ---- xGMI / PCIe peer probe ------------------------------
// `bytes` of a nonce-derived pattern filled in src's HBM, copied src -> dst
// HBM by the DMA engines over the link between them (`reps` times, best time
// kept), then dst -> host and verified word by word. Link properties are ROCr's
// view of dst's HBM pool from src. src == dst exercises the same path on one
// device (single-GPU boxes).
typedef struct {
  int src, dst;              // HSA GPU agent ordinals
  int ok;
  int hsa_error;
  uint32_t value;            // fill pattern
  int access;                // hsa_amd_memory_pool_access_t of dst HBM from src
  int link_type;             // hsa_amd_link_info_type_t of the first hop (4 = xGMI, 2 = PCIe)
  uint32_t hops;
  uint32_t numa_distance;
  uint32_t link_max_bw_mbps; // ROCr's link bandwidth figure for the first hop
  int reps;
  uint64_t bytes;
  uint64_t mismatches;
  double copy_us_best;
  double gbps_best;
  double total_us;
  char src_bus_id[32];
  char dst_bus_id[32];
  char error[160];
} mi355x_peer_result;

int mi355x_hsa_peer_probe(int src, int dst, uint32_t nonce, uint64_t bytes, int reps, double timeout_s,
                          mi355x_peer_result* out);

// ---- full-chip sweep (every CU of every XCD) --------------------------------
// One workgroup per CU (each holds the CU's whole 160 KiB LDS), all resident
// at once (bounded wait), each checks 4 MFMA tiles against the VALU, writes
// and cross-reads the whole LDS, and reports its XCC / CU ids; the host
// verifies records and wave 0's tiles bit-exactly and counts the distinct
// CUs and XCDs that ran.
typedef struct {
  int ordinal;
  int ok;                 // every record present and correct, every tile exact, all XCDs seen
  int hsa_error;
  uint32_t nonce;
  int iters;
  int grid;               // workgroups launched (= agent CU count)
  int cu_count;           // HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT
  int num_xcc;            // HSA_AMD_AGENT_INFO_NUM_XCC
  int records_ok;         // workgroups whose record is present, echoed the nonce and found no fault
  uint32_t mfma_bad;      // MFMA elements differing from the VALU recomputation (all waves)
  uint32_t lds_bad;       // LDS words read back wrong
  uint32_t tile_bad;      // wave-0 tile elements differing from the host reference
  int cus_covered;        // distinct (XCC, SE, SH, CU) that ran a workgroup
  int xccs_covered;
  int all_resident;       // every workgroup saw the whole grid resident before working
  int wgs_per_xcc[16];
  double kernel_us;       // dispatch start -> end (HSA profiling)
  double arrival_spread_us;  // first to last workgroup arrival (s_memrealtime)
  double total_us;
  // > 0: an earlier sweep on this device has not completed for this long; its
  // queue and buffers stay allocated and no new sweep is submitted (at most one
  // outstanding sweep per device, so a wedged GPU leaks one queue, not one per cadence)
  double in_flight_s;
  int kept_queue;         // ran on the device's kept probe queue (--serve --keep), no queue of its own
  char error[160];
} mi355x_sweep_result;

int mi355x_hsa_chip_sweep(int ordinal, uint32_t nonce, int iters, double timeout_s, mi355x_sweep_result* out);

// ---- throughput check (idle GPUs only: it owns the chip for a few ms) --------
// HBM: fill `bytes` of device memory with an address-derived pattern (write
// bandwidth), read it back and verify every word (read bandwidth). MFMA: two
// register-resident bf16 v_mfma_f32_32x32x16 chains per wave, two waves per
// SIMD on every CU (sustained TFLOP/s), with each workgroup's shader clock
// from s_memtime / s_memrealtime, folded per XCD; every wave's accumulator
// checksum must be bit-identical (same operands everywhere).
typedef struct {
  int ordinal;
  int ok;                    // pattern exact, checksums identical, every record present, all XCDs ran
  int hsa_error;
  uint32_t nonce;
  uint64_t bytes;
  int cu_count;
  int num_xcc;
  double fill_us;            // kernel times (HSA dispatch profiling)
  double check_us;           // first read pass (right after the fill)
  double check2_us;          // second read pass
  double hbm_write_gbps;
  double hbm_read_gbps;      // from the faster read pass
  uint64_t hbm_bad_words;    // 32-bit words read back wrong (the pass that found more)
  uint64_t hbm_bad_words_pass2;
  int64_t hbm_first_bad;     // lowest failing 16-byte unit, -1 if none
  int mfma_iters;            // MFMA pairs per wave
  int mfma_grid;             // workgroups (MI355X_BURN_WGS_PER_CU per CU)
  int mfma_records_ok;
  int mfma_checksum_mismatch;  // waves whose checksum differs from workgroup 0 wave 0
  int mfma_xccs;             // distinct XCDs that ran burn workgroups
  double mfma_us;
  double mfma_tflops;        // dense bf16, from the dispatch time
  double clock_mhz_min;      // per-workgroup shader clock during the MFMA loop
  double clock_mhz_median;
  double clock_mhz_max;
  double xcd_clock_mhz[16];  // median per XCD (0 = no workgroup seen)
  double total_us;
  double in_flight_s;        // > 0: an earlier sweep / check on this device has not completed
  int kept_queue;            // ran on the device's kept probe queue (--serve --keep)
  char error[160];
} mi355x_perf_result;

int mi355x_hsa_perf_check(int ordinal, uint32_t nonce, uint64_t bytes, int mfma_iters, double timeout_s,
                          mi355x_perf_result* out);
// Debug fault injection: the fill pass writes 16-byte unit `unit` with its
// first word inverted, so the check pass must report exactly one bad word
// there (UINT64_MAX = off).
void mi355x_hsa_perf_poison(uint64_t unit);

#ifdef __cplusplus
}
#endif
