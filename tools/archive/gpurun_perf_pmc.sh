#!/bin/bash
# PMC counters of the throughput check's kernels (mi355x_hbm_fill / _check /
# mi355x_mfma_burn): MFMA busy cycles vs GPU-active cycles, HBM bytes fetched
# and written. One counter group per run, --kernel-trace only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc
P=$GRAFT_REPO_ROOT/rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe
cd /tmp && export TMPDIR=/tmp
run() {  # tag, counters
  local tag=$1 ctr=$2
  timeout -s KILL 60 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag -o $tag \
    -- $P --perf --perf-mib 4096 --perf-iters 65536 --devices 0 --timeout 20 > $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log 2>&1 \
    || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log; return 1; }
  find $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag -name "*counter_collection.csv" -exec cat {} \; | cut -d, -f9,16-19
}
run perf_a "SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
 && run perf_b "FETCH_SIZE" \
 && run perf_c "WRITE_SIZE" \
 && run perf_d "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
