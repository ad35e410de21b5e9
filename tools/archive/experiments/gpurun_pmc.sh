#!/bin/bash
# PMC counters of the chip sweep and the one-wave probe (counter runs use
# --kernel-trace/--stats only, as required).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc
P=$GRAFT_REPO_ROOT/rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe
cd /tmp && export TMPDIR=/tmp
run() {  # tag, counters, probe args...
  local tag=$1 ctr=$2; shift 2
  timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag -o $tag \
    -- $P "$@" > $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log; return 1; }
  find $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag -name "*counter_collection.csv" -exec cat {} \; | cut -d, -f1-3,11- | head -20
}
run sweep_a "SQ_WAVES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CU_CYCLES" --sweep --devices 0 --timeout 10 \
 && run sweep_b "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU" --sweep --devices 0 --timeout 10 \
 && run tile_a "SQ_WAVES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU" --devices 0 --iters 4
