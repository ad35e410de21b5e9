#!/bin/bash
# Full-chip MFMA/LDS sweep: correctness, CU/XCD coverage, kernel time.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P=rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe
timeout -k 10 60 $P --sweep --devices 0 --iters 8 --timeout 10 > gpurun_out/sweep1.json || { cat gpurun_out/sweep1.json; exit 1; }
cat gpurun_out/sweep1.json; echo
for i in 1 2 3; do timeout -k 10 60 $P --sweep --devices 0 --timeout 10 >> gpurun_out/sweep_reps.jsonl || exit 1; done
python -c "
import json
for l in open('gpurun_out/sweep_reps.jsonl'):
    d=json.loads(l)['devices'][0]; print({k:d[k] for k in ('ok','records_ok','cus_covered','xccs_covered','all_resident','kernel_us','arrival_spread_us','wgs_per_xcc')})"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_sweep -o sweep -- $GRAFT_REPO_ROOT/$P --sweep --devices 0 --timeout 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_sweep.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_sweep.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_sweep -name "*kernel_stats.csv" -exec cat {} \;
