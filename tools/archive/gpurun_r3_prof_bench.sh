#!/bin/bash
# Round 3: rocprofv3 kernel stats of a short bench through the native daemon
# (container MFMA probes, throughput-check kernels, peer-probe copy).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof_r3_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3_bench -o bench -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof_r3_bench.log 2>&1 || { tail -20 gpurun_out/prof_r3_bench.log; exit 1; }
find gpurun_out/prof_r3_bench -name "*kernel_stats.csv"
