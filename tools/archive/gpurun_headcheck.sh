#!/bin/bash
# HEAD check on MI355X: what the round-end driver runs (GPU tests, smoke, default
# bench), a 100-admission headline run and a rocprofv3 kernel-stats profile of a
# short bench (the probe kernel inside the admission path).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/archive/gpurun_roundcheck.sh || exit 1
bash tools/archive/gpurun_bench100.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
find gpurun_out/prof_bench -name "*kernel_stats.csv" | head -3
