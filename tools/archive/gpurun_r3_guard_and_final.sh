#!/bin/bash
# Round 3, last HEAD check: the bench extras deadline on MI355X, then what the
# round-end driver runs (smoke, -m gpu suite, default bench), then rocprofv3
# kernel stats of a short bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/archive/gpurun_r3_extras_guard.sh || exit 1
bash tools/archive/gpurun_r3_final.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
find gpurun_out/prof_bench -name "*kernel_stats.csv"
