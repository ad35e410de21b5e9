#!/bin/bash
# GPU session: 1-GPU bench, default settle (kfd teardown) and back-to-back.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 400 python bench.py --gpus 1 --steps 40 --warmup 3 --hip-compare 10 --b2b-compare 10 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
timeout -k 10 300 python bench.py --gpus 1 --steps 40 --warmup 3 --settle none --hip-compare 0 > gpurun_out/bench1_b2b.json 2> gpurun_out/bench1_b2b.err || { tail gpurun_out/bench1_b2b.err; exit 1; }
cat gpurun_out/bench1_b2b.json
cat /proc/loadavg
