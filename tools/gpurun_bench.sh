#!/bin/bash
# GPU session: gpu tests + 1-GPU bench (both container runtimes) + sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu.py -q -m gpu -rA > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --gpus 1 --steps 40 --warmup 3 --hip-compare 15 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 1
cat gpurun_out/bench1.json
timeout -k 10 300 python bench.py --gpus 1 --steps 40 --warmup 3 --container-runtime hip --hip-compare 0 > gpurun_out/bench1_hip.json 2> gpurun_out/bench1_hip.err || exit 1
cat gpurun_out/bench1_hip.json
