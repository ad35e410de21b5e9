#!/bin/bash
# GPU session 2: full gpu test suite (incl. rocprof dispatch-count tests), health sweep with the
# MFMA liveness probe through the real plugin + trace, 1-GPU bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu.py -q -m gpu -rA > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/archive/experiments/health_sweep_gpu.py --sweeps 20 --out gpurun_out/health_sweep.json --trace gpurun_out/health_trace.json > gpurun_out/health_sweep.log 2>&1 || exit 1
tail -5 gpurun_out/health_sweep.log
timeout -k 10 300 python bench.py --gpus 1 --steps 40 --warmup 3 --hip-compare 10 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 1
cat gpurun_out/bench1.json
