#!/bin/bash
# GPU tests, persistent vs spawn liveness: sweep cost and interference with container start-up.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/archive/experiments/health_sweep_gpu.py --sweeps 20 --pulse 0.5 --liveness-mode persistent \
  --out gpurun_out/health_sweep_persistent.json --trace gpurun_out/health_trace_persistent.json > gpurun_out/health_sweep_persistent.log 2>&1 || { tail -30 gpurun_out/health_sweep_persistent.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/health_sweep_persistent.json'));d.pop('verdicts');print(d)"
timeout -k 10 400 python tools/health_interference.py --containers 15 --pulse 0.3 \
  --out gpurun_out/health_interference.json > gpurun_out/health_interference.log 2>&1 || { tail -30 gpurun_out/health_interference.log; exit 1; }
cat gpurun_out/health_interference.log; cat /proc/loadavg
