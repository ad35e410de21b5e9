#!/bin/bash
# Health loop with kept probe queues (default): sweep cost through the real plugin,
# and container start-up next to the loop.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/archive/experiments/health_sweep_gpu.py --sweeps 20 --pulse 0.5 --liveness-mode persistent \
  --out gpurun_out/health_sweep_kept.json --trace gpurun_out/health_trace_kept.json > gpurun_out/health_sweep_kept.log 2>&1 || { tail -30 gpurun_out/health_sweep_kept.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/health_sweep_kept.json'));d.pop('verdicts');print(d)"
timeout -k 10 400 python tools/health_interference.py --containers 15 --pulse 0.3 \
  --out gpurun_out/health_interference_kept.json > gpurun_out/health_interference_kept.log 2>&1 || { tail -30 gpurun_out/health_interference_kept.log; exit 1; }
cat gpurun_out/health_interference_kept.log; cat /proc/loadavg
