#!/bin/bash
# Kept-queue probe server on the GPU, then the tenant-interference comparison
# (a GEMM workload timed per kernel while the liveness loop probes the same GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "persistent_probe_server" > gpurun_out/pytest_gpu_keep.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_keep.log; exit 1; }
tail -4 gpurun_out/pytest_gpu_keep.log
timeout -k 10 300 python -u tools/tenant_interference.py --seconds 6 --pulse ${PULSE:-0.05} \
  --modes none,per_sweep,keep,none,per_sweep,keep --out gpurun_out/tenant_interference.json \
  > gpurun_out/tenant_interference.log 2>&1 || { tail -30 gpurun_out/tenant_interference.log; exit 1; }
cat gpurun_out/tenant_interference.log
