#!/bin/bash
# Session-3 GPU checks: device set-up cost split, new GPU tests (models, fabric
# links, RCCL collectives CLI).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 240 bash tools/gpurun_devsetup.sh > gpurun_out/devsetup.log 2>&1 || { tail -20 gpurun_out/devsetup.log; exit 1; }
cat gpurun_out/devsetup.log
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "model or fabric or collectives" > gpurun_out/pytest_gpu_s3.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_s3.log; exit 1; }
tail -6 gpurun_out/pytest_gpu_s3.log
