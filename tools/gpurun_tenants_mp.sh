#!/bin/bash
# GPU tests + smoke at HEAD, then the multi-process tenant interference case:
# 8 tenant processes x 4 GEMM streams on GPU 0, with and without the kept-queue probe server.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 500 python -u tools/tenant_interference.py --procs 8 --streams 4 --n 4096 --seconds 5 --pulse 0.05 --modes none,keep,per_sweep,none --out gpurun_out/tenant_mp_box.json > gpurun_out/tenant_mp.log 2>&1 || { tail -30 gpurun_out/tenant_mp.log; exit 1; }
cat gpurun_out/tenant_mp.log
