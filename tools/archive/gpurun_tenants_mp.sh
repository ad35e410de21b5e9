#!/bin/bash
# Multi-process tenant interference (num_cp_queues of the GPU first):
# 8 tenant processes x 4 GEMM streams on GPU 0: no prober, kept-queue server, the monitor (crowded step-off).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cat /sys/class/kfd/kfd/topology/nodes/*/properties 2>/dev/null | grep -E "num_cp_queues|num_xcc" | sort | uniq -c || true
timeout -k 10 500 python -u tools/tenant_interference.py --procs 8 --streams 4 --n 4096 --seconds 5 --pulse 0.05 --modes none,keep,monitor,none --out gpurun_out/tenant_mp_box.json > gpurun_out/tenant_mp.log 2>&1 || { tail -30 gpurun_out/tenant_mp.log; exit 1; }
cat gpurun_out/tenant_mp.log
