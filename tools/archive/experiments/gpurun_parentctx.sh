#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=hsa:rocr_visible,hip:rocr_visible
timeout -k 10 200 python tools/container_ready_sweep.py --reps 20 --only $V > gpurun_out/sweep_noparent.log 2>&1 || exit 1
timeout -k 10 200 python tools/container_ready_sweep.py --reps 20 --only $V --parent-gpu > gpurun_out/sweep_parentgpu.log 2>&1 || exit 1
timeout -k 10 200 python tools/container_ready_sweep.py --reps 20 --only $V > gpurun_out/sweep_noparent2.log 2>&1 || exit 1
cat gpurun_out/sweep_noparent.log gpurun_out/sweep_parentgpu.log gpurun_out/sweep_noparent2.log
nproc; uptime
