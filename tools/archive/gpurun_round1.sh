#!/bin/bash
# Round-1 GPU session: gpu tests, container-ready sweep, rocprof of both probe paths, 1-GPU bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 400 python -m pytest tests/test_gpu.py -q -m gpu -rA > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python tools/container_ready_sweep.py --reps 10 --out gpurun_out/container_sweep.json > gpurun_out/container_sweep.log 2>&1 || exit 1
echo "sweep ok"
cat gpurun_out/container_sweep.log
export TMPDIR=/tmp
P="$GRAFT_REPO_ROOT/rocm_k8s_device_plugin_amd/bin"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/hsa" -o probe -- "$P/mi355x-liveness-probe" --devices all --iters 4 > gpurun_out/prof_probe_hsa.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/hip" -o probe -- "$P/mi355x-liveness-probe-hip" --devices all --iters 4 > gpurun_out/prof_probe_hip.log 2>&1 || exit 1
echo "rocprof ok"
timeout -k 10 300 python bench.py --gpus 1 --steps 30 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 1
echo "bench ok"
cat gpurun_out/bench1.json
