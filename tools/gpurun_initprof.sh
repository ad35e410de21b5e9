#!/bin/bash
# dlopen(ROCr) overlapped with the /dev/kfd open: start-up split + bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/container_ready_sweep.py --reps 15 --sample-init 250 --wait-kfd --tag "@wait_kfd" \
    --only hsa:rocr_visible,hip:rocr_visible --out gpurun_out/container_dlopen.json > gpurun_out/container_dlopen.log 2>&1 || { cat gpurun_out/container_dlopen.log; exit 1; }
cat gpurun_out/container_dlopen.log
timeout -k 10 400 python bench.py --gpus 1 --steps 40 --warmup 3 --hip-compare 10 --b2b-compare 10 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json; cat /proc/loadavg
