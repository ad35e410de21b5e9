#!/bin/bash
# ROCr start-up breakdown of the container entrypoint (HSA and HIP builds),
# ROCr env knobs, and a sampled wall-clock profile of runtime init.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python tools/container_ready_sweep.py --reps 15 \
  --only hsa:rocr_visible,hip:rocr_visible,hsa:rocr_visible+disable_image,hsa:rocr_visible+tools_disable_register,hsa:rocr_visible+cu_mask_skip_init,hsa:rocr_visible+no_pc_sampling,hsa:rocr_visible+lean \
  --out gpurun_out/container_phases.json > gpurun_out/container_phases.log 2>&1 || { cat gpurun_out/container_phases.log; exit 1; }
cat gpurun_out/container_phases.log
timeout -k 10 300 python tools/container_ready_sweep.py --reps 15 --sample-init 250 \
  --only hsa:rocr_visible,hip:rocr_visible --out gpurun_out/container_init_profile.json \
  > gpurun_out/container_init_profile.log 2>&1 || { cat gpurun_out/container_init_profile.log; exit 1; }
cat gpurun_out/container_init_profile.log
uptime
