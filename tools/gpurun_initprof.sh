#!/bin/bash
# Does waiting for the previous process' kfd procfs entry to vanish remove the
# next process' open("/dev/kfd") wait?
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/container_ready_sweep.py --reps 15 --sample-init 250 --wait-kfd --tag "@wait_kfd" \
    --only hsa:rocr_visible --out gpurun_out/container_wait_kfd.json > gpurun_out/container_wait_kfd.log 2>&1 || { cat gpurun_out/container_wait_kfd.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/container_wait_kfd.json'));print({k:(v['hip_init_ms'],v['ready_ms'],v.get('kfd_linger_ms'),v['init_profile']) for k,v in d.items()})"
