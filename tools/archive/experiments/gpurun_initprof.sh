#!/bin/bash
# ROCr start-up CPU split (user vs kernel) and blocking-syscall attribution.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/container_ready_sweep.py --reps 15 --sample-init 100 --wait-kfd --tag "@wait_kfd" \
    --only hsa:rocr_visible,hsa:rocr_visible+identify_only --out gpurun_out/container_cpusplit.json > gpurun_out/container_cpusplit.log 2>&1 || { cat gpurun_out/container_cpusplit.log; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/container_cpusplit.json'))
for k,v in d.items(): print(k, 'init',v['hip_init_ms'],'ready',v['ready_ms'],'cpu',v['cpu_ms_runtime'],'user',v['cpu_user_ms_runtime'],'reads',v['read_syscalls_runtime'],v['init_us'],v['init_profile'])"
