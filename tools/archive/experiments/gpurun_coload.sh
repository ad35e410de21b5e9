#!/bin/bash
# Device setup phases (code object load, queue creation) vs ROCr loader knobs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in default "HSA_CO_DMACOPY_SIZE=1073741824" "HSA_CO_DMACOPY_SIZE=0" "HSA_ENABLE_SDMA=0" "HSA_ALLOCATE_QUEUE_DEV_MEM=1"; do
  args=(); [ "$v" != default ] && args=(--env "$v")
  timeout -k 10 200 python tools/container_ready_sweep.py --reps 10 --wait-kfd --only hsa:rocr_visible --tag "@$v" "${args[@]}" \
    --out "gpurun_out/coload.json" > gpurun_out/coload.log 2>&1 || { cat gpurun_out/coload.log; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/coload.json'))
for k,v in d.items(): print(k, 'ready', v['ready_ms'], 'device', v['device_ms'], v['phase_us'], 'total', v.get('setup_us'))"
done
