#!/bin/bash
# One process, K device setups on parallel threads (same GPU): does queue /
# code-object setup serialise inside a process?
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P=rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe
for k in 1 2 4 8; do
  devs=$(python -c "print(','.join(['0']*$k))")
  for r in 1 2 3; do
    timeout -k 10 60 $P --devices $devs > gpurun_out/threads_$k.json || exit 1
    python -c "
import json;d=json.load(open('gpurun_out/threads_$k.json'))
ds=d['devices']; print($k, 'ok',d['ok'], 'init_ms',round((d['t_runtime_ns']-d['t_start_ns'])/1e6,1), 'device_ms', round((d['t_ready_ns']-d['t_runtime_ns'])/1e6,1), 'setup_us max', round(max(x['setup_us'] for x in ds)), 'queue_us', [round(x['phase_us']['queue']) for x in ds])"
    sleep 0.3
  done
done
