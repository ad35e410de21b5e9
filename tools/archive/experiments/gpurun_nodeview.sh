#!/bin/bash
# Container entrypoint end to end (ROCr init + MFMA probe) against an emulated
# -node_view / -topology_view (path interposition; bind mounts need root here).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
HSACO="$PWD/rocm_k8s_device_plugin_amd/kernels/liveness_gfx950.hsaco"
g++ -O2 -std=c++17 -rdynamic -DMI355X_PROBE_HSA=1 -DMI355X_HSACO_PATH="\"$HSACO\"" -Inative/include -Inative/src/health \
  -I/opt/rocm/include native/src/health/probe_main.cpp native/src/health/hsa_probe.cpp native/tools/probe_emu.cpp \
  -o gpurun_out/probe_emu -ldl -pthread || exit 1
python tools/archive/experiments/view_emulation.py /tmp/mi355x_views > gpurun_out/view_emulation.json || exit 1
spec() { python -c "import json;print(json.load(open('gpurun_out/view_emulation.json'))['$1'])"; }
NODE=$(spec node); BOTH=$(spec both)
sweep() {  # tag, extra args...
  local tag=$1; shift
  timeout -k 10 300 python tools/container_ready_sweep.py --reps 15 --wait-kfd --only hsa:rocr_visible --tag "$tag" \
    --exe gpurun_out/probe_emu "$@" --out "gpurun_out/nodeview_$tag.json" > "gpurun_out/nodeview_$tag.log" 2>&1 \
    || { cat "gpurun_out/nodeview_$tag.log"; return 1; }
  cut -c1-330 "gpurun_out/nodeview_$tag.log"
}
sweep @emu_plain && sweep @emu_node_view --env "MI355X_INITPROF_REDIRECT=$NODE" \
  && sweep @emu_both_views --env "MI355X_INITPROF_REDIRECT=$BOTH" && sweep @emu_plain_again || exit 1
cat /proc/loadavg
