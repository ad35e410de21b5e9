#!/bin/bash
# Concurrent container start-up: plain vs emulated -node_view.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
HSACO="$PWD/rocm_k8s_device_plugin_amd/kernels/liveness_gfx950.hsaco"
g++ -O2 -std=c++17 -rdynamic -DMI355X_PROBE_HSA=1 -DMI355X_HSACO_PATH="\"$HSACO\"" -Inative/include -Inative/src/health \
  -I/opt/rocm/include native/src/health/probe_main.cpp native/src/health/hsa_probe.cpp native/tools/probe_emu.cpp \
  -o gpurun_out/probe_emu -ldl -pthread || exit 1
python tools/archive/experiments/view_emulation.py /tmp/mi355x_views > gpurun_out/view_emulation.json || exit 1
NODE=$(python -c "import json;print(json.load(open('gpurun_out/view_emulation.json'))['node'])")
timeout -k 10 400 python tools/concurrent_containers.py --ks 1,2,4,8 --rounds 6 --exe gpurun_out/probe_emu \
  --env "MI355X_INITPROF_REDIRECT=$NODE" --out gpurun_out/concurrent_node_view.json > gpurun_out/concurrent_nv.log 2>&1 || { cat gpurun_out/concurrent_nv.log; exit 1; }
echo node_view; cat gpurun_out/concurrent_nv.log
timeout -k 10 400 python tools/concurrent_containers.py --ks 8 --rounds 6 --exe gpurun_out/probe_emu \
  --env "MI355X_INITPROF_HIDE=/sys/devices/virtual/kfd/kfd/topology/nodes/N/io_links" --out gpurun_out/concurrent_ctl.json > gpurun_out/concurrent_ctl.log 2>&1 || { cat gpurun_out/concurrent_ctl.log; exit 1; }
echo plain_emu_binary; cat gpurun_out/concurrent_ctl.log; cat /proc/loadavg
