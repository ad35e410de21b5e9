#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python tools/archive/experiments/topology_read_cost.py > gpurun_out/topology_read_cost.json 2>&1 || exit 1
cat gpurun_out/topology_read_cost.json
ls /sys/class/kfd/kfd/topology/nodes/9/ 2>&1 | head; ls /sys/class/kfd/kfd/topology/nodes/9/caches | wc -l
cat /sys/class/kfd/kfd/topology/nodes/2/properties 2>&1 | head -3
