#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python tools/archive/experiments/topology_view_experiment.py 12 > gpurun_out/topology_view_experiment.json 2>&1
echo "rc=$?"
cat gpurun_out/topology_view_experiment.json
