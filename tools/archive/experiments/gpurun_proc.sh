#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python tools/archive/experiments/proc_read_cost.py --out gpurun_out/proc_read_cost.json > gpurun_out/proc_read_cost.log 2>&1 || { cat gpurun_out/proc_read_cost.log; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/proc_read_cost.json'))
print({k:v for k,v in d.items() if k!='kfd_nodes'})
for k,v in d['kfd_nodes'].items(): print(k, v)"
grep -c processor /proc/cpuinfo
