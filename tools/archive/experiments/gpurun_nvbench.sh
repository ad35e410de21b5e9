#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --hip-compare 0 --b2b-compare 0 --node-view-compare 6 > gpurun_out/bench_nv.json 2> gpurun_out/bench_nv.err || { tail -30 gpurun_out/bench_nv.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_nv.json'));e=d['extra'];print(d['value'], e['latency_p50_ms_node_view_emulated'], e['node_view_emulated_runtime_init_p50_ms'], e['container_phases_p50_ms'])"
tail -5 gpurun_out/bench_nv.err
