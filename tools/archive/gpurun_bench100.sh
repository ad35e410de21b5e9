#!/bin/bash
# 100 timed admissions at N=1 (headline statistics).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 100 --warmup 3 --json-out gpurun_out/bench_100.json > gpurun_out/bench_100.out 2> gpurun_out/bench_100.err || { tail -20 gpurun_out/bench_100.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_100.json")); e = d["extra"]
print("p50", d["value"], "p99", e["latency_p99_ms"], "mean", e["latency_mean_ms"], "rpc", e["plugin_rpc_p50_ms"],
      "phases", e["container_phases_p50_ms"])
PY
cat /proc/loadavg
