#!/bin/bash
# Round-3 GPU session: the default 1-GPU bench (gloo-only coordination: no GPU
# context in the bench process) and a 100-step run for the tail attribution.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/r3_bench_default.json 2> gpurun_out/r3_bench_default.err || { tail gpurun_out/r3_bench_default.err; exit 1; }
cat gpurun_out/r3_bench_default.json
timeout -k 10 500 python bench.py --gpus 1 --steps 100 --warmup 3 --hip-compare 20 > gpurun_out/r3_bench100.json 2> gpurun_out/r3_bench100.err || { tail gpurun_out/r3_bench100.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r3_bench_default.json", "gpurun_out/r3_bench100.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    e = d["extra"]
    print(f, d["value"], e["latency_p99_ms"], e["latency_p50_ms_with_hip_runtime_container"], e["bench_process_gpu"], e["launcher"])
    print(json.dumps(e["tail_attribution"]["by_phase"]), e["tail_attribution"]["phase_p50_ms"], e["tail_attribution"]["p99_over_p50"])
PY
