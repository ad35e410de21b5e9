#!/bin/bash
# Does any ROCr environment knob (something the plugin could set through the
# Allocate envs, no mounts needed) skip the hsa_init sysfs walk?
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
g++ -O2 -std=c++17 -rdynamic -I/opt/rocm/include -Inative/tools native/tools/rocr_initprof.cpp -o gpurun_out/rocr_initprof -ldl -pthread || exit 1
run() {  # label, env assignment...; 10 fresh processes, 300 ms apart (past the previous kfd teardown)
  local label=$1; shift
  for i in $(seq 10); do
    env "$@" ROCR_VISIBLE_DEVICES=0 timeout -k 5 60 gpurun_out/rocr_initprof >> "gpurun_out/knob_$label.jsonl" || return 1
    sleep 0.3
  done
}
rm -f gpurun_out/knob_*.jsonl
run base X=1 && run disable_cache HSA_DISABLE_CACHE=1 && run no_copy_agents HSA_DISCOVER_COPY_AGENTS=0 \
  && run no_interrupt HSA_ENABLE_INTERRUPT=0 && run no_dtif HSA_ENABLE_DTIF=0 && run base2 X=1 || exit 1
python - <<'PY'
import json, statistics, glob
res = {}
for f in sorted(glob.glob("gpurun_out/knob_*.jsonl")):
    rows = [json.loads(l) for l in open(f)]
    k = f.split("knob_")[1][:-6]
    res[k] = {"ok": all(r["ok"] for r in rows), "agents": rows[0]["agents"],
              "hsa_init_ms_p50": round(statistics.median(r["hsa_init_ms"] for r in rows), 2),
              "hsa_init_ms_min": round(min(r["hsa_init_ms"] for r in rows), 2),
              "opens": rows[0]["walk"]["opens"] if isinstance(rows[0].get("walk"), dict) else None}
    print(k, res[k])
json.dump(res, open("gpurun_out/rocr_knobs.json", "w"), indent=1)
PY
