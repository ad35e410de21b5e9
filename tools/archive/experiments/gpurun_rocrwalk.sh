#!/bin/bash
# ROCr's sysfs walk at hsa_init and what the -node_view / -topology_view
# container views would save (emulated in-process, native/tools/rocr_initprof.cpp).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
g++ -O2 -std=c++17 -rdynamic -I/opt/rocm/include native/tools/rocr_initprof.cpp -o gpurun_out/rocr_initprof -ldl -pthread || exit 1
python tools/archive/experiments/view_emulation.py /tmp/mi355x_views > gpurun_out/view_emulation.json || exit 1
cat gpurun_out/view_emulation.json | cut -c1-400; echo
spec() { python -c "import json;print(json.load(open('gpurun_out/view_emulation.json'))['$1'])"; }
run() {  # label, env assignment...; 12 fresh processes, 300 ms apart (past the previous kfd teardown)
  local label=$1; shift
  for i in $(seq 12); do
    env "$@" ROCR_VISIBLE_DEVICES=0 timeout -k 5 60 gpurun_out/rocr_initprof >> "gpurun_out/walk_$label.jsonl" || return 1
    sleep 0.3
  done
}
rm -f gpurun_out/walk_*.jsonl
run base X=1 && run node_view "MI355X_INITPROF_REDIRECT=$(spec node)" \
  && run topology_view "MI355X_INITPROF_REDIRECT=$(spec topology)" \
  && run both_views "MI355X_INITPROF_REDIRECT=$(spec both)" \
  && run hide_cpu_caches "MI355X_INITPROF_HIDE=/sys/devices/system/node/nodeN/cpuN/cache" \
  && run hide_gpu_caches "MI355X_INITPROF_HIDE=/sys/devices/virtual/kfd/kfd/topology/nodes/N/caches" || exit 1
python - <<'PY'
import json, statistics, glob
res = {}
for f in sorted(glob.glob("gpurun_out/walk_*.jsonl")):
    rows = [json.loads(l) for l in open(f)]
    k = f.split("walk_")[1][:-6]
    res[k] = {"ok": all(r["ok"] for r in rows), "agents": rows[0]["agents"],
              "hsa_init_ms_p50": round(statistics.median(r["hsa_init_ms"] for r in rows), 2),
              "hsa_init_ms_min": round(min(r["hsa_init_ms"] for r in rows), 2),
              "opens": rows[0]["opens"], "hidden": rows[0]["hidden"], "redirected": rows[0]["redirected"],
              "top": dict(list(rows[0]["by_template"].items())[:6])}
    print(k, {kk: v for kk, v in res[k].items() if kk != "top"})
json.dump(res, open("gpurun_out/rocr_walk_views.json", "w"), indent=1)
PY
