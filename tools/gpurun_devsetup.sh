#!/bin/bash
# Per-call cost of the container entrypoint's device set-up after hsa_init
# (queue, signal, allocations, code object, first dispatch), one ROCr call at a
# time with the blocking syscall sampled (native/tools/rocr_devsetup.cpp).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
g++ -O2 -std=c++17 -I/opt/rocm/include native/tools/rocr_devsetup.cpp -o gpurun_out/rocr_devsetup -ldl -pthread || exit 1
CO=rocm_k8s_device_plugin_amd/kernels/liveness_gfx950.hsaco
rm -f gpurun_out/devsetup_*.jsonl
for order in queue-first alloc-first code-first; do
  for i in $(seq 6); do
    ROCR_VISIBLE_DEVICES=0 timeout -k 5 60 gpurun_out/rocr_devsetup "$CO" --order "$order" \
      >> "gpurun_out/devsetup_$order.jsonl" || exit 1
    sleep 0.4   # past the previous process' kfd teardown
  done
done
python - <<'PY'
import json, statistics, glob, collections
res = {}
for f in sorted(glob.glob("gpurun_out/devsetup_*.jsonl")):
    rows = [json.loads(l) for l in open(f)]
    order = rows[0]["order"]
    steps = collections.OrderedDict()
    prof = collections.defaultdict(collections.Counter)
    for r in rows:
        for s in r["steps"]:
            steps.setdefault(s["name"], []).append(s["ms"])
            prof[s["name"]].update(s["profile"]["buckets"])
    res[order] = {"ok": all(r["ok"] for r in rows), "runs": len(rows),
                  "hsa_init_ms_p50": round(statistics.median(r["hsa_init_ms"] for r in rows), 2),
                  "device_setup_ms_p50": round(statistics.median(r["device_setup_ms"] for r in rows), 2),
                  "steps_ms_p50": {k: round(statistics.median(v), 3) for k, v in steps.items()},
                  "steps_samples_100us": {k: dict(prof[k].most_common(4)) for k in steps}}
    print(order, res[order]["device_setup_ms_p50"], res[order]["steps_ms_p50"])
json.dump(res, open("gpurun_out/devsetup_box.json", "w"), indent=1)
PY
