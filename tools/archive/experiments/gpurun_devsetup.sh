#!/bin/bash
# Per-call cost of the container entrypoint's device set-up after hsa_init
# (queue, signal, allocations, code object, first dispatch), one ROCr call at a
# time with the blocking syscall sampled and this process' kfd queues counted
# after each call (native/tools/rocr_devsetup.cpp), under a few ROCr env knobs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
g++ -O2 -std=c++17 -I/opt/rocm/include native/tools/rocr_devsetup.cpp -o gpurun_out/rocr_devsetup -ldl -pthread || exit 1
CO=rocm_k8s_device_plugin_amd/kernels/liveness_gfx950.hsaco
rm -f gpurun_out/devsetup_*.jsonl
run() {  # label, env assignments...
  local label=$1; shift
  for order in queue-first code-first; do
    for i in $(seq ${REPS:-4}); do
      env "$@" ROCR_VISIBLE_DEVICES=0 timeout -k 5 60 gpurun_out/rocr_devsetup "$CO" --order "$order" \
        | sed "s/^{/{\"variant\":\"$label\",/" >> "gpurun_out/devsetup_$label.jsonl" || return 1
      sleep 0.4   # past the previous process' kfd teardown
    done
  done
}
run default X=1 && run sdma_off HSA_ENABLE_SDMA=0 && run co_dmacopy_1g HSA_CO_DMACOPY_SIZE=1073741824 \
  && run co_dmacopy_0 HSA_CO_DMACOPY_SIZE=0 || exit 1
python - <<'PY'
import json, statistics, glob, collections
res = {}
for f in sorted(glob.glob("gpurun_out/devsetup_*.jsonl")):
    rows = [json.loads(l) for l in open(f)]
    for order in sorted({r["order"] for r in rows}):
        rs = [r for r in rows if r["order"] == order]
        key = f'{rs[0]["variant"]}:{order}'
        steps = collections.OrderedDict()
        prof = collections.defaultdict(collections.Counter)
        queues = {}
        for r in rs:
            for s in r["steps"]:
                steps.setdefault(s["name"], []).append(s["ms"])
                prof[s["name"]].update(s["profile"]["buckets"])
                queues[s["name"]] = s.get("kfd_queues")
        res[key] = {"ok": all(r["ok"] for r in rs), "runs": len(rs),
                    "hsa_init_ms_p50": round(statistics.median(r["hsa_init_ms"] for r in rs), 2),
                    "device_setup_ms_p50": round(statistics.median(r["device_setup_ms"] for r in rs), 2),
                    "steps_ms_p50": {k: round(statistics.median(v), 3) for k, v in steps.items()},
                    "kfd_queues_after": queues,
                    "steps_samples_100us": {k: dict(prof[k].most_common(3)) for k in steps}}
        slow = {k: v for k, v in res[key]["steps_ms_p50"].items() if v > 0.5}
        print(key, res[key]["ok"], res[key]["device_setup_ms_p50"], slow, queues.get("queue_create"),
              queues.get("exe_freeze"), queues.get("dispatch_wait_2nd"))
json.dump(res, open("gpurun_out/devsetup_box.json", "w"), indent=1)
PY
