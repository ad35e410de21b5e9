#!/bin/bash
# Verdict r2 item 8: which ROCr call creates the kept-queue probe server's
# second kfd queue (and its 181 MB CWSR area), and does any ROCr knob avoid it.
#  1. rocr_queue_origin: CREATE_QUEUE args + call stack per step, both orders.
#  2. the same under env variants.
#  3. the real probe server's RSS / kfd queues under the same variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
g++ -O1 -g -std=c++17 -rdynamic -I/opt/rocm/include native/tools/rocr_queue_origin.cpp \
    -o gpurun_out/rqo -ldl -pthread || exit 1
CO=rocm_k8s_device_plugin_amd/kernels/liveness_gfx950.hsaco
OUT=gpurun_out/queue_origin.jsonl
RSS=gpurun_out/queue_origin_rss.jsonl
rm -f $OUT $RSS
run() {
  local label=$1; shift
  env "$@" ROCR_VISIBLE_DEVICES=0 timeout -k 5 60 gpurun_out/rqo "$CO" \
    | sed "s/^{/{\"variant\":\"$label\",/" >> $OUT || return 1
  env "$@" ROCR_VISIBLE_DEVICES=0 timeout -k 5 60 gpurun_out/rqo "$CO" --code-first \
    | sed "s/^{/{\"variant\":\"$label\",/" >> $OUT || return 1
  env "$@" timeout -k 5 90 python3 tools/archive/experiments/queue_origin_rss.py "$label" >> $RSS || return 1
  echo "variant $label done"
}
run default X=1 \
  && run max_queues_1 HSA_MAX_QUEUES=1 \
  && run scratch_async_reclaim_0 HSA_ENABLE_SCRATCH_ASYNC_RECLAIM=0 \
  && run no_scratch_reclaim HSA_NO_SCRATCH_RECLAIM=1 \
  && run sdma_0 HSA_ENABLE_SDMA=0 \
  && run debug_1 HSA_ENABLE_DEBUG=1 \
  && run interrupt_0 HSA_ENABLE_INTERRUPT=0 \
  && run queue_devmem HSA_ALLOCATE_QUEUE_DEV_MEM=1 \
  && run copy_agents_0 HSA_DISCOVER_COPY_AGENTS=0 \
  && run pc_sampling_off HSA_DISABLE_PC_SAMPLING=1 || exit 1
python3 - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/queue_origin.jsonl")]
rss = {r["variant"]: r for r in (json.loads(l) for l in open("gpurun_out/queue_origin_rss.jsonl"))}
out = {}
for r in rows:
    key = f'{r["variant"]}/{r.get("order")}'
    steps = {}
    for s in r.get("steps", []):
        steps[s["step"]] = {"rss_mb": s["rss_kb"] // 1024, "kfd_queues": s["kfd_queues"],
                            "svm_mb": [x >> 20 for x in s["svm_sizes"]],
                            "create_queue": [{k: v for k, v in q.items() if k != "stack"} | {"stack": q["stack"][:8]}
                                             for q in s["create_queue"]]}
    out[key] = steps
    print(key, {k: (v["rss_mb"], v["kfd_queues"], [q["queue_type"] for q in v["create_queue"]], v["svm_mb"])
                for k, v in steps.items()})
for v, r in rss.items():
    print("server", v, r["server_mb"], r["probes"])
json.dump({"tool": out, "probe_server": rss}, open("gpurun_out/queue_origin_box.json", "w"), indent=1)
PY
