#!/bin/bash
# Does any ROCr knob make its internal (trap handler / blit) queue an SDMA queue
# (no CWSR area, no AMDKFD_IOC_SVM)? rocr_devsetup with the ioctl timer,
# code-first order, per env variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
g++ -O2 -std=c++17 -DMI355X_IOCTL_TRACE -rdynamic -I/opt/rocm/include native/tools/rocr_devsetup.cpp \
    -o gpurun_out/rocr_devsetup_io -ldl -pthread || exit 1
CO=rocm_k8s_device_plugin_amd/kernels/liveness_gfx950.hsaco
OUT=gpurun_out/devsetup_knobs_ioctl.jsonl
rm -f $OUT
run() {
  local label=$1; shift
  for i in 1 2 3; do
    env "$@" timeout -k 5 60 gpurun_out/rocr_devsetup_io "$CO" --order code-first \
      | sed "s/^{/{\"variant\":\"$label\",/" >> $OUT || return 1
    sleep 0.4
  done
}
run default X=1 && run sdma_on HSA_ENABLE_SDMA=1 && run sdma_off HSA_ENABLE_SDMA=0 \
  && run force_sdma_0 HSA_FORCE_SDMA_SIZE=0 && run force_sdma_1 HSA_FORCE_SDMA_SIZE=1 \
  && run sdma_override HSA_ENABLE_SDMA_COPY_SIZE_OVERRIDE=1 && run co_dma_0 HSA_CO_DMACOPY_SIZE=0 \
  && run queue_devmem HSA_ALLOCATE_QUEUE_DEV_MEM=1 || exit 1
python - <<'PY'
import json, statistics, collections
rows = [json.loads(l) for l in open("gpurun_out/devsetup_knobs_ioctl.jsonl")]
res = {}
for v in dict.fromkeys(r["variant"] for r in rows):
    rs = [r for r in rows if r["variant"] == v]
    out = {}
    for step in ("exe_freeze", "queue_create", "queue_create_2nd", "dispatch_wait"):
        ms = [s["ms"] for r in rs for s in r["steps"] if s["name"] == step]
        io = collections.defaultdict(list)
        for r in rs:
            for s in r["steps"]:
                if s["name"] == step:
                    for k, x in (s.get("ioctls") or {}).items():
                        io[k].append(x["ms"])
        out[step] = {"ms_p50": round(statistics.median(ms), 3) if ms else None,
                     "ioctl_ms_p50": {k: round(statistics.median(x), 3) for k, x in io.items() if statistics.median(x) > 0.05}}
    out["ok"] = all(r["ok"] for r in rs)
    out["device_setup_ms_p50"] = round(statistics.median(r["device_setup_ms"] for r in rs), 2)
    res[v] = out
    print(v, out["ok"], out["device_setup_ms_p50"], {k: (x["ms_p50"], x["ioctl_ms_p50"]) for k, x in out.items() if isinstance(x, dict)})
json.dump(res, open("gpurun_out/devsetup_knobs_ioctl_box.json", "w"), indent=1)
PY
