#!/bin/bash
# Which kfd ioctls the container entrypoint's device set-up spends its time in:
# rocr_devsetup built with the ioctl timer (native/tools/ioctl_trace.h), one
# ROCr call at a time, after the previous process' kfd teardown. Also reads the
# GPU node's CWSR / control-stack sizes from the kfd topology.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
g++ -O2 -std=c++17 -DMI355X_IOCTL_TRACE -rdynamic -I/opt/rocm/include native/tools/rocr_devsetup.cpp \
    -o gpurun_out/rocr_devsetup_io -ldl -pthread || exit 1
CO=rocm_k8s_device_plugin_amd/kernels/liveness_gfx950.hsaco
OUT=gpurun_out/devsetup_ioctl.jsonl
rm -f $OUT
for n in /sys/class/kfd/kfd/topology/nodes/*; do
  if grep -q "^simd_count [1-9]" $n/properties 2>/dev/null; then
    echo "node $(basename $n): $(grep -E '^(cwsr_size|ctl_stack_size|num_xcc|simd_count|max_waves_per_simd|drm_render_minor|gpu_id) ' $n/properties | tr '\n' ' ')"
  fi
done > gpurun_out/kfd_cwsr_props.txt
for order in queue-first code-first; do
  for i in $(seq ${REPS:-5}); do
    timeout -k 5 60 gpurun_out/rocr_devsetup_io "$CO" --order "$order" >> $OUT || exit 1
    sleep 0.4
  done
done
python - <<'PY'
import json, statistics, collections
rows = [json.loads(l) for l in open("gpurun_out/devsetup_ioctl.jsonl")]
res = {}
for order in ("queue-first", "code-first"):
    rs = [r for r in rows if r["order"] == order]
    agg = collections.OrderedDict()
    for r in rs:
        for s in r["steps"]:
            a = agg.setdefault(s["name"], {"ms": [], "io": collections.defaultdict(list)})
            a["ms"].append(s["ms"])
            for k, v in (s.get("ioctls") or {}).items():
                a["io"][k].append((v["n"], v["ms"]))
    init_io = collections.defaultdict(list)
    for r in rs:
        for k, v in (r.get("hsa_init_ioctls") or {}).items():
            init_io[k].append((v["n"], v["ms"]))
    out = {"runs": len(rs), "ok": all(r["ok"] for r in rs),
           "hsa_init_ms_p50": round(statistics.median(r["hsa_init_ms"] for r in rs), 2),
           "hsa_init_ioctls_p50": {k: {"n": statistics.median(x[0] for x in v), "ms": round(statistics.median(x[1] for x in v), 3)}
                                   for k, v in sorted(init_io.items())},
           "steps": {}}
    for name, a in agg.items():
        out["steps"][name] = {"ms_p50": round(statistics.median(a["ms"]), 3),
                              "ioctls_p50": {k: {"n": statistics.median(x[0] for x in v),
                                                 "ms": round(statistics.median(x[1] for x in v), 3)}
                                             for k, v in sorted(a["io"].items())}}
    res[order] = out
    print(order, out["hsa_init_ms_p50"], {k: (v["ms_p50"], v["ioctls_p50"]) for k, v in out["steps"].items() if v["ms_p50"] > 0.3})
json.dump(res, open("gpurun_out/devsetup_ioctl_box.json", "w"), indent=1)
PY
cat gpurun_out/kfd_cwsr_props.txt
