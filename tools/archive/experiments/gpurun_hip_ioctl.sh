#!/bin/bash
# What does the HIP runtime add to a container's start-up over ROCr-direct?
# Both liveness entrypoints linked with the ioctl timer (native/tools/
# ioctl_trace_main.cpp), 6 fresh processes each after the previous teardown.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
# both entrypoints are linked on the build host (the object files stay there):
#   build/measure/probe_{hsa,hip}_io  (see the commit that added this script)
for rt in hsa hip; do test -x build/measure/probe_${rt}_io || { echo "missing build/measure/probe_${rt}_io"; exit 1; }; done
for rt in hsa hip; do
  for i in 1 2 3 4 5 6; do
    ROCR_VISIBLE_DEVICES=0 timeout -k 5 60 build/measure/probe_${rt}_io --devices 0 --iters 4 \
        > gpurun_out/hipio_${rt}_$i.json 2> gpurun_out/hipio_${rt}_$i.err || { tail gpurun_out/hipio_${rt}_$i.err; exit 1; }
    sleep 0.5
  done
done
python - <<'PY'
import json, glob, statistics, collections
res = {}
for rt in ("hsa", "hip"):
    io = collections.defaultdict(list); ready = []; init = []
    for i in range(1, 7):
        doc = json.loads(open(f"gpurun_out/hipio_{rt}_{i}.json").read().strip().splitlines()[-1])
        ready.append((doc["t_ready_ns"] - doc["t_start_ns"]) / 1e6)
        init.append((doc["t_runtime_ns"] - doc["t_start_ns"]) / 1e6)
        for line in open(f"gpurun_out/hipio_{rt}_{i}.err"):
            if line.startswith("IOCTL_TRACE "):
                for k, v in json.loads(line[12:]).items():
                    io[k].append((v["n"], v["ms"]))
    res[rt] = {"main_to_ready_ms_p50": round(statistics.median(ready), 2), "runtime_init_ms_p50": round(statistics.median(init), 2),
               "ioctls_p50": {k: {"n": statistics.median(x[0] for x in v), "ms": round(statistics.median(x[1] for x in v), 3)}
                              for k, v in sorted(io.items())}}
    print(rt, res[rt]["main_to_ready_ms_p50"], res[rt]["runtime_init_ms_p50"],
          {k: v for k, v in res[rt]["ioctls_p50"].items() if v["ms"] > 0.2})
json.dump(res, open("gpurun_out/hip_vs_hsa_ioctl_box.json", "w"), indent=1)
PY
