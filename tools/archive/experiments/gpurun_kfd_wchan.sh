#!/bin/bash
# Where does open("/dev/kfd") block while the previous GPU process is torn down?
# Back-to-back container starts with the init sampler naming the kernel wait
# function (wchan) of every thread in uninterruptible sleep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/container_ready_sweep.py --reps 12 --sample-init 250 --tag "@b2b" \
    --only hsa:rocr_visible --out gpurun_out/kfd_wchan_b2b.json > gpurun_out/kfd_wchan_b2b.log 2>&1 || { tail -20 gpurun_out/kfd_wchan_b2b.log; exit 1; }
timeout -k 10 300 python tools/container_ready_sweep.py --reps 12 --sample-init 250 --wait-kfd --tag "@settled" \
    --only hsa:rocr_visible --out gpurun_out/kfd_wchan_settled.json > gpurun_out/kfd_wchan_settled.log 2>&1 || { tail -20 gpurun_out/kfd_wchan_settled.log; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/kfd_wchan_b2b.json", "gpurun_out/kfd_wchan_settled.json"):
    d = json.load(open(f))
    for k, v in d.items():
        prof = v.get("init_profile") or {}
        top = sorted(((ms, b) for b, ms in prof.items() if " D " in b), reverse=True)[:6]
        print(f, k, "init", v.get("hip_init_ms"), "ready", v.get("ready_ms"))
        print("   D-state ms/run:", [(b, ms) for ms, b in top])
PY
