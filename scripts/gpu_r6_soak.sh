#!/bin/bash
# Round-6 GPU evidence: the probe server's per-device deadline under a long-kernel
# tenant, the PreStart gate under the same tenant, the GPU suite, then soaks of the
# native daemon (plain and TSan) with every health source and the PreStart gate
# on, a real HIP container every second. Each step has its own time limit and
# the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
FLAGS="-liveness -prestart_liveness -liveness_chip_sweep_every 10 -perf_check_every 60 -smi_ecc -smi_events -smi_xgmi"
step() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "$name failed: $?"; exit 1; }; }
[ -n "$SKIP_DEADLINE" ] || step probe_deadline_tenant 200 python -u tools/probe_deadline_tenant.py --out gpurun_out/probe_deadline_tenant.json
[ -n "$SKIP_TENANT" ] || step prestart_tenant_after 300 python -u tools/prestart_tenant.py --out gpurun_out/prestart_tenant_after.json
[ -n "$SKIP_SUITE" ] || step r6_gpu_suite 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider
[ -n "$SKIP_SOAK" ] || step soak_prestart_r6 $(( ${SOAK_SECONDS:-240} + 180 )) python -u tools/soak_native.py --seconds ${SOAK_SECONDS:-240} --report 30 \
  --container-interval 1 --extra "$FLAGS" --out gpurun_out/soak_prestart_r6.json
[ -n "$SKIP_TSAN" ] || TSAN_OPTIONS="halt_on_error=1" step soak_prestart_tsan_r6 $(( ${TSAN_SECONDS:-180} + 240 )) python -u tools/soak_native.py \
  --seconds ${TSAN_SECONDS:-180} --report 30 --container-interval 1 --exe tsan_bin/mi355x-device-plugin --extra "$FLAGS" \
  --out gpurun_out/soak_prestart_tsan_r6.json
echo done
