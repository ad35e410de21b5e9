#!/bin/bash
# Round-6 GPU evidence: the probe server's per-device deadline under a long-kernel
# tenant, then soaks of the native daemon (plain and TSan) with every health
# source and the PreStart gate on, a real HIP container every second.
set -o pipefail
mkdir -p gpurun_out
FLAGS="-liveness -prestart_liveness -liveness_chip_sweep_every 10 -perf_check_every 60 -smi_ecc -smi_events -smi_xgmi"
timeout -k 10 200 python -u tools/probe_deadline_tenant.py --out gpurun_out/probe_deadline_tenant.json \
  > gpurun_out/probe_deadline_tenant.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/soak_native.py --seconds ${SOAK_SECONDS:-300} --report 30 --container-interval 1 \
  --extra "$FLAGS" --out gpurun_out/soak_prestart_r6.json > gpurun_out/soak_prestart_r6.log 2>&1 || exit $?
TSAN_OPTIONS="halt_on_error=1" timeout -k 10 300 python -u tools/soak_native.py --seconds ${TSAN_SECONDS:-180} --report 30 \
  --container-interval 1 --exe tsan_bin/mi355x-device-plugin --extra "$FLAGS" --out gpurun_out/soak_prestart_tsan_r6.json \
  > gpurun_out/soak_prestart_tsan_r6.log 2>&1
