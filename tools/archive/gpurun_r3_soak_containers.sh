#!/bin/bash
# Round 3: the native daemon with every feature on, admissions back to back and
# every second one admission's container started for real on the GPU the
# liveness loop is probing (5 minutes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 450 python -u tools/soak_native.py --seconds 300 --report 30 --pulse 1 --metrics-port 19200 \
  --container-interval 1.0 \
  --extra "-liveness -liveness_chip_sweep_every 10 -perf_check_every 60 -perf_mib 1024 -smi_ecc -smi_events -smi_xgmi -topology_watch 5" \
  --out gpurun_out/soak_native_containers_box.json
