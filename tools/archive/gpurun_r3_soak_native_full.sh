#!/bin/bash
# Round 3: the native daemon with every health source and feature on (liveness,
# chip sweep, throughput check, amd-smi ECC / events / xGMI, CDI, topology
# watch, /metrics) on the box's own /sys, admissions back to back for 180 s.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/soak_native.py --seconds 180 --report 15 --pulse 1 --metrics-port 19200 \
  --extra "-liveness -liveness_chip_sweep_every 10 -perf_check_every 60 -perf_mib 1024 -smi_ecc -smi_events -smi_xgmi -device_list_strategy device-specs,cdi-cri -cdi_spec_dir /tmp/cdi-soak -topology_watch 5" \
  --out gpurun_out/soak_native_full_box.json
