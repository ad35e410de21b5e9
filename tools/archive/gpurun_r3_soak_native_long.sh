#!/bin/bash
# Round 3: the native daemon with every feature on (as gpurun_r3_soak_native_full.sh) for 15 minutes:
# admissions back to back, health sweeps every second, chip sweeps, throughput checks; memory and fds tracked.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1050 python -u tools/soak_native.py --seconds 900 --report 30 --pulse 1 --metrics-port 19200 \
  --extra "-liveness -liveness_chip_sweep_every 10 -perf_check_every 60 -perf_mib 1024 -smi_ecc -smi_events -smi_xgmi -device_list_strategy device-specs,cdi-cri -cdi_spec_dir /tmp/cdi-soak -topology_watch 5" \
  --out gpurun_out/soak_native_900s_box.json
