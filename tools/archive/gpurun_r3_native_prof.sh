#!/bin/bash
# Round 3: rocprofv3 kernel trace of the native daemon's health path on MI355X
# (-dry_run: one sweep with the full-chip sweep and the throughput check, then
# exit), and the headline through the native daemon after the RPC-path changes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
DP=rocm_k8s_device_plugin_amd/bin/mi355x-device-plugin
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_native_daemon -o sweep -- \
  $DP -dry_run -pulse 1 -liveness -liveness_chip_sweep_every 1 -perf_check_every 1 -perf_mib 1024 -exporter_socket "" \
  > gpurun_out/native_daemon_dryrun_prof.json 2> gpurun_out/native_daemon_dryrun_prof.err || { tail -30 gpurun_out/native_daemon_dryrun_prof.err; exit 1; }
find gpurun_out/prof_native_daemon -name "*stats*" | head
timeout -k 10 600 python -u bench.py > gpurun_out/r3n2_bench_default.json 2> gpurun_out/r3n2_bench_default.err || { tail -30 gpurun_out/r3n2_bench_default.err; exit 1; }
echo "default: $(head -c 300 gpurun_out/r3n2_bench_default.json)"
