#!/bin/bash
# Round 3: the native daemons' GPU tests against their ASan/UBSan builds (host
# code only: the daemon and labeller; the probe server they drive is the normal
# gfx950 build). Needs asan_bin/ (copied from build/native-address-undefined/pkg/bin).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
export UBSAN_OPTIONS=print_stacktrace=1
# evidence the sanitizer runtime is live in these binaries on the box
ASAN_OPTIONS=help=1 timeout -k 5 30 asan_bin/mi355x-device-plugin -dry_run -sysfs_root /nonexistent > gpurun_out/r3_asan_runtime.txt 2>&1 || true
head -2 gpurun_out/r3_asan_runtime.txt
MI355X_NATIVE_DAEMON_EXE=$PWD/asan_bin/mi355x-device-plugin MI355X_NATIVE_LABELLER_EXE=$PWD/asan_bin/mi355x-node-labeller \
  timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_native_labeller.py -m gpu -v --timeout 240 \
  --timeout-method thread -k "native_daemon or real_node_labels" > gpurun_out/r3_gpu_asan.log 2>&1 || { tail -60 gpurun_out/r3_gpu_asan.log; exit 1; }
tail -5 gpurun_out/r3_gpu_asan.log
timeout -k 5 120 asan_bin/mi355x-device-plugin -dry_run -liveness -liveness_probe rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe \
  -pulse 1 -liveness_chip_sweep_every 1 -perf_check_every 1 -perf_mib 512 -smi_ecc -smi_events -smi_xgmi -exporter_socket "" \
  > gpurun_out/r3_asan_dryrun.json 2> gpurun_out/r3_asan_dryrun.err
echo "dry run rc=$? sanitizer reports: $(grep -c -E 'ERROR: AddressSanitizer|runtime error:' gpurun_out/r3_asan_dryrun.err || true)"
