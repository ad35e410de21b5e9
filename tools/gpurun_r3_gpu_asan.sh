#!/bin/bash
# Round 3: the native daemons' GPU tests against their ASan/UBSan builds (host
# code only: the daemon and labeller; the probe server they drive is the normal
# gfx950 build). Needs asan_bin/ (copied from build/native-address-undefined/pkg/bin).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
export UBSAN_OPTIONS=print_stacktrace=1
MI355X_NATIVE_DAEMON_EXE=$PWD/asan_bin/mi355x-device-plugin MI355X_NATIVE_LABELLER_EXE=$PWD/asan_bin/mi355x-node-labeller \
  timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_native_labeller.py -m gpu -v --timeout 240 \
  --timeout-method thread -k "native_daemon or real_node_labels" > gpurun_out/r3_gpu_asan.log 2>&1 || { tail -60 gpurun_out/r3_gpu_asan.log; exit 1; }
tail -5 gpurun_out/r3_gpu_asan.log
