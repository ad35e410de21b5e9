#!/bin/bash
# Round-3 GPU tests: the native daemon's MFMA liveness path first, then the whole -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -v -m gpu -x --timeout 240 --timeout-method thread -k native_daemon > gpurun_out/r3_native_gpu.log 2>&1 || { tail -80 gpurun_out/r3_native_gpu.log; exit 1; }
tail -5 gpurun_out/r3_native_gpu.log
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu -x --timeout 240 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r3_pytest_gpu.log
