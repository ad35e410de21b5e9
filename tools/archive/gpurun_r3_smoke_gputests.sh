#!/bin/bash
# Round-3 end-of-round rehearsal: build check, smoke() (admission through the native daemon), then the -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r3_smoke.log 2>&1 || { tail -60 gpurun_out/r3_smoke.log; exit 1; }
tail -3 gpurun_out/r3_smoke.log
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu -x --timeout 240 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r3_pytest_gpu.log
