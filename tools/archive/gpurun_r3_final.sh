#!/bin/bash
# Round 3, HEAD check: smoke(), the -m gpu suite and the default bench (what the round-end driver runs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r3_smoke.log 2>&1 || { tail -60 gpurun_out/r3_smoke.log; exit 1; }
tail -3 gpurun_out/r3_smoke.log
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu -x --timeout 240 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r3_pytest_gpu.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3_head_bench.json 2> gpurun_out/r3_head_bench.err || { tail -30 gpurun_out/r3_head_bench.err; exit 1; }
echo "default: $(head -c 300 gpurun_out/r3_head_bench.json)"
