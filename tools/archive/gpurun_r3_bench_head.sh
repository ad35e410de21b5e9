#!/bin/bash
# Round 3, HEAD check: the driver's default bench invocation (native daemon) on MI355X.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r3_head_bench.json 2> gpurun_out/r3_head_bench.err || { tail -30 gpurun_out/r3_head_bench.err; exit 1; }
echo "default: $(head -c 400 gpurun_out/r3_head_bench.json)"
