#!/bin/bash
# Round 3: the headline through the native daemon (bench default), 20 and 100
# admissions, and the Python CLI's plugin on the same box for comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r3n_bench_default.json 2> gpurun_out/r3n_bench_default.err || { tail -30 gpurun_out/r3n_bench_default.err; exit 1; }
echo "default: $(head -c 400 gpurun_out/r3n_bench_default.json)"
timeout -k 10 900 python -u bench.py --steps 100 > gpurun_out/r3n_bench100.json 2> gpurun_out/r3n_bench100.err || { tail -30 gpurun_out/r3n_bench100.err; exit 1; }
echo "100: $(head -c 400 gpurun_out/r3n_bench100.json)"
timeout -k 10 600 python -u bench.py --plugin python > gpurun_out/r3n_bench_python.json 2> gpurun_out/r3n_bench_python.err || { tail -30 gpurun_out/r3n_bench_python.err; exit 1; }
echo "python: $(head -c 400 gpurun_out/r3n_bench_python.json)"
