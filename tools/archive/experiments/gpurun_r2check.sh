#!/bin/bash
# Round-2 check: GPU tests, smoke(), default bench, rocprofv3 kernel stats of the probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json; cat /proc/loadavg
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_probe -o probe -- rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe --devices all --iters 4 > gpurun_out/prof_probe.log 2>&1 || { tail -20 gpurun_out/prof_probe.log; exit 1; }
find gpurun_out/prof_probe -name '*kernel_stats.csv' -exec cat {} \;
