#!/bin/bash
# What the driver runs at round end: GPU tests, smoke(), default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json; cat /proc/loadavg
timeout -k 10 200 python tools/plugin_startup.py --reps 5 --out gpurun_out/plugin_startup.json > gpurun_out/plugin_startup.log 2>&1 || { tail -20 gpurun_out/plugin_startup.log; exit 1; }
cat gpurun_out/plugin_startup.log
timeout -k 10 60 python -m rocm_k8s_device_plugin_amd.cli.node_labeller -dry_run -vram -cu-count -family -device-id -product-name -simd-count -driver-version -firmware -compute-memory-partition -compute-partitioning-supported -memory-partitioning-supported > gpurun_out/labels_box.json 2> gpurun_out/labels_box.err || { tail gpurun_out/labels_box.err; exit 1; }
echo "labels: $(grep -c '"' gpurun_out/labels_box.json)"
