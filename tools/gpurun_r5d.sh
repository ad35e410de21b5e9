# Round-5 evidence on the current tree: the driver's GPU suite line, smoke, the
# headline bench and rocprofv3 kernel stats (profiles/r5/).
set -o pipefail
out=gpurun_out/r5d; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { echo pytest_fail; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke_fail; cat $out/smoke.log; exit 1; }
cat $out/smoke.log
timeout -k 10 400 python -u bench.py --json-out $out/bench_default.json > $out/bench_default.log 2>&1 || { echo bench_fail; tail -20 $out/bench_default.log; exit 1; }
python -c "import json; d=json.load(open('$out/bench_default.json')); e=d['extra']; print('headline', d['value'], 'p99', e['latency_p99_ms'], e['container_phases_p50_ms'])"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof_probe -o probe -- rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe-hip --devices all --iters 4 > $out/prof_probe.log 2>&1 || { echo prof_fail; tail -20 $out/prof_probe.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_bench -o bench -- python3 bench.py --steps 5 --warmup 1 --runtime-compare 0 --node-view-compare 0 --visibility-compare 0 --b2b-compare 0 > $out/prof_bench.log 2>&1 || { echo profbench_fail; tail -20 $out/prof_bench.log; exit 1; }
find $out -name "*kernel_stats.csv" | head
