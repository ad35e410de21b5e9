set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5b/smoke.log 2>&1 || { echo smoke_fail; cat gpurun_out/r5b/smoke.log; exit 1; }
cat gpurun_out/r5b/smoke.log
timeout -k 10 400 python -u bench.py --json-out gpurun_out/r5b/bench_default.json > gpurun_out/r5b/bench_default.log 2>&1 || { echo bench_fail; tail -20 gpurun_out/r5b/bench_default.log; exit 1; }
tail -c 400 gpurun_out/r5b/bench_default.json; echo
for mode in persistent spawn; do
timeout -k 10 400 python -u bench.py --steps 40 --warmup 3 --health-pulse 2 --health-liveness-mode $mode --runtime-compare 0 --throughput-check 0 --peer-check 0 --json-out gpurun_out/r5b/bench_health_$mode.json > gpurun_out/r5b/bench_health_$mode.log 2>&1 || { echo health_fail $mode; tail -20 gpurun_out/r5b/bench_health_$mode.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r5b/bench_health_$mode.json')); print('$mode', d['value'], d['extra']['latency_p99_ms'], d['extra']['health_loop'])"
done
