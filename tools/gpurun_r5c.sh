# Health DaemonSet default: persistent kept-queue server vs -liveness_mode=spawn at -pulse=2
# (VERDICT r4 item 6): admission latency under the loop, host memory, sweep cost, tenant GEMM stalls.
set -o pipefail
mkdir -p gpurun_out/r5c
for mode in persistent spawn; do
timeout -k 10 500 python -u bench.py --steps 100 --warmup 3 --health-pulse 2 --health-liveness-mode $mode --runtime-compare 0 --throughput-check 0 --peer-check 0 --node-view-compare 0 --visibility-compare 0 --b2b-compare 0 --json-out gpurun_out/r5c/bench_health_$mode.json > gpurun_out/r5c/bench_health_$mode.log 2>&1 || { echo health_fail $mode; tail -20 gpurun_out/r5c/bench_health_$mode.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r5c/bench_health_$mode.json')); print('$mode', d['value'], d['extra']['latency_p99_ms'], d['extra']['health_loop'])"
done
timeout -k 10 300 python -u tools/tenant_interference.py --seconds 20 --pulse 2 --modes none,spawn,keep,none --out gpurun_out/r5c/tenant_interference_pulse2.json > gpurun_out/r5c/tenant.log 2>&1 || { echo tenant_fail; tail -20 gpurun_out/r5c/tenant.log; exit 1; }
cat gpurun_out/r5c/tenant.log | cut -c1-400
