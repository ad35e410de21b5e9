# Tail study: 100 headline admissions with the kfd-open timing per step (profiles/r5/).
set -o pipefail
out=gpurun_out/r5e; mkdir -p $out
timeout -k 10 600 python -u bench.py --steps 100 --warmup 3 --runtime-compare 40 --json-out $out/bench100.json > $out/bench100.log 2>&1 || { echo bench_fail; tail -20 $out/bench100.log; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r5e/bench100.json')); e=d['extra']
print('headline', d['value'], 'p99', e['latency_p99_ms'], e['container_counters_p50'])
for s in e['tail_attribution'].get('slow_steps', []): print(' slow', s['step'], s['latency_ms'], s['phase'], s.get('kfd_open_ms'), s.get('hsa_init_ms'))
r=e['comparisons']['rocr_direct_container']
print('rocr', r['latency_p50_ms'], r['latency_p99_ms'], r['counters_p50'])
for s in r['tail_attribution'].get('slow_steps', []): print(' slow', s['step'], s['latency_ms'], s['phase'], s.get('kfd_open_ms'), s.get('hsa_init_ms'))
PY
