#!/bin/bash
# Headline benchmark with the plugin configured as the health DaemonSet
# (liveness via the kept-queue probe server + amd-smi ECC/events/xGMI) at two
# pulses, next to the plain run, on the same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for hp in 0 1.0 0.1; do
  timeout -k 10 400 python bench.py --steps 30 --warmup 3 --health-pulse $hp --hip-compare 0 --b2b-compare 0 \
    --node-view-compare 0 --visibility-compare 0 --peer-check 0 \
    > gpurun_out/bench_health_$hp.json 2> gpurun_out/bench_health_$hp.err || { tail -20 gpurun_out/bench_health_$hp.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_health_$hp.json')); e=d['extra']
print('pulse $hp', d['value'], e['latency_p99_ms'], e['container_phases_p50_ms'], e['health_loop'])"
done
