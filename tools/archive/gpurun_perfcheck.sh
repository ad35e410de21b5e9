#!/bin/bash
# Throughput check (HBM pattern fill/check + sustained bf16 MFMA + per-XCD
# clocks) on the box's GPU: a size / length sweep, the same under the kept
# probe server, and rocprofv3 kernel stats of one check.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe
: > gpurun_out/perf_sweep.jsonl
for mib in 1024 4096 16384; do
  for it in 16384 65536 262144; do
    timeout -k 10 60 $P --perf --perf-mib $mib --perf-iters $it --timeout 20 >> gpurun_out/perf_sweep.jsonl || { echo "perf $mib $it failed rc=$?"; tail -c 2000 gpurun_out/perf_sweep.jsonl; exit 1; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/perf_sweep.jsonl"):
    d = json.loads(l)["devices"][0]
    print({k: d[k] for k in ("ok", "bytes", "hbm_write_gbps", "hbm_read_gbps", "hbm_bad_words", "mfma_iters", "mfma_us",
                             "mfma_tflops", "clock_mhz_min", "clock_mhz_median", "clock_mhz_max", "xcd_clock_mhz",
                             "mfma_checksum_mismatch", "mfma_xccs", "total_us", "error")})
PY
timeout -k 10 60 $P --sweep --timeout 10 > gpurun_out/sweep_after_perf.json && python -c "import json;d=json.load(open('gpurun_out/sweep_after_perf.json'))['devices'][0];print('sweep ok', d['ok'], d['cus_covered'], d['kernel_us'])" || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_perf -o perf -- $P --perf --perf-mib 4096 --perf-iters 65536 --timeout 20 > gpurun_out/prof_perf.log 2>&1 || { tail -20 gpurun_out/prof_perf.log; exit 1; }
find gpurun_out/prof_perf -name '*kernel_stats.csv' -exec cat {} \;
