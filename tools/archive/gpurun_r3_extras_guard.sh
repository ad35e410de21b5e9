#!/bin/bash
# bench.py's --extras-deadline on MI355X: (1) under torchrun with a deadline that
# lands inside the GPU extras (throughput check / peer probe / RCCL): one headline
# line, exit 0, no daemon left; (2) the default run under torchrun (RCCL extra on);
# (3) the bench GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 1 --steps 5 --warmup 1 --extras-deadline 1.5 \
  --node-view-compare 0 --visibility-compare 0 --hip-compare 0 --b2b-compare 0 --fragmented-compare 0 > gpurun_out/guard_bench.json 2> gpurun_out/guard_bench.err \
  || { tail -30 gpurun_out/guard_bench.err; exit 1; }
echo "guard: $(grep -o '"extras_incomplete": {[^}]*}' gpurun_out/guard_bench.json)"
grep "secondary measurements" gpurun_out/guard_bench.err || true
sleep 5
echo "left: $(ps -eo cmd | grep -c '[m]i355x-device-plugin' || true)"
timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 \
  bench.py --gpus 1 > gpurun_out/torchrun_bench.json 2> gpurun_out/torchrun_bench.err \
  || { tail -30 gpurun_out/torchrun_bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/torchrun_bench.json") if l.startswith("{")][-1])
e = d["extra"]
print("torchrun default:", d["value"], "ms p50;", "incomplete:", e.get("extras_incomplete"), "rccl:", json.dumps(e.get("rccl"))[:300],
      "peer:", json.dumps(e.get("peer_probe"))[:200], "launcher:", e["launcher"], "clean:", e["bench_process_gpu"]["clean"])
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -v -m gpu -k "collectives or admission or smoke" -x --timeout 300 --timeout-method thread > gpurun_out/gpu_bench_tests.log 2>&1 || { tail -40 gpurun_out/gpu_bench_tests.log; exit 1; }
tail -3 gpurun_out/gpu_bench_tests.log
