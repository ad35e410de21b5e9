#!/bin/bash
# The one maintained GPU-box script (gpurun): each argument is a step, run in
# order; a failed step ends the call (no further GPU work after a failure).
#
#   smoke   __graft_entry__.smoke()                       -> gpurun_out/smoke.log
#   tests   pytest -m gpu                                 -> gpurun_out/gputests.log
#   bench   default bench (N=1, 20 steps)                 -> gpurun_out/bench.json
#   torchrun1 the driver's torchrun launch at N = 1       -> gpurun_out/bench_torchrun1.json
#   bench100  100 timed admissions                        -> gpurun_out/bench100.json
#   health  bench with the health DaemonSet loop (-pulse 2, liveness, amd-smi) -> gpurun_out/bench_health.json
#   healthpre  the same with -prestart_liveness                     -> gpurun_out/bench_health_prestart.json
#   prof    rocprofv3 kernel stats of a short bench       -> gpurun_out/prof_bench/
#   profprobe  rocprofv3 kernel stats of one HIP container entrypoint -> gpurun_out/prof_probe/
#   hipvariants  tools/hip_setup_variants.py (own vs null stream)     -> gpurun_out/hip_setup_variants.json
#   asan    the native-daemon GPU tests against the ASan/UBSan builds in asan_bin/
#   tsan    the same against the ThreadSanitizer builds in tsan_bin/
#   asansoak  the same soak against the ASan/UBSan daemon in asan_bin/ -> gpurun_out/soak_asan.json
#   tsansoak  2 min (SOAK_SECONDS) soak of the ThreadSanitizer daemon, every health source on, HIP containers -> gpurun_out/soak_tsan.json
#   soak    4 min native daemon soak, every health source on, a HIP container every second -> gpurun_out/soak_native.json
#   soakpre the soak with -prestart_liveness (a GPU check per admission)  -> gpurun_out/soak_prestart.json
#   cov     pytest -m gpu against the gcov build in cov_bin/ -> gpurun_out/gcov (merged by tools/native_coverage.py)
#
#   gpurun --timeout 900 -- bash tools/gpurun_check.sh smoke tests bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
# TSan's fixed shadow layout needs ASLR off for its processes (the box's kernel randomises
# with more bits than the runtime accepts): launchers that start each tsan_bin/ binary
# under setarch -R, in a fresh directory printed on stdout
tsan_launchers() {
  local w b
  w=$(mktemp -d)
  for b in mi355x-device-plugin mi355x-node-labeller; do
    printf '#!/bin/bash\nexec setarch "$(uname -m)" -R %s "$@"\n' "$PWD/tsan_bin/$b" > "$w/$b" && chmod +x "$w/$b"
  done
  echo "$w"
}
TSAN_ENV="halt_on_error=1 second_deadlock_stack=1 suppressions=$PWD/native/tsan.supp"
for s in "$@"; do
  case "$s" in
    smoke)
      step smoke
      timeout -k 10 240 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || { tail -30 gpurun_out/smoke.log; exit 1; }
      tail -3 gpurun_out/smoke.log ;;
    tests)
      step tests
      timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
      tail -3 gpurun_out/gputests.log ;;
    bench)
      step bench
      timeout -k 10 400 python3 bench.py --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 \
        || { tail -20 gpurun_out/bench.log; exit 1; }
      cut -c1-600 gpurun_out/bench.json ;;
    torchrun1)
      # the driver's launch line at N = 1
      step torchrun1
      timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 3 --json-out gpurun_out/bench_torchrun1.json \
        > gpurun_out/bench_torchrun1.log 2>&1 || { tail -20 gpurun_out/bench_torchrun1.log; exit 1; }
      cut -c1-400 gpurun_out/bench_torchrun1.json ;;
    bench100)
      step bench100
      timeout -k 10 600 python3 bench.py --steps 100 --warmup 5 --json-out gpurun_out/bench100.json \
        > gpurun_out/bench100.log 2>&1 || { tail -20 gpurun_out/bench100.log; exit 1; }
      cut -c1-600 gpurun_out/bench100.json ;;
    health)
      step health
      timeout -k 10 400 python3 bench.py --steps 30 --health-pulse 2 --runtime-compare 0 \
        --json-out gpurun_out/bench_health.json > gpurun_out/bench_health.log 2>&1 \
        || { tail -20 gpurun_out/bench_health.log; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/bench_health.json')); print(d['value'], d['extra']['health_loop'])" ;;
    healthpre)
      # the health DaemonSet configuration plus -prestart_liveness (kubelet's PreStartContainer probes the pod's GPU)
      step healthpre
      timeout -k 10 400 python3 bench.py --steps 30 --health-pulse 2 --health-prestart 1 --runtime-compare 0 \
        --json-out gpurun_out/bench_health_prestart.json > gpurun_out/bench_health_prestart.log 2>&1 \
        || { tail -20 gpurun_out/bench_health_prestart.log; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/bench_health_prestart.json')); e=d['extra']; print(d['value'], e['plugin_rpc_p50_ms'], e['prestart_rpc_p50_ms'], e['health_loop'])" ;;
    prof)
      step prof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench \
        -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof_bench.log 2>&1 \
        || { tail -20 gpurun_out/prof_bench.log; exit 1; }
      find gpurun_out/prof_bench -name "*kernel_stats.csv" ;;
    profprobe)
      step profprobe
      timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_probe -o probe \
        -- ./rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe-hip --devices 0 > gpurun_out/prof_probe.log 2>&1 \
        || { tail -20 gpurun_out/prof_probe.log; exit 1; }
      find gpurun_out/prof_probe -name "*kernel_stats.csv" ;;
    hipvariants)
      step hipvariants
      timeout -k 10 300 python3 tools/hip_setup_variants.py --runs 20 --json-out gpurun_out/hip_setup_variants.json \
        > gpurun_out/hip_setup_variants.log 2>&1 || { tail -20 gpurun_out/hip_setup_variants.log; exit 1; }
      cat gpurun_out/hip_setup_variants.json ;;
    soak)
      step soak
      timeout -k 10 420 python3 tools/soak_native.py --seconds 240 --report 30 --container-interval 1 \
        --extra "-liveness -liveness_chip_sweep_every 10 -perf_check_every 60 -smi_ecc -smi_events -smi_xgmi" \
        --out gpurun_out/soak_native.json > gpurun_out/soak_native.log 2>&1 \
        || { tail -20 gpurun_out/soak_native.log; exit 1; }
      tail -c 1500 gpurun_out/soak_native.json ;;
    soakpre)
      # the same soak with -prestart_liveness: every admission's PreStartContainer probes its GPU
      step soakpre
      timeout -k 10 420 python3 tools/soak_native.py --seconds 240 --report 30 --container-interval 1 --metrics-port 9437 \
        --extra "-liveness -prestart_liveness -liveness_chip_sweep_every 10 -perf_check_every 60 -smi_ecc -smi_events -smi_xgmi" \
        --out gpurun_out/soak_prestart.json > gpurun_out/soak_prestart.log 2>&1 \
        || { tail -20 gpurun_out/soak_prestart.log; exit 1; }
      tail -c 1500 gpurun_out/soak_prestart.json ;;
    asan)
      # the GPU tests that drive the native daemons, against their ASan/UBSan builds (host code only;
      # asan_bin/ holds build/native-address-undefined/pkg/bin/*, copied before the call)
      step asan
      MI355X_NATIVE_DAEMON_EXE=$PWD/asan_bin/mi355x-device-plugin MI355X_NATIVE_LABELLER_EXE=$PWD/asan_bin/mi355x-node-labeller \
        timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "native or daemon or labeller" \
        > gpurun_out/gputests_asan.log 2>&1 || { tail -40 gpurun_out/gputests_asan.log; exit 1; }
      tail -3 gpurun_out/gputests_asan.log ;;
    tsan)
      # the same GPU tests against the ThreadSanitizer builds (host code only; tsan_bin/ holds
      # build/native-thread/pkg/bin/*): the health engine, probe-server supervision and RPC threads
      # racing for real, with the GPU liveness path on; the first report fails the daemon
      step tsan
      w=$(tsan_launchers)
      # first the binary alone on the real node (a runtime that cannot map its shadow fails here)
      TSAN_OPTIONS="$TSAN_ENV" timeout -k 10 60 "$w/mi355x-device-plugin" -dry_run \
        > gpurun_out/tsan_dry_run.json 2> gpurun_out/tsan_dry_run.err || { tail -30 gpurun_out/tsan_dry_run.err; exit 1; }
      TSAN_OPTIONS="$TSAN_ENV" \
      MI355X_NATIVE_DAEMON_EXE=$w/mi355x-device-plugin MI355X_NATIVE_LABELLER_EXE=$w/mi355x-node-labeller \
        timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "native or daemon or labeller" \
        > gpurun_out/gputests_tsan.log 2>&1 || { tail -40 gpurun_out/gputests_tsan.log; exit 1; }
      tail -3 gpurun_out/gputests_tsan.log ;;
    tsansoak)
      # 2 minutes of the soak against the ThreadSanitizer daemon: admissions back to back (each with its
      # PreStartContainer GPU check), a HIP container every 2 s, liveness + chip sweep + throughput check +
      # the three amd-smi sources
      step tsansoak
      w=$(tsan_launchers)
      TSAN_OPTIONS="$TSAN_ENV" timeout -k 10 $(( ${SOAK_SECONDS:-120} + 180 )) python3 tools/soak_native.py --seconds "${SOAK_SECONDS:-120}" \
        --report 20 --container-interval 2 --metrics-port 9438 --exe "$w/mi355x-device-plugin" \
        --extra "-liveness -prestart_liveness -liveness_probe $PWD/rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe -liveness_chip_sweep_every 5 -perf_check_every 20 -smi_ecc -smi_events -smi_xgmi" \
        --out gpurun_out/soak_tsan.json > gpurun_out/soak_tsan.log 2>&1 || { tail -c 3000 gpurun_out/soak_tsan.json; exit 1; }
      tail -c 800 gpurun_out/soak_tsan.json ;;
    asansoak)
      # the same 2-minute soak against the ASan/UBSan daemon (asan_bin/)
      step asansoak
      UBSAN_OPTIONS="print_stacktrace=1" timeout -k 10 $(( ${SOAK_SECONDS:-120} + 180 )) python3 tools/soak_native.py --seconds "${SOAK_SECONDS:-120}" \
        --report 20 --container-interval 2 --metrics-port 9439 --exe "$PWD/asan_bin/mi355x-device-plugin" \
        --extra "-liveness -prestart_liveness -liveness_probe $PWD/rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe -liveness_chip_sweep_every 5 -perf_check_every 20 -smi_ecc -smi_events -smi_xgmi" \
        --out gpurun_out/soak_asan.json > gpurun_out/soak_asan.log 2>&1 || { tail -c 3000 gpurun_out/soak_asan.json; exit 1; }
      tail -c 800 gpurun_out/soak_asan.json ;;
    cov)
      # the GPU tests against the gcov build staged in cov_bin/ (tools/native_coverage.py --no-build
      # --stage cov_bin); the counts land under gpurun_out/gcov for --no-build --merge gpurun_out/gcov
      step cov
      so=(cov_bin/_native*.so)
      GCOV_PREFIX=$PWD/gpurun_out/gcov GCOV_PREFIX_STRIP=3 MI355X_NATIVE_CORE_SO=$PWD/${so[0]} \
      MI355X_NATIVE_DAEMON_EXE=$PWD/cov_bin/mi355x-device-plugin MI355X_NATIVE_LABELLER_EXE=$PWD/cov_bin/mi355x-node-labeller \
        timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
        > gpurun_out/gputests_cov.log 2>&1 || { tail -40 gpurun_out/gputests_cov.log; exit 1; }
      tail -3 gpurun_out/gputests_cov.log ;;
    *)
      echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
