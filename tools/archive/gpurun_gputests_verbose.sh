set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_full.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_full.log
cat gpurun_out/native_labeller_box.json | tail -5
