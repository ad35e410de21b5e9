set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value tools/archive/experiments/hbm_stream_variants.hip -o /tmp/hbmv || exit 1
timeout -k 10 120 /tmp/hbmv | tee gpurun_out/hbm_stream_variants_box.jsonl
