#!/bin/bash
# Write shapes for the throughput check's fill pass (hbm_fill_variants.hip).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 tools/archive/experiments/hbm_fill_variants.hip -o /tmp/hfv || exit 1
timeout -k 10 120 /tmp/hfv | tee gpurun_out/hbm_fill_variants_box.jsonl
