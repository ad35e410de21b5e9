#!/bin/bash
# The native daemon on the MI355X box's own /sys: admissions back to back for 180 s with a 1 s health pulse.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 260 python -u tools/soak_native.py --seconds 180 --report 15 --out gpurun_out/soak_native_box.json
