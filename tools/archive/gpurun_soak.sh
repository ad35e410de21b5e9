#!/bin/bash
# Soak of the real plugin CLI with every health source on while pods come and go (tools/soak.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
S=${SOAK_SECONDS:-300}
timeout -k 10 $((S + 240)) python -u tools/soak.py --seconds $S --report 30 --perf-every 20 --log gpurun_out/soak_plugin.log --out gpurun_out/soak${SOAK_IDLE:+_idle}.json ${SOAK_IDLE:+--idle}
