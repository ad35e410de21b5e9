#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for p in /sys/class/kfd/kfd/proc/*; do echo "$p: $(ls $p | tr '\n' ' ')"; ls $p/queues 2>/dev/null | head -3; for q in $p/queues/*; do [ -d "$q" ] && echo "  $q: $(ls $q | tr '\n' ' ') gpuid=$(cat $q/gpuid 2>&1)"; done; done 2>&1 | head -40
cat /sys/class/kfd/kfd/topology/nodes/*/gpu_id 2>&1 | tr '\n' ' '
