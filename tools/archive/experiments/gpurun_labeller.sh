#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -m pytest tests/test_gpu.py -q -k labeller -x 2>&1 | tail -30
timeout -k 10 60 python -m rocm_k8s_device_plugin_amd.cli.node_labeller -dry_run -vram -cu-count -family -device-id -product-name -simd-count -driver-version -firmware -compute-memory-partition 2>&1 | tail -30
