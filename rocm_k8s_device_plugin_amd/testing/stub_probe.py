#!/usr/bin/env python3
"""Fault-injection stand-in for ``mi355x-liveness-probe`` (CPU tests).

Speaks the same CLI and JSON contract. Behaviour per ROCr ordinal comes from
the JSON file named by $MI355X_STUB_PROBE_CONTROL, e.g.
``{"0": "ok", "3": "fail", "5": "hang", "6": "stale", "7": "garbage"}``
(missing ordinals are "ok"). Exercises the real LivenessProber code path:
process spawn, deadline kill, output parsing, nonce check, hysteresis.
"""
import json
import os
import sys
import time


def main(argv):
    nonce = 0
    for i, a in enumerate(argv):
        if a == "--nonce":
            nonce = int(argv[i + 1], 0)
    ordinal = os.environ.get("ROCR_VISIBLE_DEVICES", "0").split(",")[0]
    ctl = {}
    path = os.environ.get("MI355X_STUB_PROBE_CONTROL")
    if path and os.path.exists(path):
        with open(path) as f:
            ctl = json.load(f)
    mode = ctl.get(ordinal, "ok")
    if mode == "hang":
        time.sleep(3600)
    if mode == "garbage":
        print("segfault-ish noise")
        return 139
    t = time.monotonic_ns()
    ok = mode == "ok"
    dev = {"ordinal": 0, "ok": ok or mode == "stale", "hip_error": 0, "mismatches": 0 if ok else 17,
           "nonce": nonce if mode != "stale" else (nonce + 1) & 0xFFFFFFFF, "xcc_id": 0, "hw_id": 0, "iters": 4,
           "dispatches": 1, "kfd_node_id": -1, "runtime": "stub", "kernel_us": 3.0, "setup_us": 1.0,
           "total_us": 5.0, "pci_bus_id": "", "arch": "gfx950", "name": "", "uuid": "", "pci_domain": 0,
           "pci_bus": 0, "pci_device": 0, "cu_count": 256, "total_mem": 0,
           "error": "" if ok or mode == "stale" else "17/1024 MFMA results differ from host reference"}
    doc = {"ok": dev["ok"], "hip_device_count": 1, "identify": False, "t_start_ns": t, "t_runtime_ns": t,
           "t_ready_ns": t, "devices": [dev]}
    print(json.dumps(doc))
    return 0 if dev["ok"] else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
