#!/usr/bin/env python3
"""Cost of the amd-smi queries the health loop makes per pulse (smi_snapshot for
ECC, smi_xgmi_links for -smi_xgmi), each a full amdsmi_init/shut_down cycle
unless --hold keeps amd-smi initialised (as the monitor does).

  python tools/smi_timing.py [--hold] [OUT.json]
"""
import json
import os
import sys
import time

if "-h" in sys.argv or "--help" in sys.argv:
    print(__doc__)
    sys.exit(0)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rocm_k8s_device_plugin_amd.ops.native import core  # noqa: E402

n = core()
rows = []
if "--hold" in sys.argv:
    n.smi_hold()
for i in range(5):
    t = time.perf_counter()
    r = n.smi_xgmi_links()
    a = (time.perf_counter() - t) * 1e3
    t = time.perf_counter()
    s = n.smi_snapshot()
    b = (time.perf_counter() - t) * 1e3
    rows.append({"xgmi_links_ms": round(a, 2), "xgmi_ok": r["ok"], "snapshot_ms": round(b, 2), "snapshot_ok": s["ok"]})
    print(json.dumps(rows[-1]), flush=True)
out = [a for a in sys.argv[1:] if not a.startswith("-")]
if out:
    with open(out[0], "w") as f:
        json.dump(rows, f, indent=1)
