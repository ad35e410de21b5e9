#!/usr/bin/env python3
"""Cost of the amd-smi queries the health loop makes per pulse (smi_snapshot for
ECC, smi_xgmi_links for -smi_xgmi), each a full amdsmi_init/shut_down cycle
unless --hold keeps amd-smi initialised (as the monitor does).

  python tools/smi_timing.py [--hold] [--rounds N] [OUT.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--hold", action="store_true", help="keep amd-smi initialised between queries")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("out", nargs="?", default="", help="write the rows here as JSON")
    return ap


def main(argv=None) -> int:
    a = make_parser().parse_args(argv)
    from rocm_k8s_device_plugin_amd.ops.native import core
    n = core()
    rows = []
    if a.hold:
        n.smi_hold()
    for _ in range(a.rounds):
        t = time.perf_counter()
        r = n.smi_xgmi_links()
        x = (time.perf_counter() - t) * 1e3
        t = time.perf_counter()
        s = n.smi_snapshot()
        y = (time.perf_counter() - t) * 1e3
        rows.append({"xgmi_links_ms": round(x, 2), "xgmi_ok": r["ok"], "snapshot_ms": round(y, 2),
                     "snapshot_ok": s["ok"]})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
