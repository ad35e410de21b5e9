#!/usr/bin/env python3
"""What a HIP container pays to reach its first verified kernel, by variant.

Runs the HIP container entrypoint (mi355x-probe-hip-devemu: the HIP probe with
the container /dev view of one GPU) as fresh processes, alternating variants,
each start after the previous process' kfd teardown (as bench.py does), and
prints one JSON document: per variant the p50 of ready time (exec -> verified
tile) and of each phase (library load before main, runtime init, and the
device set-up phases the probe times itself).

  --variants own,null        own: hipStreamCreateWithFlags (the default container);
                             null: the null stream (HIP creates its queue at the launch)

  python tools/hip_setup_variants.py --runs 20 --ordinal 0 --json-out out.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from rocm_k8s_device_plugin_amd.container_runtime import kfd_processes, wait_kfd_released  # noqa: E402
from rocm_k8s_device_plugin_amd.ops.native import probe_executable  # noqa: E402
from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals  # noqa: E402


def run_once(exe, dev_paths, variant):
    env = {k: v for k, v in os.environ.items() if k not in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                                            "CUDA_VISIBLE_DEVICES")}
    env["MI355X_DEV_ALLOW"] = ";".join(p for p in dev_paths if p.startswith("/dev/dri/"))
    env["MI355X_INITPROF_COUNT"] = "0"
    before = kfd_processes()
    t0 = time.monotonic_ns()
    p = subprocess.run([exe, "--devices", "0", "--iters", "4", "--timeout", "30", "--hip-stream", variant],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=60)
    doc = json.loads(p.stdout.decode().strip().splitlines()[-1])
    lingering = kfd_processes() - before
    dev = doc["devices"][0]
    out = {"ok": bool(doc.get("ok")), "ready_ms": (doc["t_ready_ns"] - t0) / 1e6,
           "exec_and_library_load_ms": (doc["t_start_ns"] - t0) / 1e6,
           "runtime_init_ms": (doc["t_runtime_ns"] - doc["t_start_ns"]) / 1e6,
           "device_ms": (doc["t_ready_ns"] - doc["t_runtime_ns"]) / 1e6,
           **{f"phase_{k}_us": v for k, v in dev.get("phase_us", {}).items()}}
    wait_kfd_released(lingering, timeout_s=1.0)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--variants", default="own,null")
    ap.add_argument("--ordinal", type=int, default=0, help="host ROCr ordinal of the GPU to use")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)
    inv = discover("/sys")
    ords = hip_ordinals(inv, "/dev")
    dev = next(d for d in inv.devices if ords.get(d.id) == a.ordinal)
    paths = ["/dev/kfd"] + dev.dev_paths()
    exe = str(probe_executable("hip-devemu"))
    variants = a.variants.split(",")
    rows = {v: [] for v in variants}
    for v in variants:       # one untimed start each
        run_once(exe, paths, v)
    for i in range(a.runs):
        for v in (variants if i % 2 == 0 else variants[::-1]):
            rows[v].append(run_once(exe, paths, v))
        print(f"run {i + 1}/{a.runs}", file=sys.stderr, flush=True)
    summary = {}
    for v, rs in rows.items():
        keys = sorted({k for r in rs for k in r if k != "ok"})
        summary[v] = {"runs": len(rs), "ok": all(r["ok"] for r in rs),
                      **{f"{k}_p50": round(statistics.median(r[k] for r in rs if k in r), 3) for k in keys}}
    doc = {"device": dev.id, "ordinal": a.ordinal, "variants": summary}
    line = json.dumps(doc)
    print(line)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
