#!/usr/bin/env python3
"""K container entrypoints started at once (what an N-GPU admission does on an
N-GPU node, one process per GPU): does GPU-runtime start-up serialise?

All K processes use GPU 0 here (1-GPU box); the per-process kfd work is the
same. Between rounds the previous processes' kfd teardown is waited out.

  python tools/concurrent_containers.py --ks 1,2,4,8 --rounds 8 --out gpurun_out/concurrent.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rocm_k8s_device_plugin_amd.container_runtime import kfd_processes, wait_kfd_released  # noqa: E402
from rocm_k8s_device_plugin_amd.health.liveness import _VISIBILITY_VARS  # noqa: E402
from rocm_k8s_device_plugin_amd.ops.native import probe_executable  # noqa: E402


def one_round(k: int, exe: str, extra_env: dict) -> dict:
    env = {kk: v for kk, v in os.environ.items() if kk not in _VISIBILITY_VARS}
    env["ROCR_VISIBLE_DEVICES"] = "0"
    env.update(extra_env)
    before = kfd_processes()
    t0 = time.monotonic_ns()
    procs = [subprocess.Popen([exe, "--devices", "0", "--iters", "4"], stdout=subprocess.PIPE,
                              stderr=subprocess.DEVNULL, env=env) for _ in range(k)]
    docs = []
    for p in procs:
        out, _ = p.communicate(timeout=120)
        docs.append(json.loads(out.decode().strip().splitlines()[-1]))
    lingering = kfd_processes() - before
    waited = wait_kfd_released(lingering, timeout_s=min(5.0, 0.25 + 0.25 * len(lingering)))
    ready = [(d["t_ready_ns"] - t0) / 1e6 for d in docs]
    return {"ok": all(d["ok"] for d in docs), "ready_max_ms": max(ready), "ready_min_ms": min(ready),
            "kfd_open_ms_max": max(d["init_us"]["kfd_open"] for d in docs) / 1e3,
            "hsa_init_ms_max": max(d["init_us"]["hsa_init"] for d in docs) / 1e3,
            "hsa_init_ms_min": min(d["init_us"]["hsa_init"] for d in docs) / 1e3,
            "teardown_wait_ms": waited}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="1,2,4,8")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--out", default="")
    ap.add_argument("--exe", default="", help="entrypoint binary (e.g. the path-interposing measurement build)")
    ap.add_argument("--env", action="append", default=[], help="K=V for every process")
    a = ap.parse_args()
    exe = a.exe or str(probe_executable("hsa"))
    extra = dict(kv.split("=", 1) for kv in a.env)
    res = {}
    for k in (int(x) for x in a.ks.split(",")):
        rows = [one_round(k, exe, extra) for _ in range(a.rounds)]
        res[k] = {key: round(statistics.median(r[key] for r in rows), 2) for key in rows[0] if key != "ok"}
        res[k]["all_ok"] = all(r["ok"] for r in rows)
        print(k, json.dumps(res[k]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
