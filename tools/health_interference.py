#!/usr/bin/env python3
"""Does the plugin's liveness loop slow down pod start-up on the same node?

Starts "containers" (the HSA entrypoint, as bench.py does) at random spacing
while a LivenessProber sweeps the GPU every --pulse seconds, and reports the
p50 Allocate->ready latency of those containers for:

  none        no health loop (reference point)
  spawn       a fresh probe process per device per sweep
  persistent  one long-lived probe server (--serve)

Every GPU process that exits leaves kfd teardown work behind that blocks the
next process' open("/dev/kfd") (profiles/archive/measurements_r1_r3.md §3c), so the spawn mode is
expected to inject that wait into container start-up; the server does not.

  python tools/health_interference.py --containers 15 --pulse 0.3 --out gpurun_out/health_interference.json
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rocm_k8s_device_plugin_amd.container_runtime import start_container  # noqa: E402
from rocm_k8s_device_plugin_amd.health.liveness import LivenessProber  # noqa: E402


async def run_mode(mode: str, a) -> dict:
    prober = LivenessProber(timeout_s=30, mode=mode) if mode != "none" else None
    stop = asyncio.Event()
    sweep_ms = []

    async def health_loop():
        while not stop.is_set():
            t0 = time.perf_counter()
            res = await prober.probe({"gpu0": 0})
            assert all(r.ok for r in res.values()), res
            sweep_ms.append((time.perf_counter() - t0) * 1e3)
            try:
                await asyncio.wait_for(stop.wait(), a.pulse)
            except asyncio.TimeoutError:
                pass

    task = asyncio.create_task(health_loop()) if prober else None
    if prober:
        while not sweep_ms:  # server up (persistent) before the first container
            await asyncio.sleep(0.05)
    rng = random.Random(a.seed)
    ready_ms, init_ms = [], []
    for _ in range(a.containers):
        await asyncio.sleep(rng.uniform(a.min_gap, a.max_gap))
        r = await asyncio.to_thread(start_container, [0])
        assert r.ok, r.error
        ready_ms.append((r.t_ready_ns - r.t_start_ns) / 1e6)
        init_ms.append((r.doc["t_runtime_ns"] - r.doc["t_start_ns"]) / 1e6)
    stop.set()
    if task:
        await task
        await prober.close()
    q = statistics.quantiles(ready_ms, n=10)
    return {"mode": mode, "containers": len(ready_ms), "ready_ms_p50": round(statistics.median(ready_ms), 2),
            "ready_ms_p90": round(q[-1], 2), "ready_ms_min": round(min(ready_ms), 2),
            "runtime_init_ms_p50": round(statistics.median(init_ms), 2),
            "health_sweeps": len(sweep_ms),
            "health_sweep_ms_p50": round(statistics.median(sweep_ms), 2) if sweep_ms else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--containers", type=int, default=15)
    ap.add_argument("--pulse", type=float, default=0.3)
    ap.add_argument("--min-gap", type=float, default=0.3, help="idle time before each container (s)")
    ap.add_argument("--max-gap", type=float, default=0.6)
    ap.add_argument("--modes", default="none,spawn,persistent")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    for m in a.modes.split(","):
        rows.append(asyncio.run(run_mode(m, a)))
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"pulse_s": a.pulse, "gap_s": [a.min_gap, a.max_gap], "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
