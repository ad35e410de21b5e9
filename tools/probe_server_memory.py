#!/usr/bin/env python3
"""Host memory held by the persistent liveness probe server.

Each kfd queue on MI355X carries a context-save (CWSR) area of
num_xcc x cwsr_size = 8 x 22.7 MB = 181 MB that ROCr's thunk maps for the GPU
(profiles/archive/measurements_r1_r3.md §3f). The kept-queue server (`-liveness_keep_queues`,
default) holds its queues between pulses, so this measures what that costs
the node: the server's RSS / anonymous / pinned memory and the host's
MemAvailable, before and after the first sweep, with and without kept queues.

  python tools/probe_server_memory.py --out gpurun_out/probe_server_memory.json
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from rocm_k8s_device_plugin_amd.health.liveness import LivenessProber  # noqa: E402
from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals  # noqa: E402


def status_kb(pid: int) -> dict:
    out = {}
    try:
        with open(f"/proc/{pid}/status") as f:
            for line in f:
                k, _, v = line.partition(":")
                if k in ("VmRSS", "RssAnon", "RssFile", "RssShmem", "VmPin", "VmLck", "VmSize"):
                    out[k] = int(v.split()[0])
    except OSError:
        pass
    return out


def mem_available_kb() -> int:
    with open("/proc/meminfo") as f:
        for line in f:
            if line.startswith("MemAvailable:"):
                return int(line.split()[1])
    return 0


async def measure(ordinals, keep: bool) -> dict:
    p = LivenessProber(mode="persistent", keep_queues=keep, timeout_s=30)
    avail0 = mem_available_kb()
    try:
        r1 = await p.probe(ordinals)
        pid = p._server.proc.pid if p._server else None
        after1 = status_kb(pid) if pid else {}
        avail1 = mem_available_kb()
        r2 = await p.probe(ordinals)
        after2 = status_kb(pid) if pid else {}
    finally:
        await p.close()
    return {"keep_queues": keep, "devices": len(ordinals),
            "ok": all(o.ok for o in list(r1.values()) + list(r2.values())),
            "server_after_sweep1_kb": after1, "server_after_sweep2_kb": after2,
            "host_mem_available_drop_mb": round((avail0 - avail1) / 1024, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    inv = discover("/sys")
    ords = hip_ordinals(inv, "/dev")
    rows = []
    for keep in (False, True):
        rows.append(asyncio.run(measure(ords, keep)))
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
