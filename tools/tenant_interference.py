#!/usr/bin/env python3
"""Does the plugin's liveness loop disturb a pod that is computing on the GPU?

A "tenant" process runs back-to-back bf16 GEMMs (torch, hipBLASLt) on GPU 0
and times every one with HIP events, while the plugin's LivenessProber probes
the same GPU every --pulse seconds in one of these modes:

  none        no health loop (reference point)
  per_sweep   persistent probe server, queue/executable created and destroyed
              every sweep (two kfd queue operations = two HWS runlist updates
              per pulse, each of which preempts every queue on the GPU)
  keep        persistent probe server with --keep: the queue lives across
              sweeps, a sweep is one AQL packet
  spawn       a fresh probe process per sweep (-liveness_mode=spawn)

Reports, per mode, the tenant's GEMM time distribution (p50/p99/p99.9/max),
GEMMs slower than 1.5x the median ("stalls"), throughput, and the sweep
latency.

  python tools/tenant_interference.py --seconds 6 --pulse 0.05 --out gpurun_out/tenant_interference.json
  python tools/tenant_interference.py --procs 8 --streams 4 --modes none,keep,none   # multi-process tenants
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

TENANT = r"""
import json, sys, time, torch
n, seconds, nstreams = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
# one GEMM chain per stream (HIP maps streams onto up to GPU_MAX_HW_QUEUES kfd queues)
streams = [torch.cuda.Stream() for _ in range(nstreams)] if nstreams > 1 else [torch.cuda.current_stream()]
bufs = [(torch.randn(n, n, device="cuda", dtype=torch.bfloat16), torch.randn(n, n, device="cuda", dtype=torch.bfloat16),
         torch.empty(n, n, device="cuda", dtype=torch.bfloat16)) for _ in streams]
for s, (a, b, c) in zip(streams, bufs):
    with torch.cuda.stream(s):
        for _ in range(10):
            torch.matmul(a, b, out=c)
torch.cuda.synchronize()
print("READY", flush=True)
sys.stdin.readline()                      # go
evs, t_end = [], time.perf_counter() + seconds
while time.perf_counter() < t_end:        # batches of 50 GEMMs per stream, each bracketed by events
    round_ = []
    for s, (a, b, c) in zip(streams, bufs):
        with torch.cuda.stream(s):
            batch = [torch.cuda.Event(enable_timing=True) for _ in range(51)]
            batch[0].record()
            for i in range(50):
                torch.matmul(a, b, out=c)
                batch[i + 1].record()
        round_.append(batch)
    evs.append(round_)
    if len(evs) > 2:
        for batch in evs[-3]:
            batch[-1].synchronize()       # keep at most ~2 rounds queued ahead
torch.cuda.synchronize()
ms = [batch[i].elapsed_time(batch[i + 1]) for round_ in evs for batch in round_ for i in range(50)]
print(json.dumps({"n": n, "gemms": len(ms), "ms": ms}), flush=True)
"""


def kfd_queue_count(gpu_id: int) -> int:
    """User queues on the GPU, every process (kfd proc entries)."""
    root, n = "/sys/class/kfd/kfd/proc", 0
    try:
        for pid in os.listdir(root):
            qd = os.path.join(root, pid, "queues")
            try:
                for q in os.listdir(qd):
                    with open(os.path.join(qd, q, "gpuid")) as f:
                        n += int(f.read().strip() or 0) == gpu_id
            except (OSError, ValueError):
                continue
    except OSError:
        return -1
    return n


def gpu0_kfd_id() -> int:
    from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals
    inv = discover("/sys")
    ords = hip_ordinals(inv, "/dev")
    dev = min(ords, key=ords.get)
    return inv.topology.node(inv.by_id[dev].node_id).gpu_id


def stats(ms, n):
    s = sorted(ms)
    med = statistics.median(s)
    q = lambda p: s[min(len(s) - 1, int(p * (len(s) - 1)))]  # noqa: E731
    flops = 2.0 * n ** 3
    return {"gemms": len(s), "p50_ms": round(med, 4), "p99_ms": round(q(0.99), 4), "p999_ms": round(q(0.999), 4),
            "max_ms": round(s[-1], 4), "stalls_over_1p5x": sum(1 for x in s if x > 1.5 * med),
            "stall_ms_total": round(sum(x - med for x in s if x > 1.5 * med), 3),
            "tflops_mean": round(flops * len(s) / (sum(s) * 1e-3) / 1e12, 1)}


async def run_mode(mode: str, a) -> dict:
    from rocm_k8s_device_plugin_amd.health.liveness import LivenessProber
    prober = None
    monitor = None
    if mode == "monitor":
        # the health monitor as the plugin runs it: kept queues, busy grace,
        # GFX-activity corroboration and the crowded-GPU step-off
        from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig, HealthMonitor
        from rocm_k8s_device_plugin_amd.topology import Inventory, discover, hip_ordinals
        inv = discover("/sys")
        ords = hip_ordinals(inv, "/dev")
        dev = min(ords, key=ords.get)
        acc = Inventory(sysfs_root="/sys", devices=(inv.by_id[dev],), topology=inv.topology, driver_loaded=True,
                        kfd_present=True)
        monitor = HealthMonitor(acc, HealthConfig(exporter_socket=None, liveness=True,
                                                  liveness_timeout_s=a.probe_timeout),
                                ordinal_map={dev: ords[dev]})
        await monitor.check_once()
        prober = monitor.prober
    elif mode == "spawn":
        # -liveness_mode=spawn: a fresh probe process per device per sweep (ROCr start-up,
        # two queues and the kfd process teardown every pulse; nothing held between pulses)
        prober = LivenessProber(timeout_s=a.probe_timeout, mode="spawn")
    elif mode != "none":
        prober = LivenessProber(timeout_s=a.probe_timeout, mode="persistent", keep_queues=(mode == "keep"))
        res = await prober.probe({"gpu0": 0})          # server up before the tenant starts timing
        assert all(r.ok for r in res.values()), res
    tenants = [subprocess.Popen([sys.executable, "-c", TENANT, str(a.n), str(a.seconds), str(a.streams)],
                                stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                                env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
               for _ in range(a.procs)]
    for tenant in tenants:
        line = await asyncio.to_thread(tenant.stdout.readline)
        assert line.strip() == "READY", line
    queues = kfd_queue_count(a.gpu_id) if a.gpu_id else -1
    stop = asyncio.Event()
    sweep_ms = []
    counts = {"ok": 0, "ok_late": 0, "pending": 0, "failed": 0}
    rss_kb = []

    async def health_loop():
        while not stop.is_set():
            t0 = time.perf_counter()
            if monitor is not None:
                skips = monitor.crowded_skips
                await monitor.check_once()
                counts["crowded_skip" if monitor.crowded_skips > skips else "swept"] = \
                    counts.get("crowded_skip" if monitor.crowded_skips > skips else "swept", 0) + 1
                sweep_ms.append((time.perf_counter() - t0) * 1e3)
                try:
                    await asyncio.wait_for(stop.wait(), a.pulse)
                except asyncio.TimeoutError:
                    pass
                continue
            # the tenant's queue makes GPU 0 busy: a probe queued behind a long
            # kernel comes back pending and is answered late by the next sweep
            res = await prober.probe({"gpu0": 0}, busy={0})
            for r in res.values():
                counts["ok_late" if r.ok and r.detail.get("late") else "ok" if r.ok else
                       "pending" if r.pending else "failed"] += 1
            sweep_ms.append((time.perf_counter() - t0) * 1e3)
            try:
                await asyncio.wait_for(stop.wait(), a.pulse)
            except asyncio.TimeoutError:
                pass

    for tenant in tenants:
        tenant.stdin.write("go\n")
        tenant.stdin.flush()
    task = asyncio.create_task(health_loop()) if prober else None
    outs = [await asyncio.to_thread(tenant.stdout.readline) for tenant in tenants]
    server_alive_end = bool(prober is not None and prober._server is not None and prober._server.alive)
    if prober is not None and prober._server is not None:
        try:
            with open(f"/proc/{prober._server.proc.pid}/status") as f:
                rss_kb = [int(l.split()[1]) for l in f if l.startswith("VmRSS")]
        except OSError:
            pass
    stop.set()
    if task:
        await task
        if monitor is not None:
            await monitor.close()
        else:
            await prober.close()
    for tenant in tenants:
        rc = await asyncio.to_thread(tenant.wait)
        assert rc == 0, rc
    docs = [json.loads(out) for out in outs]
    ms = [x for doc in docs for x in doc["ms"]]
    r = {"mode": mode, "pulse_s": a.pulse if prober else None, "gemm_n": a.n, "tenant_procs": a.procs,
         "streams_per_proc": a.streams, "kfd_queues_on_gpu": queues, **stats(ms, a.n),
         "per_proc_gemms": [doc["gemms"] for doc in docs],
         "health_sweeps": len(sweep_ms),
         "health_sweep_ms_p50": round(statistics.median(sweep_ms), 3) if sweep_ms else None,
         # the probe's wait behind the tenant's kernels (long GEMMs: --n 32768 / 65536)
         "health_sweep_ms_p99": round(sorted(sweep_ms)[int(0.99 * (len(sweep_ms) - 1))], 3) if sweep_ms else None,
         "health_sweep_ms_max": round(max(sweep_ms), 3) if sweep_ms else None,
         "probe_timeout_s": a.probe_timeout if prober else None, "probe_outcomes": counts if prober else None,
         "probe_server_rss_mb_end": round(rss_kb[0] / 1024, 1) if rss_kb else None,
         "probe_server_starts": prober.server_starts if prober else None,
         "probe_server_alive_at_end": server_alive_end if prober else None,
         "health": (monitor.snapshot()[next(iter(monitor.snapshot()))].health if monitor is not None else None)}
    print(json.dumps(r), flush=True)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--pulse", type=float, default=0.05)
    ap.add_argument("--n", type=int, default=8192, help="GEMM size (n x n x n, bf16)")
    ap.add_argument("--modes", default="none,per_sweep,keep,none")
    ap.add_argument("--probe-timeout", type=float, default=30.0,
                    help="liveness deadline; below the tenant's kernel time probes come back pending")
    ap.add_argument("--procs", type=int, default=1, help="tenant processes on GPU 0")
    ap.add_argument("--streams", type=int, default=1, help="GEMM streams (HIP queues) per tenant process")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    try:
        a.gpu_id = gpu0_kfd_id()
    except Exception:
        a.gpu_id = 0

    async def go():
        return [await run_mode(m, a) for m in a.modes.split(",")]

    res = asyncio.run(go())
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"runs": res}, f, indent=1)


if __name__ == "__main__":
    main()
