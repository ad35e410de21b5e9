#!/usr/bin/env python3
"""How closely does the kept-queue probe server keep a short per-device
deadline while a tenant's long kernels hold every CU of the GPU?

Starts `mi355x-liveness-probe --serve --keep`, then a torch tenant running
back-to-back bf16 GEMMs (n=65536, ~430 ms each) on GPU 0, and sends tagged
probe requests with a per-device deadline of --deadline seconds, one at a
time and in pairs (two requests on the same GPU at once, as a sweep and a
PreStartContainer check can be). Reports, per request: the client-side round
trip, the server's own total_us, and whether the reply was pending or late.

  python tools/probe_deadline_tenant.py --out gpurun_out/probe_deadline_tenant.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

from prestart_tenant import TENANT  # noqa: E402


def pct(xs, p):
    s = sorted(xs)
    return round(s[min(len(s) - 1, int(p * (len(s) - 1)))], 3) if s else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--seconds", type=float, default=12.0)
    ap.add_argument("--deadline", type=float, default=0.05)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
    from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals
    inv = discover("/sys")
    ords = hip_ordinals(inv, "/dev")
    o = min(ords.values())
    env = dict(os.environ, ROCR_VISIBLE_DEVICES=str(o))
    srv = subprocess.Popen([os.path.join(str(PKG_DIR), "bin", "mi355x-liveness-probe"), "--serve", "--keep"],
                           stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)
    hello = json.loads(srv.stdout.readline())
    assert hello["ok"] and hello.get("concurrent"), hello
    lock = threading.Lock()
    replies, waiters = {}, {}
    stop = threading.Event()

    def reader():
        for line in srv.stdout:
            d = json.loads(line)
            with lock:
                replies[d.get("id")] = (time.perf_counter(), d)
                ev = waiters.get(d.get("id"))
            if ev:
                ev.set()
    threading.Thread(target=reader, daemon=True).start()
    nid = [0]

    def send(deadline):
        with lock:
            nid[0] += 1
            rid = nid[0]
            ev = waiters[rid] = threading.Event()
        t0 = time.perf_counter()
        srv.stdin.write(f"@{rid} probe 4 {deadline:.3f} 0:{rid}:{deadline:.3f}\n")
        srv.stdin.flush()
        ev.wait(30)
        t1, d = replies[rid]
        dev = d["devices"][0]
        return {"rt_ms": (t1 - t0) * 1e3, "server_ms": dev["total_us"] / 1e3, "ok": dev["ok"],
                "pending": dev.get("pending_s", 0) > 0, "late": bool(dev.get("late")),
                "wait_ms": dev["phase_us"]["dispatch_wait"] / 1e3, "error": dev["error"]}

    out = {"deadline_s": a.deadline, "idle": [send(a.deadline) for _ in range(10)]}
    ten = subprocess.Popen([sys.executable, "-c", TENANT, str(a.n), str(a.seconds)], stdin=subprocess.PIPE,
                           stdout=subprocess.PIPE, text=True)
    assert ten.stdout.readline().strip() == "READY"
    ten.stdin.write("go\n")
    ten.stdin.flush()
    single, paired = [], []
    end = time.monotonic() + a.seconds - 1.0
    while time.monotonic() < end:
        single.append(send(a.deadline))
        time.sleep(0.1)
        res = [None, None]
        ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, send(a.deadline))) for i in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        paired += res
        time.sleep(0.1)
    doc = json.loads(ten.stdout.readline())
    ten.wait()
    srv.stdin.write("quit\n")
    srv.stdin.flush()
    srv.wait(30)
    stop.set()

    def summ(rows):
        return {"n": len(rows), "rt_p50_ms": pct([r["rt_ms"] for r in rows], 0.5),
                "rt_p90_ms": pct([r["rt_ms"] for r in rows], 0.9), "rt_max_ms": round(max(r["rt_ms"] for r in rows), 3),
                "server_p50_ms": pct([r["server_ms"] for r in rows], 0.5),
                "server_max_ms": round(max(r["server_ms"] for r in rows), 3),
                "ok": sum(r["ok"] for r in rows), "pending": sum(r["pending"] for r in rows),
                "late_ok": sum(r["late"] and r["ok"] for r in rows)}
    out.update({"idle_summary": summ(out.pop("idle")), "tenant_single": summ(single), "tenant_paired": summ(paired),
                "gemm_ms_p50": statistics.median(doc["gemm_ms"]), "examples": (single + paired)[:6]})
    text = json.dumps(out, indent=1)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
