#!/usr/bin/env python3
"""Plugin process start -> kubelet sees the resource (Register + first ListAndWatch).

Starts the real ``k8s-device-plugin`` CLI as a child process against a fake
kubelet (UDS in a temp dir) and times: exec -> Register RPC received -> first
ListAndWatch device list with all devices. That is how long a node's GPUs stay
unschedulable after the plugin pod (re)starts.

  python tools/plugin_startup.py [--fixture] [--native] --reps 5 --out gpurun_out/plugin_startup.json
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import statistics
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet  # noqa: E402


async def one(sysfs: str, dev: str, expect: int, native: bool = False) -> dict:
    with tempfile.TemporaryDirectory() as d:
        k = FakeKubelet(d)
        await k.start()
        env = dict(os.environ, PYTHONPATH=REPO, MI355X_DP_NO_AUTOBUILD="1")
        t0 = time.monotonic()
        argv = ([os.path.join(REPO, "rocm_k8s_device_plugin_amd", "bin", "mi355x-device-plugin")] if native else
                [sys.executable, "-m", "rocm_k8s_device_plugin_amd.cli.device_plugin"])
        proc = await asyncio.create_subprocess_exec(
            *argv, "-kubelet_dir", d,
            "-sysfs_root", sysfs, "-dev_root", dev, "-exporter_socket", "", "-driver_type", "container",
            env=env, stdout=asyncio.subprocess.DEVNULL, stderr=asyncio.subprocess.DEVNULL)
        try:
            await k.wait_for_resource("amd.com/gpu", expect, timeout=60)
            t_law = time.monotonic()
            t_reg = k.register_times["amd.com/gpu"]
            rss_mb = None
            try:
                with open(f"/proc/{proc.pid}/status") as f:
                    rss_mb = [int(x.split()[1]) / 1024 for x in f if x.startswith("VmRSS")][0]
            except (OSError, IndexError):
                pass
        finally:
            proc.send_signal(signal.SIGTERM)
            await asyncio.wait_for(proc.wait(), 20)
            await k.stop()
    return {"register_ms": (t_reg - t0) * 1e3, "devices_listed_ms": (t_law - t0) * 1e3, "rss_mb": rss_mb}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fixture", action="store_true", help="synthetic 8x MI355X sysfs (CPU)")
    ap.add_argument("--native", action="store_true", help="the native daemon (mi355x-device-plugin) instead")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    sysfs, dev = "/sys", "/dev"
    if a.fixture:
        from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
        fi = make_mi355x_node(tempfile.mkdtemp(prefix="mi355x-startup-"))
        sysfs, dev = str(fi.sysfs), str(fi.dev)
    from rocm_k8s_device_plugin_amd.topology import discover
    expect = len(discover(sysfs).devices)
    rows = [asyncio.run(one(sysfs, dev, expect, a.native)) for _ in range(a.reps)]
    res = {"entrypoint": "mi355x-device-plugin" if a.native else "k8s-device-plugin (Python CLI)",
           "devices": expect, "reps": a.reps,
           **{f"{k}_p50": round(statistics.median(r[k] for r in rows), 1) for k in rows[0]},
           **{f"{k}_max": round(max(r[k] for r in rows), 1) for k in rows[0]}}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
