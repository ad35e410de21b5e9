#!/usr/bin/env python3
"""Soak: the real plugin CLI on a GPU node for a while, with every health
source on, while pods come and go.

The `k8s-device-plugin` CLI registers at a fake kubelet (UDS); the health loop
runs with the kept-queue probe server, the full-chip sweep and the throughput
check; admissions (GetPreferredAllocation + Allocate over gRPC) start a real
container process on the allocated GPU (MFMA kernel, ready line) back to back.
Every --report seconds one JSON line: admissions, failures, latency, and the
resources that would leak if anything did: plugin and probe-server RSS and
open fds, kfd queues of the probe server, ListAndWatch updates.

  python tools/soak.py --seconds 300 --out gpurun_out/soak.json
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import re
import signal
import socket
import statistics
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from rocm_k8s_device_plugin_amd.container_runtime import (  # noqa: E402
    render_minors_from_specs, start_container, wait_kfd_released)
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet  # noqa: E402
from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals  # noqa: E402


_TICK = os.sysconf("SC_CLK_TCK")


def proc_stats(pid: int) -> dict:
    out = {"rss_mb": None, "fds": None, "cpu_s": None}
    try:
        with open(f"/proc/{pid}/status") as f:
            for line in f:
                if line.startswith("VmRSS"):
                    out["rss_mb"] = round(int(line.split()[1]) / 1024, 1)
        out["fds"] = len(os.listdir(f"/proc/{pid}/fd"))
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        out["cpu_s"] = round((int(fields[11]) + int(fields[12])) / _TICK, 2)   # utime + stime
    except (OSError, ValueError, IndexError):
        pass
    return out


def children(pid: int) -> list:
    kids = []
    try:
        for tid in os.listdir(f"/proc/{pid}/task"):
            with open(f"/proc/{pid}/task/{tid}/children") as f:
                kids += [int(x) for x in f.read().split()]
    except OSError:
        pass
    return kids


def kfd_queues() -> dict:
    """kfd proc entry -> user queues (all processes on the host we can see)."""
    root, out = "/sys/class/kfd/kfd/proc", {}
    try:
        for e in os.listdir(root):
            try:
                out[e] = len(os.listdir(os.path.join(root, e, "queues")))
            except OSError:
                continue
    except OSError:
        pass
    return out


def scrape(port: int) -> dict:
    """The plugin's /metrics: health-loop counters and the last throughput check."""
    import urllib.request
    try:
        text = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
    except OSError:
        return {}
    out = {}
    for name in ("mi355x_dp_perf_checks_total", "mi355x_dp_health_sweep_seconds_count",
                 "mi355x_dp_perf_hbm_read_gbps", "mi355x_dp_perf_hbm_write_gbps", "mi355x_dp_perf_mfma_tflops",
                 "mi355x_dp_perf_clock_mhz", "mi355x_dp_perf_state"):
        vals = [float(m.group(1)) for m in re.finditer(rf"^{name}(?:{{[^}}]*}})? ([0-9.eE+-]+)$", text, re.M)]
        if vals:
            out[name] = vals[0] if len(vals) == 1 else vals
    return out


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def main_async(a) -> dict:
    inv = discover("/sys")
    ords = hip_ordinals(inv, "/dev")
    minor_to_ord = {inv.by_id[d].render_minor: o for d, o in ords.items()}
    with tempfile.TemporaryDirectory() as kd:
        k = FakeKubelet(kd, rpc_client="native")
        await k.start()
        env = dict(os.environ, PYTHONPATH=REPO, MI355X_DP_NO_AUTOBUILD="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
        kfd_before = set(kfd_queues())
        port = free_port()
        plugin = await asyncio.create_subprocess_exec(
            sys.executable, "-m", "rocm_k8s_device_plugin_amd.cli.device_plugin", "-kubelet_dir", kd,
            "-exporter_socket", "", "-pulse", str(a.pulse), "-liveness", "-liveness_chip_sweep_every", "5",
            "-perf_check_every", str(a.perf_every), "-perf_mib", "1024", "-smi_ecc", "-smi_events", "-smi_xgmi",
            "-metrics_port", str(port), "-v", "2", env=env, stdout=asyncio.subprocess.DEVNULL, stderr=open(a.log, "w"))
        rows, lat, fails, n = [], [], 0, 0
        try:
            st = await k.wait_for_resource("amd.com/gpu", len(ords), timeout=120)
            t_end = time.monotonic() + a.seconds
            next_report = time.monotonic() + a.report
            first = None
            while time.monotonic() < t_end:
                if a.idle:   # no pods: what the daemon itself costs between admissions
                    await asyncio.sleep(max(0.0, min(1.0, next_report - time.monotonic())))
                else:
                    t0 = time.monotonic_ns()
                    try:
                        adm = await k.admit("amd.com/gpu", 1)
                        car = adm.response.container_responses[0]
                        ol = [minor_to_ord[m] for m in render_minors_from_specs(car)]
                        paths = ["/dev/kfd"] + [ds.host_path for ds in car.devices if "/dri/" in ds.host_path]
                        r = await asyncio.to_thread(start_container, ol, timeout_s=60, device_paths=paths)
                        k.release("amd.com/gpu", adm.device_ids)
                        if r.ok:
                            lat.append((r.t_ready_ns - t0) / 1e6)
                        else:
                            fails += 1
                        await asyncio.to_thread(wait_kfd_released, r.kfd_lingering, 1.0)
                    except Exception as e:  # noqa: BLE001
                        fails += 1
                        print(json.dumps({"error": f"{type(e).__name__}: {e}"[:300]}), flush=True)
                    n += 1
                if time.monotonic() >= next_report:
                    next_report += a.report
                    kids = children(plugin.pid)
                    q = kfd_queues()
                    srv = [dict(proc_stats(c), pid=c, kfd_queues=q.get(str(c))) for c in kids]
                    row = {"t_s": round(a.seconds - (t_end - time.monotonic()), 1), "admissions": n, "failures": fails,
                           "ready_p50_ms": round(statistics.median(lat[-50:]), 2) if lat else None,
                           "plugin": proc_stats(plugin.pid), "plugin_children": srv,
                           # kfd entries that appeared since start-up, not the plugin's children:
                           # containers still running or still being torn down
                           "kfd_other_new_entries": sum(1 for e in q if e not in kfd_before and
                                                        int(e) not in kids),
                           "listandwatch_updates": st.updates,
                           "healthy": sum(h == "Healthy" for h in st.devices.values()),
                           "metrics": scrape(port)}
                    first = first or row
                    rows.append(row)
                    print(json.dumps(row), flush=True)
        finally:
            plugin.send_signal(signal.SIGTERM)
            try:
                rc = await asyncio.wait_for(plugin.wait(), 30)
            except asyncio.TimeoutError:
                plugin.kill()
                rc = "killed"
            await k.stop()
        return {"seconds": a.seconds, "pulse_s": a.pulse, "idle": a.idle, "admissions": n, "failures": fails,
                "ready_p50_ms": round(statistics.median(lat), 2) if lat else None,
                "ready_p99_ms": round(sorted(lat)[int(0.99 * (len(lat) - 1))], 2) if lat else None,
                "plugin_exit": rc, "first": rows[0] if rows else None, "last": rows[-1] if rows else None,
                "rows": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300)
    ap.add_argument("--pulse", type=int, default=1, help="plugin -pulse (whole seconds, as upstream)")
    ap.add_argument("--perf-every", type=int, default=40, help="throughput check every N pulses")
    ap.add_argument("--report", type=float, default=30)
    ap.add_argument("--idle", action="store_true", help="no admissions: the daemon's own steady-state cost")
    ap.add_argument("--log", default="/tmp/soak_plugin.log")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = asyncio.run(main_async(a))
    print(json.dumps({k: v for k, v in res.items() if k != "rows"}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
