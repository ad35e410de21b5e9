#!/usr/bin/env python3
"""Soak of the native daemon (`mi355x-device-plugin`) on a real node.

The daemon registers at a fake kubelet over UDS on the node's own /sys, with a
1 s health pulse; admissions (GetPreferredAllocation + Allocate of every size
1..N over the native gRPC server) run back to back with no pause. Every
--report seconds one JSON line: admissions, errors, RPC latency percentiles,
and what would leak if anything did: the daemon's RSS, open fds and threads.
With --container-interval S, every S seconds one admission's container is
started for real (container_runtime.start_container: a fresh process whose
/dev is the Allocate DeviceSpecs runs the MFMA kernel), on the GPU the
daemon's liveness loop is probing: containers must all come up, and the
device must stay Healthy in ListAndWatch.

  python tools/soak_native.py --seconds 120 --out gpurun_out/soak_native.json
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR  # noqa: E402
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet  # noqa: E402

EXE = os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")
CONTAINER_RUNTIME = "hip"   # the container is a HIP program, --container-runtime


def proc_stats(pid: int) -> dict:
    out = {}
    with open(f"/proc/{pid}/status") as f:
        for line in f:
            k, _, v = line.partition(":")
            if k in ("VmRSS", "Threads"):
                out[k] = int(v.split()[0])
    out["fds"] = len(os.listdir(f"/proc/{pid}/fd"))
    return {"rss_kb": out.get("VmRSS"), "threads": out.get("Threads"), "fds": out["fds"]}


def children(ppid: int) -> list:
    out = []
    for d in os.listdir("/proc"):
        if d.isdigit():
            try:
                with open(f"/proc/{d}/stat") as f:
                    if int(f.read().rsplit(")", 1)[1].split()[1]) == ppid:
                        out.append(int(d))
            except (OSError, ValueError, IndexError):
                pass
    return out


def pct(xs, q):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(q * len(xs)))], 4) if xs else None



SANITIZER_MARKERS = (b"WARNING: ThreadSanitizer", b"ERROR: AddressSanitizer", b"ERROR: LeakSanitizer", b"runtime error:")


def sanitizer_reports(f):
    """(count, first report text) of sanitizer findings in the daemon's whole stderr
    file, read in chunks (a long soak logs every Allocate: hundreds of MB)."""
    f.seek(0)
    count, first, tail = 0, "", b""
    while True:
        chunk = f.read(1 << 22)
        if not chunk:
            break
        buf = tail + chunk
        for m in SANITIZER_MARKERS:
            # markers wholly inside the carried-over tail were counted with the previous chunk
            count += buf.count(m) - tail.count(m)
            if not first and m in buf:
                i = buf.index(m)
                first = buf[i:i + 3000].decode(errors="replace")
        tail = buf[-64:]
    return count, first


async def run_container(adm, minor_to_ord: dict, cont: dict) -> None:
    """The admitted pod's container, for real (blocking; the kfd teardown of the
    previous one is waited out first, as kubelet does before reusing devices)."""
    from rocm_k8s_device_plugin_amd.container_runtime import (render_minors_from_specs, start_container,
                                                              wait_kfd_released)
    car = adm.response.container_responses[0]
    ordl = [minor_to_ord[m] for m in render_minors_from_specs(car)]
    paths = ["/dev/kfd"] + [d.host_path for d in car.devices if d.host_path.startswith("/dev/dri/")]
    res = await asyncio.to_thread(start_container, ordl, 60.0, device_paths=paths, runtime=CONTAINER_RUNTIME)
    cont["started"] += 1
    if res.ok:
        cont["ready_ms"].append((res.t_ready_ns - res.t_start_ns) / 1e6)
    else:
        cont["failed"] += 1
        cont["errors"].append(res.error[:200])
    await asyncio.to_thread(wait_kfd_released, res.kfd_lingering, 1.0)


def probe_endpoints(port: int) -> dict:
    """/healthz and /readyz as kubelet's probes read them: status code and time to the answer."""
    import urllib.error
    import urllib.request
    out = {}
    for path in ("/healthz", "/readyz"):
        t0 = time.monotonic()
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=10) as r:
                code = r.status
        except urllib.error.HTTPError as e:
            code = e.code
        except OSError:
            code = 0
        out[path.strip("/")] = code
        out[path.strip("/") + "_ms"] = round((time.monotonic() - t0) * 1e3, 2)
    return out


async def main(a) -> int:
    global CONTAINER_RUNTIME
    CONTAINER_RUNTIME = a.container_runtime
    kdir = tempfile.mkdtemp(prefix="soak-native-")
    k = FakeKubelet(kdir)
    await k.start()
    extra = a.extra.split() if a.extra else []
    if a.metrics_port:
        extra += ["-metrics_port", str(a.metrics_port)]
    # the daemon logs every Allocate (as the reference does): its stderr goes to a file, a
    # pipe nobody reads would fill and block its control loop (and with it the health pulses)
    errf = open(os.path.join(kdir, "daemon.stderr"), "w+b")
    proc = await asyncio.create_subprocess_exec(a.exe, "-kubelet_dir", kdir, "-sysfs_root", a.sysfs_root,
                                                "-pulse", str(a.pulse), "-exporter_socket", "", *extra,
                                                stdout=asyncio.subprocess.DEVNULL, stderr=errf)
    rows = []
    try:
        # the first health sweep (with -perf_check_every: a throughput check) runs before
        # registration; a sanitizer build takes a while longer
        st = await k.wait_for_resource("amd.com/gpu", 1, timeout=120)
        n = len(st.devices)
        t_end = time.monotonic() + a.seconds
        next_report = time.monotonic() + a.report
        adm = errors = 0
        lat = []
        first = proc_stats(proc.pid)
        cont = {"started": 0, "failed": 0, "ready_ms": [], "errors": [], "unhealthy_seen": 0}
        minor_to_ord = {}
        if a.container_interval > 0:
            from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals
            inv = discover(a.sysfs_root)
            ords = hip_ordinals(inv, "/dev", check_access=True)
            minor_to_ord = {dv.render_minor: ords[dv.id] for dv in inv.devices if dv.id in ords}
        next_container = time.monotonic() + (a.container_interval if a.container_interval > 0 else 1e18)
        while time.monotonic() < t_end:
            healthy = len(k.healthy_free("amd.com/gpu")) + 0
            size = adm % max(1, min(n, healthy)) + 1
            try:
                r = await k.admit("amd.com/gpu", 1 if time.monotonic() >= next_container else size)
                lat.append(r.total_ms)
                adm += 1
                if time.monotonic() >= next_container:
                    next_container = time.monotonic() + a.container_interval
                    await run_container(r, minor_to_ord, cont)
                    unhealthy = [d for d, h in k.resources["amd.com/gpu"].devices.items() if h != "Healthy"]
                    cont["unhealthy_seen"] += any(d in r.device_ids for d in unhealthy)
                k.release("amd.com/gpu", r.device_ids)
            except Exception as e:  # noqa: BLE001
                errors += 1
                print(f"admission error: {e}", file=sys.stderr)
            if time.monotonic() >= next_report:
                next_report += a.report
                row = {"t_s": round(a.seconds - (t_end - time.monotonic()), 1), "admissions": adm, "errors": errors,
                       "rpc_ms_p50": pct(lat, 0.5), "rpc_ms_p99": pct(lat, 0.99), **proc_stats(proc.pid),
                       "children": [proc_stats(c) for c in children(proc.pid)]}
                if a.container_interval > 0:
                    row["containers"] = {"started": cont["started"], "failed": cont["failed"],
                                         "ready_ms_p50": pct(cont["ready_ms"], 0.5),
                                         "ready_ms_p99": pct(cont["ready_ms"], 0.99),
                                         "device_unhealthy_after": cont["unhealthy_seen"]}
                if a.metrics_port:
                    row["probes"] = await asyncio.to_thread(probe_endpoints, a.metrics_port)
                rows.append(row)
                print(json.dumps(row), flush=True)
                lat = []
        metrics = None
        if a.metrics_port:
            import urllib.request
            with urllib.request.urlopen(f"http://127.0.0.1:{a.metrics_port}/metrics", timeout=5) as r:
                metrics = {ln.rsplit(" ", 1)[0]: float(ln.rsplit(" ", 1)[1]) for ln in r.read().decode().splitlines()
                           if ln and not ln.startswith("#") and "_bucket" not in ln}
        doc = {"exe": os.path.basename(a.exe), "exe_path": a.exe, "devices": n, "pulse_s": a.pulse, "seconds": a.seconds,
               "flags": extra, "metrics_end": metrics,
               "containers": ({"interval_s": a.container_interval, "started": cont["started"],
                               "failed": cont["failed"], "errors": cont["errors"][:5],
                               "ready_ms_p50": pct(cont["ready_ms"], 0.5), "ready_ms_p99": pct(cont["ready_ms"], 0.99),
                               "device_unhealthy_after": cont["unhealthy_seen"]}
                              if a.container_interval > 0 else None),
               "start": first, "reports": rows, "admissions": adm, "errors": errors,
               "listandwatch_updates": k.state("amd.com/gpu").updates if hasattr(k, "state") else None}
    finally:
        if proc.returncode is None:
            proc.terminate()
        await asyncio.wait_for(proc.wait(), 20)
        await k.stop()
        errf.seek(0, os.SEEK_END)
        errf.seek(max(0, errf.tell() - 4000))
        err = errf.read()
        reports, first_report = sanitizer_reports(errf)
        errf.close()
    doc["exit_code"] = proc.returncode
    # kubelet's liveness / readiness probes (the chart's, with a metrics port) at every report
    doc["probe_failures"] = sum(1 for r in doc["reports"] if "probes" in r
                                and (r["probes"]["healthz"] != 200 or r["probes"]["readyz"] != 200))
    doc["sanitizer_reports"] = reports
    # stopping the daemon must not flip a device (a check cut short by the shutdown is no verdict)
    tail_text = err.decode(errors="replace")
    after = tail_text[tail_text.find("Received signal"):] if "Received signal" in tail_text else ""
    doc["transitions_after_shutdown"] = after.count("-> Unhealthy") + after.count("-> failed")
    if first_report:
        doc["first_sanitizer_report"] = first_report
    doc["stderr_tail"] = err.decode(errors="replace")[-500:]
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)
    print(json.dumps({k_: doc[k_] for k_ in ("admissions", "errors", "exit_code")}))
    bad_containers = doc["containers"] and (doc["containers"]["failed"] or doc["containers"]["device_unhealthy_after"])
    ok = doc["errors"] == 0 and doc["exit_code"] == 0 and not bad_containers and not reports and not doc["probe_failures"]
    return 0 if ok and not doc["transitions_after_shutdown"] else 1


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--report", type=float, default=15)
    ap.add_argument("--pulse", type=int, default=1)
    ap.add_argument("--sysfs-root", default="/sys")
    ap.add_argument("--out", default="")
    ap.add_argument("--extra", default="", help="more daemon flags, space-separated")
    ap.add_argument("--exe", default=os.environ.get("MI355X_NATIVE_DAEMON_EXE") or EXE,
                    help="the daemon binary (e.g. a ThreadSanitizer build; default: this tree's)")
    ap.add_argument("--metrics-port", type=int, default=0)
    ap.add_argument("--container-runtime", default="hip", choices=["hip", "hsa"])
    ap.add_argument("--container-interval", type=float, default=0.0,
                    help="every S seconds start one admission's container on the GPU (0 = never)")
    sys.exit(asyncio.run(main(ap.parse_args())))
