#!/usr/bin/env python3
"""PreStartContainer latency and health-sweep time of the native daemon while
a tenant runs long kernels on the same GPU.

The shipped path end to end: `mi355x-device-plugin -liveness -prestart_liveness`
with its kept-queue probe server, a fake kubelet calling PreStartContainer over
the plugin socket, and a torch tenant running back-to-back bf16 GEMMs (n=65536:
~440 ms each, every CU held) on GPU 0. Phases:

  idle     no tenant: PreStartContainer on the GPU, --calls times
  tenant   the tenant runs: PreStartContainer every --interval s, and the
           daemon's 1 s health sweeps go on meanwhile

The sweep and gate times come from the daemon's own Chrome trace
(-trace_file: `health.sweep`, `liveness.prestart` spans); the client times
every PreStartContainer call. The reference's PreStartContainer is a no-op
(internal/pkg/plugin/plugin.go:139-141); kubelet gives it 30 s
(vendor/k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/constants.go:44).

  python tools/prestart_tenant.py --out gpurun_out/prestart_tenant.json
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import socket
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

TENANT = r"""
import json, sys, time, torch
n, seconds = int(sys.argv[1]), float(sys.argv[2])
a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
torch.matmul(a, b, out=c)
torch.cuda.synchronize()
print("READY", flush=True)
sys.stdin.readline()
ms, t_end = [], time.perf_counter() + seconds
while time.perf_counter() < t_end:
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.matmul(a, b, out=c)
    e1.record()
    e1.synchronize()
    ms.append(e0.elapsed_time(e1))
print(json.dumps({"n": n, "gemm_ms": ms}), flush=True)
"""


def pct(xs, p):
    s = sorted(xs)
    return round(s[min(len(s) - 1, int(p * (len(s) - 1)))], 3) if s else None


def summary(xs):
    return {"n": len(xs), "p50_ms": pct(xs, 0.5), "p90_ms": pct(xs, 0.9), "max_ms": round(max(xs), 3) if xs else None,
            "mean_ms": round(statistics.mean(xs), 3) if xs else None}


def spans(trace_path, name, t0_us, t1_us):
    with open(trace_path) as f:
        ev = json.load(f)["traceEvents"]
    return [e["dur"] / 1e3 for e in ev if e.get("name") == name and e.get("ph") == "X" and t0_us <= e["ts"] <= t1_us]


async def run(a) -> dict:
    from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet, NativeRpcError
    from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals

    inv = discover("/sys")
    ords = hip_ordinals(inv, "/dev")
    dev_id = min(ords, key=ords.get)
    exe = os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")
    probe = os.path.join(str(PKG_DIR), "bin", "mi355x-liveness-probe")
    work = os.path.abspath(a.workdir)
    os.makedirs(work, exist_ok=True)
    kdir, trace = os.path.join(work, "dp"), os.path.join(work, "daemon_trace.json")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    k = FakeKubelet(kdir, rpc_client="native")
    await k.start()
    args = [exe, "-kubelet_dir", kdir, "-exporter_socket", "", "-pulse", str(a.pulse), "-liveness", "-liveness_probe",
            probe, "-liveness_timeout", str(a.liveness_timeout), "-prestart_liveness", "-trace_file", trace,
            "-metrics_port", str(port), *a.daemon_args.split()]
    proc = await asyncio.create_subprocess_exec(*args, stdout=asyncio.subprocess.DEVNULL,
                                                stderr=asyncio.subprocess.PIPE)
    out = {"device": dev_id, "daemon_args": args[1:], "gemm_n": a.n}
    req = pb.PreStartContainerRequest(devices_ids=[dev_id])
    tenant = None

    async def prestart():
        t0 = time.perf_counter()
        try:
            await k._call(st, "PreStartContainer", req, pb.PreStartContainerResponse, timeout=35.0)
            status = 0
        except NativeRpcError as e:
            status = e.status
        return (time.perf_counter() - t0) * 1e3, status

    try:
        st = await k.wait_for_resource("amd.com/gpu", 1, timeout=90)
        idle = []
        for _ in range(a.calls):
            idle.append(await prestart())
            await asyncio.sleep(0.05)
        out["idle_prestart"] = summary([x for x, _ in idle])
        out["idle_prestart_failed"] = sum(1 for _, s in idle if s)
        t_idle_end = time.monotonic_ns() / 1e3
        tenant = subprocess.Popen([sys.executable, "-c", TENANT, str(a.n), str(a.seconds)], stdin=subprocess.PIPE,
                                  stdout=subprocess.PIPE, text=True)
        line = await asyncio.to_thread(tenant.stdout.readline)
        assert line.strip() == "READY", line
        tenant.stdin.write("go\n")
        tenant.stdin.flush()
        t_ten0 = time.monotonic_ns() / 1e3
        print(f"tenant running ({a.seconds:.0f} s)", flush=True)
        busy = []
        end = time.monotonic() + a.seconds - 1.0
        while time.monotonic() < end:
            busy.append(await prestart())
            await asyncio.sleep(a.interval)
            if len(busy) % 10 == 0:
                print(f"  {len(busy)} PreStart calls under the tenant, last {busy[-1][0]:.1f} ms", flush=True)
        t_ten1 = time.monotonic_ns() / 1e3
        doc = json.loads(await asyncio.to_thread(tenant.stdout.readline))
        await asyncio.to_thread(tenant.wait)
        tenant = None
        g = doc["gemm_ms"]
        out["tenant_gemm"] = summary(g[1:] if len(g) > 1 else g)
        out["tenant_prestart"] = summary([x for x, _ in busy])
        out["tenant_prestart_failed"] = sum(1 for _, s in busy if s)
        out["tenant_prestart_statuses"] = sorted({s for _, s in busy})
    finally:
        if tenant is not None:
            tenant.kill()
        if proc.returncode is None:
            proc.send_signal(signal.SIGTERM)
        _, err = await asyncio.wait_for(proc.communicate(), 60)
        await k.stop()
    out["daemon_rc"] = proc.returncode
    err = err.decode(errors="replace")
    out["daemon_log_tail"] = err[-1500:]
    out["idle_sweep"] = summary(spans(trace, "health.sweep", 0, t_idle_end))
    out["tenant_sweep"] = summary(spans(trace, "health.sweep", t_ten0, t_ten1))
    out["tenant_gate_span"] = summary(spans(trace, "liveness.prestart", t_ten0, t_ten1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536, help="tenant GEMM size (n x n x n bf16)")
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--interval", type=float, default=0.25)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--pulse", type=int, default=1)
    ap.add_argument("--liveness-timeout", type=float, default=10.0)
    ap.add_argument("--daemon-args", default="", help="extra daemon flags, space-separated")
    ap.add_argument("--workdir", default="gpurun_out/prestart_tenant")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = asyncio.run(run(a))
    text = json.dumps(res, indent=1)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
