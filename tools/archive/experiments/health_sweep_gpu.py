#!/usr/bin/env python3
"""Health sweeps with the MFMA liveness probe on real hardware, through the
real plugin (fake kubelet, ListAndWatch), with a Chrome trace.

Reports per-sweep latency, per-device probe latency and the verdicts; every
accessible device must stay Healthy for the whole run.

  python tools/archive/experiments/health_sweep_gpu.py --sweeps 20 --out gpurun_out/health_sweep.json --trace t.json
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

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig, HealthMonitor  # noqa: E402
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl  # noqa: E402
from rocm_k8s_device_plugin_amd.plugin.manager import ManagerConfig, PluginManager  # noqa: E402
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet  # noqa: E402
from rocm_k8s_device_plugin_amd.topology import Inventory, discover, hip_ordinals  # noqa: E402
from rocm_k8s_device_plugin_amd.utils import log  # noqa: E402
from rocm_k8s_device_plugin_amd.utils.trace import TRACER  # noqa: E402


async def main_async(a):
    inv = discover(a.sysfs_root)
    ords = hip_ordinals(inv, a.dev_root)
    acc = Inventory(sysfs_root=a.sysfs_root, devices=tuple(inv.by_id[i] for i in ords), topology=inv.topology,
                    driver_loaded=True, kfd_present=True)
    mon = HealthMonitor(acc, HealthConfig(exporter_socket=None, liveness=True, liveness_timeout_s=30,
                                          dev_root=a.dev_root, liveness_mode=a.liveness_mode), ordinal_map=ords)
    impl = ContainerImpl("single", a.sysfs_root, inventory=acc, monitor=mon)
    sweep_ms, probe_ms, kernel_us = [], [], []
    orig = mon.prober.probe

    async def timed(ordinals):
        res = await orig(ordinals)
        for r in res.values():
            probe_ms.append(r.latency_ms)
            kernel_us.append(float(r.detail.get("kernel_us", 0.0)))
        return res

    mon.prober.probe = timed
    with tempfile.TemporaryDirectory() as d:
        k = FakeKubelet(d)
        await k.start()
        mgr = PluginManager(impl, ManagerConfig(pulse_s=a.pulse, plugin_dir=d, handle_signals=False))
        task = asyncio.create_task(mgr.run())
        st = await k.wait_for_resource("amd.com/gpu", len(acc), timeout=60)
        t_end = time.monotonic() + 600
        while mon.sweeps < a.sweeps and time.monotonic() < t_end:
            await asyncio.sleep(a.pulse / 2)
        devices = dict(st.devices)
        mgr.request_stop()
        await task
        await k.stop()
    from rocm_k8s_device_plugin_amd.utils.metrics import REGISTRY
    h = REGISTRY.histogram("mi355x_dp_health_sweep_seconds")
    sweep_ms = list(h.samples)
    res = {
        "devices": list(ords), "sweeps": mon.sweeps, "listandwatch_health": devices,
        "all_healthy": all(v.health == "Healthy" for v in mon.snapshot().values()),
        "verdicts": {k: [v.health, list(v.reasons)] for k, v in mon.snapshot().items()},
        "sweep_ms_p50": round(statistics.median(sweep_ms), 2) if sweep_ms else None,
        "sweep_ms_max": round(max(sweep_ms), 2) if sweep_ms else None,
        "probe_ms_p50": round(statistics.median(probe_ms), 2) if probe_ms else None,
        "probe_ms_max": round(max(probe_ms), 2) if probe_ms else None,
        "kernel_us_p50": round(statistics.median(kernel_us), 2) if kernel_us else None,
        "liveness_mode": a.liveness_mode, "probe_server_starts": mon.prober.server_starts,
        "probe_fallbacks": mon.prober.fallbacks,
    }
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweeps", type=int, default=10)
    ap.add_argument("--pulse", type=float, default=1.0)
    ap.add_argument("--sysfs-root", default="/sys")
    ap.add_argument("--dev-root", default="/dev")
    ap.add_argument("--out", default="")
    ap.add_argument("--trace", default="")
    ap.add_argument("--liveness-mode", default="persistent", choices=("persistent", "spawn"))
    a = ap.parse_args()
    log.setup(0)
    TRACER.configure(a.trace or None)
    res = asyncio.run(main_async(a))
    TRACER.flush()
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    sys.exit(0 if res["all_healthy"] else 1)


if __name__ == "__main__":
    main()
