#!/usr/bin/env python3
"""CPU benchmarks of the plugin-owned part of admission (no GPU needed).

1. Allocator: the C++ set search vs a faithful re-implementation of the
   reference's ordered-BFS enumeration (internal/pkg/allocator/device.go:353-442)
   on the same weights, same requests: time per call and candidates scored.
   Topologies: 8x MI355X SPX one hive, 8x SPX in two hives of 4, 8x8 CPX, and
   the reference's own MI300X-CPX / MI210 captures when mounted.
2. Admission over UDS gRPC through the fake kubelet on a synthetic 8x MI355X
   node: GetPreferredAllocation + Allocate p50/p99 at 1/2/4/8 GPUs, whole node
   free and fragmented, and on the 8x8 CPX node; the native daemon, and the
   oracle servicer on grpc.aio for comparison.

  python tools/bench_alloc.py --out profiles/r5/alloc_bench.json
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rocm_k8s_device_plugin_amd.allocator import BestEffortPolicy, load_topology  # noqa: E402
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node  # noqa: E402
from rocm_k8s_device_plugin_amd.topology import discover  # noqa: E402

REF = "/root/reference/testdata"


def pct(xs, q):
    s = sorted(xs)
    return s[min(len(s) - 1, int(round(q * (len(s) - 1))))] if s else float("nan")


def time_call(fn, reps):
    ts = []
    out = None
    for _ in range(reps):
        t = time.perf_counter()
        out = fn()
        ts.append((time.perf_counter() - t) * 1e6)
    return ts, out


def bench_topology(name, pol, ids, sizes, rng, frag_trials=20, ref_cap_us=2e6):
    rows = []
    for k in sizes:
        # whole node free
        ours_t, ours = time_call(lambda: pol.explain(ids, [], k), 50)
        t0 = time.perf_counter()
        ref = pol.reference_allocate(ids, [], k)
        ref_us = (time.perf_counter() - t0) * 1e6
        reps = 1 if ref_us > 20000 else 10
        ref_t, ref = time_call(lambda: pol.reference_allocate(ids, [], k), reps)
        # fragmented: random availability
        f_ours, f_ref, agree = [], [], 0
        for _ in range(frag_trials):
            av = rng.sample(ids, rng.randint(k, len(ids)))
            a = time_call(lambda: pol.explain(av, [], k), 3)
            b = time_call(lambda: pol.reference_allocate(av, [], k), 1)
            f_ours.append(statistics.median(a[0]))
            f_ref.append(b[0][0])
            agree += a[1]["weight"] == b[1]["weight"]
        rows.append({
            "topology": name, "k": k,
            "ours_us_p50": round(pct(ours_t, .5), 2), "ours_candidates": ours["candidates"],
            "reference_us_p50": round(pct(ref_t, .5), 2), "reference_candidates": ref["candidates"],
            "same_weight": ours["weight"] == ref["weight"], "same_ids": ours["ids"] == ref["ids"],
            "fragmented_ours_us_p50": round(pct(f_ours, .5), 2),
            "fragmented_reference_us_p50": round(pct(f_ref, .5), 2),
            "fragmented_weight_agreement": f"{agree}/{frag_trials}",
            "speedup": round(pct(ref_t, .5) / max(pct(ours_t, .5), 1e-3), 1),
        })
        print(json.dumps(rows[-1]), flush=True)
    return rows


def synthetic_ref_devices(dev_count, parts, numa_count, start, end):
    out, node = [], start
    per = dev_count // numa_count
    for i in range(dev_count):
        for j in range(parts):
            if node > end:
                break
            out.append((f"test{i + 1}" if j == 0 else f"amdgpu_xcp_{i * 8 + j}", node, i // per, str(i)))
            node += 1
    return out


async def admission(sysfs, n_adv, n_req, steps, fragment, server="native-daemon", client="native"):
    """kubelet's GetPreferredAllocation + Allocate round trips against the plugin on
    `n_adv` advertised devices: the native daemon (the product, as the images run it)
    or the oracle servicer on grpc.aio (testing/aio_plugin.py, the comparison)."""
    import signal
    import subprocess

    from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
    from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
    from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
    from rocm_k8s_device_plugin_amd.testing.aio_plugin import AioPlugin
    from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
    from rocm_k8s_device_plugin_amd.topology import Inventory

    full = discover(sysfs)
    devs = full.devices[:n_adv]
    with tempfile.TemporaryDirectory() as d:
        k = FakeKubelet(d, rpc_client=client)
        await k.start()
        proc = aio = None
        if server == "native-daemon":
            exe = os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")
            proc = subprocess.Popen([exe, "-kubelet_dir", d, "-sysfs_root", sysfs, "-dev_root",
                                     os.path.join(os.path.dirname(sysfs), "dev"), "-exporter_socket", "",
                                     "-device_ids", ",".join(x.id for x in devs)],
                                    stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        else:
            inv = Inventory(sysfs_root=sysfs, devices=devs, topology=full.topology, driver_loaded=True,
                            kfd_present=True)
            aio = AioPlugin(ContainerImpl("single", sysfs, HealthConfig(exporter_socket=None), inventory=inv), d)
            await aio.start()
        try:
            await k.wait_for_resource("amd.com/gpu", n_adv)
            rng = random.Random(5)
            lat, pref = [], []
            for i in range(steps):
                av = None
                if fragment:
                    ids = k.healthy_free("amd.com/gpu")
                    av = sorted(rng.sample(ids, rng.randint(n_req, len(ids))))
                a = await k.admit("amd.com/gpu", n_req, available=av)
                lat.append(a.total_ms)
                pref.append(a.preferred_ms)
                k.release("amd.com/gpu", a.device_ids)
        finally:
            if proc is not None:
                proc.send_signal(signal.SIGTERM)
                proc.wait(timeout=20)
            if aio is not None:
                await aio.stop()
            await k.stop()
    return {"server": server, "kubelet_client": client, "advertised": n_adv, "requested": n_req, "fragmented": fragment,
            "admission_p50_ms": round(pct(lat, .5), 4), "admission_p99_ms": round(pct(lat, .99), 4),
            "preferred_p50_ms": round(pct(pref, .5), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    rng = random.Random(11)
    res = {"allocator": [], "admission": []}
    with tempfile.TemporaryDirectory() as d:
        for name, kw, sizes in [("mi355x_spx_1hive", {}, range(1, 8)),
                                ("mi355x_spx_2hives", {"hive_size": 4}, range(1, 8)),
                                ("mi355x_cpx_8x8", {"compute_partition": "cpx"}, [1, 2, 4, 8, 12, 16, 24, 30, 32])]:
            fi = make_mi355x_node(os.path.join(d, name), **kw)
            inv = discover(str(fi.sysfs))
            pol = BestEffortPolicy()
            pol.init(inv.devices, inv.topology)
            res["allocator"] += bench_topology(name, pol, [x.id for x in inv.devices], sizes, rng)
        if os.path.isdir(REF):
            for name, args, path, sizes in [
                ("ref_mi210_2hives", (8, 1, 2, 2, 9), "topo-mi210-xgmi-pcie/nodes", range(1, 8)),
                ("ref_mi300x_cpx", (8, 8, 2, 2, 64), "topo-mi300-cpx/topology/nodes", [1, 4, 8, 16, 30, 32])]:
                devs = synthetic_ref_devices(*args)
                pol = BestEffortPolicy()
                pol.init(devs, load_topology(nodes_dir=os.path.join(REF, path)))
                res["allocator"] += bench_topology(name, pol, [x[0] for x in devs], sizes, rng)
        # the plugin-owned part of admission over UDS: kubelet's GetPreferredAllocation +
        # Allocate round trips against the native daemon, and against the oracle servicer on
        # grpc.aio for comparison, both called from the native client (kubelet itself is a
        # compiled grpc-go client)
        fi = make_mi355x_node(os.path.join(d, "adm"))
        cpx = make_mi355x_node(os.path.join(d, "adm_cpx"), compute_partition="cpx")
        # ("native-thread": the same client on a worker thread, needed when the server runs on this
        # process' event loop -- grpc.aio -- and used for both servers for a like-for-like pair)
        for server, client in (("native-daemon", "native"), ("native-daemon", "native-thread"),
                               ("aio", "native-thread")):
            runs = [(fi, n, n, False) for n in (1, 2, 4, 8)] + [(fi, 8, n, True) for n in (1, 2, 4, 7)] + \
                [(cpx, 64, n, True) for n in (1, 8, 32)]
            for node, n_adv, n_req, frag in runs:
                r = asyncio.run(admission(str(node.sysfs), n_adv, n_req, a.steps, frag, server=server,
                                          client=client))
                if node is cpx:
                    r["partition"] = "cpx"
                print(json.dumps(r), flush=True)
                res["admission"].append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
