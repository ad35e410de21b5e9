#!/usr/bin/env python3
"""How often, and by how much, the reference's candidate family loses to the
optimum on fragmented partitioned nodes.

GetPreferredAllocation's default search enumerates the reference's candidates
(internal/pkg/allocator/device.go:353-442): whole GPUs plus one partial GPU's
prefix. `-allocator_extended_search` is an exact search over every split of
the request (brute-force-verified in tests/test_allocator.py). This tool
samples fragmented availabilities — devices held by other pods at random, a
random request size, sometimes a must-include device — on

* generated MI355X nodes: CPX / QPX / DPX x NPS1 / NPS2, one 8-GPU hive and
  two hives of 4;
* the reference's own captures: MI300X CPX (topo-mi300-cpx) and MI308X CPX
  (topology-parsing-mi308), with the synthetic devices of its tests;

and reports, per layout, the share of requests where the default's total pair
weight exceeds the optimum, the mean / max excess, how many more physical GPUs
the default's set spans, and both searches' time.

  python tools/alloc_gap.py [--samples 2000] [--json-out profiles/archive/allocator_default_vs_optimum.json]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from rocm_k8s_device_plugin_amd.allocator import BestEffortPolicy  # noqa: E402

REF = "/root/reference/testdata"


def mi355x_layouts(tmp):
    from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
    from rocm_k8s_device_plugin_amd.topology import discover
    out = {}
    for cp in ("CPX", "QPX", "DPX"):
        for mp in ("NPS1", "NPS2"):
            for hive in (8, 4):
                name = f"mi355x-{cp.lower()}-{mp.lower()}-hive{hive}"
                fi = make_mi355x_node(os.path.join(tmp, name), compute_partition=cp, memory_partition=mp,
                                      hive_size=hive)
                inv = discover(str(fi.sysfs))
                gpu = {d.id: d.unique_id for d in inv.devices}
                out[name] = (inv.devices, inv.topology, gpu)
    return out


def reference_layouts():
    if not os.path.isdir(REF):
        return {}
    from test_allocator import TOPOS, synthetic_devices
    from rocm_k8s_device_plugin_amd.allocator import load_topology
    out = {}
    for name in ("mi300cpx", "mi308"):
        t = TOPOS[name]
        devs = synthetic_devices(t["dev_count"], t["parts"], t["numa"], t["start"], t["end"])
        topo = load_topology(nodes_dir=os.path.join(REF, t["path"]))
        out[f"reference-{name}"] = (devs, topo, {d[0]: d[3] for d in devs})
    return out


def measure(name, devs, topo, gpu, samples, rng):
    ref = BestEffortPolicy()
    ext = BestEffortPolicy(extended_search=True)
    ref.init(devs, topo)
    ext.init(devs, topo)
    ids = [d[0] if isinstance(d, tuple) else d.id for d in devs]
    n = len(ids)
    worse, excess, gpus_more, t_ref, t_ext, checked = 0, [], [], [], [], 0
    for _ in range(samples):
        held = rng.uniform(0.1, 0.7)
        avail = [i for i in ids if rng.random() > held]
        if len(avail) < 2:
            continue
        k = rng.randint(1, min(len(avail) - 1, 16))
        req = rng.sample(avail, 1) if rng.random() < 0.2 else []
        t0 = time.perf_counter()
        a = ref.explain(avail, req, k)
        t1 = time.perf_counter()
        b = ext.explain(avail, req, k)
        t2 = time.perf_counter()
        if a["error"] or b["error"] or a["short_circuit"]:
            continue
        checked += 1
        t_ref.append((t1 - t0) * 1e6)
        t_ext.append((t2 - t1) * 1e6)
        assert b["weight"] <= a["weight"], (name, avail, req, k, a, b)
        ga, gb = len({gpu[x] for x in a["ids"]}), len({gpu[x] for x in b["ids"]})
        if a["weight"] > b["weight"]:
            worse += 1
            excess.append((a["weight"] - b["weight"]) / max(1, b["weight"]))
        gpus_more.append(ga - gb)
    pct = lambda xs, q: sorted(xs)[min(len(xs) - 1, int(q * (len(xs) - 1)))] if xs else None  # noqa: E731
    return {"devices": n, "requests": checked,
            "default_worse_pct": round(100.0 * worse / max(1, checked), 2),
            "excess_weight_mean_pct": round(100 * statistics.mean(excess), 2) if excess else 0.0,
            "excess_weight_max_pct": round(100 * max(excess), 2) if excess else 0.0,
            "default_spans_more_gpus_pct": round(100.0 * sum(1 for g in gpus_more if g > 0) / max(1, checked), 2),
            "default_spans_fewer_gpus_pct": round(100.0 * sum(1 for g in gpus_more if g < 0) / max(1, checked), 2),
            "reference_family_us_p50": round(pct(t_ref, .5), 1) if t_ref else None,
            "extended_us_p50": round(pct(t_ext, .5), 1) if t_ext else None,
            "extended_us_p99": round(pct(t_ext, .99), 1) if t_ext else None}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--samples", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)
    rng = random.Random(a.seed)
    with tempfile.TemporaryDirectory() as tmp:
        layouts = {**mi355x_layouts(tmp), **reference_layouts()}
        res = {name: measure(name, *v, a.samples, rng) for name, v in layouts.items()}
    doc = {"samples_per_layout": a.samples, "seed": a.seed,
           "note": "default = the reference's candidate family; optimum = -allocator_extended_search (exact)",
           "layouts": res}
    line = json.dumps(doc, indent=1)
    print(line)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
