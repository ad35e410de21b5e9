#!/usr/bin/env python3
"""A/B of the -node_view mounts on this host's real GPU (measurement tool).

Alternates plain and viewed containers (ABAB..., both through the same
interposing entrypoint build with the same /dev view), for the HSA and the HIP
entrypoint, with the view built on /tmp and on /dev/shm. Per container it
records what decides the question deterministically (read syscalls, CPU ms,
per-CPU cache descriptors opened, redirected paths) next to the wall-clock
runtime init, and prints one JSON document:

  python tools/node_view_ab.py --rounds 8 --json-out gpurun_out/node_view_ab.json
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import statistics
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def host_shape() -> dict:
    node = "/sys/devices/system/node"
    nodes = sorted(n for n in os.listdir(node) if n.startswith("node") and n[4:].isdigit())
    cpus = sum(1 for n in nodes for c in os.listdir(os.path.join(node, n)) if c.startswith("cpu") and c[3:].isdigit())
    return {"numa_nodes": len(nodes), "node_cpu_entries": cpus, "os_cpu_count": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0))}


def row(r, runtime: str) -> dict:
    d = r.doc
    init_ms = (d["init_us"]["hsa_init"] / 1e3 if runtime == "hsa"
               else (d["t_runtime_ns"] - d["t_start_ns"]) / 1e6)
    return {"ok": r.ok, "runtime_init_ms": round(init_ms, 2), "wall_ms": round(r.wall_ms, 2),
            "read_syscalls": d.get("read_syscalls_runtime"), "cpu_ms": d.get("cpu_ms_runtime"),
            "cpu_user_ms": d.get("cpu_user_ms_runtime"), "view": d.get("view")}


def summarize(rows) -> dict:
    out = {}
    for k in ("runtime_init_ms", "wall_ms", "read_syscalls", "cpu_ms", "cpu_user_ms"):
        xs = [r[k] for r in rows if r.get(k) is not None]
        if xs:
            out[k] = {"p50": round(statistics.median(xs), 2), "min": round(min(xs), 2), "max": round(max(xs), 2)}
    caches = [r["view"]["node_cpu_cache_opens"] for r in rows if r.get("view")]
    out["node_cpu_cache_opens_p50"] = statistics.median(caches) if caches else None
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--runtimes", default="hsa,hip")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)

    from rocm_k8s_device_plugin_amd.container_runtime import start_container, wait_kfd_released
    from rocm_k8s_device_plugin_amd.node_view import NodeView
    from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals

    inv = discover("/sys")
    ords = hip_ordinals(inv, "/dev")
    dev_id, o = sorted(ords.items(), key=lambda kv: kv[1])[0]
    paths = ["/dev/kfd"] + inv.by_id[dev_id].dev_paths()
    roots = {"tmp": tempfile.mkdtemp(prefix="nv-"), "shm": tempfile.mkdtemp(prefix="nv-", dir="/dev/shm")}
    views = {}
    for k, root in roots.items():
        nv = NodeView(root, "/sys", alias="/sys/devices/system/node")
        views[k] = (nv, [(ctr, host) for host, ctr in nv.mounts()])
    doc = {"host": host_shape(), "device": dev_id, "hidden_cache_dirs": views["tmp"][0].hidden,
           "view_symlinks": views["tmp"][0].links, "rows": {}, "summary": {}}
    try:
        for runtime in a.runtimes.split(","):
            variants = {"plain": (), "view_tmp": views["tmp"][1], "view_shm": views["shm"][1]}
            rows = {k: [] for k in variants}
            for i in range(a.rounds):
                order = list(variants) if i % 2 == 0 else list(reversed(variants))
                for k in order:
                    r = start_container([o], timeout_s=120, runtime=runtime, device_paths=paths, mounts=variants[k])
                    wait_kfd_released(r.kfd_lingering)
                    if not r.ok:
                        raise SystemExit(f"{runtime}/{k}: container failed: {r.error}")
                    rows[k].append(row(r, runtime))
                print(f"node_view_ab: {runtime} round {i + 1}/{a.rounds}", file=sys.stderr, flush=True)
            doc["rows"][runtime] = rows
            doc["summary"][runtime] = {k: summarize(v) for k, v in rows.items()}
    finally:
        for root in roots.values():
            shutil.rmtree(root, ignore_errors=True)
    out = json.dumps(doc, indent=1)
    if a.json_out:
        os.makedirs(os.path.dirname(os.path.abspath(a.json_out)), exist_ok=True)
        with open(a.json_out, "w") as f:
            f.write(out)
    print(json.dumps({"host": doc["host"], "hidden_cache_dirs": doc["hidden_cache_dirs"], "summary": doc["summary"]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
