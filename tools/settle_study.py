#!/usr/bin/env python3
"""When has the previous pod's GPU process really gone? (measurement tool)

bench.py starts the next admission once the previous containers' kfd process
entries (/sys/class/kfd/kfd/proc/<pid>) are gone. Its 100-admission tail study
(profiles/r5/bench100_kfd_open_tails.json) shows that ~10 % of containers still
wait 50-220 ms inside open("/dev/kfd"). This runs containers one after another
on the GPU with different settle rules, alternating, and records for each
container the time its open("/dev/kfd") took (timed by the emulated
container's view) next to what the previous one left behind after it exited:
when its kfd entry went, and when the GPU's VRAM / GTT use returned to the
idle baseline.

  python tools/settle_study.py --rounds 60 --json-out gpurun_out/settle_study.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def read_int(path: str) -> int:
    try:
        with open(path) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return -1


def pct(xs, q):
    s = sorted(xs)
    return s[min(len(s) - 1, int(round(q * (len(s) - 1))))] if s else None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--rounds", type=int, default=60)
    ap.add_argument("--runtime", default="hip", choices=["hip", "hsa"])
    ap.add_argument("--strategies", default="proc,proc+mem,fixed500")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)

    from rocm_k8s_device_plugin_amd.container_runtime import kfd_processes, start_container
    from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals

    inv = discover("/sys")
    ords = hip_ordinals(inv, "/dev")
    dev_id, o = sorted(ords.items(), key=lambda kv: kv[1])[0]
    dev = inv.by_id[dev_id]
    paths = ["/dev/kfd"] + dev.dev_paths()
    pci = f"/sys/bus/pci/devices/{dev.bdf}"
    mem = lambda: (read_int(f"{pci}/mem_info_vram_used"), read_int(f"{pci}/mem_info_gtt_used"))  # noqa: E731
    strategies = a.strategies.split(",")
    base = mem()
    gpu_id = inv.topology.node(dev.node_id).gpu_id if dev.node_id is not None and dev.node_id >= 0 else -1

    def kfd_census():
        """kfd processes on the host, and those with a queue or VRAM on our GPU (other tenants)."""
        root = "/sys/class/kfd/kfd/proc"
        procs = sorted(kfd_processes())
        ours = []
        for pid in procs:
            q = os.path.join(root, pid, "queues")
            try:
                if any(read_int(os.path.join(q, x, "gpuid")) == gpu_id for x in os.listdir(q)):
                    ours.append(pid)
                    continue
            except OSError:
                pass
            if read_int(os.path.join(root, pid, f"vram_{gpu_id}")) > 0:
                ours.append(pid)
        return len(procs), ours
    census0 = kfd_census()
    rows = []
    prev = None
    for i in range(a.rounds + 1):
        r = start_container([o], timeout_s=120, runtime=a.runtime, device_paths=paths)
        if not r.ok:
            raise SystemExit(f"container {i} failed: {r.error}")
        t_exit = time.monotonic()
        view = r.doc.get("view") or {}
        row = {"i": i, "kfd_open_ms": round(view.get("kfd_open_us", 0.0) / 1e3, 3),
               "runtime_init_ms": round((r.doc["t_runtime_ns"] - r.doc["t_start_ns"]) / 1e6, 2),
               "after_strategy": prev}
        # what this container leaves behind: its kfd entries, the GPU's memory use
        strategy = strategies[i % len(strategies)]
        left = set(r.kfd_lingering)
        t_proc = t_mem = None
        mem_trace = []
        deadline = t_exit + 1.5
        while time.monotonic() < deadline:
            now = time.monotonic()
            if t_proc is None and not (left & kfd_processes()):
                t_proc = now
            m = mem()
            if len(mem_trace) < 400:
                mem_trace.append((round((now - t_exit) * 1e3, 1), m[0], m[1]))
            if t_mem is None and m[0] <= base[0] + (1 << 20) and m[1] <= base[1] + (1 << 20):
                t_mem = now
            done = {"proc": t_proc is not None, "proc+mem": t_proc is not None and t_mem is not None,
                    "fixed500": now - t_exit >= 0.5}[strategy]
            if done:
                break
            time.sleep(0.002)
        row.update({"strategy": strategy,
                    "proc_gone_ms": round((t_proc - t_exit) * 1e3, 1) if t_proc else None,
                    "mem_back_ms": round((t_mem - t_exit) * 1e3, 1) if t_mem else None,
                    "settle_ms": round((time.monotonic() - t_exit) * 1e3, 1),
                    "mem_trace": mem_trace[:60]})
        row["kfd_census_after"] = kfd_census()
        rows.append(row)
        prev = strategy
        print(f"settle_study: {i}/{a.rounds} kfd_open {row['kfd_open_ms']} ms after {row['after_strategy']}",
              file=sys.stderr, flush=True)
    summary = {}
    for s in strategies:
        ko = [r["kfd_open_ms"] for r in rows if r["after_strategy"] == s]
        pg = [r["proc_gone_ms"] for r in rows if r["strategy"] == s and r["proc_gone_ms"] is not None]
        mb = [r["mem_back_ms"] for r in rows if r["strategy"] == s and r["mem_back_ms"] is not None]
        summary[s] = {"next_containers": len(ko), "kfd_open_ms_p50": pct(ko, .5), "kfd_open_ms_p90": pct(ko, .9),
                      "kfd_open_ms_max": max(ko) if ko else None,
                      "waits_over_10ms": sum(1 for x in ko if x > 10),
                      "proc_gone_ms_p50": pct(pg, .5), "mem_back_ms_p50": pct(mb, .5),
                      "mem_back_ms_max": max(mb) if mb else None}
    doc = {"device": dev_id, "runtime": a.runtime, "idle_vram_gtt": base,
           "vram_total": read_int(f"{pci}/mem_info_vram_total"), "kfd_census_before": census0,
           "summary": summary, "rows": rows}
    if a.json_out:
        os.makedirs(os.path.dirname(os.path.abspath(a.json_out)), exist_ok=True)
        with open(a.json_out, "w") as f:
            json.dump(doc, f, indent=1)
    print(json.dumps({"idle_vram_gtt": base, "vram_total": doc["vram_total"], "kfd_census_before": census0,
                      "summary": summary}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
