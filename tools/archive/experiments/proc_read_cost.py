#!/usr/bin/env python3
"""Cost of the /proc and sysfs files a GPU runtime parses at start-up.

  python tools/archive/experiments/proc_read_cost.py --out gpurun_out/proc_read_cost.json
"""
import argparse
import glob
import json
import os
import statistics
import time


def timed_read(path, bufsize=4096, reps=5):
    ts, size, reads = [], 0, 0
    for _ in range(reps):
        t0 = time.perf_counter()
        try:
            fd = os.open(path, os.O_RDONLY)
        except OSError as e:
            return {"error": str(e)}
        size = reads = 0
        try:
            while True:
                try:
                    b = os.read(fd, bufsize)
                except OSError as e:
                    return {"error": str(e)}
                reads += 1
                if not b:
                    break
                size += len(b)
        finally:
            os.close(fd)
        ts.append((time.perf_counter() - t0) * 1e3)
    return {"ms_p50": round(statistics.median(ts), 3), "ms_min": round(min(ts), 3), "bytes": size, "reads": reads}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = {"cpu_count": os.cpu_count(), "sched_affinity": len(os.sched_getaffinity(0))}
    for p in ("/proc/cpuinfo", "/proc/self/maps", "/proc/meminfo", "/proc/stat",
              "/sys/devices/system/node/online", "/sys/devices/system/cpu/online"):
        res[p] = timed_read(p)
    # one accessible GPU node's properties and its caches, and one denied node
    nodes = sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*"), key=lambda x: int(x.rsplit("/", 1)[1]))
    per_node = {}
    for n in nodes:
        caches = glob.glob(n + "/caches/*/properties")
        t0 = time.perf_counter()
        ok = err = 0
        for c in caches:
            try:
                with open(c, "rb") as f:
                    f.read()
                ok += 1
            except OSError:
                err += 1
        per_node[os.path.basename(n)] = {"caches": len(caches), "readable": ok, "denied": err,
                                         "ms": round((time.perf_counter() - t0) * 1e3, 2),
                                         "properties": timed_read(n + "/properties", reps=3)}
    res["kfd_nodes"] = per_node
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
