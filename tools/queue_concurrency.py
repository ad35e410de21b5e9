#!/usr/bin/env python3
"""T kfd queue creations: T threads of one process vs T processes (1 GPU box).

The per-GPU set-up of a pod-mode container with N GPUs is 2 queue creations
per GPU; whether those serialise inside one process (the process' mmap lock
taken by AMDKFD_IOC_SVM, kfd's per-process mutex in CREATE_QUEUE) decides how
the headline grows with N. On one GPU, T queues on GPU 0 exercise the same
locks. Builds native/tools/queue_concurrency.cpp with g++ first.

  python tools/queue_concurrency.py --out gpurun_out/queue_concurrency.json
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "gpurun_out", "queue_concurrency")


def build():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-I/opt/rocm/include",
                    os.path.join(REPO, "native/tools/queue_concurrency.cpp"), "-o", EXE, "-ldl", "-pthread"],
                   check=True)


def threads_mode(t):
    p = subprocess.run([EXE, "--threads", str(t)], stdout=subprocess.PIPE, timeout=60, check=True)
    d = json.loads(p.stdout.decode().strip().splitlines()[-1])
    assert d["ok"], d
    return d["wall_ms"], d["sum_ms"] / t


def procs_mode(t):
    barrier = time.monotonic_ns() + int(2.5e9)
    ps = [subprocess.Popen([EXE, "--threads", "1", "--barrier-ns", str(barrier)], stdout=subprocess.PIPE)
          for _ in range(t)]
    docs = []
    for p in ps:
        out, _ = p.communicate(timeout=60)
        d = json.loads(out.decode().strip().splitlines()[-1])
        assert d["ok"], d
        docs.append(d)
    start = min(d["start_ns"] for d in docs)
    end = max(d["end_ns"] for d in docs)
    return (end - start) / 1e6, statistics.mean(d["sum_ms"] for d in docs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--counts", default="1,2,4,8")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    build()
    rows = []
    for t in [int(x) for x in a.counts.split(",")]:
        for mode, fn in (("threads", threads_mode), ("processes", procs_mode)):
            walls, per = [], []
            for _ in range(a.reps):
                w, q = fn(t)
                walls.append(w)
                per.append(q)
                time.sleep(0.2 + 0.2 * t)   # past the kfd teardown of what just exited
            row = {"queues": t, "mode": mode, "wall_ms_p50": round(statistics.median(walls), 2),
                   "per_queue_ms_p50": round(statistics.median(per), 2)}
            rows.append(row)
            print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
