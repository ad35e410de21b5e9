#!/usr/bin/env python3
"""Where does "container ready" time go? Run the container entrypoint (the
liveness probe) repeatedly under different runtime environments and report
p50 of each phase: spawn->main (exec + dynamic loading), main->HIP runtime
ready (ROCr/HIP init), runtime->ready (device setup + MFMA kernel + verify).

  python tools/container_ready_sweep.py --reps 15 --out gpurun_out/container_sweep.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rocm_k8s_device_plugin_amd.ops.native import probe_executable  # noqa: E402

VIS = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")

VARIANTS = {
    "rocr_visible": {"ROCR_VISIBLE_DEVICES": "0"},
    "hip_visible": {"HIP_VISIBLE_DEVICES": "0"},
    "no_visibility_env": {},
    "rocr_visible+hw_queues_1": {"ROCR_VISIBLE_DEVICES": "0", "GPU_MAX_HW_QUEUES": "1"},
    "rocr_visible+sdma_off": {"ROCR_VISIBLE_DEVICES": "0", "HSA_ENABLE_SDMA": "0"},
    "rocr_visible+no_interrupt": {"ROCR_VISIBLE_DEVICES": "0", "HSA_ENABLE_INTERRUPT": "0"},
    "rocr_visible+no_scratch_reclaim": {"ROCR_VISIBLE_DEVICES": "0", "HSA_NO_SCRATCH_RECLAIM": "1"},
    # ROCr start-up knobs (names from libhsa-runtime64's own getenv table)
    "rocr_visible+disable_image": {"ROCR_VISIBLE_DEVICES": "0", "HSA_DISABLE_IMAGE": "1"},
    "rocr_visible+tools_disable_register": {"ROCR_VISIBLE_DEVICES": "0", "HSA_TOOLS_DISABLE_REGISTER": "1"},
    "rocr_visible+cu_mask_skip_init": {"ROCR_VISIBLE_DEVICES": "0", "HSA_CU_MASK_SKIP_INIT": "1"},
    "rocr_visible+no_pc_sampling": {"ROCR_VISIBLE_DEVICES": "0", "HSA_DISABLE_PC_SAMPLING": "1"},
    "rocr_visible+lean": {"ROCR_VISIBLE_DEVICES": "0", "HSA_DISABLE_IMAGE": "1", "HSA_TOOLS_DISABLE_REGISTER": "1",
                          "HSA_CU_MASK_SKIP_INIT": "1", "HSA_DISABLE_PC_SAMPLING": "1"},
}
SAMPLE_ARGS: list = []
EXE_OVERRIDE: list = []   # --exe: e.g. the path-interposing measurement build
EXTRA_ENV: dict = {}      # --env K=V


def kfd_procs():
    try:
        return set(os.listdir("/sys/class/kfd/kfd/proc"))
    except OSError:
        return set()


def run_once(env_extra, args, runtime="hsa"):
    env = {k: v for k, v in os.environ.items() if k not in VIS}
    env.update(env_extra)
    env.update(EXTRA_ENV)
    argv = [EXE_OVERRIDE[0] if EXE_OVERRIDE else str(probe_executable(runtime)), "--devices", "0", "--iters", "4"] \
        + args + SAMPLE_ARGS
    t0 = time.monotonic_ns()
    p = subprocess.run(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=120)
    t1 = time.monotonic_ns()
    doc = json.loads(p.stdout.decode().strip().splitlines()[-1])
    return {
        "ok": p.returncode == 0 and doc["ok"],
        "spawn_to_main_ms": (doc["t_start_ns"] - t0) / 1e6,
        "hip_init_ms": (doc["t_runtime_ns"] - doc["t_start_ns"]) / 1e6,
        "device_ms": (doc["t_ready_ns"] - doc["t_runtime_ns"]) / 1e6,
        "ready_ms": (doc["t_ready_ns"] - t0) / 1e6,
        "exit_ms": (t1 - t0) / 1e6,
        "kernel_us": doc["devices"][0]["kernel_us"] if doc["devices"] else 0.0,
        "setup_us": doc["devices"][0].get("setup_us", 0.0) if doc["devices"] else 0.0,
        # ROCr start-up split (HSA build) and the process' CPU time up to each point
        "init_us": doc.get("init_us", {}),
        "phase_us": doc["devices"][0].get("phase_us", {}) if doc["devices"] else {},
        "cpu_ms_runtime": doc.get("cpu_ms_runtime", 0.0),
        "cpu_ms_ready": doc.get("cpu_ms_ready", 0.0),
        "cpu_user_ms_runtime": doc.get("cpu_user_ms_runtime", 0.0),
        "read_syscalls_runtime": doc.get("read_syscalls_runtime", -1),
        "init_profile": doc.get("init_profile"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="", help="comma list of variant names (default: all)")
    ap.add_argument("--sample-init", type=int, default=0,
                    help="probe samples its own threads every N us during runtime init (see init_sampler.h)")
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="idle time between runs (lets the previous process' kfd teardown finish)")
    ap.add_argument("--probe-args", default="", help="extra probe arguments, e.g. '--exit fast'")
    ap.add_argument("--wait-kfd", action="store_true",
                    help="after each run wait until its /sys/class/kfd/kfd/proc entry is gone (<= 2 s)")
    ap.add_argument("--exe", default="", help="entrypoint binary instead of the built probe")
    ap.add_argument("--env", action="append", default=[], help="K=V added to every run's environment")
    ap.add_argument("--tag", default="", help="suffix for the row names")
    ap.add_argument("--parent-gpu", action="store_true",
                    help="initialise HIP in this (parent) process first, like a torch-based harness would")
    a = ap.parse_args()
    if a.sample_init:
        SAMPLE_ARGS[:] = ["--sample-init", str(a.sample_init)]
    SAMPLE_ARGS.extend(a.probe_args.split())
    if a.exe:
        EXE_OVERRIDE.append(a.exe)
    for kv in a.env:
        k, v = kv.split("=", 1)
        EXTRA_ENV[k] = v
    if a.parent_gpu:
        import torch
        torch.cuda.synchronize() if torch.cuda.is_available() else None
        print("parent holds a HIP context:", torch.cuda.is_available(), flush=True)
    table = {}
    plan = [(f"{rt}:{name}", env, rt) for rt in ("hsa", "hip") for name, env in VARIANTS.items()]
    plan += [(f"{rt}:rocr_visible+identify_only", {"ROCR_VISIBLE_DEVICES": "0"}, rt) for rt in ("hsa", "hip")]
    if a.only:
        keep = set(a.only.split(","))
        plan = [p for p in plan if p[0] in keep]
    for name, env, rt in plan:
        extra = ["--identify"] if name.endswith("identify_only") else []
        runs = []
        for _ in range(a.reps):
            before = kfd_procs()
            runs.append(run_once(env, extra, rt))
            if a.wait_kfd:
                t = time.monotonic()
                left = kfd_procs() - before
                while left and time.monotonic() - t < 2.0:
                    time.sleep(0.002)
                    left = kfd_procs() & left
                runs[-1]["kfd_linger_ms"] = (time.monotonic() - t) * 1e3
            if a.gap_ms:
                time.sleep(a.gap_ms / 1e3)
        row = {}
        for k, v in runs[0].items():
            if k == "ok":
                continue
            if k == "init_profile":
                if v:  # pooled histogram over all runs, in ms of wall time per run
                    agg = {}
                    for r in runs:
                        for b, c in r[k]["buckets"].items():
                            agg[b] = agg.get(b, 0) + c
                    per = v["period_us"] / 1e3 / len(runs)
                    row[k] = dict(sorted(((b, round(c * per, 2)) for b, c in agg.items()), key=lambda x: -x[1]))
                continue
            if isinstance(v, dict):
                row[k] = {kk: round(statistics.median(r[k].get(kk, 0.0) for r in runs), 1) for kk in v}
            else:
                row[k] = round(statistics.median(r[k] for r in runs), 3)
        row["all_ok"] = all(r["ok"] for r in runs)
        row["ready_ms_min"] = round(min(r["ready_ms"] for r in runs), 3)
        name = name + a.tag
        table[name] = row
        print(f"{name:40s} {json.dumps(row)}", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(table, f, indent=1)


if __name__ == "__main__":
    main()
