#!/usr/bin/env python3
"""Does a filtered kfd topology view (bind-mounted the way a pod would get it
from the plugin's Allocate mounts) speed up ROCr start-up? Uses an unprivileged
user+mount namespace (unshare -Urm) to emulate the container mount."""
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rocm_k8s_device_plugin_amd.ops.native import probe_executable  # noqa: E402
from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals  # noqa: E402
from rocm_k8s_device_plugin_amd.topology_view import KFD_TOPOLOGY_CONTAINER_PATH, build_view  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
out = {}
if not shutil.which("unshare"):
    print(json.dumps({"error": "no unshare"}))
    sys.exit(0)
r = subprocess.run(["unshare", "-Urm", "true"], capture_output=True)
out["unshare_ok"] = r.returncode == 0
out["unshare_err"] = r.stderr.decode()[-300:]
inv = discover("/sys")
ords = hip_ordinals(inv, "/dev")
dev = inv.by_id[next(iter(ords))]
view = tempfile.mkdtemp(prefix="topoview-")
t0 = time.perf_counter()
remap = build_view("/sys/devices/virtual/kfd/kfd/topology", view, [dev.node_id])
out["build_view_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
out["remap"] = remap
out["view_files"] = sum(len(f) for _, _, f in os.walk(view))
exe = str(probe_executable("hsa"))


def run(mode):
    env = {k: v for k, v in os.environ.items() if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES")}
    if mode == "plain":
        argv = [exe, "--devices", "0"]
    elif mode == "ns_only":
        argv = ["unshare", "-Urm", exe, "--devices", "0"]
    else:
        argv = ["unshare", "-Urm", "sh", "-c",
                f"mount --bind {view} {KFD_TOPOLOGY_CONTAINER_PATH} && exec {exe} --devices 0"]
    t0 = time.monotonic_ns()
    p = subprocess.run(argv, capture_output=True, env=env, timeout=120)
    try:
        doc = json.loads(p.stdout.decode().strip().splitlines()[-1])
    except Exception:
        return {"ok": False, "err": (p.stderr.decode() + p.stdout.decode())[-400:]}
    return {"ok": doc["ok"], "ready_ms": (doc["t_ready_ns"] - t0) / 1e6,
            "init_ms": (doc["t_runtime_ns"] - doc["t_start_ns"]) / 1e6,
            "err": "" if doc["ok"] else json.dumps(doc)[-400:]}


if out["unshare_ok"]:
    for mode in ("plain", "ns_only", "view", "plain", "ns_only", "view"):
        rs = [run(mode) for _ in range(reps)]
        ok = [x for x in rs if x["ok"]]
        key = mode if mode not in out else mode + "_2"
        out[key] = {"ok": f"{len(ok)}/{reps}",
                    "init_ms_p50": round(statistics.median(x["init_ms"] for x in ok), 2) if ok else None,
                    "ready_ms_p50": round(statistics.median(x["ready_ms"] for x in ok), 2) if ok else None,
                    "ready_ms_min": round(min(x["ready_ms"] for x in ok), 2) if ok else None,
                    "first_err": next((x["err"] for x in rs if not x["ok"]), "")}
print(json.dumps(out, indent=1))
