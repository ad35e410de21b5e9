"""RSS and kfd queues of the kept-queue probe server under the current env.

Runs by tools/archive/experiments/gpurun_queue_origin.sh once per ROCr env variant
(the prober passes its environment to the server): two probes, then the
server's VmRSS and the types of its kfd queues. One JSON line.
"""
import asyncio
import json
import os
import sys

sys.path.insert(0, ".")
from rocm_k8s_device_plugin_amd.health.liveness import LivenessProber  # noqa: E402
from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals  # noqa: E402


def status(pid):
    out = {}
    with open(f"/proc/{pid}/status") as f:
        for line in f:
            k, _, v = line.partition(":")
            if k in ("VmRSS", "RssAnon", "RssFile", "RssShmem", "VmPin"):
                out[k] = int(v.split()[0]) // 1024
    qdir = f"/sys/class/kfd/kfd/proc/{pid}/queues"
    types = []
    for q in sorted(os.listdir(qdir)) if os.path.isdir(qdir) else []:
        with open(f"{qdir}/{q}/type") as f:
            types.append(f.read().strip())
    out["kfd_queue_types"] = types
    return out


async def go(variant):
    inv = discover("/sys")
    o = sorted(hip_ordinals(inv, "/dev").values())[0]
    p = LivenessProber(timeout_s=60, keep_queues=True)
    rows = []
    try:
        for _ in range(2):
            r = (await p.probe({"g": o}))["g"]
            rows.append({"ok": r.ok, "kept_queue": r.detail.get("kept_queue")})
        st = status(p._server.proc.pid)
    finally:
        await p.close()
    return {"variant": variant, "probes": rows, "server_mb": st}


print(json.dumps(asyncio.run(go(sys.argv[1] if len(sys.argv) > 1 else "default"))))
