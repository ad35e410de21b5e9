import asyncio, json, sys
sys.path.insert(0, ".")
from rocm_k8s_device_plugin_amd.health.liveness import LivenessProber
from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals
inv = discover("/sys"); o = sorted(hip_ordinals(inv, "/dev").values())[0]
p = LivenessProber(timeout_s=60); p.perf_mib, p.perf_iters = 1024, 8192
def rss():
    with open(f"/proc/{p._server.proc.pid}/status") as f:
        return [int(l.split()[1]) // 1024 for l in f if l.startswith("VmRSS")][0]
async def go():
    out = []
    for step in ("probe", "probe", "sweep", "sweep", "perf", "perf", "probe"):
        r = (await getattr(p, step)({"g": o}))["g"]
        out.append((step, r.ok, r.detail.get("kept_queue"), rss()))
    await p.close()
    return out
for row in asyncio.run(go()): print(row)
