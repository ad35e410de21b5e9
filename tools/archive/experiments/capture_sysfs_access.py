"""Capture which GPU identity sources a process can read when the device
cgroup denies most GPUs (gpurun box, non-privileged plugin pod).

For every amdgpu PCI function: unique_id, xgmi_hive_info/xgmi_hive_id,
xgmi_device_id / xgmi_physical_id, partition files, drm minors; for every
amdgpu_xcp_* platform device: its drm minors and directory entries; for every
kfd node: which files are readable and the errno of those that are not.
Writes JSON to --out (default stdout).
"""
from __future__ import annotations

import argparse
import errno
import json
import os


def rd(path):
    try:
        with open(path) as f:
            return {"ok": True, "value": f.read().strip()[:400]}
    except OSError as e:
        return {"ok": False, "errno": errno.errorcode.get(e.errno, str(e.errno))}


def ls(path):
    try:
        return sorted(os.listdir(path))
    except OSError as e:
        return {"errno": errno.errorcode.get(e.errno, str(e.errno))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sysfs", default="/sys")
    ap.add_argument("--out")
    a = ap.parse_args()
    s = a.sysfs
    out = {"pci": {}, "xcp": {}, "kfd_nodes": {}, "class_drm": {}}
    drv = os.path.join(s, "module/amdgpu/drivers/pci:amdgpu")
    for bdf in ls(drv) if isinstance(ls(drv), list) else []:
        if ":" not in bdf:
            continue
        d = os.path.join(drv, bdf)
        ent = {"entries": ls(d), "realpath": os.path.realpath(d)}
        for f in ("unique_id", "xgmi_hive_info/xgmi_hive_id", "xgmi_device_id", "xgmi_physical_id",
                  "current_compute_partition", "current_memory_partition", "available_compute_partition",
                  "numa_node", "device", "serial_number", "product_name", "compute_partition_config/xcp_config",
                  "mem_info_vram_total"):
            ent[f] = rd(os.path.join(d, f))
        ent["xgmi_hive_info"] = ls(os.path.join(d, "xgmi_hive_info"))
        ent["drm"] = ls(os.path.join(d, "drm"))
        ent["compute_partition_config"] = ls(os.path.join(d, "compute_partition_config"))
        out["pci"][bdf] = ent
    plat = os.path.join(s, "devices/platform")
    for name in sorted(x for x in (ls(plat) if isinstance(ls(plat), list) else []) if x.startswith("amdgpu_xcp_")):
        p = os.path.join(plat, name)
        out["xcp"][name] = {"entries": ls(p), "drm": ls(os.path.join(p, "drm")),
                            "uevent": rd(os.path.join(p, "uevent")),
                            "modalias": rd(os.path.join(p, "modalias"))}
    cd = os.path.join(s, "class/drm")
    for name in ls(cd) if isinstance(ls(cd), list) else []:
        out["class_drm"][name] = os.path.realpath(os.path.join(cd, name))
    nodes = os.path.join(s, "class/kfd/kfd/topology/nodes")
    for n in ls(nodes) if isinstance(ls(nodes), list) else []:
        nd = os.path.join(nodes, n)
        ent = {}
        for f in ("properties", "name", "gpu_id", "io_links/0/properties", "p2p_links/0/properties",
                  "mem_banks/0/properties", "caches"):
            r = rd(os.path.join(nd, f)) if f != "caches" else {"ok": True, "value": ls(os.path.join(nd, f))}
            if f == "properties" and r.get("ok"):
                kv = dict(line.split(" ", 1) for line in r["value"].splitlines() if " " in line)
                r = {"ok": True, "value": {k: kv.get(k) for k in ("drm_render_minor", "unique_id", "location_id",
                                                                 "hive_id", "num_xcc", "gfx_target_version")}}
            ent[f] = r
        ent["io_links"] = ls(os.path.join(nd, "io_links"))
        out["kfd_nodes"][n] = ent
    js = json.dumps(out, indent=1, sort_keys=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    else:
        print(js)


if __name__ == "__main__":
    main()
