#!/usr/bin/env python3
"""Build the -node_view and -topology_view directories for this host and print
the MI355X_INITPROF_REDIRECT specs that make native/tools/rocr_initprof.cpp
see them where the container would (in-process stand-in for the bind mounts).

  python tools/archive/experiments/view_emulation.py OUTDIR   -> JSON {"node": spec, "topology": spec, "both": spec, ...}
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from rocm_k8s_device_plugin_amd.node_view import build_node_view  # noqa: E402
from rocm_k8s_device_plugin_amd.topology_view import build_view  # noqa: E402

KFD = "/sys/devices/virtual/kfd/kfd/topology"


def accessible_gpu_nodes(root=KFD):
    out = []
    for n in sorted(os.listdir(os.path.join(root, "nodes")), key=int):
        try:
            with open(os.path.join(root, "nodes", n, "properties")) as f:
                props = f.read()
        except OSError:
            continue
        kv = dict(l.split(None, 1) for l in props.splitlines() if len(l.split(None, 1)) == 2)
        if kv.get("simd_count", "0").strip() != "0":
            out.append(int(n))
    return out


def main():
    out = os.path.abspath(sys.argv[1])
    os.makedirs(out, exist_ok=True)
    links, hidden = build_node_view("/sys/devices/system/node", os.path.join(out, "node"),
                                    alias="/sys/devices/system/node")
    keep = accessible_gpu_nodes()
    remap = build_view(KFD, os.path.join(out, "topology"), keep)
    node = f"/sys/devices/system/node={out}/node"
    topo = f"{KFD}={out}/topology"
    print(json.dumps({"node": node, "topology": topo, "both": node + ";" + topo, "node_links": links,
                      "node_hidden_cache_dirs": hidden, "kept_gpu_nodes": keep, "remap": remap}))


if __name__ == "__main__":
    main()
