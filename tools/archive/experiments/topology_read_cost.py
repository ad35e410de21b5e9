#!/usr/bin/env python3
"""How expensive is reading the kfd topology sysfs tree (what ROCr's thunk does at init)?"""
import json
import os
import sys
import time

root = sys.argv[1] if len(sys.argv) > 1 else "/sys/class/kfd/kfd/topology"
res = {}
for rep in range(3):
    files = errs = nbytes = 0
    per_node = {}
    t0 = time.perf_counter()
    for dp, dn, fn in os.walk(root):
        for f in fn:
            p = os.path.join(dp, f)
            try:
                with open(p, "rb") as fh:
                    nbytes += len(fh.read())
                files += 1
            except OSError:
                errs += 1
            parts = p[len(root):].split("/")
            if len(parts) > 2 and parts[1] == "nodes":
                per_node[parts[2]] = per_node.get(parts[2], 0) + 1
    dt = (time.perf_counter() - t0) * 1e3
    res[f"rep{rep}"] = {"files": files, "errors": errs, "bytes": nbytes, "ms": round(dt, 2)}
res["files_per_node"] = per_node
print(json.dumps(res, indent=1))
