"""-node_view applied with real bind mounts (CPU; needs root for a private mount
namespace — skipped otherwise).

The GPU box cannot bind-mount (no root, no user namespaces), so the view's
effect on ROCr is measured there with the mounts emulated by path
redirection (profiles/archive/measurements_r1_r3.md §3e). What a container runtime does with the
Allocate mounts — bind the real node directory at the alias, then the view
over /sys/devices/system/node, both read-only and in that order — is done here
for real on this host's sysfs, and generic consumers are checked inside the
namespace: the node files read the live values, each node's CPUs keep every
entry but `cache`, /sys/devices/system/cpu still has its caches, lscpu works.
"""
import json
import os
import shutil
import subprocess
import sys

import pytest

from rocm_k8s_device_plugin_amd.node_view import NODE_ALIAS, NODE_CONTAINER_PATH, NodeView

CHECK = r'''
import glob, json, os
node = "/sys/devices/system/node"
out = {}
nodes = sorted(glob.glob(node + "/node[0-9]*"))
out["nodes"] = len(nodes)
out["meminfo"] = open(nodes[0] + "/meminfo").read().split("\n")[0]
out["cpulist"] = open(nodes[0] + "/cpulist").read().strip()
cpus = sorted(glob.glob(nodes[0] + "/cpu[0-9]*"))
out["cpus"] = len(cpus)
out["cache_under_node"] = sum(os.path.exists(c + "/cache") for c in cpus)
out["topology_under_node"] = sum(os.path.exists(c + "/topology/core_id") for c in cpus)
out["cache_under_cpu"] = os.path.isdir("/sys/devices/system/cpu/cpu0/cache")
# the files ROCr's thunk reads per CPU through the node directories (bounded
# glob: sysfs symlinks form cycles, so no recursive walk)
out["cache_files_via_node"] = len(glob.glob(node + "/node[0-9]*/cpu[0-9]*/cache/index[0-9]*/*"))
print(json.dumps(out))
'''


def _can_unshare() -> bool:
    if os.geteuid() != 0 or not shutil.which("unshare") or not shutil.which("mount"):
        return False
    r = subprocess.run(["unshare", "-m", "--propagation", "private", "true"], capture_output=True)
    return r.returncode == 0


@pytest.mark.skipif(not _can_unshare(), reason="needs root and mount namespaces")
def test_node_view_with_real_bind_mounts(tmp_path):
    if not os.path.isdir("/sys/devices/system/node/node0"):
        pytest.skip("no NUMA node directory in this sysfs")
    nv = NodeView(str(tmp_path / "nv"), "/sys")
    mounts = nv.mounts()
    assert mounts[0] == ("/sys/devices/system/node", NODE_ALIAS) and mounts[-1][1] == NODE_CONTAINER_PATH
    script = ["set -e"]
    for host, ctr in mounts:               # what the runtime does, in the Allocate order
        script += [f"mkdir -p {ctr}", f"mount --bind {host} {ctr}", f"mount -o remount,bind,ro {ctr}"]
    check = tmp_path / "check.py"
    check.write_text(CHECK)
    script += [f"{sys.executable} {check}", "lscpu > /dev/null", "echo LSCPU_OK"]
    before = subprocess.run([sys.executable, str(check)], capture_output=True, text=True, check=True, timeout=60)
    r = subprocess.run(["unshare", "-m", "--propagation", "private", "sh", "-c", "\n".join(script)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert lines[-1] == "LSCPU_OK"
    host, inside = json.loads(before.stdout), json.loads(lines[-2])
    # live node data unchanged, same CPUs, same per-CPU topology entries
    for k in ("nodes", "meminfo", "cpulist", "cpus", "topology_under_node"):
        assert inside[k] == host[k], (k, inside[k], host[k])
    # only the cache walk is gone, and only through the node directories
    assert host["cache_under_node"] == host["cpus"] and host["cache_files_via_node"] > 0
    assert inside["cache_under_node"] == 0 and inside["cache_files_via_node"] == 0
    assert inside["cache_under_cpu"]
    # the host's own view is untouched (private mount namespace)
    assert os.path.isdir("/sys/devices/system/node/node0/cpu0/cache") or host["cpus"] == 0
