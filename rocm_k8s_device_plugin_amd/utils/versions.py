"""Runtime/platform versions for the start-up banner and the labeller.

Reference: the device plugin prints the hwloc compile-time and runtime
versions in its usage banner (cmd/k8s-device-plugin/main.go:36-41,
internal/pkg/hwloc/hwloc.go:29-36) because hwloc is its NUMA source. Here NUMA
locality comes straight from PCI sysfs (``numa_locality``), so the banner
reports what this build actually depends on instead: the ROCm release the
native code was built against, the loaded amdgpu driver and the libraries the
GPU paths dlopen.
"""
from __future__ import annotations

import ctypes.util
import os
from typing import Dict, List, Optional


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip() or None
    except OSError:
        return None


def rocm_version(rocm_path: str = os.environ.get("ROCM_PATH", "/opt/rocm")) -> Optional[str]:
    return _read(os.path.join(rocm_path, ".info", "version"))


def amdgpu_driver_version(sysfs_root: str = "/sys") -> Optional[str]:
    # in-tree amdgpu has no module version; DKMS (amdgpu-dkms) exposes one
    return _read(os.path.join(sysfs_root, "module", "amdgpu", "version")) or (
        "in-tree" if os.path.isdir(os.path.join(sysfs_root, "module", "amdgpu")) else None)


def versions(sysfs_root: str = "/sys") -> Dict[str, Optional[str]]:
    return {
        "rocm": rocm_version(),
        "amdgpu": amdgpu_driver_version(sysfs_root),
        "libdrm_amdgpu": ctypes.util.find_library("drm_amdgpu"),
        "numa_source": "sysfs",
    }


def banner_line(sysfs_root: str = "/sys") -> str:
    v = versions(sysfs_root)
    return ", ".join(f"{k}: {v[k] or 'n/a'}" for k in ("rocm", "amdgpu", "libdrm_amdgpu", "numa_source"))


def _cpulist(text: str) -> List[int]:
    out: List[int] = []
    for part in (text or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def numa_locality(bdf: str, sysfs_root: str = "/sys") -> Dict[str, list]:
    """NUMA nodes and CPUs local to a PCI function.

    Same answer as the reference's ``Hwloc.GetNUMANodes`` (the memory children
    of the GPU's first non-I/O ancestor, hwloc.go:69-98) on Linux, where hwloc
    derives that ancestor from the device's ``numa_node`` / ``local_cpulist``.
    A device without NUMA affinity (``numa_node`` = -1) is local to every
    node, like hwloc's machine-level ancestor.
    """
    dev = os.path.join(sysfs_root, "bus", "pci", "devices", bdf)
    if not os.path.isdir(dev):
        raise FileNotFoundError(f"Fail to find GPU with bus ID: {bdf}")
    node = _read(os.path.join(dev, "numa_node"))
    cpus = _cpulist(_read(os.path.join(dev, "local_cpulist")) or "")
    if node is not None and int(node) >= 0:
        return {"numa_nodes": [int(node)], "cpus": cpus}
    nodes_dir = os.path.join(sysfs_root, "devices", "system", "node")
    try:
        nodes = sorted(int(n[4:]) for n in os.listdir(nodes_dir) if n.startswith("node") and n[4:].isdigit())
    except OSError:
        nodes = []
    return {"numa_nodes": nodes, "cpus": cpus}
