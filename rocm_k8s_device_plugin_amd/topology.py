"""Node GPU inventory: immutable snapshots over the native discovery.

``discover()`` is the Python face of the C++ ``discover_gpus`` (reference
GetAMDGPUs, internal/pkg/amdgpu/amdgpu.go:448-568). Snapshots are frozen
dataclasses: health updates build new device lists instead of mutating shared
objects, which removes the reference's data race between UpdateHealth and
concurrent RPCs.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from .ops.native import core


@dataclass(frozen=True)
class Gpu:
    id: str
    bdf: str
    is_partition: bool
    xcp_index: int
    card: int
    render_minor: int
    unique_id: str
    compute_partition: str
    memory_partition: str
    numa_node: int
    node_id: int
    gfx_target_version: int = 0
    simd_count: int = 0
    simd_per_cu: int = 0
    num_xcc: int = 0
    pci_device_id: int = 0
    location_id: int = 0
    domain: int = 0
    hive_id: int = 0
    vram_bytes: int = 0
    # "kfd" | "sysfs" (kfd node unreadable, identity from PCI sysfs) | "" (unknown)
    identity: str = ""

    @property
    def partition_type(self) -> str:
        if not self.compute_partition or not self.memory_partition:
            return ""
        return f"{self.compute_partition}_{self.memory_partition}"

    @property
    def cu_count(self) -> int:
        return self.simd_count // self.simd_per_cu if self.simd_per_cu else 0

    @property
    def is_gfx950(self) -> bool:
        return self.gfx_target_version == 90500

    def dev_paths(self) -> List[str]:
        """/dev nodes a container needs for this device: card then renderD
        (fixed order; the reference's order depended on Go map iteration,
        SURVEY Appendix B #13)."""
        out = []
        if self.card >= 0:
            out.append(f"/dev/dri/card{self.card}")
        if self.render_minor >= 0:
            out.append(f"/dev/dri/renderD{self.render_minor}")
        return out

    @classmethod
    def from_native(cls, g) -> "Gpu":
        return cls(id=g.id, bdf=g.bdf, is_partition=g.is_partition, xcp_index=g.xcp_index, card=g.card,
                   render_minor=g.render_minor, unique_id=g.unique_id, compute_partition=g.compute_partition,
                   memory_partition=g.memory_partition, numa_node=g.numa_node, node_id=g.node_id,
                   gfx_target_version=g.gfx_target_version, simd_count=g.simd_count, simd_per_cu=g.simd_per_cu,
                   num_xcc=g.num_xcc, pci_device_id=g.pci_device_id, location_id=g.location_id, domain=g.domain,
                   hive_id=g.hive_id, vram_bytes=g.vram_bytes, identity=g.identity)


@dataclass
class Inventory:
    sysfs_root: str
    devices: Tuple[Gpu, ...]
    topology: object  # native KfdTopology
    driver_loaded: bool
    kfd_present: bool
    warnings: List[str] = field(default_factory=list)
    # kfd node dirs whose properties this process cannot read (EPERM: the device
    # cgroup denies those GPUs) and devices whose identity could not be recovered
    kfd_unreadable_nodes: Tuple[int, ...] = ()
    unresolved: Tuple[str, ...] = ()

    def __post_init__(self):
        self.by_id: Dict[str, Gpu] = {d.id: d for d in self.devices}

    def __len__(self) -> int:
        return len(self.devices)

    def partition_counts(self) -> Dict[str, int]:
        out: Dict[str, int] = {}
        for d in self.devices:
            t = d.partition_type
            if t:
                out[t] = out.get(t, 0) + 1
        return out

    @property
    def homogeneous(self) -> bool:
        return len(self.partition_counts()) <= 1

    @property
    def recovered(self) -> List[str]:
        """Devices identified from PCI sysfs because kfd denied their nodes."""
        return [d.id for d in self.devices if d.identity == "sysfs"]

    @property
    def placement_trusted(self) -> bool:
        """Every device has a known physical-GPU identity and fabric position
        (from kfd or recovered from sysfs): topology-aware placement is sound."""
        ids = set(self.by_id)
        return not any(u in ids for u in self.unresolved)

    def physical_gpus(self) -> Dict[str, List[Gpu]]:
        """unique_id -> devices (partitions) of that physical GPU, in device order."""
        out: Dict[str, List[Gpu]] = {}
        for d in self.devices:
            out.setdefault(d.unique_id, []).append(d)
        return out

    def hives(self) -> Dict[int, List[str]]:
        out: Dict[int, List[str]] = {}
        for d in self.devices:
            out.setdefault(d.hive_id, []).append(d.id)
        return out

    def compute_partition_supported(self) -> bool:
        return core().compute_partition_supported(self.sysfs_root)

    def memory_partition_supported(self) -> bool:
        return core().memory_partition_supported(self.sysfs_root)


def _limit_physical(devs: List[Gpu], limit: Optional[int]) -> List[Gpu]:
    """Keep the devices of the first `limit` physical GPUs (BDF order)."""
    if limit is None or limit < 0:
        return devs
    keep = []
    seen: List[str] = []
    for d in devs:
        if (d.unique_id or d.bdf) not in seen:
            seen.append(d.unique_id or d.bdf)
    allowed = set(seen[:limit])
    for d in devs:
        if (d.unique_id or d.bdf) in allowed:
            keep.append(d)
    return keep


def device_count_limit_from_env(env=None) -> Optional[int]:
    """AMD_GPU_DEVICE_COUNT: documented by the reference
    (docs/user-guide/configuration.md:11) but never implemented there; here it
    caps the number of advertised physical GPUs."""
    env = os.environ if env is None else env
    v = env.get("AMD_GPU_DEVICE_COUNT", "").strip()
    if not v:
        return None
    try:
        n = int(v)
    except ValueError:
        return None
    return n if n >= 0 else None


def discover(sysfs_root: str = "/sys", device_count_limit: Optional[int] = None) -> Inventory:
    n = core()
    topo = n.KfdTopology.load_sysfs(sysfs_root)
    res = n.discover_gpus_with(sysfs_root, topo)
    devs = [Gpu.from_native(g) for g in res.devices]
    devs = _limit_physical(devs, device_count_limit)
    from .models import check_inventory
    return Inventory(sysfs_root=sysfs_root, devices=tuple(devs), topology=topo, driver_loaded=res.driver_loaded,
                     kfd_present=res.kfd_present, warnings=list(res.warnings) + check_inventory(devs),
                     kfd_unreadable_nodes=tuple(res.kfd_unreadable_nodes), unresolved=tuple(res.unresolved))


def hip_ordinals(inv: Inventory, dev_root: str = "/dev", check_access: bool = True) -> Dict[str, int]:
    """kubelet device ID -> ROCr/HIP ordinal on this host (all devices visible).

    ROCr enumerates GPU agents in kfd node order and skips render nodes it
    cannot open, so the ordinal of a device is its position among accessible
    GPU nodes sorted by kfd node id. In CPX mode every partition is its own
    agent and gets its own ordinal.
    """
    gpu_nodes = []
    for nid in inv.topology.gpu_node_ids():
        node = inv.topology.node(nid)
        minor = node.drm_render_minor
        if minor <= 0:
            continue
        if check_access and os.path.isdir(os.path.join(dev_root, "dri")):
            p = os.path.join(dev_root, "dri", f"renderD{minor}")
            if not os.access(p, os.R_OK | os.W_OK):
                continue
        gpu_nodes.append(nid)
    pos = {nid: i for i, nid in enumerate(gpu_nodes)}
    return {d.id: pos[d.node_id] for d in inv.devices if d.node_id in pos}


class KfdBusyUnknown(Exception):
    """Another process' kfd queues could not be read (permissions): which GPUs
    are busy is unknown, so callers must treat every GPU as busy."""


def kfd_gpu_load(sysfs_root: str = "/sys", exclude=()) -> Dict[int, Tuple[int, int]]:
    """kfd gpu_id -> (processes with user queues on it, user queues on it),
    from every process on the host (``/sys/class/kfd/kfd/proc/<pid>/queues/<qid>/gpuid``)
    except the ``exclude``d entries (the plugin's own probe server). Raises
    KfdBusyUnknown when a process' queues are unreadable (not when it merely
    exited meanwhile)."""
    load: Dict[int, List[int]] = {}
    root = os.path.join(sysfs_root, "class/kfd/kfd/proc")
    try:
        pids = os.listdir(root)
    except FileNotFoundError:
        return {}               # no kfd process list at all: no process has queues
    except OSError as e:
        # the list itself is unreadable: every GPU may be running work
        raise KfdBusyUnknown(f"{root}: {e}") from e
    skip = set(exclude)
    for pid in pids:
        if pid in skip:
            continue
        qdir = os.path.join(root, pid, "queues")
        try:
            qids = os.listdir(qdir)
        except PermissionError as e:
            raise KfdBusyUnknown(f"{qdir}: {e}") from e
        except OSError:
            continue            # the process exited meanwhile
        mine: Dict[int, int] = {}
        for q in qids:
            try:
                with open(os.path.join(qdir, q, "gpuid")) as f:
                    g = int(f.read().strip() or 0)
            except PermissionError as e:
                raise KfdBusyUnknown(f"{qdir}/{q}: {e}") from e
            except (OSError, ValueError):
                continue
            mine[g] = mine.get(g, 0) + 1
        for g, nq in mine.items():
            cur = load.setdefault(g, [0, 0])
            cur[0] += 1
            cur[1] += nq
    return {g: (v[0], v[1]) for g, v in load.items()}


def kfd_busy_gpu_ids(sysfs_root: str = "/sys", exclude=()) -> set:
    """kfd gpu_ids that currently have user queues, from any process on the host
    except the ``exclude``d entries (the plugin's own probe server). A GPU
    without queues runs no work; the liveness loop runs its full-chip sweep
    only on those. Raises KfdBusyUnknown (see kfd_gpu_load)."""
    return set(kfd_gpu_load(sysfs_root, exclude))


def topology_signature(sysfs_root: str = "/sys") -> tuple:
    """Cheap fingerprint of the GPU topology: kfd's generation_id (bumped by the
    driver when kfd nodes come or go) and every amdgpu PCI function's current
    partition modes (~17 small reads on 8 GPUs). Used by the plugin's and the
    labeller's ``-topology_watch``."""
    def rd(path):
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            return None
    gen = rd(os.path.join(sysfs_root, "class/kfd/kfd/topology/generation_id"))
    drv = os.path.join(sysfs_root, "module/amdgpu/drivers/pci:amdgpu")
    try:
        bdfs = sorted(e for e in os.listdir(drv) if ":" in e)
    except OSError:
        bdfs = []
    parts = tuple((b, rd(os.path.join(drv, b, "current_compute_partition")),
                   rd(os.path.join(drv, b, "current_memory_partition"))) for b in bdfs)
    return gen, parts
