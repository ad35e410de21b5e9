"""Hardware models of the AMD Instinct parts the plugin can meet on a node.

The reference has no notion of a GPU model: it reads whatever sysfs says and
trusts it (internal/pkg/amdgpu/amdgpu.go:448-568). Here a small registry,
keyed by the kfd/PCI device id, says what a *consistent* node of that part
looks like — XCDs, CUs, HBM, xGMI links, partition modes — so that

* discovery can flag a node whose partitions do not add up (a half-applied
  partition switch, stale ``amdgpu_xcp_*`` platform devices: both seen on real
  MI355X hosts, profiles/archive/measurements_r1_r3.md §5) instead of advertising it silently
  (``check_inventory``);
* the fabric model (``parallel/fabric.py``) has a per-link bandwidth when the
  kfd io_links do not report one;
* the fixture generator (``testing/fixtures.py``) writes MI355X trees from the
  same numbers the checks use.

Every entry says where its numbers come from: ``measured`` = read on a real
MI355X gpurun box (profiles/archive/real_sysfs_inventory_box.json,
amdsmi_snapshot_box.json, drm_info_box.json); ``reference-fixture`` = the
captured sysfs trees under /root/reference/testdata;
``spec`` = vendor specification, not verified here.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

# partitions per GPU for each compute mode; CPX = one per XCD (filled per model)
_FIXED_PARTS = {"spx": 1, "dpx": 2, "qpx": 4}


@dataclass(frozen=True)
class GpuModel:
    name: str
    device_ids: Tuple[int, ...]             # PF device ids (kfd `device_id`, PCI `device`)
    gfx: str                                # LLVM target
    gfx_target_version: int                 # kfd `gfx_target_version`
    xcds: int                               # accelerator complex dies (XCCs) per GPU
    cus: int                                # compute units per GPU (all XCDs)
    vram_bytes: int                         # HBM per GPU
    hbm: str
    family: str                             # libdrm family name (labeller `family`)
    xgmi_links: int                         # xGMI links per GPU
    xgmi_link_mbps: int                     # per link, one direction, MB/s (kfd io_link units)
    compute_partitions: Tuple[str, ...]     # lower-case, as in resource names
    memory_partitions: Tuple[str, ...]
    vf_device_ids: Tuple[int, ...] = ()
    source: Dict[str, str] = field(default_factory=dict, compare=False, hash=False)

    def partitions_per_gpu(self, compute_partition: str) -> Optional[int]:
        """Logical devices one physical GPU splits into in this compute mode."""
        cp = compute_partition.lower()
        if cp not in self.compute_partitions:
            return None
        if cp == "cpx":
            return self.xcds
        return _FIXED_PARTS.get(cp)

    def cus_per_partition(self, compute_partition: str) -> Optional[int]:
        n = self.partitions_per_gpu(compute_partition)
        return self.cus // n if n else None

    def supports(self, compute_partition: str, memory_partition: str = "") -> bool:
        if compute_partition and compute_partition.lower() not in self.compute_partitions:
            return False
        if memory_partition and memory_partition.lower() not in self.memory_partitions:
            return False
        return True


MI355X = GpuModel(
    name="AMD Instinct MI355X", device_ids=(0x75A3,), vf_device_ids=(0x75B3,), gfx="gfx950",
    gfx_target_version=90500, xcds=8, cus=256, vram_bytes=288 * 1024 ** 3, hbm="HBM3E", family="AI",
    xgmi_links=7, xgmi_link_mbps=76000,
    compute_partitions=("spx", "dpx", "qpx", "cpx"), memory_partitions=("nps1", "nps2"),
    source={"device_ids": "measured (asic id 0x75a3)", "cus": "measured (256)",
            "vram_bytes": "measured (294,896 MiB)", "family": "measured (libdrm family 141 = AI)",
            "compute_partitions": "measured (available_compute_partition)",
            "gfx_target_version": "measured (90500)",
            "xgmi_link_mbps": "measured (kfd io_link max_bandwidth 76000 MB/s, type 11, weight 15; 7 per GPU)",
            "vf_device_ids": "assumed, unverified", "memory_partitions": "spec"},
)

MI300X = GpuModel(
    name="AMD Instinct MI300X", device_ids=(0x74A1,), gfx="gfx942", gfx_target_version=90402, xcds=8, cus=304,
    vram_bytes=192 * 1024 ** 3, hbm="HBM3", family="AI", xgmi_links=7, xgmi_link_mbps=64000,
    compute_partitions=("spx", "dpx", "qpx", "cpx"), memory_partitions=("nps1", "nps4"),
    source={"device_ids": "reference-fixture (testdata/topo-mi300-cpx)", "xcds": "reference-fixture (8 partitions)",
            "gfx_target_version": "reference-fixture (90402)", "cus": "spec", "vram_bytes": "spec",
            "xgmi_link_mbps": "spec"},
)

MI308X = GpuModel(
    name="AMD Instinct MI308X", device_ids=(0x74A2,), gfx="gfx942", gfx_target_version=90402, xcds=4, cus=80,
    vram_bytes=192 * 1024 ** 3, hbm="HBM3", family="AI", xgmi_links=7, xgmi_link_mbps=64000,
    compute_partitions=("spx", "cpx"), memory_partitions=("nps1",),
    source={"device_ids": "reference-fixture (testdata/topology-parsing-mi308)",
            "xcds": "reference-fixture (4 partitions per GPU in CPX)", "gfx_target_version": "reference-fixture",
            "cus": "spec", "vram_bytes": "spec"},
)

MI210 = GpuModel(
    name="AMD Instinct MI210", device_ids=(0x740F,), gfx="gfx90a", gfx_target_version=90010, xcds=1, cus=104,
    vram_bytes=64 * 1024 ** 3, hbm="HBM2e", family="AI", xgmi_links=3, xgmi_link_mbps=50000,
    compute_partitions=(), memory_partitions=(),
    source={"device_ids": "reference-fixture (testdata/topo-mi210-xgmi-pcie)",
            "gfx_target_version": "reference-fixture (90010)", "cus": "spec", "vram_bytes": "spec"},
)

REGISTRY: Tuple[GpuModel, ...] = (MI355X, MI300X, MI308X, MI210)
_BY_ID: Dict[int, GpuModel] = {i: m for m in REGISTRY for i in m.device_ids + m.vf_device_ids}
_BY_GFX: Dict[int, GpuModel] = {}
for _m in REGISTRY:
    _BY_GFX.setdefault(_m.gfx_target_version, _m)


def model_for(device_id: int = 0, gfx_target_version: int = 0) -> Optional[GpuModel]:
    """The model of a device: by PCI/kfd device id, else by gfx target (first
    registered part of that target), else None."""
    if device_id and device_id in _BY_ID:
        return _BY_ID[device_id]
    if gfx_target_version and gfx_target_version in _BY_GFX:
        return _BY_GFX[gfx_target_version]
    return None


def check_inventory(devices: Sequence) -> List[str]:
    """Consistency of discovered devices against their models.

    ``devices`` are ``topology.Gpu`` snapshots. Per physical GPU (kfd
    ``unique_id``, else BDF): all partitions share one mode, the number of
    partitions matches the mode, and each partition's CU count is the model's
    share. Devices without kfd data (gfx_target_version 0: EPERM'd nodes in a
    restricted container) and unknown parts are skipped. Returns warnings;
    empty means consistent.
    """
    groups: Dict[str, list] = {}
    for d in devices:
        groups.setdefault(d.unique_id or d.bdf, []).append(d)
    out: List[str] = []
    for key, parts in groups.items():
        first = parts[0]
        if not first.gfx_target_version:
            continue
        m = model_for(first.pci_device_id, first.gfx_target_version)
        if m is None:
            continue
        modes = sorted({p.compute_partition for p in parts if p.compute_partition})
        if len(modes) > 1:
            out.append(f"{first.bdf}: partitions in different compute modes {modes}")
            continue
        if not modes:
            continue
        mode = modes[0]
        if not m.supports(mode):
            out.append(f"{first.bdf}: {m.name} does not support compute partition {mode!r}")
            continue
        want = m.partitions_per_gpu(mode)
        if want and len(parts) != want:
            out.append(f"{first.bdf}: {len(parts)} {mode} partitions discovered, {m.name} has {want}")
        want_cu = m.cus_per_partition(mode)
        for p in parts:
            if want_cu and p.cu_count and p.cu_count != want_cu:
                out.append(f"{p.id}: {p.cu_count} CUs, {m.name} {mode} partitions have {want_cu}")
    return out
