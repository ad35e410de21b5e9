"""xGMI fabric model of an allocated device set.

The plugin's placement rule (GetPreferredAllocation, ``allocator.py``) keeps a
pod's GPUs in one xGMI hive so that the workload's RCCL collectives never
leave the fabric. This module says, for a concrete set of kubelet device IDs,
what fabric the pod got: which pairs are on the same package, which are
direct xGMI links and which fall back to PCIe, and the bandwidth bound that
implies for a ring all-reduce. ``bench.py`` prints it next to the RCCL
bus bandwidth it measures on the same GPUs (``parallel/collectives.py``).

Ring bound. xGMI is point-to-point: on a fully connected hive of k whole
GPUs, RCCL can run k-1 directed rings at once, each using one outgoing link
per GPU, so every GPU's k-1 links to the others carry traffic and the bus
bandwidth of an all-reduce is bounded by one GPU's egress over those links:
``min_i sum_{j != i} bw(i, j)``. A set that needs a PCIe hop between two GPUs
is bounded by that hop instead. Partitions of one GPU share its links, so the
bound is computed over physical GPUs.

The reference has no equivalent: its pair weights only rank candidate sets
(internal/pkg/allocator/device.go:135-157) and ignore link bandwidth and hive
ids.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from ..models import model_for

LINK_XGMI = 11
LINK_PCIE = 2


@dataclass
class FabricReport:
    devices: List[str]
    physical_gpus: int
    one_hive: bool
    pairs: Dict[str, int] = field(default_factory=dict)   # same_gpu / xgmi / pcie / unknown
    min_xgmi_degree: int = 0          # fewest direct xGMI peers (other GPUs of the set) of any GPU
    egress_mbps_min: int = 0          # min over GPUs of the summed link bandwidth to the others
    allreduce_bound_gbs: Optional[float] = None
    note: str = ""

    def as_dict(self) -> dict:
        return {"devices": self.devices, "physical_gpus": self.physical_gpus, "one_hive": self.one_hive,
                "pairs": dict(self.pairs), "min_xgmi_degree": self.min_xgmi_degree,
                "egress_mbps_min": self.egress_mbps_min,
                "allreduce_bound_gbs": None if self.allreduce_bound_gbs is None else round(self.allreduce_bound_gbs, 1),
                "note": self.note}


class Fabric:
    """Link graph between the kfd GPU nodes of one node's inventory."""

    def __init__(self, inventory):
        self.inv = inventory
        # (from_node, to_node) -> (type, max_bandwidth MB/s); io_links win over p2p_links
        self.links: Dict[Tuple[int, int], Tuple[int, int]] = {}
        topo = inventory.topology
        for nid in topo.gpu_node_ids():
            node = topo.node(nid)
            if node is None:
                continue
            for l in list(node.p2p_links) + list(node.io_links):
                self.links[(l["node_from"], l["node_to"])] = (l["type"], int(l["max_bandwidth"]))

    def link(self, a, b) -> Tuple[str, int]:
        """Class and bandwidth (MB/s, 0 = unknown) between two devices."""
        if a.unique_id and a.unique_id == b.unique_id:
            return "same_gpu", 0
        t = self.links.get((a.node_id, b.node_id)) or self.links.get((b.node_id, a.node_id))
        if t is None:
            return "unknown", 0
        typ, bw = t
        if typ == LINK_XGMI:
            if bw <= 0:
                m = model_for(a.pci_device_id, a.gfx_target_version)
                bw = m.xgmi_link_mbps if m else 0
            return "xgmi", bw
        if typ == LINK_PCIE:
            return "pcie", bw
        return "unknown", bw

    def report(self, device_ids: Sequence[str]) -> FabricReport:
        devs = [self.inv.by_id[i] for i in device_ids if i in self.inv.by_id]
        gpus: Dict[str, object] = {}
        for d in devs:
            gpus.setdefault(d.unique_id or d.bdf, d)   # one representative partition per physical GPU
        hives = {d.hive_id for d in devs}
        rep = FabricReport(devices=[d.id for d in devs], physical_gpus=len(gpus),
                           one_hive=len(hives) == 1 and 0 not in hives)
        pairs = {"same_gpu": 0, "xgmi": 0, "pcie": 0, "unknown": 0}
        for i, a in enumerate(devs):
            for b in devs[i + 1:]:
                pairs[self.link(a, b)[0]] += 1
        rep.pairs = pairs
        reps = list(gpus.values())
        if len(reps) <= 1:
            rep.note = "single GPU: collectives stay on the package"
            return rep
        degrees, egress, slow_hops = [], [], []
        for a in reps:
            deg = eg = 0
            for b in reps:
                if b is a:
                    continue
                cls, bw = self.link(a, b)
                if cls == "xgmi":
                    deg += 1
                    eg += bw
                else:
                    slow_hops.append((cls, bw))
            degrees.append(deg)
            egress.append(eg)
        rep.min_xgmi_degree = min(degrees)
        rep.egress_mbps_min = min(egress)
        if not slow_hops and rep.egress_mbps_min > 0:
            rep.allreduce_bound_gbs = rep.egress_mbps_min / 1000.0
            rep.note = f"all {len(reps)} GPUs directly xGMI-connected: {len(reps) - 1} concurrent ring(s)"
        elif any(cls == "unknown" for cls, _ in slow_hops):
            rep.note = (f"{sum(cls == 'unknown' for cls, _ in slow_hops) // 2} GPU pairs with no kfd link "
                        "(node properties not readable here): no bound")
        elif slow_hops:
            bws = [bw for _, bw in slow_hops if bw > 0]
            rep.allreduce_bound_gbs = (min(bws) / 1000.0) if bws else None
            rep.note = f"{len(slow_hops) // 2} GPU pairs without a direct xGMI link: a ring crosses PCIe"
        return rep
