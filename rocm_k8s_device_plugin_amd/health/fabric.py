"""xGMI link state as a placement input (``-smi_xgmi``).

No reference counterpart: the reference weighs GPU pairs by the kfd io_link
type it reads once (internal/pkg/allocator/device.go:135-157), so a pair
whose xGMI link has failed keeps scoring as xGMI-connected and multi-GPU pods
keep landing on it. kfd's topology does not change when a link goes down;
amd-smi reports the live state (``amdsmi_get_gpu_xgmi_link_status``: up /
down / disabled per link) and which peer each link reaches
(``amdsmi_get_link_metrics``: destination BDF, link type).

A link that is *up* in the first reading and later *down* is a degraded
link. Measured on an 8x MI355X node: 8 link slots per GPU, 7 up (one to each
peer) and 1 disabled by design, so "disabled" is never counted as a failure
and the baseline is whatever the plugin saw first. Links go down without the
peer being named in every firmware, so:

* a peer listed by the link metrics at baseline that is gone from the list
  (or whose link reports a zero bit rate) degrades exactly that GPU pair;
* if the count of up links dropped but no peer can be named, every xGMI pair
  of that GPU is degraded.

The devices stay Healthy (a single-GPU pod does not care): the allocator is
re-initialised with the degraded pairs scoring as the worst link, so
GetPreferredAllocation stops packing multi-GPU pods across them, and they
are exported as ``mi355x_dp_xgmi_links_down``.
"""
from __future__ import annotations

from typing import Callable, Dict, FrozenSet, Optional, Set, Tuple

from ..allocator import group_key
from ..topology import Inventory
from ..utils import log

_log = log.get("health")

LINK_DOWN, LINK_UP, LINK_DISABLED = 0, 1, 2
LINK_TYPE_XGMI = 2

Pair = Tuple[str, str]


def _pair(a: str, b: str) -> Pair:
    return (a, b) if a <= b else (b, a)


class FabricWatcher:
    def __init__(self, inventory: Inventory, source: Optional[Callable[[], dict]] = None):
        self.inv = inventory
        self._source = source
        # physical GPU (allocator group key) by the BDF amd-smi reports for it
        self._gpu_by_bdf: Dict[str, str] = {}
        for d in inventory.devices:
            self._gpu_by_bdf.setdefault(d.bdf.lower(), group_key(d))
        self._baseline: Dict[str, dict] = {}     # bdf -> {"up": n, "peers": {peer_bdf}}
        self.degraded: FrozenSet[Pair] = frozenset()
        self.links_down: Dict[str, int] = {}     # bdf -> links down vs baseline
        self.version = 0
        self.error = ""
        self.readings = 0

    @property
    def reads_amd_smi(self) -> bool:
        return self._source is None

    def _read(self) -> dict:
        if self._source is not None:
            return self._source()
        from ..ops.native import core
        return core().smi_xgmi_links()

    def check(self) -> bool:
        """One reading; True if the set of degraded GPU pairs changed."""
        try:
            snap = self._read()
        except Exception as e:  # never fail a health sweep over amd-smi
            snap = {"ok": False, "error": str(e), "gpus": []}
        if not snap.get("ok"):
            if snap.get("error") != self.error:
                _log.warning("xGMI link state unavailable: %s", snap.get("error"))
            self.error = snap.get("error", "")
            return False
        self.error = ""
        self.readings += 1
        degraded: Set[Pair] = set()
        down: Dict[str, int] = {}
        for g in snap.get("gpus", []):
            bdf = g.get("bdf", "").lower()
            me = self._gpu_by_bdf.get(bdf)
            if me is None:
                continue            # a GPU this plugin does not advertise
            status = list(g.get("status") or []) if g.get("status_ok") else None
            up = sum(1 for s in status if s == LINK_UP) if status is not None else None
            peers = {p["peer_bdf"].lower(): p for p in (g.get("peers") or []) if g.get("metrics_ok")
                     and p.get("link_type") == LINK_TYPE_XGMI and p["peer_bdf"].lower() in self._gpu_by_bdf}
            live = {b for b, p in peers.items() if int(p.get("bit_rate_gbps", 1)) > 0}
            base = self._baseline.get(bdf)
            if base is None:
                self._baseline[bdf] = {"up": up, "peers": set(live)}
                continue
            lost_peers = base["peers"] - live
            lost_links = (base["up"] - up) if (base["up"] is not None and up is not None) else 0
            if lost_peers:
                for pb in lost_peers:
                    degraded.add(_pair(me, self._gpu_by_bdf[pb]))
            elif lost_links > 0:
                for pb in base["peers"] or set(self._gpu_by_bdf) - {bdf}:
                    other = self._gpu_by_bdf.get(pb)
                    if other is not None and other != me:
                        degraded.add(_pair(me, other))
            if lost_links > 0 or lost_peers:
                down[bdf] = max(lost_links, len(lost_peers))
        self.links_down = down
        new = frozenset(degraded)
        if new == self.degraded:
            return False
        added, cleared = new - self.degraded, self.degraded - new
        for a, b in sorted(added):
            _log.warning("xGMI link between GPUs %s and %s is down: multi-GPU placement avoids the pair", a, b)
        for a, b in sorted(cleared):
            _log.warning("xGMI link between GPUs %s and %s is back up", a, b)
        self.degraded = new
        self.version += 1
        from ..utils.metrics import REGISTRY
        REGISTRY.set("mi355x_dp_xgmi_links_down", float(sum(down.values())),
                     help="xGMI links down vs the first reading")
        return True
