"""xGMI / PCIe peer-link probe.

Runs ``mi355x-liveness-probe --peer`` over a set of GPUs in a child process
(same isolation and deadline model as the liveness probe): for every ordered
pair a nonce-derived pattern is DMA-copied from one GPU's HBM to the other's
over the link between them, read back and verified word by word, and the best
copy time gives the link's achieved bandwidth. ROCr's view of the link (type,
hops, NUMA distance, nominal bandwidth) is reported next to it, so a pair that
should be one xGMI hop but is routed over PCIe, or an xGMI link running far
below its peers, is visible.

With a single GPU the device is copied to itself (same code path, no link).
"""
from __future__ import annotations

import json
import os
import statistics
import subprocess
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from ..ops.native import probe_executable
from .liveness import _VISIBILITY_VARS

LINK_TYPES = {0: "hypertransport", 1: "qpi", 2: "pcie", 3: "infiniband", 4: "xgmi"}


@dataclass
class PeerReport:
    ok: bool
    pairs: List[dict] = field(default_factory=list)
    error: str = ""
    wall_ms: float = 0.0

    def summary(self) -> Dict[str, object]:
        bw = [p["gbps_best"] for p in self.pairs if p.get("ok")]
        return {
            "ok": self.ok, "pairs": len(self.pairs), "pairs_ok": sum(bool(p.get("ok")) for p in self.pairs),
            "link_types": sorted({LINK_TYPES.get(p.get("link_type", -1), str(p.get("link_type")))
                                  for p in self.pairs if p.get("src") != p.get("dst")}),
            "gbps_min": round(min(bw), 2) if bw else None,
            "gbps_p50": round(statistics.median(bw), 2) if bw else None,
            "gbps_max": round(max(bw), 2) if bw else None,
            "bytes": self.pairs[0]["bytes"] if self.pairs else 0,
            "errors": [p["error"] for p in self.pairs if p.get("error")][:4] or ([self.error] if self.error else []),
        }


def probe_peers(ordinals: Sequence[int], nbytes: int = 64 << 20, reps: int = 3, timeout_s: float = 120.0,
                exe: Optional[str] = None) -> PeerReport:
    """Probe every ordered pair of host ROCr `ordinals` (ROCR_VISIBLE_DEVICES order)."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in _VISIBILITY_VARS}
    env["ROCR_VISIBLE_DEVICES"] = ",".join(str(o) for o in ordinals)
    local = ",".join(str(i) for i in range(len(ordinals)))
    argv = [exe or str(probe_executable("hsa")), "--peer", "--devices", local, "--peer-bytes", str(int(nbytes)),
            "--peer-reps", str(int(reps)), "--timeout", f"{max(1.0, timeout_s / 4):.1f}"]
    t0 = time.perf_counter()
    try:
        p = subprocess.run(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=timeout_s,
                           start_new_session=True)
    except subprocess.TimeoutExpired:
        return PeerReport(False, error=f"peer probe exceeded {timeout_s:.0f}s",
                          wall_ms=(time.perf_counter() - t0) * 1e3)
    wall = (time.perf_counter() - t0) * 1e3
    try:
        doc = json.loads(p.stdout.decode().strip().splitlines()[-1])
    except (ValueError, IndexError):
        return PeerReport(False, error=f"unparseable peer probe output (rc={p.returncode}): "
                                       f"{p.stderr.decode(errors='replace')[-200:]}", wall_ms=wall)
    pairs = doc.get("pairs") or []
    for q in pairs:  # local indices -> host ordinals
        q["src"] = ordinals[q["src"]] if 0 <= q.get("src", -1) < len(ordinals) else q.get("src")
        q["dst"] = ordinals[q["dst"]] if 0 <= q.get("dst", -1) < len(ordinals) else q.get("dst")
    return PeerReport(bool(doc.get("ok")) and p.returncode == 0, pairs, doc.get("error", ""), wall)
