"""Statistics and per-step reports of the admission benchmark (bench.py)."""
from __future__ import annotations

import os
import statistics
import sys


def pct(xs, q):
    s = sorted(xs)
    if not s:
        return float("nan")
    return s[min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))]


def alloc_summary(pl, steps):
    """GetPreferredAllocation over admissions that all start from the same
    availability: RPC time, whether the search ran (no short-circuit), its
    candidate count, and the chosen set against the reference's ordered BFS
    (C++ re-simulation) on that availability."""
    if not steps:
        return {}
    avail = pl.available()
    n = len(steps[0][3])
    ref = pl.allocator.reference_allocate(avail, [], n) if len(avail) > n else None
    chosen = {tuple(x[3]) for x in steps}
    return {"available": len(avail),
            "preferred_rpc_p50_ms": round(pct([x[0] for x in steps], .5), 4),
            "preferred_used": all(x[4] for x in steps),
            "short_circuit_steps": sum(1 for x in steps if x[1]),
            "candidates": max(x[2] for x in steps),
            "chosen": [list(c) for c in sorted(chosen)],
            "reference_candidates": ref["candidates"] if ref else None,
            "same_set_as_reference": (chosen == {tuple(sorted(ref["ids"]))}) if ref else None}


def fragment(ids, n, hold=-1):
    """Devices other pods hold: alternating positions (every hive loses some),
    (M-N)//2 of them by default, never leaving fewer than n free."""
    m = len(ids)
    h = (m - n) // 2 if hold < 0 else hold
    h = max(0, min(h, m - n))
    return (list(ids[1::2]) + list(ids[0::2]))[:h]


def process_gpu_state() -> dict:
    """This process's hold on the GPU right now: a torch HIP context, open
    /dev/kfd and render-node descriptors (a kubelet node has none of these)."""
    torch = sys.modules.get("torch")
    kfd = render = 0
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                t = os.readlink(f"/proc/self/fd/{fd}")
            except OSError:
                continue
            kfd += t == "/dev/kfd"
            render += t.startswith("/dev/dri/renderD")
    except OSError:
        pass
    return {"torch_cuda_initialized": bool(torch is not None and torch.cuda.is_initialized()),
            "kfd_fds": kfd, "render_fds": render}


def tail_attribution(lat, phases, factor=1.5, details=None) -> dict:
    """Every step slower than factor x p50: which phase carries the excess.
    ``phases`` maps a phase name to its per-step ms (aligned with ``lat``); a
    slow step is attributed to the phase with the largest excess over its own
    p50. ``details``: more per-step series (e.g. the kfd open inside the
    runtime init) reported with each slow step, not used for attribution."""
    if not lat:
        return {}
    p50 = pct(lat, .5)
    med = {k: pct(v, .5) for k, v in phases.items()}
    slow, by_phase = [], {}
    for i, x in enumerate(lat):
        if x <= factor * p50:
            continue
        excess = {k: round(v[i] - med[k], 2) for k, v in phases.items()}
        top = max(excess, key=excess.get)
        by_phase.setdefault(top, []).append(excess[top])
        row = {"step": i, "latency_ms": round(x, 2), "phase": top, "excess_ms": excess}
        for k, v in (details or {}).items():
            if i < len(v) and v[i] is not None:
                row[k] = round(v[i], 2)
        slow.append(row)
    return {"threshold_ms": round(factor * p50, 2), "p99_over_p50": round(pct(lat, .99) / p50, 3) if p50 else None,
            "phase_p50_ms": {k: round(v, 3) for k, v in med.items()},
            "slow_steps": slow,
            "by_phase": {k: {"steps": len(v), "excess_ms_mean": round(statistics.mean(v), 2)}
                         for k, v in sorted(by_phase.items())}}
