"""Allocation policy facade (reference: internal/pkg/allocator/allocator.go:21-30
``Policy{Init, Allocate}`` and BestEffortPolicy, besteffort_policy.go:45-151).

The search itself is native (C++ ``HiveAllocator``, native/src/alloc/hive_allocator.cpp).
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence

from .ops.native import core
from .utils.trace import TRACER


class AllocationError(Exception):
    pass


@dataclass
class AllocStats:
    calls: int = 0
    total_us: float = 0.0
    last_us: float = 0.0
    last_candidates: int = 0
    last_weight: int = -1
    last_short_circuit: bool = False


class Policy:
    """Interface kept for parity with the reference Policy."""

    def init(self, devices, topology, degraded_links: Iterable = ()) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def allocate(self, available: Sequence[str], required: Sequence[str], size: int) -> List[str]:
        raise NotImplementedError  # pragma: no cover


def group_key(d) -> str:
    """Physical-GPU identity the allocator groups partitions by: kfd's
    unique_id, or — for a device whose kfd node is unreadable (e.g.
    cgroup-denied inside a container) — its own PCI function."""
    return d.unique_id or f"bdf:{getattr(d, 'bdf', '') or d.id}"


class BestEffortPolicy(Policy):
    """Hive-aware optimal subset selection with the reference's tie-breaks."""

    SEARCH_MODES = ("auto", "reference", "extended")

    def __init__(self, missing_pair_is_worst: bool = True, cross_hive_penalty: int = 100,
                 extended_search=False):
        """`extended_search`: True searches every split of the request over
        classes of interchangeable devices (several partial GPUs; kfd link
        weight / bandwidth tie-breaks) instead of the reference's candidate
        family; "auto" does so only on nodes with partitioned GPUs (the
        plugins' default, see AllocatorOptions::extended_search_auto)."""
        n = core()
        self._opts = n.AllocatorOptions(missing_pair_is_worst=missing_pair_is_worst,
                                        cross_hive_penalty=cross_hive_penalty)
        self._opts.extended_search_auto = extended_search == "auto"
        self._opts.extended_search = extended_search is True or extended_search == "extended"
        self._alloc = n.HiveAllocator()
        self.stats = AllocStats()

    @staticmethod
    def to_alloc_devices(devices: Iterable) -> list:
        """Accepts topology.Gpu objects or (id, node_id, numa, unique_id[, hive]) tuples."""
        n = core()
        out = []
        for d in devices:
            if isinstance(d, tuple):
                out.append(n.AllocDevice(*d))
            else:
                # a device whose kfd node is unreadable (e.g. cgroup-denied inside a
                # container) is grouped by its sysfs unique_id, else by its own PCI
                # function; with a sysfs identity its links are inferred from the hive
                inferred = d.node_id < 0 and getattr(d, "identity", "") == "sysfs"
                out.append(n.AllocDevice(d.id, d.node_id, d.numa_node, group_key(d), int(getattr(d, "hive_id", 0)),
                                         inferred))
        return out

    def init(self, devices, topology, degraded_links: Iterable = ()) -> None:
        """``degraded_links``: pairs of physical-GPU keys (``group_key``) whose
        direct xGMI link is down (health/fabric.py); they score as the worst
        link until the next init without them."""
        self._opts.degraded_links = sorted(tuple(sorted(p)) for p in degraded_links)
        # a fresh native allocator per init: the native gRPC server may still be
        # answering with the previous one (it holds a shared snapshot)
        alloc = core().HiveAllocator()
        err = alloc.init(self.to_alloc_devices(devices), topology, self._opts)
        if err:
            raise AllocationError(err)
        self._alloc = alloc

    @property
    def native(self):
        return self._alloc

    def allocate(self, available: Sequence[str], required: Sequence[str], size: int) -> List[str]:
        t0 = time.perf_counter()
        with TRACER.span("allocator.allocate", "alloc", size=size, available=len(available)):
            r = self._alloc.allocate(list(available), list(required or ()), int(size))
        dt = (time.perf_counter() - t0) * 1e6
        self.stats.calls += 1
        self.stats.total_us += dt
        self.stats.last_us = dt
        self.stats.last_candidates = r["candidates"]
        self.stats.last_weight = r["weight"]
        self.stats.last_short_circuit = bool(r["short_circuit"])
        if r["error"]:
            raise AllocationError(r["error"])
        return list(r["ids"])

    def reference_allocate(self, available: Sequence[str], required: Sequence[str], size: int) -> dict:
        """The reference's ordered-BFS enumeration on the same weights (benchmarks/parity)."""
        return self._alloc.reference_allocate(list(available), list(required or ()), int(size))

    def explain(self, available: Sequence[str], required: Sequence[str], size: int) -> dict:
        return self._alloc.allocate(list(available), list(required or ()), int(size))


def load_topology(nodes_dir: Optional[str] = None, sysfs_root: Optional[str] = None):
    n = core()
    if nodes_dir:
        return n.KfdTopology.load(nodes_dir)
    return n.KfdTopology.load_sysfs(sysfs_root or "/sys")
