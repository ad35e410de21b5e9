"""Per-device health aggregation for the container (KFD) mode.

Reference behaviour (internal/pkg/amdgpu/amdgpu.go:322-345,865-974): one
node-global verdict — "Healthy" if *any* kfd node is a live GPU — copied onto
every device, then overridden per PCI BDF by the metrics exporter. Partitions
never get their own verdict and the verdict objects are mutated in place while
RPCs read them.

Here each device gets its own verdict from up to four sources, and a device is
Healthy only if every *available* source agrees:

1. kfd: the device's own kfd node still exists and is a live GPU node;
2. exporter: per-BDF verdict, applied to every partition of that BDF;
3. liveness: the gfx950 MFMA probe on that exact HIP device, with hysteresis
   (``fail_threshold`` consecutive failures to go Unhealthy,
   ``recover_threshold`` successes to come back);
4. amd-smi: a rise in uncorrectable ECC errors since the last sweep;
5. amd-smi events (push-style, drained every sweep): a ``gpu_pre_reset`` keeps
   the device Unhealthy until its ``gpu_post_reset``; VM faults, thermal
   throttling and queue evictions are counted
   (``mi355x_dp_gpu_events_total``) and logged.

Not a verdict but read in the same sweep: the xGMI link state (``smi_xgmi``,
health/fabric.py). A GPU pair whose link went down stays Healthy; the
allocator stops treating it as xGMI-connected (``degraded_links``).

Verdicts are published as immutable snapshots with a version number, so
ListAndWatch streams can send on change without locks.
"""
from __future__ import annotations

import asyncio
import os
import time
from dataclasses import dataclass
from typing import Callable, Dict, Mapping, Optional, Tuple

from ..ops.native import core
from ..proto import deviceplugin as dp
from ..topology import Inventory, KfdBusyUnknown, hip_ordinals, kfd_busy_gpu_ids, kfd_gpu_load
from ..utils import log
from ..utils.trace import TRACER
from . import exporter
from .fabric import FabricWatcher
from .liveness import LivenessProber, ProbeOutcome

_log = log.get("health")


@dataclass(frozen=True)
class Verdict:
    health: str
    reasons: Tuple[str, ...] = ()


@dataclass
class HealthConfig:
    exporter_socket: Optional[str] = exporter.DEFAULT_SOCKET
    exporter_timeout_s: float = 10.0
    liveness: bool = False
    liveness_timeout_s: float = 10.0
    liveness_iters: int = 4
    liveness_parallel: int = 8
    liveness_mode: str = "persistent"  # persistent probe server | spawn per device per sweep
    liveness_keep_queues: bool = True  # persistent server keeps per-device queues between sweeps
    # every N-th sweep (and the first), GPUs with no user queues from any process
    # get the full-chip sweep (every CU of every XCD) instead of the one-wave probe
    chip_sweep_every: int = 0
    fail_threshold: int = 2
    # a probe whose dispatch stays queued behind other processes' work on the
    # GPU (a tenant kernel holding every CU) is inconclusive for this long
    # before it counts as a failure
    liveness_busy_grace_s: float = 300.0
    # the same grace while which GPUs are busy is unknown (kfd process list
    # unreadable, or the probe server's own kfd entry unresolved): every GPU
    # then counts as busy, so the grace is kept short to bound the blind spot
    liveness_unknown_busy_grace_s: float = 30.0
    # a pending probe on a "busy" GPU is only inconclusive while the GPU is
    # actually executing: amd-smi reporting 0% GFX activity on this many
    # consecutive sweeps ends the grace (a wedged queue, not a long kernel)
    liveness_corroborate: bool = True
    liveness_idle_sweeps: int = 2
    # crowded GPUs: with this many other processes holding queues on a GPU
    # (or their queues leaving fewer than 2 of the GPU's kfd num_cp_queues)
    # the HWS runlist is oversubscribed and every extra process/queue lengthens
    # the tenants' time slices (measured: 8 tenant processes x 4 queues, p99.9
    # GEMM 14 -> 34 ms with the kept probe queue, profiles/archive/measurements_r1_r3.md §3n). The
    # probe server then steps off that GPU (no queue, no runlist slot); while
    # the GPU reports GFX activity its tenants are the liveness evidence, at 0%
    # it is probed from a fresh process. 0 = off.
    liveness_crowded_procs: int = 7
    liveness_crowded_release_sweeps: int = 5   # uncrowded sweeps before the server takes the GPU back
    recover_threshold: int = 1
    # throughput check (opt-in): every N-th sweep (and the first), GPUs with no
    # other process's queues get HBM write/read bandwidth over a verified
    # pattern, the sustained bf16 MFMA rate and per-XCD shader clocks
    # (LivenessProber.perf, ~40 ms of the chip per GPU at the defaults). Data
    # read back wrong is always a failure; rates under the floors (scaled by the
    # device's share of a whole MI355X's 256 CUs) or an XCD clocked far below
    # its siblings make the GPU "degraded": logged and exported, and with
    # perf_action "unhealthy" withdrawn until a later check passes. Floors are
    # about half of what an MI355X measures (profiles/archive/measurements_r1_r3.md §10).
    perf_check_every: int = 0
    perf_mib: int = 4096
    perf_mfma_iters: int = 65536
    perf_action: str = "report"             # report | unhealthy
    perf_min_hbm_read_gbps: float = 3000.0
    perf_min_hbm_write_gbps: float = 2000.0
    perf_min_mfma_tflops: float = 700.0
    perf_min_xcd_clock_ratio: float = 0.6   # slowest XCD's clock over the median XCD's
    smi_ecc: bool = False
    smi_events: bool = False
    smi_xgmi: bool = False             # watch xGMI link state (placement input, health/fabric.py)
    dev_root: str = "/dev"


@dataclass
class _Track:
    fails: int = 0
    oks: int = 0
    live: bool = True
    last_reason: str = ""
    pending_since: Optional[float] = None   # first inconclusive (busy GPU) probe
    idle_pending: int = 0                   # consecutive pending sweeps with 0% GFX activity


class HealthMonitor:
    def __init__(self, inventory: Inventory, cfg: Optional[HealthConfig] = None,
                 prober: Optional[LivenessProber] = None,
                 ordinal_map: Optional[Mapping[str, int]] = None,
                 exporter_fn: Optional[Callable] = None, event_source=None,
                 fabric_source: Optional[Callable[[], dict]] = None,
                 activity_source: Optional[Callable[[], Dict[str, int]]] = None):
        self.inv = inventory
        self.cfg = cfg or HealthConfig()
        self.prober = prober
        if self.cfg.liveness and self.prober is None:
            self.prober = LivenessProber(timeout_s=self.cfg.liveness_timeout_s, iters=self.cfg.liveness_iters,
                                         max_parallel=self.cfg.liveness_parallel, mode=self.cfg.liveness_mode,
                                         keep_queues=self.cfg.liveness_keep_queues,
                                         kfd_proc_dir=os.path.join(self.inv.sysfs_root, "class/kfd/kfd/proc"))
        self._ordinals = dict(ordinal_map) if ordinal_map is not None else None
        # amd-smi event watcher (or a test double with start/poll/stop)
        self._events = event_source
        self._events_started = False
        self._resetting: Dict[str, str] = {}   # bdf -> message of the pending pre-reset
        self.event_counts: Dict[Tuple[str, str], int] = {}
        self.chip_sweeps = 0
        self._exporter_fn = exporter_fn or exporter.get_gpu_health
        self._track: Dict[str, _Track] = {d.id: _Track() for d in inventory.devices}
        self._ecc: Dict[str, int] = {}
        self._snapshot: Dict[str, Verdict] = {d.id: Verdict(dp.HEALTHY) for d in inventory.devices}
        self.version = 0
        self.sweeps = 0
        self.last_sweep_ms = 0.0
        self.fabric = FabricWatcher(inventory, fabric_source) if self.cfg.smi_xgmi else None
        self._smi_held = False   # amd-smi kept initialised while its sources are on (smi_hold)
        self.busy_state_known = True   # last sweep could tell busy GPUs from idle ones
        self.identity_remaps = 0       # sweeps whose probe replies did not match the positional ordinals
        self._activity_source = activity_source   # bdf -> GFX activity % (amd-smi by default)
        self._load: Dict[int, Tuple[int, int]] = {}  # kfd gpu_id -> (other processes, their queues)
        self._crowded: Dict[str, int] = {}          # device -> uncrowded sweeps seen since it got crowded
        self.crowded_skips = 0
        self._perf: Dict[str, Tuple[str, str]] = {}  # device -> (ok | degraded | failed, reason)
        self.perf_last: Dict[str, dict] = {}         # device -> last throughput-check reply
        self.perf_checks = 0

    # ------------------------------------------------------------------ fabric
    def degraded_links(self):
        """Physical-GPU pairs (allocator group keys) whose xGMI link is down."""
        return self.fabric.degraded if self.fabric is not None else frozenset()

    @property
    def fabric_version(self) -> int:
        return self.fabric.version if self.fabric is not None else 0

    # ------------------------------------------------------------------ views
    def snapshot(self) -> Dict[str, Verdict]:
        return self._snapshot

    def health(self, dev_id: str) -> str:
        v = self._snapshot.get(dev_id)
        return v.health if v else dp.UNHEALTHY

    def ordinals(self) -> Dict[str, int]:
        if self._ordinals is None:
            self._ordinals = hip_ordinals(self.inv, self.cfg.dev_root)
        return self._ordinals

    # ---------------------------------------------------------------- sources
    def _kfd_verdicts(self) -> Dict[str, Optional[str]]:
        n = core()
        nodes_dir = os.path.join(self.inv.sysfs_root, "class/kfd/kfd/topology/nodes")
        out: Dict[str, Optional[str]] = {}
        if not os.path.isdir(nodes_dir):
            return {d.id: "kfd topology unavailable" for d in self.inv.devices}
        for d in self.inv.devices:
            if d.node_id < 0:
                out[d.id] = None
                continue
            kv = n.parse_kv_file(os.path.join(nodes_dir, str(d.node_id), "properties"))
            if kv is None:
                out[d.id] = f"kfd node {d.node_id} missing"
                continue
            try:
                cores = int(kv.get("cpu_cores_count", "0"), 0)
                gfx = int(kv.get("gfx_target_version", "0"), 0)
            except ValueError:
                out[d.id] = f"kfd node {d.node_id} unparseable"
                continue
            out[d.id] = None if (cores == 0 and gfx > 0) else f"kfd node {d.node_id} not a live GPU"
        return out

    def _smi_hold(self) -> None:
        # one amdsmi_init for the monitor's lifetime instead of one per query
        # (~26 ms each on MI355X, tools/smi_timing.py)
        if not self._smi_held:
            n = core()
            self._smi_held = bool(n.smi_available() and n.smi_hold())

    def _smi_ecc(self) -> Dict[str, str]:
        n = core()
        if not n.smi_available():
            return {}
        self._smi_hold()
        snap = n.smi_snapshot()
        if not snap["ok"]:
            return {}
        bad: Dict[str, str] = {}
        by_bdf = {g["bdf"]: g for g in snap["gpus"] if g["ecc_ok"]}
        for d in self.inv.devices:
            g = by_bdf.get(d.bdf)
            if not g:
                continue
            prev = self._ecc.get(d.id)
            cur = int(g["ecc_uncorrectable"])
            self._ecc[d.id] = cur
            if prev is not None and cur > prev:
                bad[d.id] = f"uncorrectable ECC errors rose {prev}->{cur}"
        return bad

    EVENT_MASK_NAMES = ("vmfault", "thermal_throttle", "gpu_pre_reset", "gpu_post_reset", "queue_eviction")
    _EVENT_TYPES = {"vmfault": 1, "thermal_throttle": 2, "gpu_pre_reset": 3, "gpu_post_reset": 4,
                    "queue_eviction": 9}

    def _drain_events(self) -> None:
        if self._events is None:
            self._events = core().SmiEventWatcher()
        if not self._events_started:
            mask = 0
            for nm in self.EVENT_MASK_NAMES:
                mask |= 1 << (self._EVENT_TYPES[nm] - 1)
            err = self._events.start(mask)
            self._events_started = True
            if err:
                _log.warning("amd-smi event notification unavailable: %s", err)
                return
        if not getattr(self._events, "running", True):
            return
        from ..utils.metrics import REGISTRY
        for ev in self._events.poll(0):
            bdf, name = ev.get("bdf", ""), ev.get("name", "unknown")
            key = (bdf, name)
            self.event_counts[key] = self.event_counts.get(key, 0) + 1
            REGISTRY.inc("mi355x_dp_gpu_events_total", help="amd-smi GPU events", bdf=bdf, event=name)
            if name == "gpu_pre_reset":
                self._resetting[bdf] = ev.get("message", "")
                _log.warning("GPU %s: reset starting (%s)", bdf, ev.get("message", ""))
            elif name == "gpu_post_reset":
                self._resetting.pop(bdf, None)
                _log.warning("GPU %s: reset finished", bdf)
            else:
                _log.info("GPU %s: %s %s", bdf, name, ev.get("message", ""))

    def _idle_devices(self, dev_ids) -> set:
        """Devices whose kfd gpu_id has no user queue in any process right now."""
        own = self._own_entries()
        try:
            busy = kfd_busy_gpu_ids(self.inv.sysfs_root, exclude=own)
        except KfdBusyUnknown as e:
            # cannot tell which GPUs run work: sweep none (the sweep holds every CU)
            _log.warning("full-chip sweep skipped: %s", e)
            return set()
        idle = set()
        for dev_id in dev_ids:
            d = self.inv.by_id.get(dev_id)
            node = self.inv.topology.node(d.node_id) if d is not None and d.node_id >= 0 else None
            gid = int(getattr(node, "gpu_id", 0) or 0) if node is not None else 0
            if gid and gid not in busy:
                idle.add(dev_id)
        return idle

    def _gpu_id(self, dev_id: str) -> int:
        d = self.inv.by_id.get(dev_id)
        node = self.inv.topology.node(d.node_id) if d is not None and d.node_id >= 0 else None
        return int(getattr(node, "gpu_id", 0) or 0) if node is not None else 0

    def _own_entries(self):
        """The probe server's kfd proc entries (see LivenessProber.own_kfd_entries_for)."""
        if self.prober is None:
            return ()
        probed = self._ordinals.keys() if self._ordinals else ()
        return self.prober.own_kfd_entries_for({self._gpu_id(d) for d in probed})

    def _busy_devices(self, dev_ids) -> set:
        """Devices whose GPU runs other processes' queues (unknown -> all, and
        busy_state_known is cleared so the short grace applies)."""
        own = self._own_entries()
        unresolved = not own and self.prober is not None and self.prober.server_running and \
            self.prober.keep_queues
        try:
            self._load = kfd_gpu_load(self.inv.sysfs_root, exclude=own)
            busy = set(self._load)
        except KfdBusyUnknown as e:
            self._load = {}
            self._set_busy_known(False, str(e))
            return set(dev_ids)
        # the server's own kept queues could not be told apart from a tenant's
        self._set_busy_known(not unresolved, "probe server's kfd entry unresolved")
        out = set()
        for dev_id in dev_ids:
            d = self.inv.by_id.get(dev_id)
            node = self.inv.topology.node(d.node_id) if d is not None and d.node_id >= 0 else None
            gid = int(getattr(node, "gpu_id", 0) or 0) if node is not None else 0
            if gid and gid in busy:
                out.add(dev_id)
        return out

    def _gfx_activity(self) -> Dict[str, int]:
        """bdf -> GFX engine activity % (amd-smi); {} when unavailable."""
        if self._activity_source is not None:
            return self._activity_source()
        n = core()
        if not n.smi_available():
            return {}
        self._smi_hold()
        snap = n.smi_snapshot()
        if not snap["ok"]:
            return {}
        return {g["bdf"]: int(g.get("gfx_activity", -1)) for g in snap["gpus"] if g.get("gfx_activity", -1) >= 0}

    def _set_busy_known(self, known: bool, why: str) -> None:
        if known != self.busy_state_known:
            if known:
                _log.info("busy-GPU state readable again")
            else:
                _log.warning("busy-GPU state unknown (%s): every GPU counts as busy, pending probes get "
                             "a %.0fs grace instead of %.0fs", why, self.cfg.liveness_unknown_busy_grace_s,
                             self.cfg.liveness_busy_grace_s)
        self.busy_state_known = known
        from ..utils.metrics import REGISTRY
        REGISTRY.set("mi355x_dp_busy_state_known", 1.0 if known else 0.0,
                     help="1 if busy GPUs can be told from idle ones (kfd process list readable)")

    @staticmethod
    def _reply_identity(detail: dict):
        """(kfd node id, pci domain, kfd-style location_id) of the agent that
        answered, from the probe reply; None when the reply carries none."""
        nid = int(detail.get("kfd_node_id", -1) if detail.get("kfd_node_id") is not None else -1)
        loc = dom = None
        bus_id = detail.get("pci_bus_id") or ""
        try:
            d, b, df = bus_id.split(":")
            dev, fn = df.split(".")
            dom, loc = int(d, 16), (int(b, 16) << 8) | (int(dev, 16) << 3) | int(fn, 16)
        except ValueError:
            pass
        if nid < 0 and loc is None:
            return None
        return nid, dom, loc

    def _identity_matches(self, dev_id: str, ident) -> bool:
        d = self.inv.by_id.get(dev_id)
        if d is None or ident is None:
            return True
        nid, dom, loc = ident
        # the PCI location (partition index in the function bits) is exact; the
        # agent's node id is the thunk's index, renumbered when the device
        # cgroup hides GPUs (measured on MI355X), so it is only a fallback
        if loc is not None and d.location_id:
            return (dom, loc) == (d.domain, d.location_id)
        if nid >= 0 and d.node_id >= 0:
            return nid == d.node_id
        return True

    def _verify_identity(self, ords: Dict[str, int], outcomes: Dict[str, ProbeOutcome]) -> Dict[str, ProbeOutcome]:
        """Check that every reply came from the device its verdict is written to.

        Ordinals are positional (ROCr enumerates accessible GPU nodes in kfd node
        order, hip_ordinals); a different enumeration (a hidden node, CPX
        partitions ordered differently) would put verdicts on the wrong kubelet
        IDs. Each reply names its agent's PCI location (kfd location_id, with
        the partition index in the function bits), so on any mismatch the verdicts of this
        sweep are re-keyed by identity, the ordinal map is rebuilt from the
        replies, and a device no reply identifies loses its ordinal (reported
        "no HIP device for this ID")."""
        idents = {dev: self._reply_identity(o.detail) for dev, o in outcomes.items()}
        bad = sorted(dev for dev in outcomes if not self._identity_matches(dev, idents[dev]))
        if not bad:
            return outcomes
        from ..utils.metrics import REGISTRY
        by_node, by_loc = {}, {}
        for dev, o in outcomes.items():
            ident = idents[dev]
            if ident is None:
                continue
            nid, dom, loc = ident
            if loc is not None:
                by_loc[(dom, loc)] = (ords[dev], o)
            elif nid >= 0:
                by_node[nid] = (ords[dev], o)
        fixed: Dict[str, ProbeOutcome] = {}
        new_ords: Dict[str, int] = {}
        for dev in ords:
            d = self.inv.by_id.get(dev)
            hit = None
            if d is not None:
                hit = by_loc.get((d.domain, d.location_id)) if d.location_id else None
                if hit is None and d.node_id >= 0:
                    hit = by_node.get(d.node_id)
            if hit is not None and self._identity_matches(dev, self._reply_identity(hit[1].detail)):
                new_ords[dev] = hit[0]
                fixed[dev] = hit[1]
        for dev, ordinal in new_ords.items():
            if ords.get(dev) != ordinal:
                _log.error("probe identity: device %s is ordinal %d, not %s (verdict re-keyed)", dev, ordinal,
                           ords.get(dev))
        lost = sorted(set(ords) - set(new_ords))
        if lost:
            _log.error("probe identity: no probed agent matches %s; they lose their ordinal", lost)
        keep = {k: v for k, v in (self._ordinals or {}).items() if k not in ords}
        self._ordinals = {**keep, **new_ords}
        self.identity_remaps += 1
        REGISTRY.inc("mi355x_dp_probe_identity_mismatch_total",
                     help="sweeps whose probe replies came from other devices than the positional ordinal map")
        return fixed

    def _update_crowded(self, dev_ids) -> set:
        """Devices whose GPU is crowded now or was within the release window."""
        lim = self.cfg.liveness_crowded_procs
        if lim <= 0:
            self._crowded.clear()
            return set()
        out = set()
        for dev_id in dev_ids:
            d = self.inv.by_id.get(dev_id)
            node = self.inv.topology.node(d.node_id) if d is not None and d.node_id >= 0 else None
            gid = self._gpu_id(dev_id)
            procs, queues = self._load.get(gid, (0, 0))
            cp = int(node.prop("num_cp_queues", 0)) if node is not None else 0
            crowded = procs >= lim or (cp > 0 and queues + 2 > cp)
            if crowded:
                if dev_id not in self._crowded:
                    _log.info("GPU of %s is crowded (%d other processes, %d queues): the probe server steps off it",
                              dev_id, procs, queues)
                self._crowded[dev_id] = 0
            elif dev_id in self._crowded:
                self._crowded[dev_id] += 1
                if self._crowded[dev_id] >= self.cfg.liveness_crowded_release_sweeps:
                    del self._crowded[dev_id]
                    _log.info("GPU of %s is no longer crowded: probing it again", dev_id)
            if dev_id in self._crowded:
                out.add(dev_id)
        return out

    async def _liveness(self, ords: Dict[str, int], busy_devs=frozenset()):
        every = self.cfg.chip_sweep_every
        busy = {o for d, o in ords.items() if d in busy_devs}
        if every <= 0 or self.sweeps % every != 0:
            return await self.prober.probe(ords, busy=busy)
        idle = self._idle_devices(ords)
        out = {}
        if idle:
            swept = await self.prober.sweep({k: v for k, v in ords.items() if k in idle})
            out.update(swept)
            self.chip_sweeps += 1
            from ..utils.metrics import REGISTRY
            REGISTRY.inc("mi355x_dp_chip_sweeps_total", help="full-chip sweeps run (every CU of every XCD on the idle GPUs)")
        rest = {k: v for k, v in ords.items() if k not in idle}
        if rest:
            out.update(await self.prober.probe(rest, busy=busy))
        return out

    # ------------------------------------------------------------ throughput
    PERF_STATES = {"ok": 0.0, "degraded": 1.0, "failed": 2.0}

    def perf_problems(self, d: dict) -> list:
        """Why a (correct) throughput-check reply counts as degraded; [] if not."""
        c = self.cfg
        cus = int(d.get("cu_count") or 0)
        share = min(1.0, cus / 256.0) if cus > 0 else 1.0   # a CPX partition has 1/8 of the CUs
        out = []
        for key, floor, what, unit in (("hbm_read_gbps", c.perf_min_hbm_read_gbps, "HBM read", "GB/s"),
                                       ("hbm_write_gbps", c.perf_min_hbm_write_gbps, "HBM write", "GB/s"),
                                       ("mfma_tflops", c.perf_min_mfma_tflops, "bf16 MFMA", "TFLOP/s")):
            v = float(d.get(key) or 0.0)
            if floor > 0 and v < floor * share:
                out.append(f"{what} {v:.0f} {unit} < {floor * share:.0f}")
        clocks = [float(x) for x in (d.get("xcd_clock_mhz") or []) if x and float(x) > 0]
        if len(clocks) >= 2 and c.perf_min_xcd_clock_ratio > 0:
            med = sorted(clocks)[len(clocks) // 2]
            i = min(range(len(clocks)), key=clocks.__getitem__)
            if clocks[i] < c.perf_min_xcd_clock_ratio * med:
                out.append(f"XCD {i} at {clocks[i]:.0f} MHz vs median {med:.0f} MHz under MFMA load")
        return out

    async def _perf_check(self, ords: Dict[str, int]) -> None:
        from ..utils.metrics import REGISTRY
        p = self.prober
        p.perf_mib, p.perf_iters = self.cfg.perf_mib, self.cfg.perf_mfma_iters
        with TRACER.span("health.perf_check", "health", devices=len(ords)):
            res = await p.perf(ords)
        self.perf_checks += 1
        REGISTRY.inc("mi355x_dp_perf_checks_total", help="throughput checks run (HBM pattern + MFMA + clocks)")
        for dev, o in res.items():
            d = o.detail or {}
            self.perf_last[dev] = d
            if not o.ok:
                state, why = "failed", f"throughput check: {o.reason}"
            else:
                probs = self.perf_problems(d)
                state, why = ("degraded", "throughput check: " + "; ".join(probs)) if probs else ("ok", "")
            prev = self._perf.get(dev, ("ok", ""))[0]
            if state != prev:
                (_log.info if state == "ok" else _log.warning)("device %s: throughput check %s -> %s %s", dev, prev,
                                                               state, why)
            self._perf[dev] = (state, why)
            if log.V(2) and o.ok:
                _log.info("device %s: throughput HBM write %.0f / read %.0f GB/s, bf16 MFMA %.0f TFLOP/s at %.0f MHz "
                          "(XCD clocks %s)", dev, d.get("hbm_write_gbps", 0), d.get("hbm_read_gbps", 0),
                          d.get("mfma_tflops", 0), d.get("clock_mhz_median", 0), d.get("xcd_clock_mhz"))
            REGISTRY.set("mi355x_dp_perf_state", self.PERF_STATES[state],
                         help="last throughput check: 0 ok, 1 degraded (rates under the floors), 2 failed", device=dev)
            if o.ok:
                for key, name, hlp in (("hbm_read_gbps", "mi355x_dp_perf_hbm_read_gbps", "HBM read bandwidth"),
                                       ("hbm_write_gbps", "mi355x_dp_perf_hbm_write_gbps", "HBM write bandwidth"),
                                       ("mfma_tflops", "mi355x_dp_perf_mfma_tflops", "sustained dense bf16 MFMA rate"),
                                       ("clock_mhz_median", "mi355x_dp_perf_clock_mhz",
                                        "median workgroup shader clock under MFMA load")):
                    REGISTRY.set(name, float(d.get(key) or 0.0), help=f"last throughput check: {hlp}", device=dev)
                for x, mhz in enumerate(d.get("xcd_clock_mhz") or []):
                    REGISTRY.set("mi355x_dp_perf_xcd_clock_mhz", float(mhz),
                                 help="last throughput check: median shader clock per XCD", device=dev, xcd=str(x))

    def perf_verdicts(self) -> Dict[str, Tuple[str, str]]:
        return dict(self._perf)

    # ------------------------------------------------------------------ sweep
    async def close(self) -> None:
        if self.prober is not None:
            await self.prober.close()
        if self._events is not None and self._events_started:
            self._events.stop()
            self._events_started = False
        if self._smi_held:
            core().smi_unhold()
            self._smi_held = False

    async def check_once(self) -> bool:
        """Run one sweep; returns True if any verdict changed."""
        with TRACER.span("health.sweep", "health", devices=len(self.inv.devices)):
            return await self._check_once()

    async def _check_once(self) -> bool:
        t0 = time.perf_counter()
        reasons: Dict[str, list] = {d.id: [] for d in self.inv.devices}
        for dev, r in self._kfd_verdicts().items():
            if r:
                reasons[dev].append(r)

        if self.cfg.exporter_socket:
            hmap = await self._exporter_fn(self.cfg.exporter_socket, self.cfg.exporter_timeout_s)
            if hmap:
                for d in self.inv.devices:
                    if hmap.get(d.bdf) == dp.UNHEALTHY:
                        reasons[d.id].append(f"exporter reports {d.bdf} unhealthy")

        if self.cfg.liveness and self.prober is not None:
            ords = {k: v for k, v in self.ordinals().items() if k in reasons}
            busy_devs = self._busy_devices(ords)
            crowded = self._update_crowded(ords)
            probe_ords = {k: v for k, v in ords.items() if k not in crowded}
            if hasattr(self.prober, "set_visible"):
                self.prober.set_visible(sorted(set(probe_ords.values())) if crowded else None)
            if not probe_ords and crowded and getattr(self.prober, "server_running", False):
                await self.prober.close()       # every GPU crowded: hold nothing on any of them
            outcomes = self._verify_identity(probe_ords, await self._liveness(probe_ords, busy_devs)) \
                if probe_ords else {}
            if crowded:
                act = await asyncio.to_thread(self._gfx_activity)
                from ..utils.metrics import REGISTRY
                for dev_id in sorted(crowded):
                    d = self.inv.by_id.get(dev_id)
                    if d is not None and act.get(d.bdf, -1) == 0:
                        # crowded but idle: nothing to disturb, probe it from a fresh process
                        outcomes[dev_id] = await self.prober.probe_ordinal(ords[dev_id])
                    else:
                        self.crowded_skips += 1
                        REGISTRY.inc("mi355x_dp_liveness_crowded_skips_total",
                                     help="probes skipped on GPUs crowded with tenant processes", device=dev_id)
            ords = {k: v for k, v in self.ordinals().items() if k in reasons}
            from ..utils.metrics import REGISTRY
            now = time.monotonic()
            grace = self.cfg.liveness_busy_grace_s if self.busy_state_known else \
                min(self.cfg.liveness_busy_grace_s, self.cfg.liveness_unknown_busy_grace_s)
            idle_wedged = set()
            waiting = [d for d, o in outcomes.items() if o.pending and d in busy_devs]
            if waiting and self.cfg.liveness_corroborate:
                act = await asyncio.to_thread(self._gfx_activity)
                for dev_id in waiting:
                    d = self.inv.by_id.get(dev_id)
                    a = act.get(d.bdf, -1) if d is not None else -1
                    tr = self._track[dev_id]
                    tr.idle_pending = tr.idle_pending + 1 if a == 0 else 0
                    if tr.idle_pending >= self.cfg.liveness_idle_sweeps:
                        idle_wedged.add(dev_id)
            for dev_id, o in outcomes.items():
                REGISTRY.set("mi355x_dp_liveness_probe_ms", float(o.latency_ms),
                             help="last liveness probe round trip", device=dev_id)
                tr = self._track[dev_id]
                if not o.pending:
                    tr.idle_pending = 0
                if o.ok:
                    tr.fails, tr.oks = 0, tr.oks + 1
                    tr.pending_since = None
                    if not tr.live and tr.oks >= self.cfg.recover_threshold:
                        tr.live = True
                elif o.pending and dev_id in busy_devs and dev_id not in idle_wedged and \
                        now - (tr.pending_since or now) < grace:
                    # queued behind a tenant's kernel: neither a pass nor a failure yet
                    tr.pending_since = tr.pending_since or now
                    REGISTRY.inc("mi355x_dp_liveness_inconclusive_total", help="probes queued behind a busy GPU",
                                 device=dev_id)
                else:
                    tr.oks, tr.fails = 0, tr.fails + 1
                    tr.last_reason = o.reason
                    if dev_id in idle_wedged:
                        tr.last_reason += (f" while the GPU reports 0% GFX activity ({tr.idle_pending} sweeps): "
                                           "no tenant kernel is running")
                        from ..utils.metrics import REGISTRY as _R
                        _R.inc("mi355x_dp_liveness_idle_pending_total", help="pending probes on an idle GFX engine",
                               device=dev_id)
                    if not o.pending:
                        tr.pending_since = None
                    if tr.live and tr.fails >= self.cfg.fail_threshold:
                        tr.live = False
                if not tr.live:
                    reasons[dev_id].append(f"liveness probe: {tr.last_reason}")
            for dev_id in reasons:
                if dev_id not in ords:
                    reasons[dev_id].append("no HIP device for this ID (render node inaccessible?)")
            every = self.cfg.perf_check_every
            if every > 0 and self.sweeps % every == 0:
                idle = self._idle_devices(probe_ords)
                cand = {k: v for k, v in probe_ords.items() if k in idle and self._track[k].live and k in ords}
                if cand:
                    await self._perf_check(cand)
            for dev_id, (state, why) in self._perf.items():
                if dev_id in reasons and (state == "failed" or
                                          (state == "degraded" and self.cfg.perf_action == "unhealthy")):
                    reasons[dev_id].append(why)

        if self.cfg.smi_ecc:
            for dev_id, r in (await asyncio.to_thread(self._smi_ecc)).items():   # amd-smi off the event loop
                reasons[dev_id].append(r)

        if self.cfg.smi_events:
            self._drain_events()
            for d in self.inv.devices:
                if d.bdf in self._resetting:
                    reasons[d.id].append("GPU reset in progress (amd-smi gpu_pre_reset, no post_reset yet)")

        if self.fabric is not None:
            if self.fabric.reads_amd_smi:
                self._smi_hold()
            await asyncio.to_thread(self.fabric.check)   # amd-smi queries run off the event loop

        new = {dev: Verdict(dp.UNHEALTHY if rs else dp.HEALTHY, tuple(rs)) for dev, rs in reasons.items()}
        changed = any(new[k].health != self._snapshot.get(k, Verdict("")).health for k in new)
        if changed:
            for k, v in new.items():
                old = self._snapshot.get(k)
                if old is None or old.health != v.health:
                    _log.warning("device %s: %s -> %s %s", k, old.health if old else "?", v.health,
                                 "; ".join(v.reasons))
            self.version += 1
        self._snapshot = new
        from ..utils.metrics import REGISTRY
        for dev, v in new.items():
            REGISTRY.set("mi355x_dp_device_healthy", 1.0 if v.health == dp.HEALTHY else 0.0,
                         help="1 if the device is advertised Healthy", device=dev)
        self.sweeps += 1
        self.last_sweep_ms = (time.perf_counter() - t0) * 1e3
        return changed
