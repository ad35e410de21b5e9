"""One pod admission as bench.py times it, and the per-step records.

A step (``Admissions.step``) is what kubelet and the CRI runtime do for one
pod requesting amd.com/gpu=N:

1. rank 0's fake kubelet runs GetPreferredAllocation + Allocate against the
   plugin under test;
2. the Allocate response becomes the container: one fresh process whose /dev
   holds exactly the DeviceSpecs (``--container-mode pod``), or one process
   per allocated GPU, one per rank (``per-gpu``); it initialises the GPU
   runtime and runs the MFMA liveness kernel on its GPUs;
3. ready = the slowest container's verified tile; latency = ready - the start
   of GetPreferredAllocation, both CLOCK_MONOTONIC;
4. the pod terminates and, with ``--settle kfd``, the next step waits until
   the driver has torn its kfd processes down (untimed in the latency).

Every rank takes part in every step (the allocation is broadcast, the
containers' results gathered over gloo); only rank 0 records the plugin's
side.
"""
from __future__ import annotations

import asyncio
import functools
import os
import statistics
import sys
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from .stats import pct, process_gpu_state, tail_attribution

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
STUB_PROBE = os.path.join(REPO, "rocm_k8s_device_plugin_amd", "testing", "stub_probe.py")


@dataclass
class StepRecords:
    """Per timed step (aligned lists)."""
    latency_ms: List[float] = field(default_factory=list)
    rpc_ms: List[float] = field(default_factory=list)          # GetPreferredAllocation + Allocate round trips
    allocate_rpc_ms: List[float] = field(default_factory=list)
    prestart_rpc_ms: List[float] = field(default_factory=list)  # PreStartContainer (-prestart_liveness), in rpc_ms
    ready_ms: List[float] = field(default_factory=list)        # latency - rpc
    kernel_us: List[float] = field(default_factory=list)
    prespawn_ms: List[float] = field(default_factory=list)     # after the RPCs, before the container's spawn
    exec_ms: List[float] = field(default_factory=list)         # spawn -> main (exec + library load)
    runtime_ms: List[float] = field(default_factory=list)      # main -> GPU runtime initialised
    device_ms: List[float] = field(default_factory=list)       # runtime -> verified tile
    setup_ms: List[float] = field(default_factory=list)        # device set-up part of device_ms
    launch_ms: List[float] = field(default_factory=list)       # launch -> verified part of device_ms
    settle_ms: List[float] = field(default_factory=list)
    device_phases: List[Dict[str, float]] = field(default_factory=list)
    alloc: List[tuple] = field(default_factory=list)           # (preferred ms, short circuit, candidates, ids, used)
    # the slowest container's own counters up to "GPU runtime initialised": read
    # syscalls (/proc/self/io syscr), CPU ms, hsa_init us (HSA entrypoint only) and
    # the emulated view's counters (cache descriptors opened, paths redirected)
    read_syscalls: List[int] = field(default_factory=list)
    cpu_ms_runtime: List[float] = field(default_factory=list)
    hsa_init_ms: List[float] = field(default_factory=list)
    kfd_open_ms: List[float] = field(default_factory=list)   # open("/dev/kfd") inside the runtime init
    kfd_foreign_exits: List[int] = field(default_factory=list)  # other programs' kfd processes gone meanwhile
    node_cache_opens: List[int] = field(default_factory=list)

    def phases(self) -> Dict[str, List[float]]:
        """Per-step ms of each admission phase (aligned with latency_ms)."""
        return {"plugin_rpc": self.rpc_ms, "runtime_prep": self.prespawn_ms, "exec_and_library_load": self.exec_ms,
                "gpu_runtime_init": self.runtime_ms, "device_setup": self.setup_ms,
                "launch_and_verify": self.launch_ms}

    def row(self) -> Optional[dict]:
        """A comparison row: latency p50 / p99, phase p50s, tail attribution and
        the containers' start-up counters (None without steps)."""
        if not self.latency_ms:
            return None
        med = lambda xs: round(pct(xs, .5), 3) if xs else None
        return {"steps": len(self.latency_ms), "latency_p50_ms": med(self.latency_ms),
                "latency_p99_ms": round(pct(self.latency_ms, .99), 3),
                "phases_p50_ms": {k: med(v) for k, v in self.phases().items()},
                "tail_attribution": tail_attribution(self.latency_ms, self.phases(), details=self.details()),
                "counters_p50": self.counters()}

    def details(self) -> dict:
        """Per-step detail reported with slow steps: inside the runtime init (HSA
        entrypoint), the kfd open, which waits for other processes' kfd teardown."""
        if not any(self.kfd_open_ms):
            return {}
        return {"kfd_open_ms": self.kfd_open_ms, "hsa_init_ms": self.hsa_init_ms,
                "host_kfd_exits_meanwhile": self.kfd_foreign_exits}

    def counters(self) -> dict:
        med = lambda xs: round(pct(xs, .5), 3) if xs else None
        return {"read_syscalls": med(self.read_syscalls), "cpu_ms_runtime": med(self.cpu_ms_runtime),
                "hsa_init_ms": med([x for x in self.hsa_init_ms if x > 0]),
                "kfd_open_ms": med([x for x in self.kfd_open_ms if x > 0]),
                "node_cpu_cache_opens": med(self.node_cache_opens)}


class Admissions:
    """Runs admissions against rank 0's plugin under test (``plug``; None on
    the other ranks) for an N-GPU pod."""

    def __init__(self, args, dist, n: int, loop=None, plug=None):
        self.args, self.d, self.n, self.loop, self.plug = args, dist, n, loop, plug
        self.rec = StepRecords()
        # worst seen in the timed loop: does a bench / plugin process hold the GPU?
        self.gpu_state = {"torch_cuda_initialized": False, "kfd_fds": 0, "render_fds": 0}

    # ------------------------------------------------------------------ helpers
    def _blocking(self, fn, *a, **kw):
        """Run fn; with the Python plugin's health loop on, on a worker thread
        while rank 0's event loop keeps sweeping (so sweeps overlap the start)."""
        a_ = self.args
        if (self.loop is not None and a_.health_pulse > 0 and not a_.fixture and a_.plugin == "python"):
            return self.loop.run_until_complete(asyncio.to_thread(functools.partial(fn, *a, **kw)))
        return fn(*a, **kw)

    def _admit(self, pl):
        """Rank 0: kubelet's GetPreferredAllocation + Allocate; what the containers need."""
        from rocm_k8s_device_plugin_amd.container_runtime import render_minors_from_specs
        import time
        t0 = time.monotonic_ns()
        adm = self.loop.run_until_complete(pl.kubelet.admit("amd.com/gpu", self.n))
        car = adm.response.container_responses[0]
        minors = render_minors_from_specs(car)
        ordl = [pl.minor_to_ord[m] for m in minors]
        mounts = [(m.container_path, m.host_path) for m in car.mounts]
        # the container's /dev: the DeviceSpecs, per allocated GPU (card + render node)
        spec_paths = {ds.host_path for ds in car.devices}
        groups = [[p for p in pl.minor_to_paths[m] if p in spec_paths] for m in minors]
        return adm, (t0, ordl, adm.total_ms, adm.allocate_ms, list(adm.device_ids), mounts, groups, adm.prestart_ms)

    def _container(self, runtime, mode, dev_view, ordl, mounts, groups):
        """This rank's container (if it has one): (ok, t_ready, kernel us, error, phases), lingering kfd procs."""
        from rocm_k8s_device_plugin_amd.container_runtime import start_container
        d, a_ = self.d, self.args
        if mode == "pod" and d.rank != 0:
            # the pod's single container runs on rank 0; other ranks only keep step
            return (True, 0, 0.0, "", (0, 0, 0, 0.0, {}, (None, None, 0.0, None, 0.0, 0))), frozenset()
        pod = mode == "pod" or d.world == 1
        mine_ord = ordl if pod else [ordl[d.rank]]
        paths = None
        if dev_view == "specs":
            paths = ["/dev/kfd"] + [p for g in (groups if pod else [groups[d.rank]]) for p in g]
        # CPU rehearsal (--fixture): the stub probe stands in for the GPU entrypoint,
        # through the same runtime path (/dev view, per-GPU split, result parsing)
        stub = dict(exe=STUB_PROBE, argv_prefix=[sys.executable]) if a_.fixture else {}
        r = self._blocking(start_container, mine_ord, timeout_s=a_.container_timeout, runtime=runtime,
                           mounts=mounts if not a_.fixture else (), device_paths=paths, **stub)
        devs = r.doc.get("devices", [])
        kus = max((dv.get("kernel_us", 0.0) for dv in devs), default=0.0)
        # device set-up (HIP: hipSetDevice .. stream/buffers/events; HSA: queue, code object, buffers)
        sus = max((dv.get("setup_us", 0.0) for dv in devs), default=0.0)
        slow_dev = max(devs, key=lambda dv: dv.get("total_us", 0.0), default={})
        view = r.doc.get("view") or {}
        init_us = r.doc.get("init_us") or {}
        # open("/dev/kfd"): timed by the container's view (either entrypoint), else by the HSA entrypoint
        kfd_us = view.get("kfd_open_us", init_us.get("kfd_open", 0.0))
        counters = (r.doc.get("read_syscalls_runtime"), r.doc.get("cpu_ms_runtime"), init_us.get("hsa_init", 0.0) / 1e3,
                    view.get("node_cpu_cache_opens"), kfd_us / 1e3, r.kfd_foreign_exits)
        phases = (r.t_start_ns, int(r.doc.get("t_start_ns", 0)), int(r.doc.get("t_runtime_ns", 0)), sus / 1e3,
                  slow_dev.get("phase_us") or {}, counters)
        return (r.ok, r.t_ready_ns, kus, r.error, phases), r.kfd_lingering

    # ------------------------------------------------------------------ one step
    def step(self, record, runtime: Optional[str] = None, settle: Optional[str] = None,
             mode: Optional[str] = None, dev_view: Optional[str] = None, pl=None, alloc_sink=None) -> None:
        """One admission. ``record``: True for a timed step (goes into ``rec``),
        a StepRecords a comparison row collects its steps in, or False (warm-up);
        ``alloc_sink``: a list a comparison collects the allocation outcome in; the
        other keywords override the run's --container-runtime / --settle /
        --container-mode / --dev-view and the plugin admitted against."""
        from rocm_k8s_device_plugin_amd.container_runtime import wait_kfd_released
        a_, d, n, rec = self.args, self.d, self.n, self.rec
        runtime = runtime or a_.container_runtime
        settle = settle or a_.settle
        mode = mode or a_.container_mode
        dev_view = dev_view or a_.dev_view
        adm = None
        if d.rank == 0:
            pl = pl or self.plug
            adm, payload = self._admit(pl)
        else:
            payload = None
        t0, ordl, tot, amsl, ids, mounts, groups, pre_ms = d.bcast(payload)
        mine, lingering = self._container(runtime, mode, dev_view, ordl, mounts, groups)
        into = rec if record is True else (record or None)
        if record is True:   # the containers are up: does the bench / plugin process hold the GPU?
            st_now = process_gpu_state()
            self.gpu_state["torch_cuda_initialized"] |= st_now["torch_cuda_initialized"]
            self.gpu_state["kfd_fds"] = max(self.gpu_state["kfd_fds"], st_now["kfd_fds"])
            self.gpu_state["render_fds"] = max(self.gpu_state["render_fds"], st_now["render_fds"])
        allr = d.gather(mine)
        if d.rank == 0:
            # the allocator's outcome for this admission, read once the pod is up (the
            # native daemon reports it in its log: waiting for that must not delay the pod)
            st = pl.allocator.stats
            a_rec = (adm.preferred_ms, bool(st.last_short_circuit), int(st.last_candidates),
                     sorted(adm.device_ids), adm.preferred_used)
            if into is not None:
                into.alloc.append(a_rec)
            if alloc_sink is not None:
                alloc_sink.append(a_rec)
        bad = [m[3] for m in allr if not m[0]]
        if bad:
            raise SystemExit(f"container failed to become ready: {bad[0]}")
        slowest = max(allr, key=lambda m: m[1])
        t_ready = slowest[1]
        if d.rank == 0:
            pl.kubelet.release("amd.com/gpu", ids)
        # pod termination: the driver finishes tearing down each container's kfd
        # process ~150 ms after it exits (the latency excludes this wait). N
        # containers exiting together may be torn down one after another: allow
        # ~0.25 s each (measured ~0.15 s), capped so a stuck entry cannot stall the run
        cap = min(3.0, 0.25 + 0.25 * max(len(lingering), n))  # one process with N GPUs tears down N VMs
        waited = self._blocking(wait_kfd_released, lingering, timeout_s=cap) if settle == "kfd" else 0.0
        # spawn, main(), GPU runtime ready (CLOCK_MONOTONIC), set-up ms, phases, counters
        sp, tm, trt, su, dph, (syscr, cpu_rt, hsa_ms, cache_opens, kfd_ms, foreign) = slowest[4]
        lat = (t_ready - t0) / 1e6
        if into is None:
            return
        rec = into
        dev = (t_ready - trt) / 1e6
        if syscr is not None:
            rec.read_syscalls.append(syscr)
        if cpu_rt is not None:
            rec.cpu_ms_runtime.append(cpu_rt)
        rec.hsa_init_ms.append(hsa_ms or 0.0)
        rec.kfd_open_ms.append(kfd_ms or 0.0)
        rec.kfd_foreign_exits.append(foreign or 0)
        if cache_opens is not None:
            rec.node_cache_opens.append(cache_opens)
        rec.settle_ms.append(waited)
        rec.latency_ms.append(lat)
        rec.rpc_ms.append(tot)
        rec.allocate_rpc_ms.append(amsl)
        rec.prestart_rpc_ms.append(pre_ms)
        rec.ready_ms.append(lat - tot)
        rec.kernel_us.append(max(m[2] for m in allr))
        rec.exec_ms.append((tm - sp) / 1e6)
        rec.runtime_ms.append((trt - tm) / 1e6)
        rec.device_ms.append(dev)
        rec.setup_ms.append(min(su, dev))
        rec.launch_ms.append(max(0.0, dev - su))
        rec.device_phases.append(dph)
        rec.prespawn_ms.append(max(0.0, (sp - t0) / 1e6 - tot))

    # ------------------------------------------------------------------ report
    def timed_report(self) -> dict:
        """Rank 0: the timed steps' numbers for extra (latency, RPCs, phases, tail)."""
        rec, a_ = self.rec, self.args
        return {
            "plugin_rpc_p50_ms": round(pct(rec.rpc_ms, .5), 4), "plugin_rpc_p99_ms": round(pct(rec.rpc_ms, .99), 4),
            "allocate_rpc_p50_ms": round(pct(rec.allocate_rpc_ms, .5), 4),
            # kubelet's PreStartContainer when the plugin requires it (-prestart_liveness: a probe of the GPUs)
            "prestart_rpc_p50_ms": (round(pct(rec.prestart_rpc_ms, .5), 4)
                                    if any(x > 0 for x in rec.prestart_rpc_ms) else None),
            "container_start_to_ready_p50_ms": round(pct(rec.ready_ms, .5), 3),
            "latency_p99_ms": round(pct(rec.latency_ms, .99), 3),
            "latency_mean_ms": round(statistics.mean(rec.latency_ms), 3) if rec.latency_ms else None,
            "container_runtime": a_.container_runtime,
            "settle": a_.settle,
            "settle_wait_p50_ms": round(pct(rec.settle_ms, .5), 2) if rec.settle_ms else None,
            "container_mode": a_.container_mode,
            "container_dev_view": a_.dev_view,
            "mfma_kernel_us_p50": round(pct(rec.kernel_us, .5), 2),
            # per timed step, for tail analysis: latency, runtime init, settle wait before the next step
            "steps_ms": [[round(x, 2), round(y, 2), round(z, 1)]
                         for x, y, z in zip(rec.latency_ms, rec.runtime_ms, rec.settle_ms)],
            # exec_and_library_load: fork/exec + the dynamic loader (HIP: libamdhip64 and its
            # constructors, before main); gpu_runtime_init: hipGetDeviceCount (hipInit, ROCr start-up;
            # HSA: hsa_init); device_setup: hipSetDevice .. stream, buffers, events (HSA: queue, code
            # object, buffers); launch_and_verify: first launch to the verified MFMA tile
            "container_phases_p50_ms": {"exec_and_library_load": round(pct(rec.exec_ms, .5), 3),
                                        "gpu_runtime_init": round(pct(rec.runtime_ms, .5), 3),
                                        "device_setup": round(pct(rec.setup_ms, .5), 3),
                                        "launch_and_verify": round(pct(rec.launch_ms, .5), 3)},
            # device_setup + launch_and_verify of the slowest GPU, as the container entrypoint timed them
            # (HIP: hipSetDevice + identity, stream = its hardware queue, pinned / device buffers + events,
            # launch -> verified tile; HSA: code object, queue, buffers, dispatch)
            "device_phases_p50_us": {k: round(pct([p[k] for p in rec.device_phases if k in p], .5), 1)
                                     for k in sorted({k for p in rec.device_phases for k in p})},
            # every timed step above 1.5 x p50, attributed to the admission phase with the largest excess
            "tail_attribution": tail_attribution(rec.latency_ms, rec.phases(), details=rec.details()),
            # the containers' own start-up counters (read syscalls, CPU ms): what a comparison row's
            # view or runtime changes deterministically, next to its wall-clock time
            "container_counters_p50": rec.counters(),
        }
