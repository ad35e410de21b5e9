#!/usr/bin/env python3
"""Headline benchmark: p50 Allocate->ContainerReady latency at N advertised MI355X GPUs.

Metric and config come from BASELINE.json ("p50 Allocate→ContainerReady latency;
GPUs advertised at 1/2/4/8 MI355X"). One timed step is one pod admission:

  1. (rank 0) the fake kubelet runs kubelet's devicemanager sequence against
     the real device plugin over UDS gRPC: GetPreferredAllocation for a pod
     requesting amd.com/gpu=N out of the N advertised devices, then Allocate;
  2. the DeviceSpecs in the Allocate response are turned into a "container":
     one fresh process (rank 0) whose /dev/dri holds exactly the allocated
     nodes (--dev-view specs: opens of any other render node fail as in a
     container, so ROCr initialises only the pod's GPUs; container_runtime.py)
     (--container-mode pod, what kubelet starts for a
     pod), or one process per allocated GPU, one per rank, like a torchrun
     workload inside the pod would start (--container-mode per-gpu; reported
     as a comparison at N > 1);
  3. the container initialises the GPU runtime and runs the gfx950 MFMA
     liveness kernel on each of its GPUs (parallel host threads); it is
     "ready" when every tile verifies bit-exactly;
  4. latency = (last container ready) - (kubelet starts GetPreferredAllocation),
     both on CLOCK_MONOTONIC;
  5. (untimed in the latency, inside the timed loop) the pod terminates: its
     processes exit and the driver tears down their kfd processes. The next
     admission starts once /sys/class/kfd/kfd/proc no longer lists them
     (--settle kfd); with --settle none it would start inside that teardown and
     block ~100-150 ms in open("/dev/kfd") (profiles/archive/measurements_r1_r3.md §3c) — reported
     as latency_p50_ms_back_to_back.

The plugin is the real one: by default the native daemon mi355x-device-plugin
(the primary entrypoint: real /sys discovery, C++ allocator and gRPC server;
--plugin python runs the Python CLI's plugin instead); only kubelet and the
CRI runtime are stand-ins (see rocm_k8s_device_plugin_amd/testing/
fake_kubelet.py, container_runtime.py).

  python bench.py --gpus N --steps K --warmup W
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "p50 Allocate→ContainerReady latency; GPUs advertised at 1/2/4/8 MI355X"
STUB_PROBE = os.path.join(REPO, "rocm_k8s_device_plugin_amd", "testing", "stub_probe.py")


def make_parser():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sysfs-root", default="/sys")
    ap.add_argument("--dev-root", default="/dev")
    ap.add_argument("--fixture", action="store_true",
                    help="CPU-only: synthetic 8x MI355X sysfs, containers are no-op processes")
    ap.add_argument("--container-timeout", type=float, default=120.0)
    ap.add_argument("--container-runtime", default="hip", choices=["hip", "hsa"],
                    help="how the container entrypoint reaches the GPU: hip = a HIP program (BASELINE.md: the "
                         "container finishes HIP init and one MFMA liveness kernel; the headline), hsa = the "
                         "same kernel launched through ROCr directly (no libamdhip64, no HIP device set-up)")
    ap.add_argument("--runtime-compare", type=int, default=-1,
                    help="admissions with the other --container-runtime after the timed loop, reported for "
                         "comparison (-1 = as many as --steps; 0 = off)")
    ap.add_argument("--settle", default="kfd", choices=["kfd", "none"],
                    help="between admissions wait until the previous containers' kfd processes are torn down "
                         "(the previous pod has terminated) or start the next one immediately")
    ap.add_argument("--container-mode", default="pod", choices=["pod", "per-gpu"],
                    help="pod: ONE container process gets all N allocated GPUs (rank 0 starts it; what kubelet "
                         "does for a pod); per-gpu: each rank starts a process for its GPU (torchrun-style workload)")
    ap.add_argument("--mode-compare", type=int, default=5,
                    help="for N > 1: extra untimed admissions in the other --container-mode, reported for comparison")
    ap.add_argument("--node-view-compare", type=int, default=5,
                    help="extra untimed admissions with the plugin's -node_view mounts applied to the containers "
                         "(by path redirection: no root for bind mounts), reported for comparison")
    ap.add_argument("--dev-view", default="specs", choices=["specs", "visible-devices"],
                    help="container GPU visibility: specs = the container's /dev holds exactly the Allocate "
                         "DeviceSpecs (ROCr skips the other GPUs' render nodes, as in a real container); "
                         "visible-devices = every host GPU openable, restricted with ROCR_VISIBLE_DEVICES")
    ap.add_argument("--visibility-compare", type=int, default=5,
                    help="extra untimed admissions with the other --dev-view, reported for comparison")
    ap.add_argument("--b2b-compare", type=int, default=5,
                    help="extra untimed admissions with --settle none, reported for comparison")
    ap.add_argument("--throughput-check", type=int, default=1,
                    help="after the timed steps, the throughput check (HBM pattern bandwidth, bf16 MFMA rate, "
                         "per-XCD clocks) on the advertised GPUs, reported in extra.gpu_throughput (1 = on)")
    ap.add_argument("--peer-check", type=int, default=1,
                    help="after the timed loop, DMA-copy + verify over every pair of the N GPUs' links (H2); "
                         "reported in extra.peer_probe, never part of the metric")
    ap.add_argument("--collectives", type=int, default=1,
                    help="for N > 1: after the timed loop, verify + time RCCL all-reduce / all-gather / "
                         "reduce-scatter / all-to-all on the N ranks' GPUs (parallel/collectives.py); "
                         "reported in extra.rccl next to the allocated set's xGMI fabric bound, never part of the metric")
    ap.add_argument("--collective-sizes", default="",
                    help="per-rank bytes for --collectives (default 1M,64M,256M on GPUs, 64K on CPU)")
    ap.add_argument("--health-pulse", type=float, default=0.0,
                    help="> 0: run the plugin as the health DaemonSet does (MFMA liveness via the kept-queue probe "
                         "server, amd-smi ECC / events / xGMI link state) with this pulse in seconds, while pods "
                         "are admitted (BASELINE config: health-check DaemonSet enabled)")
    ap.add_argument("--advertise", type=int, default=0,
                    help="advertise M devices and request --gpus N of them per pod (default M = N: the headline, "
                         "'GPUs advertised at N'). With M > N the timed admissions start from a fragmented "
                         "availability (--hold devices held by other pods), so GetPreferredAllocation searches")
    ap.add_argument("--hold", type=int, default=-1,
                    help="with M > N: devices held by other pods during the run (default (M-N)//2, alternating "
                         "positions so every hive is fragmented)")
    ap.add_argument("--fragmented-compare", type=int, default=5,
                    help="with M = N and more accessible devices than N: extra untimed admissions of N out of "
                         "every accessible device from a fragmented availability (a second plugin instance), "
                         "reported in extra.fragmented_n_of_m (BASELINE config: full-node hive-aware allocation)")
    ap.add_argument("--plugin", default="native", choices=["native", "python"],
                    help="the device plugin under test: native = the mi355x-device-plugin daemon (the primary "
                         "entrypoint, what ./k8s-device-plugin runs); python = the Python CLI's plugin in this "
                         "process (--grpc-server picks its transport; used automatically with --health-pulse)")
    ap.add_argument("--grpc-server", default="native", choices=["native", "aio"],
                    help="with --plugin python: the plugin's kubelet-facing gRPC server (-grpc_server)")
    ap.add_argument("--kubelet-client", default="", choices=["", "native", "native-thread", "aio"],
                    help="the fake kubelet's admission RPC client: native (a native HTTP/2 client, like kubelet's "
                         "grpc-go) or aio (grpc.aio in the bench's event loop); default native with the native server")
    ap.add_argument("--extras-deadline", type=float, default=300.0,
                    help="seconds after the timed loop for every secondary measurement (comparisons, RCCL, peer "
                         "probe, throughput check); past it rank 0 prints the headline line with what it has and "
                         "every rank exits 0, so a hung extra cannot take the measured headline with it (0 = none)")
    ap.add_argument("--json-out", default="")
    return ap


def parse_args(argv=None):
    return make_parser().parse_args(argv)


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


class _AllocStats:
    last_short_circuit = False
    last_candidates = -1


class _DaemonAllocator:
    """The daemon's allocator as the bench's microbenchmarks see it: the same
    C++ HiveAllocator on the same devices (BestEffortPolicy, -allocator_search
    auto), plus the last GetPreferredAllocation outcome the daemon logged."""

    def __init__(self, devs, topology, stats):
        from rocm_k8s_device_plugin_amd.allocator import BestEffortPolicy
        self._pol = BestEffortPolicy(extended_search="auto")
        self._pol.init(list(devs), topology)
        self.stats = stats

    @property
    def native(self):
        return self._pol.native

    def reference_allocate(self, *a):
        return self._pol.reference_allocate(*a)


class NativePluginUnderTest:
    """Rank 0: the native daemon mi355x-device-plugin (the primary entrypoint)
    advertising `devs` (-device_ids) behind a fake kubelet on its own UDS dir.
    Its per-RPC records (-log_format json -v 2: server-side latency, the
    allocator's candidates / short-circuit) are read from its stderr."""

    def __init__(self, loop, tmp, name, sysfs, devroot, devs, full, ords, kubelet_client="native", extra=(),
                 metrics_port=0):
        import subprocess
        import threading
        from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
        from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
        self.loop = loop
        self.devs = tuple(devs)
        pdir = os.path.join(tmp, name)
        self.kubelet = FakeKubelet(pdir, rpc_client=kubelet_client)
        loop.run_until_complete(self.kubelet.start())
        self.stats = _AllocStats()
        self.recent = {}
        self._cv = threading.Condition()
        self._allocates_seen = 0
        self._allocates_made = 0
        exe = os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")
        self.metrics_port = metrics_port
        if metrics_port:
            extra = (*extra, "-metrics_port", str(metrics_port))
        self.proc = subprocess.Popen(
            [exe, "-kubelet_dir", pdir, "-sysfs_root", sysfs, "-dev_root", devroot, "-exporter_socket", "",
             "-device_ids", ",".join(dv.id for dv in self.devs), "-log_format", "json", "-v", "2", *extra],
            stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        self._reader = threading.Thread(target=self._read, daemon=True)
        self._reader.start()
        admit = self.kubelet.admit

        async def counted_admit(*a, **kw):
            r = await admit(*a, **kw)
            with self._cv:
                self._allocates_made += 1
            return r
        self.kubelet.admit = counted_admit
        loop.run_until_complete(self.kubelet.wait_for_resource("amd.com/gpu", len(self.devs), timeout=30))
        self._alloc = _DaemonAllocator(self.devs, full.topology, self.stats)
        self.minor_to_ord = {dv.render_minor: ords[dv.id] for dv in self.devs}
        self.minor_to_paths = {dv.render_minor: dv.dev_paths() for dv in self.devs}
        self.held = []

    def _read(self):
        for line in self.proc.stderr:
            try:
                r = json.loads(line)
            except ValueError:
                continue
            if r.get("msg") != "rpc":
                continue
            with self._cv:
                self.recent.setdefault(r["rpc"], []).append(float(r["latency_ms"]))
                if r["rpc"] == "GetPreferredAllocation" and "candidates" in r:
                    self.stats.last_candidates = int(r["candidates"])
                    self.stats.last_short_circuit = r.get("short_circuit") == "True"
                if r["rpc"] == "Allocate":
                    self._allocates_seen += 1
                    self._cv.notify_all()

    def sync(self, timeout=2.0):
        """Wait until the daemon has logged every Allocate the kubelet made."""
        with self._cv:
            self._cv.wait_for(lambda: self._allocates_seen >= self._allocates_made, timeout)

    def hold(self, ids):
        self.kubelet.resources["amd.com/gpu"].allocated.update(ids)
        self.held = list(ids)

    @property
    def allocator(self):
        self.sync()
        return self._alloc

    def server_ms(self, reset=False):
        self.sync()
        with self._cv:
            out = {rpc: list(v) for rpc, v in self.recent.items()}
            if reset:
                self.recent.clear()
        return out

    def available(self):
        return self.kubelet.healthy_free("amd.com/gpu")

    def metrics(self) -> dict:
        """The daemon's /metrics as {series name (with labels): value}."""
        import urllib.request
        if not self.metrics_port:
            return {}
        with urllib.request.urlopen(f"http://127.0.0.1:{self.metrics_port}/metrics", timeout=5) as r:
            text = r.read().decode()
        out = {}
        for line in text.splitlines():
            if line and not line.startswith("#"):
                k, _, v = line.rpartition(" ")
                try:
                    out[k] = float(v)
                except ValueError:
                    pass
        return out

    def health_report(self, pulse_s) -> dict:
        """The health DaemonSet loop as the daemon reports it (/metrics) and as
        kubelet sees it (the ListAndWatch device table)."""
        m = self.metrics()
        n = int(m.get("mi355x_dp_health_sweep_seconds_count", 0))
        st = self.kubelet.resources.get("amd.com/gpu")
        return {"plugin": "native-daemon", "pulse_s": pulse_s, "sweeps": n,
                "sweep_ms_mean": round(m.get("mi355x_dp_health_sweep_seconds_sum", 0.0) * 1e3 / n, 3) if n else None,
                "health_changes": int(m.get("mi355x_dp_health_changes_total", 0)),
                "unhealthy": sorted(d for d, h in (st.devices.items() if st else ()) if h != "Healthy")}

    def stop(self):
        import signal
        self.loop.run_until_complete(self.kubelet.stop())
        if self.proc.poll() is None:
            self.proc.send_signal(signal.SIGTERM)
        try:
            self.proc.wait(timeout=20)
        except Exception:  # noqa: BLE001
            self.proc.kill()
            self.proc.wait()
        self._reader.join(timeout=5)


class PluginUnderTest:
    """Rank 0: the Python CLI's plugin advertising `devs` (real discovery data,
    real allocator and gRPC servicer) behind a fake kubelet on its own UDS dir."""

    def __init__(self, loop, tmp, name, sysfs, devs, full, ords, hcfg, pulse_s, grpc_server="native",
                 kubelet_client="native"):
        from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
        from rocm_k8s_device_plugin_amd.plugin.manager import ManagerConfig, PluginManager
        from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
        from rocm_k8s_device_plugin_amd.topology import Inventory
        self.loop = loop
        self.devs = tuple(devs)
        self.inv = Inventory(sysfs_root=sysfs, devices=self.devs, topology=full.topology,
                             driver_loaded=full.driver_loaded, kfd_present=full.kfd_present)
        self.impl = ContainerImpl("single", sysfs, hcfg, inventory=self.inv)
        pdir = os.path.join(tmp, name)
        self.kubelet = FakeKubelet(pdir, rpc_client=kubelet_client)
        loop.run_until_complete(self.kubelet.start())
        self.mgr = PluginManager(self.impl, ManagerConfig(pulse_s=pulse_s, plugin_dir=pdir, handle_signals=False,
                                                          grpc_server=grpc_server))
        self.task = loop.create_task(self.mgr.run())
        loop.run_until_complete(self.kubelet.wait_for_resource("amd.com/gpu", len(self.devs), timeout=30))
        self.minor_to_ord = {dv.render_minor: ords[dv.id] for dv in self.devs}
        self.minor_to_paths = {dv.render_minor: dv.dev_paths() for dv in self.devs}
        self.held = []

    def hold(self, ids):
        """Mark `ids` allocated to other pods (kubelet's view: not available)."""
        self.kubelet.resources["amd.com/gpu"].allocated.update(ids)
        self.held = list(ids)

    @property
    def allocator(self):
        self.mgr.plugins["gpu"].sync()     # native server: apply its pending call events first
        return self.mgr.plugins["gpu"].ctx.allocator

    def server_ms(self, reset=False):
        """Native server: server-side time per RPC (request read -> response queued)."""
        p = self.mgr.plugins["gpu"]
        p.sync()
        if p.native is None:
            return {}
        out = {rpc: list(q) for rpc, q in p.native.recent_ms.items()}
        if reset:
            p.native.recent_ms.clear()
        return out

    def available(self):
        return self.kubelet.healthy_free("amd.com/gpu")

    def stop(self):
        self.loop.run_until_complete(self.kubelet.stop())
        self.mgr.request_stop()
        self.loop.run_until_complete(self.task)


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def throughput_check(ordinals) -> dict:
    """The health monitor's throughput check on the pod's GPUs, once, after the
    timed steps (context for the latency numbers: what the GPUs deliver)."""
    import subprocess
    from rocm_k8s_device_plugin_amd.ops.native import probe_executable
    env = {k: v for k, v in os.environ.items() if k not in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
    env["ROCR_VISIBLE_DEVICES"] = ",".join(str(o) for o in ordinals)
    try:
        p = subprocess.run([str(probe_executable("hsa")), "--perf", "--perf-mib", "4096", "--perf-iters", "65536",
                            "--devices", "all", "--timeout", "30"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           env=env, timeout=120)
        devs = json.loads(p.stdout.decode().strip().splitlines()[-1])["devices"]
    except Exception as e:  # noqa: BLE001 -- context only, never fails the run
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    keys = ("ok", "hbm_write_gbps", "hbm_read_gbps", "hbm_bad_words", "mfma_tflops", "clock_mhz_median",
            "xcd_clock_mhz", "error")
    return {"bytes": 4 << 30, "mfma_pairs_per_wave": 65536,
            "devices": [{"ordinal": o, **{k: d.get(k) for k in keys}} for o, d in zip(ordinals, devs)]}


class Dist:
    """Rank coordination for the bench. The measured thing is a kubelet node
    admitting pods, and a kubelet node has no resident GPU process: the bench
    and plugin processes must not hold a GPU context, kfd queues or an RCCL
    communicator while containers initialise their GPUs. So:

    * step barriers and object exchange run over gloo (CPU, TCP) under torchrun;
      at world = 1 nothing is initialised and torch is not even imported;
    * ``sync()`` synchronises the GPU only if this process already has a HIP
      context (it never creates one); the containers' GPU work is complete by
      construction when a step ends (ready = every MFMA tile verified);
    * RCCL is created only after the timed loop, for the collectives extra
      (``rccl_group()``).
    """

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.launcher = "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ or self.world > 1 else "single-process"
        self.torch = None
        self.dist = None
        self.cuda = False   # this process drives a GPU (only ever for the RCCL extra)
        if self.world > 1:
            import torch
            import torch.distributed as dist
            self.torch, self.dist = torch, dist
            dist.init_process_group("gloo")

    def sync(self):
        if self.world > 1:
            self.dist.barrier()
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_initialized():
            torch.cuda.synchronize()

    def rccl_group(self):
        """After the timed loop: (group, on_gpu) for the collectives extra, one
        rank per GPU over RCCL when GPUs are visible, else the gloo group."""
        torch, dist = self.torch, self.dist
        if not torch.cuda.is_available():
            return None, False
        torch.cuda.set_device(self.local_rank)
        self.cuda = True
        return dist.new_group(backend="nccl", device_id=torch.device("cuda", self.local_rank)), True

    def bcast(self, obj):
        if self.world == 1:
            return obj
        box = [obj]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]

    def gather(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def max(self, x: float) -> float:
        return max(self.gather(x))

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


class ExtrasGuard:
    """Bounds the secondary measurements that follow the timed loop.

    Everything after the timed loop (comparison admissions, RCCL collectives,
    the xGMI peer probe, the throughput check) is context, not the metric, and
    some of it runs code that can hang on a sick node (an RCCL communicator, a
    DMA that never completes). The headline is complete when the timed loop
    ends, so a timer armed there bounds the rest: when it fires, or when a
    stage raises (its own failure, or a peer rank that already left), rank 0 prints
    the headline line with ``extra.extras_incomplete`` naming the stage that
    was running, and every rank leaves with status 0 (``os._exit``: a thread
    stuck in a collective cannot be joined). Exactly one line is printed
    whichever path gets there first."""

    def __init__(self, rank: int, deadline_s: float):
        import threading
        self.rank, self.deadline_s = rank, deadline_s
        self.stage = "start"
        self.fallback = None          # rank 0: (error) -> the headline line without the unfinished extras
        self._lock = threading.Lock()
        self._printed = False
        self._written = threading.Event()   # the printed line (and --json-out) is complete
        self._timer = None
        self._plugins = []            # plugin daemons to SIGKILL when the timer fires (no orphans)
        self.tmp = None               # rank 0's scratch directory (sockets, logs, fixture tree)
        if deadline_s > 0:
            # ranks > 0 leave a little later, so rank 0's line is out first
            self._timer = threading.Timer(deadline_s + (0 if rank == 0 else 5.0), self._fire)
            self._timer.daemon = True
            self._timer.start()

    def enter(self, stage: str) -> None:
        self.stage = stage

    def kill_on_fire(self, plugin) -> None:
        self._plugins.append(plugin)

    def emit(self, line: str, json_out: str = "") -> bool:
        """Print the JSON line (and write it to ``json_out``) unless the other
        path already has; True if written here. Whoever wins writes both, so
        stdout and --json-out always carry the same line."""
        with self._lock:
            if self._printed:
                return False
            self._printed = True
        try:
            data = memoryview((line + "\n").encode())
            while data:   # a blocking pipe can still take a large line in parts
                data = data[os.write(1, data):]
            if json_out:
                with open(json_out, "w") as f:
                    f.write(line + "\n")
        finally:
            self._written.set()
        return True

    def _fire(self) -> None:
        self.abandon(None)

    def abandon(self, error) -> None:
        """Leave now: rank 0 prints the headline line (unless it already has)
        with the unfinished stage, plugin daemons are killed, exit status 0.
        ``error`` is None when the deadline passed, else why the stage failed."""
        why = (f"exceeded --extras-deadline {self.deadline_s:g}s" if error is None else f"failed: {error}")
        msg = f"bench: secondary measurements {why} in stage '{self.stage}'"
        if self.rank == 0 and self.fallback is not None:
            with self._lock:
                printed = self._printed
            if printed:
                # the full line is out or being written by the main thread: let it finish
                self._written.wait(10.0)
                msg = f"bench: {why} in stage '{self.stage}' after the headline line was written"
            else:
                try:
                    self.emit(*self.fallback(error))
                except Exception as e:  # noqa: BLE001
                    msg += f"; headline line failed: {type(e).__name__}: {e}"
        for pl in self._plugins:
            proc = getattr(pl, "proc", None)
            if proc is not None and proc.poll() is None:
                try:
                    proc.kill()
                except OSError:
                    pass
        if self.tmp:
            import shutil
            shutil.rmtree(self.tmp, ignore_errors=True)
        try:
            sys.stdout.flush()
            os.write(2, (msg + "\n").encode())
        finally:
            os._exit(0)

    def cancel(self) -> None:
        if self._timer is not None:
            self._timer.cancel()


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


def tail_attribution(lat, phases, factor=1.5) -> dict:
    """Every step slower than factor x p50: which phase carries the excess.
    ``phases`` maps a phase name to its per-step ms (aligned with ``lat``); a
    slow step is attributed to the phase with the largest excess over its own
    p50."""
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
        slow.append({"step": i, "latency_ms": round(x, 2), "phase": top, "excess_ms": excess})
    return {"threshold_ms": round(factor * p50, 2), "p99_over_p50": round(pct(lat, .99) / p50, 3) if p50 else None,
            "phase_p50_ms": {k: round(v, 3) for k, v in med.items()},
            "slow_steps": slow,
            "by_phase": {k: {"steps": len(v), "excess_ms_mean": round(statistics.mean(v), 2)}
                         for k, v in sorted(by_phase.items())}}


def main():
    args = parse_args()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    d = Dist()
    n = args.gpus
    if d.world > 1 and d.world != n:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE {d.world}: launch one rank per GPU")

    from rocm_k8s_device_plugin_amd import _build
    if d.rank == 0:
        _build.ensure_built(hip=not args.fixture)
    d.sync()

    from rocm_k8s_device_plugin_amd.container_runtime import render_minors_from_specs, start_container

    loop = None
    plug = impl = None
    plugin_kind = None
    tmp = None
    m_adv = args.advertise or n
    if m_adv < n:
        raise SystemExit(f"--advertise {m_adv} < --gpus {n}")
    if d.rank == 0:
        from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
        from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals
        from rocm_k8s_device_plugin_amd.utils import log as ulog
        ulog.setup(0)
        import logging
        logging.getLogger("mi355x").setLevel(logging.WARNING)

        tmp = tempfile.mkdtemp(prefix="mi355x-bench-")
        sysfs, devroot = args.sysfs_root, args.dev_root
        if args.fixture:
            from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
            fi = make_mi355x_node(os.path.join(tmp, "node"))
            sysfs, devroot = str(fi.sysfs), str(fi.dev)
        full = discover(sysfs)
        ords = hip_ordinals(full, devroot, check_access=not args.fixture)
        usable = sorted((dv for dv in full.devices if dv.id in ords), key=lambda dv: ords[dv.id])
        if len(usable) < m_adv:
            raise SystemExit(f"only {len(usable)} accessible GPU devices on this node, need {m_adv}")
        adv = tuple(usable[:m_adv])     # "GPUs advertised at N" (or M with --advertise)
        adv_ordinals = [ords[dv.id] for dv in adv]
        # the Python plugin's health loop needs a GPU; the daemon's runs on the fixture with its sysfs sources
        hp = args.health_pulse if not args.fixture or args.plugin == "native" else 0.0
        hcfg = (HealthConfig(exporter_socket=None, liveness=True, smi_ecc=True, smi_events=True, smi_xgmi=True)
                if hp > 0 else HealthConfig(exporter_socket=None))
        loop = asyncio.new_event_loop()
        plugin_kind = "native-daemon" if args.plugin == "native" else "python"
        # the health DaemonSet variant (k8s-ds-amdgpu-dp-health.yaml: -pulse=2 plus the MFMA liveness
        # probe server and amd-smi ECC / events / xGMI) on the daemon; -pulse is whole seconds
        health_flags = ()
        if hp > 0 and plugin_kind == "native-daemon":
            health_flags = ("-pulse", str(max(1, int(round(hp)))),
                            *(() if args.fixture else ("-liveness", "-smi_ecc", "-smi_events", "-smi_xgmi")))

        def make_plugin(name, devs, extra=()):
            if plugin_kind == "native-daemon":
                main_plugin = name == "device-plugins"
                return NativePluginUnderTest(loop, tmp, name, sysfs, devroot, devs, full, ords,
                                             kubelet_client=kclient,
                                             extra=(*extra, *(health_flags if main_plugin else ())),
                                             metrics_port=free_port() if main_plugin and health_flags else 0)
            return PluginUnderTest(loop, tmp, name, sysfs, devs, full, ords,
                                   hcfg if name == "device-plugins" else HealthConfig(exporter_socket=None),
                                   hp if name == "device-plugins" else 0.0, grpc_server=args.grpc_server,
                                   kubelet_client=kclient)
        grpc_native = plugin_kind == "native-daemon" or args.grpc_server == "native"
        kclient = args.kubelet_client or ("native" if grpc_native else "aio")
        if kclient == "native" and not grpc_native:
            kclient = "native-thread"   # a blocking call on the loop that serves grpc.aio would deadlock
        plug = make_plugin("device-plugins", adv)
        impl = getattr(plug, "impl", None)
        inv = getattr(plug, "inv", None) or full
        if m_adv > n:
            plug.hold(fragment([dv.id for dv in adv], n, args.hold))
        gpu_info = {"ids": [dv.id for dv in adv], "gfx_target_version": sorted({dv.gfx_target_version for dv in adv}),
                    "hive_ids": sorted({str(dv.hive_id) for dv in adv}),
                    "partition": sorted({dv.partition_type for dv in adv})}
    else:
        gpu_info = None

    rpc_ms, alloc_rpc_ms, lat_ms, ready_ms, kern_us = [], [], [], [], []
    exec_ms, rt_ms, dev_ms, settle_ms, prespawn_ms, setup_ms, launch_ms = [], [], [], [], [], [], []
    dev_phases = []   # per timed step: the slowest device's set-up phases (probe phase_us)
    gpu_state = {"torch_cuda_initialized": False, "kfd_fds": 0, "render_fds": 0}   # worst seen in the timed loop
    from rocm_k8s_device_plugin_amd.container_runtime import wait_kfd_released

    def blocking(fn, *a, **kw):
        """Run fn; with the health loop on, on a worker thread while rank 0's
        event loop keeps sweeping (so sweeps overlap the container start)."""
        if loop is not None and args.health_pulse > 0 and not args.fixture and plugin_kind == "python":
            import functools
            return loop.run_until_complete(asyncio.to_thread(functools.partial(fn, *a, **kw)))
        return fn(*a, **kw)

    alloc_steps = []   # per timed admission: (preferred RPC ms, short-circuit, candidates, chosen set)

    def one_step(record: bool, runtime: str = args.container_runtime, sink=None, settle: str = args.settle,
                 init_sink=None, mode: str = args.container_mode, dev_view: str = args.dev_view, pl=None,
                 alloc_sink=None):
        if d.rank == 0:
            pl = pl or plug
            t0 = time.monotonic_ns()
            adm = loop.run_until_complete(pl.kubelet.admit("amd.com/gpu", n))
            car = adm.response.container_responses[0]
            minors = render_minors_from_specs(car)
            ordl = [pl.minor_to_ord[m] for m in minors]
            mounts = [(m.container_path, m.host_path) for m in car.mounts]
            # the container's /dev: the DeviceSpecs, per allocated GPU (card + render node)
            spec_paths = {ds.host_path for ds in car.devices}
            groups = [[p for p in pl.minor_to_paths[m] if p in spec_paths] for m in minors]
            payload = (t0, ordl, adm.total_ms, adm.allocate_ms, list(adm.device_ids), mounts, groups)
        else:
            payload = None
        payload = d.bcast(payload)
        t0, ordl, tot, amsl, ids, mounts, groups = payload
        if mode == "pod" and d.rank != 0:
            # the pod's single container runs on rank 0; other ranks only keep step
            mine = (True, 0, 0.0, "", (0, 0, 0, 0.0, {}))
            lingering = frozenset()
        else:
            pod = mode == "pod" or d.world == 1
            mine_ord = ordl if pod else [ordl[d.rank]]
            paths = None
            if dev_view == "specs":
                paths = ["/dev/kfd"] + [p for g in (groups if pod else [groups[d.rank]]) for p in g]
            # CPU rehearsal (--fixture): the stub probe stands in for the GPU entrypoint,
            # through the same runtime path (/dev view, per-GPU split, result parsing)
            stub = dict(exe=STUB_PROBE, argv_prefix=[sys.executable]) if args.fixture else {}
            r = blocking(start_container, mine_ord, timeout_s=args.container_timeout, runtime=runtime,
                         mounts=mounts if not args.fixture else (), device_paths=paths, **stub)
            kus = max((dv.get("kernel_us", 0.0) for dv in r.doc.get("devices", [])), default=0.0)
            # device set-up (HIP: hipSetDevice .. stream/buffers/events; HSA: queue, code object, buffers)
            devs = r.doc.get("devices", [])
            sus = max((dv.get("setup_us", 0.0) for dv in devs), default=0.0)
            slow_dev = max(devs, key=lambda dv: dv.get("total_us", 0.0), default={})
            phases = (r.t_start_ns, int(r.doc.get("t_start_ns", 0)), int(r.doc.get("t_runtime_ns", 0)), sus / 1e3,
                      slow_dev.get("phase_us") or {})
            mine = (r.ok, r.t_ready_ns, kus, r.error, phases)
            lingering = r.kfd_lingering
        if record:   # the containers are up: does the bench / plugin process hold the GPU?
            st_now = process_gpu_state()
            gpu_state["torch_cuda_initialized"] |= st_now["torch_cuda_initialized"]
            gpu_state["kfd_fds"] = max(gpu_state["kfd_fds"], st_now["kfd_fds"])
            gpu_state["render_fds"] = max(gpu_state["render_fds"], st_now["render_fds"])
        allr = d.gather(mine)
        if d.rank == 0:
            # the allocator's outcome for this admission, read once the pod is up (the
            # native daemon reports it in its log: waiting for that must not delay the pod)
            st = pl.allocator.stats
            a_rec = (adm.preferred_ms, bool(st.last_short_circuit), int(st.last_candidates),
                     sorted(adm.device_ids), adm.preferred_used)
            if record:
                alloc_steps.append(a_rec)
            if alloc_sink is not None:
                alloc_sink.append(a_rec)
        bad = [m[3] for m in allr if not m[0]]
        if bad:
            raise SystemExit(f"container failed to become ready: {bad[0]}")
        slowest = max(allr, key=lambda m: m[1])
        t_ready = slowest[1]
        if d.rank == 0:
            pl.kubelet.release("amd.com/gpu", ids)
        # pod termination: the driver finishes tearing down each container's
        # kfd process ~150 ms after it exits (bench latency excludes this wait)
        # N containers exiting together may be torn down one after another: allow
        # ~0.25 s each (measured ~0.15 s), capped so a stuck entry cannot stall the run
        cap = min(3.0, 0.25 + 0.25 * max(len(lingering), n))  # one process with N GPUs tears down N VMs
        waited = blocking(wait_kfd_released, lingering, timeout_s=cap) if settle == "kfd" else 0.0
        if record:
            settle_ms.append(waited)
        sp, tm, trt, su, dph = slowest[4]   # spawn, main(), GPU runtime ready (CLOCK_MONOTONIC), set-up ms, phases
        if sink is not None:
            sink.append((t_ready - t0) / 1e6)
        if init_sink is not None:
            init_sink.append((trt - tm) / 1e6)
        if record:
            lat_ms.append((t_ready - t0) / 1e6)
            rpc_ms.append(tot)
            alloc_rpc_ms.append(amsl)
            ready_ms.append((t_ready - t0) / 1e6 - tot)
            kern_us.append(max(m[2] for m in allr))
            exec_ms.append((tm - sp) / 1e6)
            rt_ms.append((trt - tm) / 1e6)
            dev_ms.append((t_ready - trt) / 1e6)
            setup_ms.append(min(su, (t_ready - trt) / 1e6))
            dev_phases.append(dph)
            launch_ms.append(max(0.0, (t_ready - trt) / 1e6 - su))
            prespawn_ms.append(max(0.0, (sp - t0) / 1e6 - tot))

    for _ in range(args.warmup):
        one_step(False)
    if d.rank == 0:
        plug.server_ms(reset=True)
    d.sync()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        one_step(True)
    d.sync()
    elapsed = time.perf_counter() - t_start
    server_ms = plug.server_ms() if d.rank == 0 else {}
    elapsed = d.max(elapsed)
    rank_gpu_state = d.gather(gpu_state)

    # the headline is measured: from here on everything is bounded by the guard
    guard = ExtrasGuard(d.rank, args.extras_deadline)
    core = {}
    if d.rank == 0:
        guard.kill_on_fire(plug)
        guard.tmp = tmp
        core = {"plugin_rpc_p50_ms": round(pct(rpc_ms, .5), 4), "plugin_rpc_p99_ms": round(pct(rpc_ms, .99), 4),
                "plugin": plugin_kind,
                "grpc_server": "native" if plugin_kind == "native-daemon" else args.grpc_server,
                "kubelet_client": kclient,
                # breakdown of plugin_rpc (kubelet's GetPreferredAllocation + Allocate round trips): the
                # plugin's own time per RPC, measured inside the native server (empty with -grpc_server aio;
                # the daemon's from its per-RPC log records)
                "plugin_server_p50_us": {rpc: round(pct(v, .5) * 1e3, 1) for rpc, v in sorted(server_ms.items())
                                         if rpc in ("GetPreferredAllocation", "Allocate")},
                "allocate_rpc_p50_ms": round(pct(alloc_rpc_ms, .5), 4),
                "container_start_to_ready_p50_ms": round(pct(ready_ms, .5), 3),
                "latency_p99_ms": round(pct(lat_ms, .99), 3), "latency_mean_ms": round(statistics.mean(lat_ms), 3),
                "container_runtime": args.container_runtime,
                "settle": args.settle, "settle_wait_p50_ms": round(pct(settle_ms, .5), 2) if settle_ms else None,
                "container_mode": args.container_mode,
                "container_dev_view": args.dev_view,
                "mfma_kernel_us_p50": round(pct(kern_us, .5), 2),
                # per timed step, for tail analysis: latency, ROCr init, settle wait before the next step
                "steps_ms": [[round(a, 2), round(b, 2), round(c, 1)] for a, b, c in zip(lat_ms, rt_ms, settle_ms)],
                # exec_and_library_load: fork/exec + the dynamic loader (HIP: libamdhip64 and its
                # constructors, before main); gpu_runtime_init: hipGetDeviceCount (hipInit, ROCr start-up;
                # HSA: hsa_init); device_setup: hipSetDevice .. stream, buffers, events (HSA: queue, code
                # object, buffers); launch_and_verify: first launch to the verified MFMA tile
                "container_phases_p50_ms": {"exec_and_library_load": round(pct(exec_ms, .5), 3),
                                            "gpu_runtime_init": round(pct(rt_ms, .5), 3),
                                            "device_setup": round(pct(setup_ms, .5), 3),
                                            "launch_and_verify": round(pct(launch_ms, .5), 3)},
                # device_setup + launch_and_verify of the slowest GPU, as the container entrypoint timed them
                # (HIP: hipSetDevice + identity, stream = its hardware queue, pinned / device buffers + events,
                # launch -> verified tile; HSA: code object, queue, buffers, dispatch)
                "device_phases_p50_us": {k: round(pct([p[k] for p in dev_phases if k in p], .5), 1)
                                         for k in sorted({k for p in dev_phases for k in p})},
                # every timed step above 1.5 x p50, attributed to the admission phase with the largest excess
                "tail_attribution": tail_attribution(lat_ms, {
                    "plugin_rpc": rpc_ms, "runtime_prep": prespawn_ms, "exec_and_library_load": exec_ms,
                    "gpu_runtime_init": rt_ms, "device_setup": setup_ms, "launch_and_verify": launch_ms}),
                # the node under test must look like a kubelet node: no GPU context in the bench /
                # plugin process(es) while the timed containers initialise (worst over the timed steps)
                "launcher": d.launcher,
                "bench_process_gpu": {"ranks": rank_gpu_state,
                                      "clean": not any(s["torch_cuda_initialized"] or s["kfd_fds"]
                                                       for s in rank_gpu_state)},
                "gpus": gpu_info}
        held = list(plug.held)

        def result_line(extra: dict) -> str:
            return json.dumps({
                "metric": METRIC,
                "value": round(pct(lat_ms, .5), 3),
                "unit": "ms",
                "n_gpus": n,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": round(elapsed / max(1, args.steps) * 1e3, 3),
                "higher_is_better": False,
                "scaling": "weak",
                "vs_baseline": None,
                "dtype": "fp32",
                "data": ("synthetic pod specs requesting amd.com/gpu=N; real /sys discovery, fake kubelet over UDS, "
                         "container = fresh process whose /dev is the Allocate DeviceSpecs running the MFMA liveness "
                         "kernel" if not args.fixture else
                         "synthetic 8xMI355X sysfs fixture; stub-probe containers (CPU only)"),
                "config": {"model": "example/pod/alexnet-gpu.yaml-style pod, amd.com/gpu=N",
                           "global_batch": n, "seq_len": None,
                           "parallelism": (f"{m_adv} GPUs advertised, 1 pod requesting {n}, " +
                                           (f"{len(held)} held by other pods, " if held else "") +
                                           ("1 container process with all N GPUs" if args.container_mode == "pod"
                                            else "1 container process per GPU")),
                           "between_admissions": ("previous pod's kfd teardown complete" if args.settle == "kfd"
                                                  else "back-to-back"),
                           "launcher": d.launcher, "plugin": plugin_kind},
                "extra": extra,
            })

        def emit(line: str) -> None:
            guard.emit(line, args.json_out)

        def partial_line(error):
            """(line, json_out) for the guard: the headline without the unfinished extras."""
            return (result_line(dict(core, extras_incomplete={"deadline_s": args.extras_deadline,
                                                              "stage": guard.stage, "error": error})),
                    args.json_out)

        guard.fallback = partial_line

    other_runtime = "hsa" if args.container_runtime == "hip" else "hip"
    rt_key = "rocr_direct_container" if other_runtime == "hsa" else "hip_runtime_container"
    rt_compare_steps = args.steps if args.runtime_compare < 0 else args.runtime_compare

    def extras():
        """The secondary measurements and, on rank 0, the JSON line."""
        rt_lat, b2b_lat, nv_lat, nv_init, other_mode_lat = [], [], [], [], []
        other_mode = "per-gpu" if args.container_mode == "pod" else "pod"
        if n > 1:
            guard.enter("container_mode_compare")
            for _ in range(args.mode_compare):
                one_step(False, sink=other_mode_lat, mode=other_mode)
        if not args.fixture and args.node_view_compare > 0:
            # the plugin returns -node_view mounts (alias = host path: the fake runtime
            # applies mounts by redirection and cannot add the alias mount)
            nvplug = None
            if d.rank == 0:
                node_dir = os.path.join(sysfs, "devices/system/node")
                if plugin_kind == "native-daemon":
                    nvplug = make_plugin("device-plugins-node-view", adv, ["-node_view", "-node_view_alias", node_dir])
                else:
                    from rocm_k8s_device_plugin_amd.node_view import NodeView
                    impl.node_view = NodeView(os.path.join(tmp, "node-view"), sysfs, alias=node_dir)
                    impl.node_view.path()  # built at plugin start-up in a real deployment
            if nvplug is not None:
                guard.kill_on_fire(nvplug)
            guard.enter("node_view_compare")
            for _ in range(args.node_view_compare):
                one_step(False, sink=nv_lat, init_sink=nv_init, pl=nvplug)
            if d.rank == 0:
                if nvplug is not None:
                    nvplug.stop()
                else:
                    impl.node_view = None
        vis_lat = []
        other_view = "visible-devices" if args.dev_view == "specs" else "specs"
        if not args.fixture:
            guard.enter("dev_view_compare")
            for _ in range(args.visibility_compare):
                one_step(False, sink=vis_lat, dev_view=other_view)
        if not args.fixture and rt_compare_steps > 0:
            # the other entrypoint, as many admissions as the headline (same settle, same view)
            guard.enter(f"{other_runtime}_runtime_compare")
            for _ in range(rt_compare_steps):
                one_step(False, runtime=other_runtime, sink=rt_lat)
        if not args.fixture and args.settle == "kfd":
            guard.enter("back_to_back_compare")
            for _ in range(args.b2b_compare):
                one_step(False, sink=b2b_lat, settle="none")

        # N of every accessible device, from a fragmented availability (second plugin
        # instance; the headline plugin keeps advertising exactly N)
        frag = None
        frag_lat, frag_alloc = [], []
        do_frag = d.bcast(d.rank == 0 and m_adv == n and args.fragmented_compare > 0 and len(usable) > n)
        if do_frag:
            fplug = None
            if d.rank == 0:
                fplug = make_plugin("device-plugins-all", usable)
                fplug.hold(fragment([dv.id for dv in usable], n, args.hold))
                guard.kill_on_fire(fplug)
            guard.enter("fragmented_compare")
            for _ in range(args.fragmented_compare):
                one_step(False, sink=frag_lat, pl=fplug, alloc_sink=frag_alloc)
            if d.rank == 0:
                frag = {"advertised": len(usable), "requested": n, "held": fplug.held,
                        "latency_p50_ms": round(pct(frag_lat, .5), 3),
                        **alloc_summary(fplug, frag_alloc)}
                fplug.stop()

        rccl = None
        if args.collectives and d.world > 1:
            # the pod's GPUs as a torchrun workload sees them: one rank per GPU, RCCL over xGMI
            from rocm_k8s_device_plugin_amd.parallel import collectives as coll
            # a secondary measurement: a failure is reported in the JSON line, not
            # allowed to take the headline down with it
            guard.enter("collectives")
            try:
                group, on_gpu = d.rccl_group()   # RCCL is created here, after the timed loop
                if on_gpu:
                    sizes = args.collective_sizes or "1M,64M,256M"
                    ops, iters, dtype = coll.DEFAULT_OPS, 20, d.torch.bfloat16
                else:
                    sizes = args.collective_sizes or "64K"
                    ops, iters, dtype = ("all_reduce", "all_gather"), 3, d.torch.float32
                rows = coll.run([coll.parse_size(x) for x in sizes.split(",") if x], ops, iters=iters, warmup=3,
                                dtype=dtype, group=group)
                rccl = coll.summary(rows)
                rccl["backend"] = d.dist.get_backend(group)
            except Exception as e:  # noqa: BLE001
                rccl = {"error": f"{type(e).__name__}: {e}"[:300]}

        def health_loop_report():
            if args.health_pulse <= 0 or (args.fixture and plugin_kind != "native-daemon"):
                return None
            if plugin_kind == "native-daemon":
                return plug.health_report(float(health_flags[1]))
            return {"plugin": "python", "pulse_s": args.health_pulse, "sweeps": impl.monitor.sweeps,
                    "sweep_ms_last": round(impl.monitor.last_sweep_ms, 3),
                    "unhealthy": sorted(k for k, v in impl.monitor.snapshot().items() if v.health != "Healthy")}

        extra = {}
        if d.rank == 0:
            guard.enter("allocator_microbench")
            # allocator microbenchmark on the same request (ours vs the reference's ordered BFS)
            pol = plug.allocator
            avail = [dv.id for dv in adv]
            t = time.perf_counter()
            for _ in range(200):  # both sides called straight into C++ (no trace/stats wrapper)
                pol.native.allocate(avail, [], n)
            ours = (time.perf_counter() - t) / 200 * 1e6
            t = time.perf_counter()
            for _ in range(20):
                ref = pol.reference_allocate(avail, [], n)
            refu = (time.perf_counter() - t) / 20 * 1e6
            # every smaller request on the same N advertised GPUs (the allocations a
            # shared node serves): our set search vs the reference's ordered BFS,
            # both in C++ on the same weights, same chosen set required
            sweep = {}
            for k in range(1, n):
                t = time.perf_counter()
                for _ in range(50):
                    mine = pol.native.allocate(avail, [], k)
                mine_us = (time.perf_counter() - t) / 50 * 1e6
                t = time.perf_counter()
                for _ in range(3):
                    refk = pol.reference_allocate(avail, [], k)
                sweep[str(k)] = {"ours_us": round(mine_us, 2), "reference_us": round((time.perf_counter() - t) / 3 * 1e6, 2),
                                 "reference_candidates": refk["candidates"], "ours_candidates": mine["candidates"],
                                 "same_set": sorted(mine["ids"]) == sorted(refk["ids"])}
            extra = dict(core, **{
                f"latency_p50_ms_{rt_key}": round(pct(rt_lat, .5), 3) if rt_lat else None,
                f"latency_p99_ms_{rt_key}": round(pct(rt_lat, .99), 3) if rt_lat else None,
                f"{rt_key}_steps": len(rt_lat),
                "latency_p50_ms_back_to_back": round(pct(b2b_lat, .5), 3) if b2b_lat else None,
                "health_loop": health_loop_report(),
                f"latency_p50_ms_dev_view_{other_view}": round(pct(vis_lat, .5), 3) if vis_lat else None,
                f"latency_p50_ms_container_mode_{other_mode}": round(pct(other_mode_lat, .5), 3) if other_mode_lat
                else None,
                "latency_p50_ms_node_view_emulated": round(pct(nv_lat, .5), 3) if nv_lat else None,
                "node_view_emulated_runtime_init_p50_ms": round(pct(nv_init, .5), 3) if nv_init else None,
                "allocator_us": round(ours, 2), "reference_algorithm_us": round(refu, 2),
                "reference_algorithm_candidates": ref["candidates"], "allocator_sweep": sweep})
            from rocm_k8s_device_plugin_amd.parallel.fabric import Fabric
            try:
                extra["fabric"] = Fabric(inv).report([dv.id for dv in adv]).as_dict()
            except Exception as e:  # noqa: BLE001
                extra["fabric"] = {"error": f"{type(e).__name__}: {e}"[:300]}
            extra["rccl"] = rccl
            # the timed admissions' GetPreferredAllocation (with M > N: a real search
            # over the fragmented availability) and the N-of-all-devices comparison
            extra["timed_allocation"] = dict({"advertised": m_adv, "requested": n, "held": plug.held},
                                             **alloc_summary(plug, alloc_steps))
            extra["fragmented_n_of_m"] = frag
            if args.throughput_check and not args.fixture:
                guard.enter("throughput_check")
                extra["gpu_throughput"] = throughput_check(adv_ordinals)
            if args.peer_check and not args.fixture:
                from rocm_k8s_device_plugin_amd.health.peer import probe_peers
                guard.enter("peer_probe")
                try:
                    rep = probe_peers(adv_ordinals, nbytes=64 << 20, reps=3, timeout_s=120)
                    extra["peer_probe"] = dict(rep.summary(), wall_ms=round(rep.wall_ms, 1))
                except Exception as e:  # noqa: BLE001
                    extra["peer_probe"] = {"error": f"{type(e).__name__}: {e}"[:300]}
            guard.enter("plugin_stop")
            plug.stop()
            # tasks still parked (watchers, event waits): cancel them before the loop goes
            rest = [t for t in asyncio.all_tasks(loop) if not t.done()]
            for t in rest:
                t.cancel()
            if rest:
                loop.run_until_complete(asyncio.gather(*rest, return_exceptions=True))
            loop.close()
            import shutil
            shutil.rmtree(tmp, ignore_errors=True)
            emit(result_line(extra))

    try:
        extras()
    except (Exception, SystemExit) as e:  # noqa: BLE001
        # a failed extra (or a peer rank that left) is reported, never fatal to the measured headline
        guard.abandon(f"{type(e).__name__}: {e}"[:300])
    d.close()
    guard.cancel()


if __name__ == "__main__":
    main()
