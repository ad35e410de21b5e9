"""The device plugin under test in the admission benchmark (bench.py): the
native daemon behind a fake kubelet (the default), or the Python oracle
plugin in the bench process; plus the throughput check run after the timed
steps."""
from __future__ import annotations

import json
import os
import threading


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


def _rss_kb(pid: int) -> int:
    try:
        with open(f"/proc/{pid}/status") as f:
            for line in f:
                if line.startswith("VmRSS:"):
                    return int(line.split()[1])
    except OSError:
        pass
    return 0


def _descendants(root: int) -> list:
    """PIDs below `root` (its probe server, spawned probes and their children)."""
    kids = {}
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open(f"/proc/{d}/stat") as f:
                ppid = int(f.read().rsplit(")", 1)[1].split()[1])
        except (OSError, ValueError, IndexError):
            continue
        kids.setdefault(ppid, []).append(int(d))
    out, todo = [], [root]
    while todo:
        for c in kids.get(todo.pop(), []):
            out.append(c)
            todo.append(c)
    return out


class RssSampler:
    """Host memory of a daemon and every process below it, sampled every
    `period_s` on a thread: what a DaemonSet's memory request has to cover
    (the persistent probe server; in spawn mode, the probe processes of a sweep)."""

    def __init__(self, pid: int, period_s: float = 0.1):
        self.pid, self.period_s = pid, period_s
        self.rows = []      # (daemon KiB, descendants KiB, descendant count)
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        while not self._stop.wait(self.period_s):
            kids = _descendants(self.pid)
            self.rows.append((_rss_kb(self.pid), sum(_rss_kb(k) for k in kids), len(kids)))

    def stop(self) -> dict:
        self._stop.set()
        self._t.join(timeout=5)
        if not self.rows:
            return {}
        from .stats import pct
        tot = [a + b for a, b, _ in self.rows]
        return {"samples": len(self.rows), "period_s": self.period_s,
                "daemon_rss_mb_p50": round(pct([a for a, _, _ in self.rows], .5) / 1024, 1),
                "children_rss_mb_p50": round(pct([b for _, b, _ in self.rows], .5) / 1024, 1),
                "children_rss_mb_max": round(max(b for _, b, _ in self.rows) / 1024, 1),
                "total_rss_mb_p50": round(pct(tot, .5) / 1024, 1), "total_rss_mb_max": round(max(tot) / 1024, 1),
                "children_max": max(c for _, _, c in self.rows)}


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
        # the health DaemonSet configuration: its host memory over the whole run
        self.rss = RssSampler(self.proc.pid) if metrics_port else None
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
        # the mean includes the start-up sweep (probe server and amd-smi start); the p50 is the
        # upper bound of the histogram bucket that holds the median sweep
        rss = self.rss.stop() if self.rss else {}
        return {"plugin": "native-daemon", "pulse_s": pulse_s, "sweeps": n, "host_memory": rss,
                "sweep_ms_mean": round(m.get("mi355x_dp_health_sweep_seconds_sum", 0.0) * 1e3 / n, 3) if n else None,
                "sweep_ms_p50_at_most": _bucket_quantile_ms(m, "mi355x_dp_health_sweep_seconds", .5),
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


def _bucket_quantile_ms(m: dict, name: str, q: float):
    """Upper bound (ms) of the Prometheus histogram bucket holding quantile q, from
    a parsed /metrics dict ({'name_bucket{le="0.005"}': count, ...}); None if empty."""
    import math
    buckets = []
    for k, v in m.items():
        if k.startswith(name + "_bucket{") and 'le="' in k:
            le = k.split('le="', 1)[1].split('"', 1)[0]
            buckets.append((math.inf if le == "+Inf" else float(le), v))
    buckets.sort()
    total = buckets[-1][1] if buckets else 0
    if not total:
        return None
    for le, cum in buckets:
        if cum >= q * total:
            return None if math.isinf(le) else round(le * 1e3, 3)
    return None


class PluginUnderTest:
    """Rank 0: the Python CLI's plugin advertising `devs` (real discovery data,
    real allocator and gRPC servicer) behind a fake kubelet on its own UDS dir."""

    def __init__(self, loop, tmp, name, sysfs, devs, full, ords, hcfg, pulse_s, kubelet_client="native"):
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
        self.mgr = PluginManager(self.impl, ManagerConfig(pulse_s=pulse_s, plugin_dir=pdir, handle_signals=False))
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
