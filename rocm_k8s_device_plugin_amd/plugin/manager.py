"""Device-plugin lifecycle manager of the Python oracle plugin.

The product is the native daemon (native/src/daemon: ``./k8s-device-plugin``
in the images); this manager is the independent Python model its behaviour
is checked against (equality tests) and the bench's ``--plugin python``. It
serves through the same C++ HTTP/2 server (plugin/native_server.py) and has no
second transport. Reference: internal/pkg/manager/manager.go:31-104 (lister, heartbeat) and the
vendored kubevirt device-plugin-manager (vendor/github.com/kubevirt/
device-plugin-manager/pkg/dpm/{manager,plugin}.go). Same externally visible
behaviour:

* one gRPC server per resource on ``<plugin_dir>/amd.com_<resource>``;
* stale socket removed before listening;
* ``Register{Version: v1beta1, Endpoint: <socket basename>,
  ResourceName: amd.com/<resource>, Options}`` against ``kubelet.sock``;
* server start retried 3 times, 3 s apart;
* kubelet restart (``kubelet.sock`` re-created) -> re-serve and re-register,
  ``kubelet.sock`` removed -> stop servers;
* SIGTERM/SIGINT/SIGQUIT -> stop everything and remove sockets;
* no DeviceImpl (every strategy failed) -> idle until signalled.

Re-designed: asyncio instead of goroutines; the kubelet socket is watched by
inode polling (works on any filesystem, catches delete+recreate between
polls); the heartbeat is a broadcast health sweep (one sweep per pulse for the
whole node, every resource's ListAndWatch woken). New: a topology watch
re-discovers the node when its GPU topology changes (partition switch) and
starts / stops per-resource servers to match.
"""
from __future__ import annotations

import asyncio
import os
import signal
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import grpc

from .. import constants as C
from ..proto import deviceplugin as pb
from ..utils import log
from ..utils.broadcast import Broadcast
from ..utils.metrics import REGISTRY, serve_metrics
from .base import DeviceImpl, PluginContext, new_context
from .native_server import NativePluginServer

_log = log.get("manager")


@dataclass
class ManagerConfig:
    pulse_s: float = 0.0
    plugin_dir: str = pb.DEVICE_PLUGIN_PATH
    kubelet_socket: Optional[str] = None   # default: <plugin_dir>/kubelet.sock
    namespace: str = C.RESOURCE_NAMESPACE
    start_retries: int = 3
    retry_wait_s: float = 3.0
    register_timeout_s: float = 10.0
    watch_interval_s: float = 0.5
    send_every_pulse: bool = False
    metrics_port: int = 0
    handle_signals: bool = True
    topology_watch_s: float = 5.0   # re-discovery check period (partition switches); 0 = off
    # GetPreferredAllocation search: "auto" (extended on partitioned nodes),
    # "reference" (the reference's candidate family), "extended" / True (allocator.py)
    allocator_extended_search: object = "auto"


class ResourcePlugin:
    def __init__(self, mgr: "PluginManager", name: str):
        self.mgr = mgr
        self.name = name
        cfg = mgr.cfg
        self.resource_name = f"{cfg.namespace}/{name}"
        self.socket = os.path.join(cfg.plugin_dir, f"{cfg.namespace}_{name}")
        self.ctx: PluginContext = new_context(name, extended_search=cfg.allocator_extended_search)
        self.stop_bc = Broadcast()
        self.native: Optional[NativePluginServer] = None
        self.running = False
        self.started = False
        self.registrations = 0
        self._lock = asyncio.Lock()

    def start(self) -> bool:
        try:
            self.mgr.impl.start(self.ctx)
            self.started = True
        except Exception as e:  # reference: log and do not start the server
            _log.error('Failed to start plugin "%s": %s', self.name, e)
            self.started = False
        if self.native is not None and self.started:
            self.native.refresh()   # new allocator / devices for the native server
        return self.started

    def sync(self) -> None:
        """Apply the native server's pending call events (stats, logs, metrics) now."""
        if self.native is not None:
            self.native.drain()

    def _cleanup(self) -> None:
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass

    async def _serve(self) -> None:
        self._cleanup()
        os.makedirs(os.path.dirname(self.socket), exist_ok=True)
        self.stop_bc = Broadcast()
        # the framework's one kubelet-facing server (C++ HTTP/2, the daemon's); a start
        # failure is retried like any other (start_server) -- there is no second transport
        native = NativePluginServer(self.mgr.impl, self.ctx, self.mgr.pulse, self.stop_bc,
                                    self.mgr.cfg.send_every_pulse)
        await native.start(self.socket)
        self.native = native

    async def _register(self) -> None:
        sock = self.mgr.kubelet_socket
        opts = self.mgr.impl.options(self.ctx)
        req = pb.RegisterRequest(version=pb.VERSION, endpoint=os.path.basename(self.socket),
                                 resource_name=self.resource_name, options=opts)
        _log.info("%s: Registration for endpoint %s", self.name, req.endpoint)
        async with grpc.aio.insecure_channel(f"unix:{sock}") as ch:
            await pb.RegistrationStub(ch).Register(req, timeout=self.mgr.cfg.register_timeout_s)
        self.registrations += 1
        REGISTRY.inc("mi355x_dp_registrations_total", resource=self.name)

    async def start_server(self) -> bool:
        async with self._lock:
            if self.running:
                return True
            cfg = self.mgr.cfg
            for attempt in range(1, cfg.start_retries + 1):
                try:
                    t0 = time.perf_counter()
                    await self._serve()
                    await self._register()
                    self.running = True
                    log.info_fields(_log, "plugin server started", resource=self.resource_name,
                                    socket=self.socket, startup_ms=f"{(time.perf_counter() - t0) * 1e3:.2f}")
                    return True
                except Exception as e:
                    await self._stop_locked()
                    if attempt == cfg.start_retries:
                        _log.error('Failed to start plugin\'s "%s" server, within given %d tries: %s', self.name,
                                   cfg.start_retries, e)
                    else:
                        _log.error('Failed to start plugin\'s "%s" server, attempt %d out of %d, waiting %.1fs '
                                   'before next try: %s', self.name, attempt, cfg.start_retries, cfg.retry_wait_s, e)
                        await asyncio.sleep(cfg.retry_wait_s)
            return False

    async def _stop_locked(self) -> None:
        self.stop_bc.close()
        if self.native is not None:
            await self.native.stop(grace=0.5)
            self.native = None
        self.running = False
        self._cleanup()

    async def stop_server(self) -> None:
        async with self._lock:
            await self._stop_locked()


class PluginManager:
    def __init__(self, impl: Optional[DeviceImpl], cfg: Optional[ManagerConfig] = None):
        self.impl = impl
        self.cfg = cfg or ManagerConfig()
        self.kubelet_socket = self.cfg.kubelet_socket or os.path.join(self.cfg.plugin_dir, "kubelet.sock")
        self.plugins: Dict[str, ResourcePlugin] = {}
        self.pulse = Broadcast()
        self.stopped = asyncio.Event()
        self.ready = asyncio.Event()
        self._tasks: List[asyncio.Task] = []
        self._metrics_server = None
        self._impl_lock: Optional[asyncio.Lock] = None   # health sweep vs topology reload
        self.topology_reloads = 0
        self._fabric_seen = 0

    # ------------------------------------------------------------- control
    def request_stop(self) -> None:
        self.stopped.set()

    def resources(self) -> List[str]:
        return list(self.plugins)

    async def _start_all(self) -> None:
        await asyncio.gather(*(p.start_server() for p in self.plugins.values() if p.started))

    async def _stop_servers(self) -> None:
        await asyncio.gather(*(p.stop_server() for p in self.plugins.values()))

    async def _health_loop(self) -> None:
        while not self.stopped.is_set():
            try:
                await asyncio.wait_for(self.stopped.wait(), self.cfg.pulse_s)
                return
            except asyncio.TimeoutError:
                pass
            t0 = time.perf_counter()
            try:
                async with self._impl_lock:
                    changed = await self.impl.refresh_health()
            except Exception as e:  # health must never take the plugin down
                _log.error("health sweep failed: %s", e)
                changed = False
            REGISTRY.histogram("mi355x_dp_health_sweep_seconds", "health sweep latency").observe(
                (time.perf_counter() - t0) * 1e3)
            if changed:
                REGISTRY.inc("mi355x_dp_health_changes_total")
            fv = self.impl.fabric_version()
            if fv != self._fabric_seen:
                # xGMI link state changed the pair weights: re-initialise every
                # resource's allocator (devices and their health are unchanged)
                self._fabric_seen = fv
                async with self._impl_lock:
                    for p in self.plugins.values():
                        p.start()
                REGISTRY.inc("mi355x_dp_fabric_reweights_total")
                _log.warning("xGMI link state changed: preferred allocation re-weighted")
            self.pulse.fire()

    async def _topology_loop(self) -> None:
        """Every topology_watch_s: has the node's GPU topology changed (e.g. an
        amd-smi partition switch)? Then advertise what is there now."""
        seen = None
        while not self.stopped.is_set():
            try:
                await asyncio.wait_for(self.stopped.wait(), self.cfg.topology_watch_s)
                return
            except asyncio.TimeoutError:
                pass
            try:
                # re-discover once a new fingerprint has held for one interval:
                # a partition switch passes through states with devices half gone
                fp = self.impl.topology_fingerprint()
                if fp is not None and fp != seen:
                    seen = fp
                    continue
                async with self._impl_lock:
                    change = await self.impl.reload_topology()
                if change:
                    await self._apply_topology_change(change)
            except Exception as e:  # never take the plugin down over a re-discovery
                _log.error("topology reload failed: %s", e)

    async def _apply_topology_change(self, change: dict) -> None:
        """Plugins of vanished resources stop (kubelet drops the resource when
        the stream ends); kept ones get their allocator re-initialised on the
        new devices and re-send their list; new resources register."""
        self.topology_reloads += 1
        REGISTRY.inc("mi355x_dp_topology_reloads_total")
        names = list(self.impl.resource_names())
        for n in [n for n in self.plugins if n not in names]:
            _log.warning("resource %s no longer exists: stopping its plugin server", n)
            await self.plugins.pop(n).stop_server()
        for n, p in self.plugins.items():
            p.start()
        new = [n for n in names if n not in self.plugins]
        for n in new:
            p = ResourcePlugin(self, n)
            self.plugins[n] = p
            p.start()
        if new:
            await asyncio.gather(*(self.plugins[n].start_server() for n in new if self.plugins[n].started))
        log.info_fields(_log, "topology reloaded", resources=",".join(names), added=len(change.get("added", [])),
                        removed=len(change.get("removed", [])))
        self.pulse.fire()

    def _sock_id(self) -> Optional[Tuple[int, int, int]]:
        # inode numbers are recycled by delete+create; ctime tells them apart
        try:
            st = os.stat(self.kubelet_socket)
            return (st.st_ino, st.st_dev, st.st_ctime_ns)
        except FileNotFoundError:
            return None

    def _open_dir_watch(self):
        """inotify on the plugin directory (the reference's dpm uses fsnotify):
        a kubelet restart is seen at once instead of at the next poll. None
        when unavailable (the poll alone then notices changes)."""
        try:
            from ..ops.native import core
            w = core().DirWatcher()
        except Exception:
            return None
        err = w.open(os.path.dirname(self.kubelet_socket) or ".")
        if err:
            _log.info("no inotify watch of the kubelet directory (%s); polling every %.1fs", err,
                      self.cfg.watch_interval_s)
            return None
        return w

    async def _watch_kubelet(self) -> None:
        last = self._sock_id()
        next_retry = 0.0
        loop = asyncio.get_running_loop()
        watch = self._open_dir_watch()
        kick = asyncio.Event()
        if watch is not None:
            sock_name = os.path.basename(self.kubelet_socket)

            def on_events():
                # only kubelet.sock (or the directory itself) matters: the
                # plugins' own sockets live in the same directory
                if any(name in (sock_name, "") for name, _ in watch.read_events()):
                    kick.set()

            loop.add_reader(watch.fileno(), on_events)
        try:
            await self._watch_kubelet_loop(last, next_retry, kick, watch)
        finally:
            if watch is not None:
                loop.remove_reader(watch.fileno())
                watch.close()

    async def _watch_kubelet_loop(self, last, next_retry, kick, watch) -> None:
        stop_wait = asyncio.ensure_future(self.stopped.wait())
        try:
            while not self.stopped.is_set():
                kick_wait = asyncio.ensure_future(kick.wait())
                # with inotify the poll is only a safety net (e.g. the directory was replaced)
                timeout = self.cfg.watch_interval_s if watch is None else max(self.cfg.watch_interval_s, 5.0)
                await asyncio.wait({stop_wait, kick_wait}, timeout=timeout, return_when=asyncio.FIRST_COMPLETED)
                kick_wait.cancel()
                kick.clear()
                if self.stopped.is_set():
                    return
                last, next_retry = await self._kubelet_check(last, next_retry)
        finally:
            stop_wait.cancel()

    async def _kubelet_check(self, last, next_retry):
        """One look at kubelet.sock: (re)start / stop servers on a change, retry
        pending registrations (rate-limited). Returns the new (last, next_retry)."""
        cur = self._sock_id()
        if cur == last:
            # kubelet is up but a plugin never got registered (e.g. the socket
            # appeared before kubelet was serving): keep retrying, rate-limited
            now = time.monotonic()
            pending = [p for p in self.plugins.values() if p.started and not p.running]
            if cur is not None and pending and now >= next_retry:
                next_retry = now + max(self.cfg.retry_wait_s, self.cfg.watch_interval_s)
                await asyncio.gather(*(p.start_server() for p in pending))
            return last, next_retry
        if cur is None:
            _log.info("kubelet socket removed; stopping plugin servers")
            await self._stop_servers()
        else:
            _log.info("kubelet socket (re)created; restarting plugin servers and re-registering")
            await self._stop_servers()
            await self._start_all()
        return cur, next_retry

    async def run(self) -> None:
        loop = asyncio.get_running_loop()
        if self.cfg.handle_signals:
            for s in (signal.SIGTERM, signal.SIGINT, signal.SIGQUIT):
                try:
                    loop.add_signal_handler(s, self.request_stop)
                except (NotImplementedError, RuntimeError):
                    pass
        if self.cfg.metrics_port:
            self._metrics_server = await serve_metrics(self.cfg.metrics_port)
        names = self.impl.resource_names() if self.impl is not None else []
        if not names:
            _log.warning("no device implementation/resources available; idling")
        for n in names:
            p = ResourcePlugin(self, n)
            self.plugins[n] = p
            p.start()
        if self.impl is not None and self.cfg.pulse_s > 0 and names:
            # one sweep before registering, so the first ListAndWatch already
            # carries real verdicts (the reference advertises everything Healthy
            # until its first pulse)
            try:
                await self.impl.refresh_health()
            except Exception as e:
                _log.error("initial health sweep failed: %s", e)
        await self._start_all()
        self._impl_lock = asyncio.Lock()
        if self.impl is not None and self.cfg.pulse_s > 0:
            self._tasks.append(asyncio.create_task(self._health_loop()))
        if self.impl is not None and self.cfg.topology_watch_s > 0:
            self._tasks.append(asyncio.create_task(self._topology_loop()))
        self._tasks.append(asyncio.create_task(self._watch_kubelet()))
        self.ready.set()
        await self.stopped.wait()
        await self.shutdown()

    async def shutdown(self) -> None:
        self.pulse.close()
        for t in self._tasks:
            t.cancel()
        await asyncio.gather(*self._tasks, return_exceptions=True)
        self._tasks.clear()
        await self._stop_servers()
        if self.impl is not None:
            await self.impl.close()
        if self._metrics_server is not None:
            self._metrics_server.close()
            await self._metrics_server.wait_closed()
        _log.info("device plugin manager stopped")
