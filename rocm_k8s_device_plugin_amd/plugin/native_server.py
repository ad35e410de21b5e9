"""The kubelet-facing v1beta1.DevicePlugin endpoint on the native gRPC server.

Reference: AMDGPUPlugin on grpc-go (internal/pkg/plugin/plugin.go:33-186).
The Python grpc.aio servicer (servicer.py) spends ~0.6-0.9 ms of interpreter
and event-loop work per admission RPC. Here the HTTP/2 server and the
admission RPCs are C++ (native/src/rpc): GetPreferredAllocation runs the
HiveAllocator on the server thread, Allocate is assembled from per-device
response fragments prepared below, ListAndWatch's first message is the
current list and later ones are pushed from the health pulse.

Python stays in charge of state and observability:

* ``refresh()`` hands the server the current options, allocator snapshot,
  Allocate fragments and device list (on start, allocator re-init, topology
  change, health change);
* whatever has no prepared state — the allocator disabled, Allocate mounts
  made per request (-topology_view / -node_view), passthrough modes — is
  answered by ``_fallback`` (the same DeviceImpl calls as the aio servicer) on
  the server thread;
* every call leaves an event (timing, allocator outcome, IDs); they are drained
  on the event loop through an eventfd into logs ("Allocating device IDs"),
  metrics (``mi355x_dp_rpc_seconds``) and trace spans, off the RPC path.
"""
from __future__ import annotations

import asyncio
import collections
from typing import Optional

from ..ops.native import core
from ..proto import deviceplugin as pb
from ..utils import log
from ..utils.broadcast import Broadcast
from ..utils.metrics import REGISTRY
from ..utils.trace import TRACER
from .base import DeviceImpl, DeviceImplError, PluginContext

_log = log.get("plugin")

_INVALID_ARGUMENT, _UNKNOWN = 3, 2


class NativePluginServer:
    def __init__(self, impl: DeviceImpl, ctx: PluginContext, pulse: Broadcast, stop: Broadcast,
                 send_every_pulse: bool = False):
        self.impl = impl
        self.ctx = ctx
        self.pulse = pulse
        self.stop_bc = stop
        self.send_every_pulse = send_every_pulse
        self.srv = core().DevicePluginServer()
        self.srv.set_fallback(self._fallback)
        self.sent = 0
        self.calls = 0
        self.fallbacks = 0
        self._task: Optional[asyncio.Task] = None
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._alloc_seen = None
        # server-side time of recent calls per RPC (ms; request complete -> response queued)
        self.recent_ms: dict = {}

    # ------------------------------------------------------------ state
    def refresh(self) -> None:
        """Hand the server the current options, allocator, Allocate fragments and list."""
        impl, ctx = self.impl, self.ctx
        self.srv.set_options(impl.options(ctx).SerializeToString())
        alloc = ctx.allocator if ctx.allocator is not None and not ctx.allocator_error else None
        native = getattr(alloc, "native", None) if alloc is not None else None
        self.srv.set_allocator(native if native is not None and native.initialized else None)
        self._alloc_seen = native
        tmpl = impl.allocate_template(ctx) if hasattr(impl, "allocate_template") else None
        if tmpl is None:
            self.srv.clear_allocate_template()
        else:
            self.srv.set_allocate_template(**tmpl)
        self.srv.set_device_list(pb.ListAndWatchResponse(devices=impl.enumerate(ctx)).SerializeToString())

    # ------------------------------------------------------------ fallback
    def _fallback(self, method: str, req: bytes):
        """Runs on the server thread (with the GIL): the DeviceImpl's own answer."""
        impl, ctx = self.impl, self.ctx
        try:
            if method == "GetPreferredAllocation":
                r = pb.PreferredAllocationRequest.FromString(req)
                with TRACER.span("GetPreferredAllocation", "rpc", resource=ctx.resource,
                                 sizes=[c.allocation_size for c in r.container_requests]):
                    return 0, "", impl.preferred_allocation(ctx, r).SerializeToString()
            if method == "Allocate":
                with TRACER.span("Allocate", "rpc", resource=ctx.resource):
                    return 0, "", impl.allocate(ctx, pb.AllocateRequest.FromString(req)).SerializeToString()
            if method == "GetDevicePluginOptions":
                return 0, "", impl.options(ctx).SerializeToString()
            if method == "ListAndWatch":
                return 0, "", pb.ListAndWatchResponse(devices=impl.enumerate(ctx)).SerializeToString()
            if method == "PreStartContainer":
                return 0, "", b""
            return 12, f"unknown method {method}", b""
        except DeviceImplError as e:
            return (_INVALID_ARGUMENT if method == "Allocate" else _UNKNOWN), str(e), b""
        except Exception as e:  # never let a handler error escape into the server thread
            return _UNKNOWN, f"{type(e).__name__}: {e}", b""

    # ------------------------------------------------------------ events
    def drain(self) -> None:
        """Logs, metrics and trace spans of the calls served since the last drain."""
        evs = self.srv.drain_events()
        if evs:
            st = self.srv.stats()
            for k in ("connections", "calls", "protocol_errors"):
                REGISTRY.set(f"mi355x_dp_grpc_{k}", float(st[k]), help=f"native gRPC server: {k.replace('_', ' ')}",
                             resource=self.ctx.resource)
            REGISTRY.set("mi355x_dp_listandwatch_open_streams", float(self.srv.open_streams()),
                         help="ListAndWatch streams open on the native server", resource=self.ctx.resource)
        for ev in evs:
            rpc, ms = ev["rpc"], ev["dur_ns"] / 1e6
            self.calls += 1
            q = self.recent_ms.setdefault(rpc, collections.deque(maxlen=4096))
            q.append(ms)
            if not ev["native"]:
                self.fallbacks += 1
            REGISTRY.histogram("mi355x_dp_rpc_seconds", "device plugin RPC latency", rpc=rpc,
                               resource=self.ctx.resource).observe(ms)
            if rpc == "ListAndWatch":
                REGISTRY.inc("mi355x_dp_listandwatch_streams_total", resource=self.ctx.resource)
            if ev["status"] != 0:
                _log.error("%s: %s", rpc, ev["message"])
                REGISTRY.inc("mi355x_dp_rpc_errors_total", rpc=rpc, resource=self.ctx.resource)
            elif rpc == "Allocate":
                _log.info("Allocating device IDs: %s", ",".join(ev["ids"]))
            if rpc == "GetPreferredAllocation" and ev["native"] and ev["candidates"] >= 0:
                st = getattr(self.ctx.allocator, "stats", None)
                if st is not None:
                    st.calls += 1
                    st.total_us += ev["alloc_us"]
                    st.last_us = ev["alloc_us"]
                    st.last_candidates = ev["candidates"]
                    st.last_weight = ev["weight"]
                    st.last_short_circuit = bool(ev["short_circuit"])
            if TRACER.enabled and ev["native"]:
                TRACER.complete(rpc, "rpc", ev["t0_ns"], ev["dur_ns"], resource=self.ctx.resource, native=True,
                                ids=",".join(ev["ids"]))
                if ev["alloc_t0_ns"]:
                    TRACER.complete("allocator.allocate", "alloc", ev["alloc_t0_ns"], int(ev["alloc_us"] * 1e3),
                                    candidates=ev["candidates"], native=True)
            if log.V(2):
                log.info_fields(_log, "rpc", rpc=rpc, resource=self.ctx.resource, latency_ms=f"{ms:.3f}",
                                native=ev["native"])

    # ------------------------------------------------------------ lifecycle
    async def start(self, socket: str) -> None:
        if hasattr(self.impl, "add_change_listener"):
            self.impl.add_change_listener(self.refresh)
        self.refresh()
        err = self.srv.start(socket)
        if err:
            raise OSError(f"native gRPC server: {err}")
        self._loop = asyncio.get_running_loop()
        self._loop.add_reader(self.srv.event_fd, self.drain)
        self._task = asyncio.create_task(self._watch())

    async def stop(self, grace: float = 0.5) -> None:
        if hasattr(self.impl, "remove_change_listener"):
            self.impl.remove_change_listener(self.refresh)
        if self._task is not None:
            self._task.cancel()
            await asyncio.gather(self._task, return_exceptions=True)
            self._task = None
        # the server thread may need the GIL (fallback) while it drains: stop off the loop thread
        await asyncio.to_thread(self.srv.stop, grace)
        if self._loop is not None:
            self._loop.remove_reader(self.srv.event_fd)
            self._loop = None
        self.drain()

    async def _watch(self) -> None:
        """Each pulse: on a health (or topology) change — or every pulse with
        -send_every_pulse — push the list to every open ListAndWatch stream."""
        gen = self.pulse.generation
        last = self.impl.health_version()
        while not self.stop_bc.closed:
            gen = await self.pulse.wait(gen)
            if self.stop_bc.closed or self.pulse.closed:
                break
            native = getattr(self.ctx.allocator, "native", None)
            if native is not self._alloc_seen:   # re-initialised (fabric / topology change)
                self.refresh()
            hv = self.impl.health_version()
            if not self.send_every_pulse and hv == last:
                continue
            last = hv
            data = pb.ListAndWatchResponse(devices=self.impl.update_health(self.ctx)).SerializeToString()
            self.srv.set_options(self.impl.options(self.ctx).SerializeToString())
            n = self.srv.publish_list(data)
            self.sent += n
            TRACER.instant("ListAndWatch.send", "rpc", resource=self.ctx.resource, health_version=hv, streams=n)
