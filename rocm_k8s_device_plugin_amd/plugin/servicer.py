"""v1beta1.DevicePlugin servicer (grpc.aio).

Reference: AMDGPUPlugin, internal/pkg/plugin/plugin.go:33-186 — a thin
adapter delegating to the DeviceImpl. Differences:

* ``ListAndWatch`` is an async generator woken by a per-node Broadcast
  (every resource sees every pulse; reference Appendix B #1), sends the full
  list on health changes (and, optionally, on every pulse like the
  reference), and ends cleanly when its plugin server stops;
* every RPC is timed into the metrics registry and logged with structured
  latency fields;
* DeviceImpl errors map to gRPC status errors instead of Go nil-derefs.
"""
from __future__ import annotations

import time

import grpc

from ..proto import deviceplugin as pb
from ..utils import log
from ..utils.broadcast import Broadcast
from ..utils.metrics import REGISTRY
from ..utils.trace import TRACER
from .base import DeviceImpl, DeviceImplError, PluginContext

_log = log.get("plugin")


class DevicePluginServicer:
    def __init__(self, impl: DeviceImpl, ctx: PluginContext, pulse: Broadcast, stop: Broadcast,
                 send_every_pulse: bool = False):
        self.impl = impl
        self.ctx = ctx
        self.pulse = pulse
        self.stop = stop
        self.send_every_pulse = send_every_pulse
        self.streams = 0
        self.sent = 0

    def _observe(self, rpc: str, t0: float) -> float:
        ms = (time.perf_counter() - t0) * 1e3
        REGISTRY.histogram("mi355x_dp_rpc_seconds", "device plugin RPC latency", rpc=rpc,
                           resource=self.ctx.resource).observe(ms)
        if log.V(2):
            log.info_fields(_log, "rpc", rpc=rpc, resource=self.ctx.resource, latency_ms=f"{ms:.3f}")
        return ms

    async def GetDevicePluginOptions(self, request, context):  # noqa: N802
        t0 = time.perf_counter()
        try:
            return self.impl.options(self.ctx)
        finally:
            self._observe("GetDevicePluginOptions", t0)

    async def PreStartContainer(self, request, context):  # noqa: N802
        return pb.PreStartContainerResponse()

    async def GetPreferredAllocation(self, request, context):  # noqa: N802
        t0 = time.perf_counter()
        try:
            with TRACER.span("GetPreferredAllocation", "rpc", resource=self.ctx.resource,
                             sizes=[c.allocation_size for c in request.container_requests]):
                return self.impl.preferred_allocation(self.ctx, request)
        except DeviceImplError as e:
            _log.error("%s", e)
            REGISTRY.inc("mi355x_dp_rpc_errors_total", rpc="GetPreferredAllocation", resource=self.ctx.resource)
            await context.abort(grpc.StatusCode.UNKNOWN, str(e))
        finally:
            self._observe("GetPreferredAllocation", t0)

    async def Allocate(self, request, context):  # noqa: N802
        t0 = time.perf_counter()
        try:
            with TRACER.span("Allocate", "rpc", resource=self.ctx.resource):
                resp = self.impl.allocate(self.ctx, request)
            for creq in request.container_requests:
                _log.info("Allocating device IDs: %s", ",".join(creq.devices_ids))
            return resp
        except DeviceImplError as e:
            _log.error("%s", e)
            REGISTRY.inc("mi355x_dp_rpc_errors_total", rpc="Allocate", resource=self.ctx.resource)
            await context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        finally:
            self._observe("Allocate", t0)

    async def ListAndWatch(self, request, context):  # noqa: N802
        self.streams += 1
        REGISTRY.inc("mi355x_dp_listandwatch_streams_total", resource=self.ctx.resource)
        try:
            devs = self.impl.enumerate(self.ctx)
            yield pb.ListAndWatchResponse(devices=devs)
            self.sent += 1
            gen = self.pulse.generation
            last_health = self.impl.health_version()
            while not self.stop.closed:
                gen = await self.pulse.wait(gen)
                if self.stop.closed or self.pulse.closed:
                    break
                hv = self.impl.health_version()
                if not self.send_every_pulse and hv == last_health:
                    continue
                last_health = hv
                TRACER.instant("ListAndWatch.send", "rpc", resource=self.ctx.resource, health_version=hv)
                yield pb.ListAndWatchResponse(devices=self.impl.update_health(self.ctx))
                self.sent += 1
        finally:
            self.streams -= 1
