"""Fake AMD device-metrics-exporter (``metricssvc.MetricsService``) on a UDS.

The reference ships the generated server interface (metricssvc_grpc.pb.go:89-128)
but never uses it in a test. Here it backs health-flip and fault-injection
tests: set ``states[bdf] = "healthy" | "unhealthy"`` and the next health sweep
sees it; ``delay_s`` simulates a slow exporter.
"""
from __future__ import annotations

import asyncio
import os
from typing import Dict, Optional

import grpc

from ..proto import metricssvc as ms


class FakeExporter:
    def __init__(self, socket_path: str, states: Optional[Dict[str, str]] = None):
        self.socket = socket_path
        self.states: Dict[str, str] = dict(states or {})
        self.delay_s = 0.0
        self.calls = 0
        self.server: Optional[grpc.aio.Server] = None

    def _resp(self, ids=None):
        r = ms.GPUStateResponse()
        for i, (bdf, h) in enumerate(sorted(self.states.items())):
            if ids and str(i) not in ids:
                continue
            r.GPUState.add(ID=str(i), UUID=f"uuid-{i}", Health=h, Device=bdf)
        return r

    async def List(self, request, context):  # noqa: N802
        self.calls += 1
        if self.delay_s:
            await asyncio.sleep(self.delay_s)
        return self._resp()

    async def GetGPUState(self, request, context):  # noqa: N802
        self.calls += 1
        return self._resp(set(request.ID))

    async def start(self) -> None:
        os.makedirs(os.path.dirname(self.socket), exist_ok=True)
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass
        self.server = grpc.aio.server()
        self.server.add_generic_rpc_handlers((ms.metrics_service_handler(self),))
        self.server.add_insecure_port(f"unix:{self.socket}")
        await self.server.start()

    async def stop(self) -> None:
        if self.server is not None:
            await self.server.stop(grace=0.1)
            self.server = None
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass
