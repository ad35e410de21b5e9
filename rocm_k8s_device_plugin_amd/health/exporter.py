"""Client for the AMD device-metrics-exporter health socket.

Reference: internal/pkg/exporter/health.go:36-79 — skip when the socket file
is missing, otherwise a short-lived connection, ``MetricsService.List`` and a
map PCI BDF -> Healthy/Unhealthy. Same semantics here over grpc.aio, with the
reference's 10 s deadline (internal/pkg/types/constants.go:92) as default.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import grpc

from ..constants import EXPORTER_HEALTH_TIMEOUT_S
from ..proto import deviceplugin as dp
from ..proto import metricssvc as ms
from ..utils import log

_log = log.get("exporter")

DEFAULT_SOCKET = ms.DEFAULT_SOCKET


async def get_gpu_health(socket_path: str = DEFAULT_SOCKET,
                         timeout: float = EXPORTER_HEALTH_TIMEOUT_S) -> Optional[Dict[str, str]]:
    """BDF -> "Healthy"/"Unhealthy", or None if the exporter is unavailable."""
    if not socket_path or not os.path.exists(socket_path):
        return None
    try:
        async with grpc.aio.insecure_channel(f"unix:{socket_path}") as ch:
            resp = await ms.MetricsServiceStub(ch).List(ms.Empty(), timeout=timeout)
    except grpc.RpcError as e:
        _log.error("Error getting health info svc : %s", e)
        return None
    out: Dict[str, str] = {}
    for g in resp.GPUState:
        out[g.Device] = dp.HEALTHY if g.Health.strip().lower() == "healthy" else dp.UNHEALTHY
    return out
