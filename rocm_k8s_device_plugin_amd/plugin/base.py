"""Device strategy interface and per-resource plugin context.

Mirrors the reference contract (internal/pkg/types/api.go:25-56):
``DeviceImpl{Start, GetResourceNames, GetOptions, Enumerate, Allocate,
GetPreferredAllocation, UpdateHealth}`` and
``DevicePluginContext{ResourceName, SetAllocatorError, GetAllocator, GetAllocatorError}``.
"""
from __future__ import annotations

import abc
import os
from dataclasses import dataclass, field
from typing import List, Optional

from ..allocator import BestEffortPolicy, Policy
from ..proto import deviceplugin as pb
from ..utils import log


class DeviceImplError(Exception):
    """Init/runtime error of a device strategy."""


@dataclass
class PluginContext:
    resource: str
    allocator: Optional[Policy] = None
    allocator_error: bool = False
    extra: dict = field(default_factory=dict)

    # reference-style accessors
    def ResourceName(self) -> str:  # noqa: N802
        return self.resource

    def SetAllocatorError(self, err: bool) -> None:  # noqa: N802
        self.allocator_error = err

    def GetAllocator(self) -> Optional[Policy]:  # noqa: N802
        return self.allocator

    def GetAllocatorError(self) -> bool:  # noqa: N802
        return self.allocator_error


def new_context(resource: str, extended_search="auto") -> PluginContext:
    """One allocator per resource, like the reference's lister.NewPlugin (manager.go:96-104)."""
    try:
        alloc = BestEffortPolicy(extended_search=extended_search)
    except ImportError:
        alloc = None
    return PluginContext(resource=resource, allocator=alloc)


class DeviceImpl(abc.ABC):
    name: str = ""

    @abc.abstractmethod
    def start(self, ctx: PluginContext) -> None:
        """Called after init and before registration with kubelet."""

    @abc.abstractmethod
    def resource_names(self) -> List[str]:
        ...

    @abc.abstractmethod
    def options(self, ctx: PluginContext) -> pb.DevicePluginOptions:
        ...

    @abc.abstractmethod
    def enumerate(self, ctx: PluginContext) -> List[pb.Device]:
        ...

    @abc.abstractmethod
    def allocate(self, ctx: PluginContext, req: pb.AllocateRequest) -> pb.AllocateResponse:
        ...

    @abc.abstractmethod
    def preferred_allocation(self, ctx: PluginContext,
                             req: pb.PreferredAllocationRequest) -> pb.PreferredAllocationResponse:
        ...

    @abc.abstractmethod
    def update_health(self, ctx: PluginContext) -> List[pb.Device]:
        """Current device list of ctx.resource with up-to-date health."""

    # optional: async health refresh hook, invoked once per pulse by the manager
    async def refresh_health(self) -> bool:
        """Re-evaluate health; return True if any verdict changed."""
        return False

    def health_version(self) -> int:
        return 0

    def fabric_version(self) -> int:
        """Bumped when the live xGMI link state changes the pair weights; the
        manager then re-initialises every resource's allocator."""
        return 0

    def topology_fingerprint(self):
        """Cheap value that changes when the GPU topology does (None: not tracked)."""
        return None

    async def reload_topology(self) -> Optional[dict]:
        """Re-discover devices if the node's GPU topology changed; None if the
        advertised devices are unchanged (see ContainerImpl.reload_topology)."""
        return None

    async def close(self) -> None:
        """Release helper processes (e.g. the liveness probe server) at shutdown."""


def driver_present(path: str) -> bool:
    """Is the driver behind `path` loaded? (reference: checkDriver,
    internal/pkg/amdgpu/utils.go:24-31 — stat plus a log line on absence)."""
    if os.path.exists(path):
        return True
    log.get("plugin").info("driver path %s not present", path)
    return False


def device_proto(dev_id: str, health: str, numa: Optional[int] = None) -> pb.Device:
    d = pb.Device(ID=dev_id, health=health)
    if numa is not None and numa >= 0:
        d.topology.nodes.add(ID=numa)
    return d
