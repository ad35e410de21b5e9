"""SR-IOV VF and PF passthrough device strategies (KubeVirt).

References: AMDGPUVFImpl (internal/pkg/amdgpu/amdgpu_sriov.go:34-308) and
AMDGPUPFImpl (internal/pkg/amdgpu/amdgpu_pf.go:32-229). One kubelet device
per IOMMU group; Allocate hands out ``/dev/vfio/<group>`` + ``/dev/vfio/vfio``
(``mrw``) and ``PCI_RESOURCE_AMD_COM_<RESOURCE>=<BDF,...>``.

Fixed: the env var lists the BDFs of *all* requested
groups (the reference overwrote it per device, keeping only the last), and
``/dev/vfio/vfio`` is emitted once per container instead of once per device.
The PF init error says "vfio-pci" instead of the reference's copy-pasted "gim".
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional

from .. import constants as C
from ..health import exporter
from ..ops.native import core
from ..proto import deviceplugin as pb
from ..utils import log
from .base import DeviceImpl, DeviceImplError, PluginContext, device_proto, driver_present

_log = log.get("passthrough")


def _group_sort_key(g: str):
    return (0, int(g)) if g.isdigit() else (1, g)


class _PassthroughBase(DeviceImpl):
    driver_rel: str = ""
    driver_missing_msg: str = ""
    mixed_resource: str = ""

    def __init__(self, naming_strategy: str = C.STRATEGY_SINGLE, sysfs_root: str = "/sys",
                 exporter_socket: Optional[str] = exporter.DEFAULT_SOCKET,
                 exporter_fn: Optional[Callable] = None):
        self.strategy = naming_strategy or C.STRATEGY_SINGLE
        self.sysfs_root = sysfs_root
        self.exporter_socket = exporter_socket
        self._exporter_fn = exporter_fn or exporter.get_gpu_health
        if not driver_present(os.path.join(sysfs_root, self.driver_rel)):
            raise DeviceImplError(self.driver_missing_msg)
        res = self._scan()
        if not res.ok:
            raise DeviceImplError(f"Failed to generate {self.name} map: {res.error}")
        self.groups: Dict[str, list] = {g: list(v) for g, v in res.groups.items()}
        self._order = sorted(self.groups, key=_group_sort_key)
        self._health: Dict[str, str] = {g: pb.HEALTHY for g in self._order}
        self._version = 0
        _log.info("Found %d %s IOMMU groups", len(self._order), self.name)

    def _scan(self):  # pragma: no cover - overridden
        raise NotImplementedError

    def resource_names(self) -> List[str]:
        return [self.mixed_resource if self.strategy == C.STRATEGY_MIXED else C.DEVICE_TYPE_GPU]

    def start(self, ctx: PluginContext) -> None:
        ctx.allocator_error = True  # no preferred allocation in passthrough modes

    def options(self, ctx: PluginContext) -> pb.DevicePluginOptions:
        return pb.DevicePluginOptions()

    def _list(self) -> List[pb.Device]:
        return [device_proto(g, self._health[g]) for g in self._order]

    def enumerate(self, ctx: PluginContext) -> List[pb.Device]:
        return self._list()

    def update_health(self, ctx: PluginContext) -> List[pb.Device]:
        return self._list()

    def health_version(self) -> int:
        return self._version

    def _bdfs(self, group: str) -> List[str]:  # pragma: no cover - overridden
        raise NotImplementedError

    def allocate(self, ctx: PluginContext, req: pb.AllocateRequest) -> pb.AllocateResponse:
        resp = pb.AllocateResponse()
        env_name = f"{C.PCI_GPU_ENV_PREFIX}_{ctx.resource.upper()}"
        for creq in req.container_requests:
            car = resp.container_responses.add()
            bdfs: List[str] = []
            for gid in creq.devices_ids:
                if gid not in self.groups:
                    raise DeviceImplError(f"device {gid} not found")
                p = f"/dev/vfio/{gid}"
                car.devices.add(container_path=p, host_path=p, permissions="mrw")
                bdfs.extend(self._bdfs(gid))
            if creq.devices_ids:
                car.devices.add(container_path="/dev/vfio/vfio", host_path="/dev/vfio/vfio", permissions="mrw")
                car.envs[env_name] = ",".join(bdfs)
        return resp

    def preferred_allocation(self, ctx, req) -> pb.PreferredAllocationResponse:
        return pb.PreferredAllocationResponse()

    def _set_health(self, new: Dict[str, str]) -> bool:
        changed = any(self._health.get(k) != v for k, v in new.items())
        self._health = new
        if changed:
            self._version += 1
        return changed


class VfImpl(_PassthroughBase):
    name = C.VF_PASSTHROUGH
    driver_rel = C.GIM_DRIVER_REL
    driver_missing_msg = "No amd gim driver loaded"
    mixed_resource = C.DEVICE_TYPE_GPU_VF

    def _scan(self):
        return core().scan_vf_mapping(self.sysfs_root)

    def _bdfs(self, group: str) -> List[str]:
        return [f.vf for f in self.groups[group]]

    async def refresh_health(self) -> bool:
        """gim driver gone -> all Unhealthy; else a group is Unhealthy iff any
        parent PF is Unhealthy per the exporter (amdgpu_sriov.go:217-308)."""
        if not driver_present(os.path.join(self.sysfs_root, C.GIM_DRIVER_REL)):
            return self._set_health({g: pb.UNHEALTHY for g in self._order})
        pf_health = None
        if self.exporter_socket:
            pf_health = await self._exporter_fn(self.exporter_socket, C.EXPORTER_HEALTH_TIMEOUT_S)
        new = {}
        for g in self._order:
            h = pb.HEALTHY
            for f in self.groups[g]:
                if pf_health and pf_health.get(f.pf) == pb.UNHEALTHY:
                    h = pb.UNHEALTHY
                    break
            new[g] = h
        return self._set_health(new)


class PfImpl(_PassthroughBase):
    name = C.PF_PASSTHROUGH
    driver_rel = C.VFIO_DRIVER_REL
    driver_missing_msg = "No vfio-pci driver loaded"
    mixed_resource = C.DEVICE_TYPE_GPU_PF

    def _scan(self):
        return core().scan_pf_mapping(self.sysfs_root)

    def _bdfs(self, group: str) -> List[str]:
        return [f.pf for f in self.groups[group]]

    async def refresh_health(self) -> bool:
        """vfio-pci driver present -> Healthy (amdgpu_pf.go:210-229)."""
        ok = driver_present(os.path.join(self.sysfs_root, C.VFIO_DRIVER_REL))
        return self._set_health({g: pb.HEALTHY if ok else pb.UNHEALTHY for g in self._order})
