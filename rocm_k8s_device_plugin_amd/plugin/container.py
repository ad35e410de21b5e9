"""Container (ROCm/KFD) device strategy.

Reference: AMDGPUKFDImpl, internal/pkg/amdgpu/amdgpu.go:47-345.

Kept identical (drop-in): device IDs (BDF / amdgpu_xcp_N), resource names
(``gpu`` | ``<compute>_<memory>``), the heterogeneous+single init error, the
``/dev/kfd`` + ``/dev/dri/card<N>`` + ``/dev/dri/renderD<N>`` spec list with
``rw`` permissions, GetPreferredAllocationAvailable unless allocator init
failed, NUMA topology hints.

Changed: per-device health (health.monitor), immutable device snapshots,
deterministic device-node order, an error (not silently empty specs) for an
unknown device ID, and a hive-aware exact allocator. New: the node is
re-discovered when its GPU topology changes (``reload_topology``: a compute /
memory partition switch done with amd-smi while the plugin runs); the
reference computes its device list once at start-up and keeps advertising
devices that no longer exist until it is restarted.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

from .. import cdi
from .. import constants as C
from ..allocator import AllocationError
from ..health.monitor import HealthConfig, HealthMonitor
from ..proto import deviceplugin as pb
from ..topology import Gpu, Inventory, discover, topology_signature
from ..node_view import NodeView
from ..topology_view import KFD_TOPOLOGY_CONTAINER_PATH, TopologyViews
from ..utils import log
from ..utils.metrics import REGISTRY
from .base import DeviceImpl, DeviceImplError, PluginContext, device_proto, driver_present

_log = log.get("container")

_HETERO_SINGLE = ("Partitions of different styles across GPUs in a node is not supported with single strategy. "
                  "Please start device plugin with mixed strategy")


class ContainerImpl(DeviceImpl):
    name = C.CONTAINER

    def __init__(self, naming_strategy: str = C.STRATEGY_SINGLE, sysfs_root: str = "/sys",
                 health_cfg: Optional[HealthConfig] = None, device_count_limit: Optional[int] = None,
                 inventory: Optional[Inventory] = None, monitor: Optional[HealthMonitor] = None,
                 topology_view_dir: Optional[str] = None, node_view_dir: Optional[str] = None,
                 device_list_strategy: Sequence[str] = (cdi.DEVICE_SPECS,), cdi_spec_dir: str = cdi.DEFAULT_SPEC_DIR):
        self.strategy = naming_strategy
        # what Allocate returns: DeviceSpecs (reference) and/or CDI device names
        self.list_strategies = tuple(device_list_strategy) or (cdi.DEVICE_SPECS,)
        self.cdi_spec_dir = cdi_spec_dir
        self._cdi = any(s != cdi.DEVICE_SPECS for s in self.list_strategies)
        self.sysfs_root = sysfs_root
        # opt-in: per-allocation filtered kfd topology bind-mounted into the container
        self._listeners: List = []   # called when what Allocate returns changes (native server templates)
        self._topology_views = (TopologyViews(topology_view_dir, os.path.join(sysfs_root, "class/kfd/kfd/topology"))
                                if topology_view_dir else None)
        # opt-in: NUMA-node sysfs without the per-CPU cache walk ROCr does at start-up
        self._node_view = NodeView(node_view_dir, sysfs_root) if node_view_dir else None
        if self.node_view is not None:  # build at start-up, not inside the first Allocate
            try:
                self.node_view.path()
            except OSError as e:
                _log.warning("node view unavailable: %s", e)
        if not driver_present(os.path.join(sysfs_root, C.KFD_CLASS_REL)):
            raise DeviceImplError("No amd gpu driver loaded")
        self.device_count_limit = device_count_limit
        self.health_cfg = health_cfg or HealthConfig()
        self._epoch = 0            # bumped by every topology reload (part of health_version)
        self._sig = self._signature()
        self._pinned = inventory is not None
        self.inv = inventory or discover(sysfs_root, device_count_limit)
        for w in self.inv.warnings:
            _log.warning("%s", w)
        self._report_kfd_access(self.inv)
        self.homogeneous = self.inv.homogeneous
        if not self.homogeneous and self.strategy == C.STRATEGY_SINGLE:
            raise DeviceImplError(_HETERO_SINGLE)
        self.monitor = monitor or HealthMonitor(self.inv, self.health_cfg)
        self._resources = self._compute_resource_names()
        self._members: Dict[str, List[Gpu]] = {r: self._devices_for(r) for r in self._resources}
        _log.info("Found %d AMDGPUs (%s)", len(self.inv), ", ".join(
            f"{r}={len(v)}" for r, v in self._members.items()))
        if self._cdi:
            try:
                self._write_cdi_specs()
            except (OSError, ValueError) as e:
                raise DeviceImplError(f"cannot write CDI specs to {self.cdi_spec_dir}: {e}") from e

    @staticmethod
    def _report_kfd_access(inv: Inventory) -> None:
        """kfd answers EPERM for the topology nodes of GPUs the plugin's device
        cgroup denies (a non-privileged pod without /dev: the drop-in Helm
        chart's default). Say so loudly: identity then comes from PCI sysfs,
        or — when even that fails — placement cannot be topology-aware."""
        REGISTRY.set("mi355x_dp_kfd_unreadable_nodes", float(len(inv.kfd_unreadable_nodes)),
                     help="kfd topology nodes whose properties the plugin cannot read (EPERM)")
        REGISTRY.set("mi355x_dp_devices_identity_from_sysfs", float(len(inv.recovered)),
                     help="devices identified from PCI sysfs because their kfd node is unreadable")
        REGISTRY.set("mi355x_dp_devices_identity_unknown", float(len(inv.unresolved)),
                     help="devices without a known physical GPU / xGMI hive (placement not topology-aware)")
        if inv.kfd_unreadable_nodes:
            _log.warning("kfd denies %d topology node(s) %s to this process; %d device(s) identified from "
                         "PCI sysfs (unique_id, xgmi_hive_id, amdgpu_xcp block layout). Run the plugin with /dev "
                         "mounted or privileged for kfd-exact topology.", len(inv.kfd_unreadable_nodes),
                         list(inv.kfd_unreadable_nodes), len(inv.recovered))
        if not inv.placement_trusted:
            _log.warning("physical-GPU identity unknown for %s: GetPreferredAllocation disabled (kubelet picks "
                         "devices itself) rather than placing by an incomplete topology", list(inv.unresolved))

    def _write_cdi_specs(self, stale=()) -> None:
        # before registration: kubelet may hand a CDI name to the runtime as
        # soon as the first Allocate returns, the spec must already be there
        paths = cdi.write_specs(self.cdi_spec_dir, self._members, stale)
        _log.info("CDI specs written: %s", ", ".join(paths))

    # ------------------------------------------------------------- resources
    def _compute_resource_names(self) -> List[str]:
        if len(self.inv) == 0:
            return []
        counts = self.inv.partition_counts()
        if self.homogeneous:
            if self.strategy == C.STRATEGY_SINGLE or not counts:
                return [C.DEVICE_TYPE_GPU]
            return sorted(t for t, c in counts.items() if c > 0)
        return sorted(t for t, c in counts.items() if c > 0)

    def _devices_for(self, resource: str) -> List[Gpu]:
        if self.homogeneous:
            return list(self.inv.devices)
        return [d for d in self.inv.devices if d.partition_type == resource]

    def resource_names(self) -> List[str]:
        return list(self._resources)

    def devices(self, resource: str) -> List[Gpu]:
        return list(self._members.get(resource, []))

    # ------------------------------------------------------------- lifecycle
    def start(self, ctx: PluginContext) -> None:
        devs = self._members.get(ctx.resource, list(self.inv.devices))
        ctx.allocator_error = False  # re-evaluated on every (re)start, e.g. after a topology reload
        if ctx.allocator is None:
            ctx.allocator_error = True
            return
        unknown = set(self.inv.unresolved) & {d.id for d in devs}
        if unknown:
            _log.error("allocator disabled for plugin %s: no physical-GPU identity for %s (kfd unreadable, no "
                       "sysfs unique_id). Falling back to kubelet default allocation.", ctx.resource, sorted(unknown))
            ctx.allocator_error = True
            return
        try:
            ctx.allocator.init(devs, self.inv.topology, degraded_links=self.monitor.degraded_links())
        except AllocationError as e:
            _log.error("allocator init failed for plugin %s. Falling back to kubelet default allocation. "
                       "Error %s", ctx.resource, e)
            ctx.allocator_error = True

    def options(self, ctx: PluginContext) -> pb.DevicePluginOptions:
        if ctx.allocator_error:
            return pb.DevicePluginOptions()
        return pb.DevicePluginOptions(get_preferred_allocation_available=True)

    # ---------------------------------------------------------------- device lists
    def _device_list(self, resource: str) -> List[pb.Device]:
        snap = self.monitor.snapshot()
        out = []
        for d in self._members.get(resource, []):
            v = snap.get(d.id)
            out.append(device_proto(d.id, v.health if v else pb.HEALTHY, d.numa_node))
        return out

    def enumerate(self, ctx: PluginContext) -> List[pb.Device]:
        return self._device_list(ctx.resource)

    def update_health(self, ctx: PluginContext) -> List[pb.Device]:
        return self._device_list(ctx.resource)

    async def refresh_health(self) -> bool:
        return await self.monitor.check_once()

    def health_version(self) -> int:
        # a reload replaces the monitor (its version restarts): the epoch keeps
        # the combined value moving so every ListAndWatch stream re-sends
        return self._epoch * 1_000_000_000 + self.monitor.version

    def fabric_version(self) -> int:
        return self._epoch * 1_000_000_000 + self.monitor.fabric_version

    # ---------------------------------------------------------------- topology reload
    def _signature(self) -> tuple:
        return topology_signature(self.sysfs_root)

    def topology_fingerprint(self):
        return None if self._pinned else self._signature()

    async def reload_topology(self) -> Optional[dict]:
        """Re-discover when the topology fingerprint changed.

        Returns None when the advertised devices did not change, else
        ``{"resources_changed": bool, "added": [...], "removed": [...],
        "resources": [...]}``. RPC handlers see the old or the new snapshots,
        never a mix (they are swapped in one step between awaits). The health
        monitor is rebuilt: a probe server's GPU agents were enumerated at its
        start and no longer match.
        """
        if self._pinned:  # the caller chose the devices (benchmarks, tests): keep them
            return None
        sig = self._signature()
        if sig == self._sig:
            return None
        inv = discover(self.sysfs_root, self.device_count_limit)
        self._sig = sig
        old_ids, new_ids = set(self.inv.by_id), set(inv.by_id)
        if old_ids == new_ids and all(self.inv.by_id[i].partition_type == inv.by_id[i].partition_type
                                      for i in new_ids):
            return None
        for w in inv.warnings:
            _log.warning("%s", w)
        self._report_kfd_access(inv)
        old_resources = list(self._resources)
        monitor = HealthMonitor(inv, self.health_cfg)
        await self.monitor.close()
        self.inv, self.homogeneous, self.monitor = inv, inv.homogeneous, monitor
        if not self.homogeneous and self.strategy == C.STRATEGY_SINGLE:
            _log.error("GPU topology changed: %s. Advertising no devices until then.", _HETERO_SINGLE)
            self._members = {r: [] for r in old_resources}
        else:
            self._resources = self._compute_resource_names()
            self._members = {r: self._devices_for(r) for r in self._resources}
        self._epoch += 1
        if self._cdi:
            try:
                self._write_cdi_specs(stale=old_resources)
            except (OSError, ValueError) as e:
                _log.error("CDI specs not updated after the topology change: %s", e)
        _log.warning("GPU topology changed (kfd generation %s): %d devices (%s); resources %s -> %s",
                     sig[0], len(inv), ", ".join(f"{r}={len(v)}" for r, v in self._members.items()),
                     old_resources, self._resources)
        return {"resources_changed": sorted(self._resources) != sorted(old_resources),
                "added": sorted(new_ids - old_ids), "removed": sorted(old_ids - new_ids),
                "resources": list(self._resources)}

    async def close(self) -> None:
        await self.monitor.close()

    # ---------------------------------------------------------------- allocation
    def allocate(self, ctx: PluginContext, req: pb.AllocateRequest) -> pb.AllocateResponse:
        resp = pb.AllocateResponse()
        specs = cdi.DEVICE_SPECS in self.list_strategies
        for creq in req.container_requests:
            car = resp.container_responses.add()
            # one /dev/kfd per container regardless of the number of GPUs
            if specs:
                car.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
            nodes = []
            for dev_id in creq.devices_ids:
                d = self.inv.by_id.get(dev_id)
                if d is None:
                    raise DeviceImplError(f"unknown device ID {dev_id!r} for resource {ctx.resource}")
                if specs:
                    for p in d.dev_paths():
                        car.devices.add(container_path=p, host_path=p, permissions="rw")
                nodes.append(d.node_id)
            if self._cdi and creq.devices_ids:
                ids = list(creq.devices_ids)
                if cdi.CDI_CRI in self.list_strategies:
                    for i in ids:
                        car.cdi_devices.add(name=cdi.qualified_name(ctx.resource, i))
                if cdi.CDI_ANNOTATIONS in self.list_strategies:
                    car.annotations[cdi.annotation_key(ctx.resource)] = cdi.annotation_value(ctx.resource, ids)
            if self.topology_views is not None and creq.devices_ids and all(n >= 0 for n in nodes):
                try:
                    view = self.topology_views.get(nodes)
                    car.mounts.add(container_path=KFD_TOPOLOGY_CONTAINER_PATH, host_path=view, read_only=True)
                except OSError as e:  # never fail an admission over an optimisation
                    _log.warning("topology view for %s unavailable: %s", list(creq.devices_ids), e)
            if self.node_view is not None and creq.devices_ids:
                try:
                    for host, ctr in self.node_view.mounts():
                        car.mounts.add(container_path=ctr, host_path=host, read_only=True)
                except OSError as e:
                    _log.warning("node view unavailable: %s", e)
        return resp

    # what Allocate returns can change at run time (views switched on/off):
    # the native server's prepared fragments follow through these listeners
    def add_change_listener(self, fn) -> None:
        self._listeners.append(fn)

    def remove_change_listener(self, fn) -> None:
        if fn in self._listeners:
            self._listeners.remove(fn)

    def _changed(self) -> None:
        for fn in list(self._listeners):
            fn()

    @property
    def topology_views(self):
        return self._topology_views

    @topology_views.setter
    def topology_views(self, v) -> None:
        self._topology_views = v
        self._changed()

    @property
    def node_view(self):
        return self._node_view

    @node_view.setter
    def node_view(self, v) -> None:
        self._node_view = v
        self._changed()

    def allocate_template(self, ctx: PluginContext) -> Optional[dict]:
        """Allocate response fragments per device for the native server's fast
        path (plugin/native_server.py); parsed, its responses equal allocate()'s.
        None when a response needs per-request work (topology views: one per
        allocated node set)."""
        if self.topology_views is not None:
            return None
        nonempty = b""
        if self.node_view is not None:
            try:
                nonempty = pb.ContainerAllocateResponse(mounts=[
                    pb.Mount(container_path=ctr, host_path=host, read_only=True)
                    for host, ctr in self.node_view.mounts()]).SerializeToString()
            except OSError:   # allocate() reports it per request
                return None
        specs = cdi.DEVICE_SPECS in self.list_strategies
        prefix = pb.ContainerAllocateResponse()
        if specs:
            prefix.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
        per_device, names = {}, {}
        annotate = self._cdi and cdi.CDI_ANNOTATIONS in self.list_strategies
        try:
            for d in self.inv.devices:
                car = pb.ContainerAllocateResponse()
                if specs:
                    for p in d.dev_paths():
                        car.devices.add(container_path=p, host_path=p, permissions="rw")
                if self._cdi and cdi.CDI_CRI in self.list_strategies:
                    car.cdi_devices.add(name=cdi.qualified_name(ctx.resource, d.id))
                if annotate:
                    names[d.id] = cdi.qualified_name(ctx.resource, d.id)
                per_device[d.id] = car.SerializeToString()
        except ValueError:   # a device ID CDI cannot name: allocate() reports it per request
            return None
        return {"resource": ctx.resource, "container_prefix": prefix.SerializeToString(), "per_device": per_device,
                "annotation_key": cdi.annotation_key(ctx.resource) if annotate else "",
                "annotation_names": names, "container_nonempty": nonempty}

    def preferred_allocation(self, ctx: PluginContext,
                             req: pb.PreferredAllocationRequest) -> pb.PreferredAllocationResponse:
        resp = pb.PreferredAllocationResponse()
        if ctx.allocator is None or ctx.allocator_error:
            raise DeviceImplError("allocator unavailable")
        for creq in req.container_requests:
            try:
                ids = ctx.allocator.allocate(list(creq.available_deviceIDs), list(creq.must_include_deviceIDs),
                                             creq.allocation_size)
            except AllocationError as e:
                raise DeviceImplError(f"unable to get preferred allocation list. Error:{e}") from e
            resp.container_responses.add(deviceIDs=ids)
        return resp
