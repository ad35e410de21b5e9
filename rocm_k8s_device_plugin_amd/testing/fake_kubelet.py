"""A fake kubelet speaking the Device Plugin v1beta1 protocol over UDS.

The reference has no protocol-level tests at all (no fake kubelet, no
bufconn). This one implements the kubelet side faithfully
enough to drive a real plugin end to end:

* ``v1beta1.Registration/Register`` server on ``<dir>/kubelet.sock``;
* on registration: dial ``<dir>/<endpoint>``, GetDevicePluginOptions, then
  consume the ListAndWatch stream into a per-resource device table;
* ``admit(resource, n)``: pick from healthy unallocated devices via
  GetPreferredAllocation (when the plugin advertises it), then Allocate —
  the same sequence kubelet's devicemanager runs for a pod — with timings;
* ``restart()``: delete and recreate the socket like a kubelet restart.
"""
from __future__ import annotations

import asyncio
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import grpc

from ..proto import deviceplugin as pb


@dataclass
class ResourceState:
    endpoint: str
    options: object
    channel: object = None
    stub: object = None
    devices: Dict[str, str] = field(default_factory=dict)   # id -> health
    numa: Dict[str, List[int]] = field(default_factory=dict)
    updates: int = 0
    allocated: set = field(default_factory=set)
    task: Optional[asyncio.Task] = None
    event: asyncio.Event = field(default_factory=asyncio.Event)
    stream_error: Optional[str] = None
    native: object = None   # core().GrpcClient when rpc_client == "native"


@dataclass
class Admission:
    resource: str
    device_ids: List[str]
    response: object
    preferred_ms: float
    allocate_ms: float
    total_ms: float
    preferred_used: bool
    prestart_ms: float = 0.0   # PreStartContainer, when the plugin's options require it


class NativeRpcError(grpc.RpcError):
    """An error status from the native client (same role as AioRpcError)."""

    def __init__(self, status: int, message: str):
        super().__init__(f"status {status}: {message}")
        self.status, self.message = status, message

    def code(self):
        return next((c for c in grpc.StatusCode if c.value[0] == self.status), grpc.StatusCode.UNAVAILABLE)

    def details(self):
        return self.message


class FakeKubelet:
    RPC_CLIENTS = ("aio", "native", "native-thread")

    def __init__(self, plugin_dir: str, rpc_client: str = "aio"):
        """`rpc_client`: how admit() calls GetPreferredAllocation / Allocate.
        "aio": grpc.aio on this event loop (works with any plugin server);
        "native": the native blocking HTTP/2 client (core().GrpcClient) -- a
        kubelet-like native caller, for timing the plugin rather than the
        interpreter. It blocks the loop for the call, so the plugin must not be
        served from this same loop (use it with the native server only);
        "native-thread": the same client called from a worker thread (works with
        any server, at the cost of a thread hop per call)."""
        if rpc_client not in self.RPC_CLIENTS:
            raise ValueError(f"rpc_client must be one of {self.RPC_CLIENTS}")
        self.rpc_client = rpc_client
        self.plugin_dir = plugin_dir
        self.socket = os.path.join(plugin_dir, "kubelet.sock")
        self.server: Optional[grpc.aio.Server] = None
        self.resources: Dict[str, ResourceState] = {}
        self.registrations: List[object] = []
        self.register_times: Dict[str, float] = {}   # resource -> time.monotonic() of its last Register
        self._registered = asyncio.Event()
        # False: after Register, only GetDevicePluginOptions is called and no
        # ListAndWatch stream is opened (a kubelet whose client cannot complete
        # calls on the plugin's transport; drives the plugin's watchdog)
        self.open_list_and_watch = True

    # -------------------------------------------------------------- server side
    async def Register(self, request, context):  # noqa: N802
        self.registrations.append(request)
        self.register_times[request.resource_name] = time.monotonic()
        if request.version != pb.VERSION:
            await context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unsupported version {request.version}")
        old = self.resources.get(request.resource_name)
        if old is not None:
            await self._drop(old)
        st = ResourceState(endpoint=request.endpoint, options=request.options)
        self.resources[request.resource_name] = st
        # kubelet connects back asynchronously, after Register returns
        st.task = asyncio.get_running_loop().create_task(self._watch(request.resource_name, st))
        self._registered.set()
        return pb.Empty()

    async def _watch(self, resource: str, st: ResourceState) -> None:
        path = os.path.join(self.plugin_dir, st.endpoint)
        st.channel = grpc.aio.insecure_channel(f"unix:{path}")
        st.stub = pb.DevicePluginStub(st.channel)
        try:
            st.options = await st.stub.GetDevicePluginOptions(pb.Empty(), timeout=10)
            while not self.open_list_and_watch:
                await asyncio.sleep(0.05)
            async for resp in st.stub.ListAndWatch(pb.Empty()):
                st.devices = {d.ID: d.health for d in resp.devices}
                st.numa = {d.ID: [n.ID for n in d.topology.nodes] for d in resp.devices}
                st.updates += 1
                st.event.set()
        except grpc.aio.AioRpcError as e:
            st.stream_error = f"{e.code().name}: {e.details()}"
        except asyncio.CancelledError:
            pass
        finally:
            st.event.set()

    async def _drop(self, st: ResourceState) -> None:
        if st.native is not None:
            st.native.close()
            st.native = None
        if st.task is not None:
            st.task.cancel()
            await asyncio.gather(st.task, return_exceptions=True)
        if st.channel is not None:
            await st.channel.close()

    async def start(self) -> None:
        os.makedirs(self.plugin_dir, exist_ok=True)
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass
        self.server = grpc.aio.server()
        self.server.add_generic_rpc_handlers((pb.registration_handler(self),))
        self.server.add_insecure_port(f"unix:{self.socket}")
        await self.server.start()

    async def stop(self, remove_socket: bool = True) -> None:
        for st in list(self.resources.values()):
            await self._drop(st)
        if self.server is not None:
            await self.server.stop(grace=0.2)
            self.server = None
        if remove_socket:
            try:
                os.unlink(self.socket)
            except FileNotFoundError:
                pass

    async def restart(self, downtime_s: float = 0.0) -> None:
        """Kubelet restart: plugins are forgotten and must re-register."""
        await self.stop()
        self.resources.clear()
        self._registered.clear()
        if downtime_s:
            await asyncio.sleep(downtime_s)
        await self.start()

    # -------------------------------------------------------------- helpers
    async def wait_for_resource(self, resource: str, min_devices: int = 1, timeout: float = 10.0) -> ResourceState:
        deadline = time.monotonic() + timeout
        while True:
            st = self.resources.get(resource)
            if st is not None and len(st.devices) >= min_devices:
                return st
            left = deadline - time.monotonic()
            if left <= 0:
                raise TimeoutError(f"resource {resource} not advertised (have {list(self.resources)})")
            if st is None:
                self._registered.clear()
                try:
                    await asyncio.wait_for(self._registered.wait(), min(left, 0.2))
                except asyncio.TimeoutError:
                    pass
            else:
                st.event.clear()
                try:
                    await asyncio.wait_for(st.event.wait(), min(left, 0.2))
                except asyncio.TimeoutError:
                    pass

    async def wait_for_update(self, resource: str, after: int, timeout: float = 10.0) -> ResourceState:
        deadline = time.monotonic() + timeout
        st = self.resources[resource]
        while st.updates <= after:
            left = deadline - time.monotonic()
            if left <= 0:
                raise TimeoutError(f"no ListAndWatch update for {resource} after #{after}")
            st.event.clear()
            try:
                await asyncio.wait_for(st.event.wait(), left)
            except asyncio.TimeoutError:
                pass
            st = self.resources.get(resource, st)
        return st

    def healthy_free(self, resource: str) -> List[str]:
        st = self.resources[resource]
        return sorted(d for d, h in st.devices.items() if h == pb.HEALTHY and d not in st.allocated)

    async def admit(self, resource: str, count: int, must_include: Sequence[str] = (),
                    available: Optional[Sequence[str]] = None, use_preferred: bool = True) -> Admission:
        """Allocate `count` devices for one container of a pod."""
        st = self.resources[resource]
        avail = list(available) if available is not None else self.healthy_free(resource)
        if len(avail) < count:
            raise RuntimeError(f"insufficient {resource}: want {count}, free {len(avail)}")
        t0 = time.perf_counter()
        chosen = list(must_include)
        pref_ms = 0.0
        used = False
        if use_preferred and st.options.get_preferred_allocation_available:
            req = pb.PreferredAllocationRequest()
            req.container_requests.add(available_deviceIDs=avail, must_include_deviceIDs=list(must_include),
                                       allocation_size=count)
            try:
                resp = await self._call(st, "GetPreferredAllocation", req, pb.PreferredAllocationResponse)
                chosen = list(resp.container_responses[0].deviceIDs)
                used = True
            except grpc.RpcError:
                chosen = list(must_include)
            pref_ms = (time.perf_counter() - t0) * 1e3
        if len(chosen) != count:  # kubelet's own fallback: fill in order
            for d in avail:
                if len(chosen) >= count:
                    break
                if d not in chosen:
                    chosen.append(d)
        t1 = time.perf_counter()
        areq = pb.AllocateRequest()
        areq.container_requests.add(devices_ids=chosen)
        aresp = await self._call(st, "Allocate", areq, pb.AllocateResponse)
        t2 = time.perf_counter()
        st.allocated.update(chosen)
        pre_ms = 0.0
        if st.options.pre_start_required:
            # kubelet's devicemanager before the container is created (its timeout: 30 s);
            # an error fails the container start
            await self._call(st, "PreStartContainer", pb.PreStartContainerRequest(devices_ids=chosen),
                             pb.PreStartContainerResponse, timeout=30.0)
            pre_ms = (time.perf_counter() - t2) * 1e3
        t3 = time.perf_counter()
        return Admission(resource, chosen, aresp, pref_ms, (t2 - t1) * 1e3, (t3 - t0) * 1e3, used, pre_ms)

    async def _call(self, st: ResourceState, method: str, req, resp_type, timeout: float = 10.0):
        if self.rpc_client == "aio":
            return await getattr(st.stub, method)(req, timeout=timeout)
        if st.native is None:
            from ..ops.native import core
            st.native = core().GrpcClient()
            err = st.native.connect(os.path.join(self.plugin_dir, st.endpoint))
            if err:
                st.native = None
                raise NativeRpcError(-1, err)
        path, data = f"/{pb.PACKAGE}.DevicePlugin/{method}", req.SerializeToString()
        if self.rpc_client == "native-thread":
            status, msg, body = await asyncio.to_thread(st.native.unary, path, data, timeout)
        else:
            status, msg, body = st.native.unary(path, data, timeout)
        if status != 0:
            if status < 0:
                st.native.close()
                st.native = None
            raise NativeRpcError(status, msg)
        return resp_type.FromString(body)

    def release(self, resource: str, ids: Sequence[str]) -> None:
        self.resources[resource].allocated.difference_update(ids)
