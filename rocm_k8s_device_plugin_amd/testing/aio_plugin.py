"""A grpc.aio DevicePlugin endpoint for one resource (test harness).

The oracle servicer (plugin/servicer.py) on grpc.aio's C-core HTTP/2 stack:
an implementation of the kubelet-facing wire independent of the framework's
own server, so tests can compare the C++ server's answers with it call by
call. Nothing in the product serves through it.
"""
from __future__ import annotations

import os

import grpc

from ..plugin.base import DeviceImpl, new_context
from ..plugin.servicer import DevicePluginServicer
from ..proto import deviceplugin as pb
from ..utils.broadcast import Broadcast


class AioPlugin:
    """Starts `impl` for `resource`, serves it on ``<plugin_dir>/amd.com_<resource>``
    and registers with ``<plugin_dir>/kubelet.sock``, as the daemon would."""

    def __init__(self, impl: DeviceImpl, plugin_dir: str, resource: str = "gpu", extended_search="auto"):
        self.impl = impl
        self.resource = resource
        self.socket = os.path.join(plugin_dir, f"amd.com_{resource}")
        self.kubelet_socket = os.path.join(plugin_dir, "kubelet.sock")
        self.ctx = new_context(resource, extended_search=extended_search)
        self.pulse = Broadcast()
        self.stop_bc = Broadcast()
        self.servicer = None
        self.server = None

    async def start(self) -> None:
        self.impl.start(self.ctx)
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass
        self.servicer = DevicePluginServicer(self.impl, self.ctx, self.pulse, self.stop_bc)
        self.server = grpc.aio.server(options=[("grpc.so_reuseport", 0)])
        self.server.add_generic_rpc_handlers((pb.device_plugin_handler(self.servicer),))
        self.server.add_insecure_port(f"unix:{self.socket}")
        await self.server.start()
        req = pb.RegisterRequest(version=pb.VERSION, endpoint=os.path.basename(self.socket),
                                 resource_name=f"amd.com/{self.resource}", options=self.impl.options(self.ctx))
        async with grpc.aio.insecure_channel(f"unix:{self.kubelet_socket}") as ch:
            await pb.RegistrationStub(ch).Register(req, timeout=10)

    async def stop(self) -> None:
        self.stop_bc.close()
        self.pulse.close()
        if self.server is not None:
            await self.server.stop(grace=0.5)
            self.server = None
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass
