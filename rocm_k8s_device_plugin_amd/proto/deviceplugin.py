"""Kubelet Device Plugin API v1beta1 — messages and service tables.

Wire contract source: vendor/k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto
(package ``v1beta1``; services ``Registration`` and ``DevicePlugin``) and
constants.go:19-48. Field names and numbers below match that file exactly;
gogoproto options only affect Go codegen and are not part of the wire format.
"""
from __future__ import annotations

import grpc

from ._builder import Field, Message, Method, Service, build_file

PACKAGE = "v1beta1"

# constants.go
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"
VERSION = "v1beta1"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
KUBELET_SOCKET = DEVICE_PLUGIN_PATH + "kubelet.sock"
PRESTART_TIMEOUT_S = 30

_MESSAGES = [
    Message("DevicePluginOptions", [Field("pre_start_required", 1, "bool"),
                                    Field("get_preferred_allocation_available", 2, "bool")]),
    Message("RegisterRequest", [Field("version", 1, "string"), Field("endpoint", 2, "string"),
                                Field("resource_name", 3, "string"),
                                Field("options", 4, "DevicePluginOptions")]),
    Message("Empty", []),
    Message("ListAndWatchResponse", [Field("devices", 1, "Device", repeated=True)]),
    Message("TopologyInfo", [Field("nodes", 1, "NUMANode", repeated=True)]),
    Message("NUMANode", [Field("ID", 1, "int64", json_name="ID")]),
    Message("Device", [Field("ID", 1, "string", json_name="ID"), Field("health", 2, "string"),
                       Field("topology", 3, "TopologyInfo")]),
    Message("PreStartContainerRequest", [Field("devices_ids", 1, "string", repeated=True)]),
    Message("PreStartContainerResponse", []),
    Message("PreferredAllocationRequest",
            [Field("container_requests", 1, "ContainerPreferredAllocationRequest", repeated=True)]),
    Message("ContainerPreferredAllocationRequest",
            [Field("available_deviceIDs", 1, "string", repeated=True, json_name="availableDeviceIDs"),
             Field("must_include_deviceIDs", 2, "string", repeated=True, json_name="mustIncludeDeviceIDs"),
             Field("allocation_size", 3, "int32")]),
    Message("PreferredAllocationResponse",
            [Field("container_responses", 1, "ContainerPreferredAllocationResponse", repeated=True)]),
    Message("ContainerPreferredAllocationResponse",
            [Field("deviceIDs", 1, "string", repeated=True, json_name="deviceIDs")]),
    Message("AllocateRequest", [Field("container_requests", 1, "ContainerAllocateRequest", repeated=True)]),
    Message("ContainerAllocateRequest", [Field("devices_ids", 1, "string", repeated=True)]),
    Message("CDIDevice", [Field("name", 1, "string")]),
    Message("AllocateResponse", [Field("container_responses", 1, "ContainerAllocateResponse", repeated=True)]),
    Message("ContainerAllocateResponse", [Field("envs", 1, "map<string,string>"),
                                          Field("mounts", 2, "Mount", repeated=True),
                                          Field("devices", 3, "DeviceSpec", repeated=True),
                                          Field("annotations", 4, "map<string,string>"),
                                          Field("cdi_devices", 5, "CDIDevice", repeated=True)]),
    Message("Mount", [Field("container_path", 1, "string"), Field("host_path", 2, "string"),
                      Field("read_only", 3, "bool")]),
    Message("DeviceSpec", [Field("container_path", 1, "string"), Field("host_path", 2, "string"),
                           Field("permissions", 3, "string")]),
]

REGISTRATION = Service("Registration", [Method("Register", "RegisterRequest", "Empty")])
DEVICE_PLUGIN = Service("DevicePlugin", [
    Method("GetDevicePluginOptions", "Empty", "DevicePluginOptions"),
    Method("ListAndWatch", "Empty", "ListAndWatchResponse", server_streaming=True),
    Method("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse"),
    Method("Allocate", "AllocateRequest", "AllocateResponse"),
    Method("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse"),
])

_classes, FILE_DESCRIPTOR = build_file(PACKAGE, "k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto",
                                       _MESSAGES, [REGISTRATION, DEVICE_PLUGIN])

DevicePluginOptions = _classes["DevicePluginOptions"]
RegisterRequest = _classes["RegisterRequest"]
Empty = _classes["Empty"]
ListAndWatchResponse = _classes["ListAndWatchResponse"]
TopologyInfo = _classes["TopologyInfo"]
NUMANode = _classes["NUMANode"]
Device = _classes["Device"]
PreStartContainerRequest = _classes["PreStartContainerRequest"]
PreStartContainerResponse = _classes["PreStartContainerResponse"]
PreferredAllocationRequest = _classes["PreferredAllocationRequest"]
ContainerPreferredAllocationRequest = _classes["ContainerPreferredAllocationRequest"]
PreferredAllocationResponse = _classes["PreferredAllocationResponse"]
ContainerPreferredAllocationResponse = _classes["ContainerPreferredAllocationResponse"]
AllocateRequest = _classes["AllocateRequest"]
ContainerAllocateRequest = _classes["ContainerAllocateRequest"]
CDIDevice = _classes["CDIDevice"]
AllocateResponse = _classes["AllocateResponse"]
ContainerAllocateResponse = _classes["ContainerAllocateResponse"]
Mount = _classes["Mount"]
DeviceSpec = _classes["DeviceSpec"]


def _path(service: Service, method: str) -> str:
    return f"/{PACKAGE}.{service.name}/{method}"


def _ser(msg) -> bytes:
    return msg.SerializeToString()


# --------------------------------------------------------------------- servers

def device_plugin_handler(servicer) -> grpc.GenericRpcHandler:
    """Generic handler routing v1beta1.DevicePlugin RPCs to `servicer`.

    `servicer` provides coroutine methods GetDevicePluginOptions, GetPreferredAllocation,
    Allocate, PreStartContainer(request, context) and an async-generator
    ListAndWatch(request, context).
    """
    handlers = {
        "GetDevicePluginOptions": grpc.unary_unary_rpc_method_handler(
            servicer.GetDevicePluginOptions, request_deserializer=Empty.FromString, response_serializer=_ser),
        "ListAndWatch": grpc.unary_stream_rpc_method_handler(
            servicer.ListAndWatch, request_deserializer=Empty.FromString, response_serializer=_ser),
        "GetPreferredAllocation": grpc.unary_unary_rpc_method_handler(
            servicer.GetPreferredAllocation, request_deserializer=PreferredAllocationRequest.FromString,
            response_serializer=_ser),
        "Allocate": grpc.unary_unary_rpc_method_handler(
            servicer.Allocate, request_deserializer=AllocateRequest.FromString, response_serializer=_ser),
        "PreStartContainer": grpc.unary_unary_rpc_method_handler(
            servicer.PreStartContainer, request_deserializer=PreStartContainerRequest.FromString,
            response_serializer=_ser),
    }
    return grpc.method_handlers_generic_handler(f"{PACKAGE}.DevicePlugin", handlers)


def registration_handler(servicer) -> grpc.GenericRpcHandler:
    handlers = {
        "Register": grpc.unary_unary_rpc_method_handler(
            servicer.Register, request_deserializer=RegisterRequest.FromString, response_serializer=_ser),
    }
    return grpc.method_handlers_generic_handler(f"{PACKAGE}.Registration", handlers)


# --------------------------------------------------------------------- clients

class RegistrationStub:
    def __init__(self, channel):
        self.Register = channel.unary_unary(_path(REGISTRATION, "Register"), request_serializer=_ser,
                                            response_deserializer=Empty.FromString)


class DevicePluginStub:
    def __init__(self, channel):
        self.GetDevicePluginOptions = channel.unary_unary(
            _path(DEVICE_PLUGIN, "GetDevicePluginOptions"), request_serializer=_ser,
            response_deserializer=DevicePluginOptions.FromString)
        self.ListAndWatch = channel.unary_stream(
            _path(DEVICE_PLUGIN, "ListAndWatch"), request_serializer=_ser,
            response_deserializer=ListAndWatchResponse.FromString)
        self.GetPreferredAllocation = channel.unary_unary(
            _path(DEVICE_PLUGIN, "GetPreferredAllocation"), request_serializer=_ser,
            response_deserializer=PreferredAllocationResponse.FromString)
        self.Allocate = channel.unary_unary(
            _path(DEVICE_PLUGIN, "Allocate"), request_serializer=_ser,
            response_deserializer=AllocateResponse.FromString)
        self.PreStartContainer = channel.unary_unary(
            _path(DEVICE_PLUGIN, "PreStartContainer"), request_serializer=_ser,
            response_deserializer=PreStartContainerResponse.FromString)
