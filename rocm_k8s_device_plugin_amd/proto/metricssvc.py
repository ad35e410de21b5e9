"""AMD device-metrics-exporter health service (``metricssvc``).

Wire contract source: internal/pkg/exporter/metricssvc/metricssvc.pb.go:46-66
(enum GPUHealth), :95-110 (GPUState), :179-186 (GPUGetRequest), :227-236
(GPUUpdateRequest), :284-291 (GPUStateResponse) and metricssvc_grpc.pb.go:44-47,169-184
(service ``metricssvc.MetricsService`` with GetGPUState and List).
``List`` takes ``google.protobuf.Empty``.
"""
from __future__ import annotations

import grpc
from google.protobuf import empty_pb2

from ._builder import EnumDef, Field, Message, Method, Service, build_file

PACKAGE = "metricssvc"
SERVICE = "MetricsService"
DEFAULT_SOCKET = "/var/lib/amd-metrics-exporter/amdgpu_device_metrics_exporter_grpc.socket"

_MESSAGES = [
    Message("GPUState", [Field("ID", 1, "string", json_name="ID"), Field("UUID", 2, "string", json_name="UUID"),
                         Field("Health", 3, "string", json_name="Health"),
                         Field("AssociatedWorkload", 4, "string", repeated=True, json_name="AssociatedWorkload"),
                         Field("Device", 5, "string", json_name="Device")]),
    Message("GPUGetRequest", [Field("ID", 1, "string", repeated=True, json_name="ID")]),
    Message("GPUUpdateRequest", [Field("ID", 1, "string", repeated=True, json_name="ID"),
                                 Field("Health", 2, "string", repeated=True, json_name="Health")]),
    Message("GPUStateResponse", [Field("GPUState", 1, "GPUState", repeated=True, json_name="GPUState")]),
]
_ENUMS = [EnumDef("GPUHealth", [("UNKNOWN", 0), ("HEALTHY", 1), ("UNHEALTHY", 2)])]
_SERVICE = Service(SERVICE, [
    Method("GetGPUState", "GPUGetRequest", "GPUStateResponse"),
    Method("List", ".google.protobuf.Empty", "GPUStateResponse"),
])

_classes, FILE_DESCRIPTOR = build_file(PACKAGE, "metricssvc.proto", _MESSAGES, [_SERVICE], _ENUMS,
                                       deps=["google/protobuf/empty.proto"])
GPUState = _classes["GPUState"]
GPUGetRequest = _classes["GPUGetRequest"]
GPUUpdateRequest = _classes["GPUUpdateRequest"]
GPUStateResponse = _classes["GPUStateResponse"]
Empty = empty_pb2.Empty


def _ser(m) -> bytes:
    return m.SerializeToString()


class MetricsServiceStub:
    def __init__(self, channel):
        self.GetGPUState = channel.unary_unary(f"/{PACKAGE}.{SERVICE}/GetGPUState", request_serializer=_ser,
                                               response_deserializer=GPUStateResponse.FromString)
        self.List = channel.unary_unary(f"/{PACKAGE}.{SERVICE}/List", request_serializer=_ser,
                                        response_deserializer=GPUStateResponse.FromString)


def metrics_service_handler(servicer) -> grpc.GenericRpcHandler:
    handlers = {
        "GetGPUState": grpc.unary_unary_rpc_method_handler(
            servicer.GetGPUState, request_deserializer=GPUGetRequest.FromString, response_serializer=_ser),
        "List": grpc.unary_unary_rpc_method_handler(
            servicer.List, request_deserializer=Empty.FromString, response_serializer=_ser),
    }
    return grpc.method_handlers_generic_handler(f"{PACKAGE}.{SERVICE}", handlers)
