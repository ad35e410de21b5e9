"""Wire-contract parity: our hand-built descriptors vs the FileDescriptorProtos
embedded in the reference's generated Go code (gogo api.pb.go, gzipped; and
metricssvc.pb.go, raw). Field names, numbers, labels, types and the service
method signatures must be identical for kubelet / the exporter to interoperate.
The reference files are read as text; nothing from them is executed."""
import gzip
import re

import pytest
from google.protobuf import descriptor_pb2

from rocm_k8s_device_plugin_amd.proto import deviceplugin as dp
from rocm_k8s_device_plugin_amd.proto import metricssvc as ms

API_PB = "vendor/k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.pb.go"
MS_PB = "internal/pkg/exporter/metricssvc/metricssvc.pb.go"


def _go_bytes(text: str, var: str) -> bytes:
    m = re.search(r"var " + re.escape(var) + r" = \[\]byte\{(.*?)\n\}", text, re.S)
    assert m, var
    body = re.sub(r"//[^\n]*", "", m.group(1))
    return bytes(int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]{2}", body))


def _fields(fdp):
    out = {}
    for m in fdp.message_type:
        for f in m.field:
            if f.type_name.endswith("Entry"):
                tn = "map"
            else:
                tn = f.type_name.split(".")[-1]
            out[(m.name, f.name)] = (f.number, f.label, f.type, tn)
    return out


def _services(fdp):
    return {(s.name, m.name): (m.input_type.split(".")[-1], m.output_type.split(".")[-1],
                               bool(m.server_streaming), bool(m.client_streaming))
            for s in fdp.service for m in s.method}


def _ours(desc):
    fdp = descriptor_pb2.FileDescriptorProto()
    desc.CopyToProto(fdp)
    return fdp


def test_deviceplugin_descriptor_matches_reference(ref_testdata):
    src = (ref_testdata.parent / API_PB).read_text()
    ref = descriptor_pb2.FileDescriptorProto.FromString(
        gzip.decompress(_go_bytes(src, "fileDescriptor_00212fb1f9d3bf1c")))
    ours = _ours(dp.FILE_DESCRIPTOR)
    assert ref.package == ours.package == "v1beta1"
    assert _fields(ours) == _fields(ref)
    assert _services(ours) == _services(ref)


def test_metricssvc_descriptor_matches_reference(ref_testdata):
    src = (ref_testdata.parent / MS_PB).read_text()
    ref = descriptor_pb2.FileDescriptorProto.FromString(_go_bytes(src, "file_metricssvc_proto_rawDesc"))
    ours = _ours(ms.FILE_DESCRIPTOR)
    assert ref.package == ours.package == "metricssvc"
    assert _fields(ours) == _fields(ref)
    assert _services(ours) == _services(ref)
    assert [e.name for e in ref.enum_type] == [e.name for e in ours.enum_type]
    assert [(v.name, v.number) for v in ref.enum_type[0].value] == [(v.name, v.number)
                                                                    for v in ours.enum_type[0].value]


def test_roundtrip_wire_bytes():
    r = dp.ContainerAllocateResponse(envs={"A": "1"})
    r.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
    b = r.SerializeToString()
    # field 1 (map entry, LEN) then field 3 (DeviceSpec, LEN)
    assert b[0] == (1 << 3 | 2) and (3 << 3 | 2) in b
    assert dp.ContainerAllocateResponse.FromString(b) == r
    d = dp.Device(ID="0000:05:00.0", health=dp.HEALTHY)
    d.topology.nodes.add(ID=1)
    assert dp.Device.FromString(d.SerializeToString()).topology.nodes[0].ID == 1


def test_constants():
    assert dp.VERSION == "v1beta1"
    assert dp.DEVICE_PLUGIN_PATH == "/var/lib/kubelet/device-plugins/"
    assert dp.KUBELET_SOCKET.endswith("device-plugins/kubelet.sock")
    assert (dp.HEALTHY, dp.UNHEALTHY) == ("Healthy", "Unhealthy")
