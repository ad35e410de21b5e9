"""Tiny DSL that builds protobuf message classes and gRPC method tables from
hand-written descriptors at import time.

The image has the protobuf runtime and grpcio but no ``grpc_tools`` codegen
(SURVEY §0.1), so the wire contracts are declared here field-by-field —
names, numbers, labels and types copied from the .proto definitions cited in
each module — and materialised through ``descriptor_pool`` +
``message_factory``. The result is wire-identical to protoc output.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto

_SCALARS = {
    "string": F.TYPE_STRING,
    "bool": F.TYPE_BOOL,
    "int32": F.TYPE_INT32,
    "int64": F.TYPE_INT64,
    "uint32": F.TYPE_UINT32,
    "uint64": F.TYPE_UINT64,
    "bytes": F.TYPE_BYTES,
    "double": F.TYPE_DOUBLE,
    "float": F.TYPE_FLOAT,
}


@dataclass
class Field:
    name: str
    number: int
    type: str                 # scalar name, message name (relative), or "map<string,string>"
    repeated: bool = False
    json_name: Optional[str] = None


@dataclass
class Message:
    name: str
    fields: List[Field] = field(default_factory=list)


@dataclass
class Method:
    name: str
    input: str
    output: str
    server_streaming: bool = False


@dataclass
class Service:
    name: str
    methods: List[Method]


@dataclass
class EnumDef:
    name: str
    values: List[Tuple[str, int]]


def _camel(s: str) -> str:
    return "".join(p[:1].upper() + p[1:] for p in s.split("_"))


def build_file(package: str, filename: str, messages: Sequence[Message], services: Sequence[Service] = (),
               enums: Sequence[EnumDef] = (), deps: Sequence[str] = (),
               pool: Optional[descriptor_pool.DescriptorPool] = None):
    """Register the file in `pool` and return {message name: class}."""
    pool = pool or descriptor_pool.Default()
    fdp = descriptor_pb2.FileDescriptorProto(name=filename, package=package, syntax="proto3")
    fdp.dependency.extend(deps)
    for e in enums:
        ed = fdp.enum_type.add(name=e.name)
        for n, v in e.values:
            ed.value.add(name=n, number=v)
    enum_names = {e.name for e in enums}
    for m in messages:
        md = fdp.message_type.add(name=m.name)
        for f in m.fields:
            fd = md.field.add(name=f.name, number=f.number)
            fd.json_name = f.json_name or _lower_camel(f.name)
            if f.type.startswith("map<"):
                k, v = f.type[4:-1].split(",")
                entry = md.nested_type.add(name=_camel(f.name) + "Entry")
                entry.options.map_entry = True
                entry.field.add(name="key", number=1, label=F.LABEL_OPTIONAL, type=_SCALARS[k.strip()],
                                json_name="key")
                entry.field.add(name="value", number=2, label=F.LABEL_OPTIONAL, type=_SCALARS[v.strip()],
                                json_name="value")
                fd.label = F.LABEL_REPEATED
                fd.type = F.TYPE_MESSAGE
                fd.type_name = f".{package}.{m.name}.{entry.name}"
                continue
            fd.label = F.LABEL_REPEATED if f.repeated else F.LABEL_OPTIONAL
            if f.type in _SCALARS:
                fd.type = _SCALARS[f.type]
            elif f.type in enum_names:
                fd.type = F.TYPE_ENUM
                fd.type_name = f".{package}.{f.type}"
            else:
                fd.type = F.TYPE_MESSAGE
                fd.type_name = f.type if f.type.startswith(".") else f".{package}.{f.type}"
    for s in services:
        sd = fdp.service.add(name=s.name)
        for mt in s.methods:
            sd.method.add(name=mt.name,
                          input_type=mt.input if mt.input.startswith(".") else f".{package}.{mt.input}",
                          output_type=mt.output if mt.output.startswith(".") else f".{package}.{mt.output}",
                          server_streaming=mt.server_streaming)
    try:
        fd_desc = pool.FindFileByName(filename)
    except KeyError:
        fd_desc = pool.Add(fdp)
        if not hasattr(fd_desc, "message_types_by_name"):
            fd_desc = pool.FindFileByName(filename)
    classes: Dict[str, type] = {}
    for m in messages:
        classes[m.name] = message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{package}.{m.name}"))
    return classes, fd_desc


def _lower_camel(s: str) -> str:
    parts = s.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])
