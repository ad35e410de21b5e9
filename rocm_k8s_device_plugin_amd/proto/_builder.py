"""Tiny DSL that builds protobuf message classes and gRPC method tables from
hand-written descriptors at import time.

The image has the protobuf runtime and grpcio but no ``grpc_tools`` codegen
(SURVEY §0.1), so the wire contracts are declared here field-by-field —
names, numbers, labels and types copied from the .proto definitions cited in
each module — and materialised through ``descriptor_pool`` +
``message_factory``. The result is wire-identical to protoc output.
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from google.protobuf import descriptor_pool, message_factory

# FieldDescriptorProto.Type / .Label values (descriptor.proto); spelled out so
# that a plugin start with a warm cache never imports descriptor_pb2 (~18 ms)
_SCALARS = {
    "double": 1, "float": 2, "int64": 3, "uint64": 4, "int32": 5, "bool": 8, "string": 9, "bytes": 12,
    "uint32": 13,
}
_TYPE_MESSAGE, _TYPE_ENUM = 11, 14
_LABEL_OPTIONAL, _LABEL_REPEATED = 1, 3

# serialized FileDescriptorProtos keyed by a hash of the declarations above
_CACHE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_fdcache")


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
    try:
        fd_desc = pool.FindFileByName(filename)
    except KeyError:
        fd_desc = None
    if fd_desc is None:
        key = hashlib.sha1(repr((package, filename, list(messages), list(services), list(enums), list(deps)))
                           .encode()).hexdigest()[:16]
        cached = os.path.join(_CACHE_DIR, f"{filename.replace('/', '_')}.{key}.pb")
        try:
            with open(cached, "rb") as f:
                pool.AddSerializedFile(f.read())
        except OSError:
            blob = _file_proto(package, filename, messages, services, enums, deps).SerializeToString()
            pool.AddSerializedFile(blob)
            try:  # best effort: a read-only install just builds every time
                os.makedirs(_CACHE_DIR, exist_ok=True)
                tmp = f"{cached}.{os.getpid()}.tmp"
                with open(tmp, "wb") as f:
                    f.write(blob)
                os.replace(tmp, cached)
            except OSError:
                pass
        fd_desc = pool.FindFileByName(filename)
    classes: Dict[str, type] = {}
    for m in messages:
        classes[m.name] = message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{package}.{m.name}"))
    return classes, fd_desc


def _file_proto(package: str, filename: str, messages: Sequence[Message], services: Sequence[Service],
                enums: Sequence[EnumDef], deps: Sequence[str]):
    from google.protobuf import descriptor_pb2
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
                entry.field.add(name="key", number=1, label=_LABEL_OPTIONAL, type=_SCALARS[k.strip()],
                                json_name="key")
                entry.field.add(name="value", number=2, label=_LABEL_OPTIONAL, type=_SCALARS[v.strip()],
                                json_name="value")
                fd.label = _LABEL_REPEATED
                fd.type = _TYPE_MESSAGE
                fd.type_name = f".{package}.{m.name}.{entry.name}"
                continue
            fd.label = _LABEL_REPEATED if f.repeated else _LABEL_OPTIONAL
            if f.type in _SCALARS:
                fd.type = _SCALARS[f.type]
            elif f.type in enum_names:
                fd.type = _TYPE_ENUM
                fd.type_name = f".{package}.{f.type}"
            else:
                fd.type = _TYPE_MESSAGE
                fd.type_name = f.type if f.type.startswith(".") else f".{package}.{f.type}"
    for s in services:
        sd = fdp.service.add(name=s.name)
        for mt in s.methods:
            sd.method.add(name=mt.name,
                          input_type=mt.input if mt.input.startswith(".") else f".{package}.{mt.input}",
                          output_type=mt.output if mt.output.startswith(".") else f".{package}.{mt.output}",
                          server_streaming=mt.server_streaming)
    return fdp


def _lower_camel(s: str) -> str:
    parts = s.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])
