"""Tiny builder for protobuf descriptors at import time.

protoc / grpcio-tools are not on the target image, so wire schemas are
declared in Python and compiled to ``FileDescriptorProto``s here; message
classes come from ``message_factory.GetMessageClass``.  The serialized file
descriptors are also what the reflection service hands to grpcurl.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple, Union

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

FDP = descriptor_pb2.FieldDescriptorProto

STRING = "string"
BYTES = "bytes"
INT32 = "int32"
INT64 = "int64"
UINT64 = "uint64"
DOUBLE = "double"
BOOL = "bool"

_SCALAR_TYPES = {
    STRING: FDP.TYPE_STRING,
    BYTES: FDP.TYPE_BYTES,
    INT32: FDP.TYPE_INT32,
    INT64: FDP.TYPE_INT64,
    UINT64: FDP.TYPE_UINT64,
    DOUBLE: FDP.TYPE_DOUBLE,
    BOOL: FDP.TYPE_BOOL,
}


@dataclass
class Map:
    key: str
    value: str


@dataclass
class Field:
    name: str
    number: int
    type: Union[str, Map]  # scalar name, ".pkg.Message", "enum:.pkg.Enum" or Map
    repeated: bool = False
    oneof: Optional[str] = None
    # proto3 `optional`: presence is tracked (HasField), so "unset" differs
    # from the zero value (a synthetic one-field oneof, declared after the
    # real ones as protoc does)
    proto3_optional: bool = False


@dataclass
class Message:
    name: str
    fields: List[Field]
    enums: Dict[str, Sequence[Tuple[str, int]]] = field(default_factory=dict)


@dataclass
class Method:
    name: str
    input: str
    output: str
    client_streaming: bool = False
    server_streaming: bool = False


@dataclass
class Service:
    name: str
    methods: List[Method]


def _camel(name: str) -> str:
    return "".join(p.capitalize() for p in name.split("_"))


def build_file(
    filename: str,
    package: str,
    messages: Sequence[Message],
    services: Sequence[Service] = (),
    dependencies: Sequence[str] = (),
) -> descriptor_pb2.FileDescriptorProto:
    fdp = descriptor_pb2.FileDescriptorProto(name=filename, package=package, syntax="proto3")
    fdp.dependency.extend(dependencies)
    for msg in messages:
        mp = fdp.message_type.add(name=msg.name)
        for enum_name, values in msg.enums.items():
            ep = mp.enum_type.add(name=enum_name)
            for vname, vnum in values:
                ep.value.add(name=vname, number=vnum)
        oneofs: List[str] = []
        optional: List = []
        for f in msg.fields:
            fp = mp.field.add(name=f.name, number=f.number, json_name=_lower_camel(f.name))
            if isinstance(f.type, Map):
                entry = mp.nested_type.add(name=_camel(f.name) + "Entry")
                entry.options.map_entry = True
                for i, (n, t) in enumerate((("key", f.type.key), ("value", f.type.value)), start=1):
                    ef = entry.field.add(name=n, number=i, label=FDP.LABEL_OPTIONAL, json_name=n)
                    _set_type(ef, t)
                fp.label = FDP.LABEL_REPEATED
                fp.type = FDP.TYPE_MESSAGE
                fp.type_name = f".{package}.{msg.name}.{entry.name}"
                continue
            fp.label = FDP.LABEL_REPEATED if f.repeated else FDP.LABEL_OPTIONAL
            _set_type(fp, f.type)
            if f.oneof is not None:
                if f.oneof not in oneofs:
                    oneofs.append(f.oneof)
                    mp.oneof_decl.add(name=f.oneof)
                fp.oneof_index = oneofs.index(f.oneof)
            elif f.proto3_optional:
                optional.append(fp)
        for fp in optional:
            mp.oneof_decl.add(name="_" + fp.name)
            fp.oneof_index = len(mp.oneof_decl) - 1
            fp.proto3_optional = True
    for svc in services:
        sp = fdp.service.add(name=svc.name)
        for m in svc.methods:
            sp.method.add(
                name=m.name,
                input_type=m.input,
                output_type=m.output,
                client_streaming=m.client_streaming,
                server_streaming=m.server_streaming,
            )
    return fdp


def _lower_camel(name: str) -> str:
    head, *rest = name.split("_")
    return head + "".join(p.capitalize() for p in rest)


def _set_type(fp, t: str) -> None:
    if t in _SCALAR_TYPES:
        fp.type = _SCALAR_TYPES[t]
    elif t.startswith("enum:"):
        fp.type = FDP.TYPE_ENUM
        fp.type_name = t[len("enum:") :]
    else:
        fp.type = FDP.TYPE_MESSAGE
        fp.type_name = t


class CompiledFile:
    """Messages of one file, registered in a private pool."""

    def __init__(self, fdp: descriptor_pb2.FileDescriptorProto, pool: descriptor_pool.DescriptorPool) -> None:
        self.proto = fdp
        self.serialized = fdp.SerializeToString()
        pool.AddSerializedFile(self.serialized)
        self.descriptor = pool.FindFileByName(fdp.name)
        self.pool = pool
        self.messages = {
            name: message_factory.GetMessageClass(desc) for name, desc in self.descriptor.message_types_by_name.items()
        }

    def __getattr__(self, name: str):
        try:
            return self.messages[name]
        except KeyError:
            raise AttributeError(name)
