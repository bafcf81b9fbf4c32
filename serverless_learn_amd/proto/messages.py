"""Message classes and method paths built from ``serverless_learn.proto``.

The image has no ``protoc`` and no ``grpc_tools``, so instead
of generated ``*_pb2.py`` stubs this module parses the normative ``.proto``
(the proto3 subset it uses: messages with scalar/repeated fields, services
with unary and streaming rpcs, comments, options) into a
``FileDescriptorProto`` and asks the protobuf runtime for message classes.
The reference generated C++ stubs with protoc + grpc_cpp_plugin instead
(/root/reference/src/Makefile:37-41).
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PROTO_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "serverless_learn.proto")

_FT = descriptor_pb2.FieldDescriptorProto
SCALARS = {
    "double": _FT.TYPE_DOUBLE, "float": _FT.TYPE_FLOAT, "int64": _FT.TYPE_INT64,
    "uint64": _FT.TYPE_UINT64, "int32": _FT.TYPE_INT32, "uint32": _FT.TYPE_UINT32,
    "bool": _FT.TYPE_BOOL, "string": _FT.TYPE_STRING, "bytes": _FT.TYPE_BYTES,
    "sint32": _FT.TYPE_SINT32, "sint64": _FT.TYPE_SINT64, "fixed32": _FT.TYPE_FIXED32,
    "fixed64": _FT.TYPE_FIXED64,
}


@dataclass
class FieldDef:
    name: str
    type: str
    number: int
    repeated: bool


@dataclass
class MethodDef:
    name: str
    input: str
    output: str
    client_streaming: bool
    server_streaming: bool


@dataclass
class ProtoDef:
    package: str = ""
    syntax: str = "proto3"
    options: dict = field(default_factory=dict)
    messages: dict = field(default_factory=dict)   # name -> [FieldDef]
    services: dict = field(default_factory=dict)   # name -> [MethodDef]


_TOKEN = re.compile(r'"[^"]*"|[A-Za-z_][A-Za-z0-9_.]*|\d+|[{}();=<>,\[\]]')


def _strip_comments(text: str) -> str:
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    return re.sub(r"//[^\n]*", " ", text)


def parse_proto(text: str) -> ProtoDef:
    toks = _TOKEN.findall(_strip_comments(text))
    pos = 0
    out = ProtoDef()

    def take(expect=None):
        nonlocal pos
        if pos >= len(toks):
            raise SyntaxError("unexpected end of .proto")
        t = toks[pos]
        pos += 1
        if expect is not None and t != expect:
            raise SyntaxError(f"expected {expect!r}, got {t!r}")
        return t

    while pos < len(toks):
        t = take()
        if t == "syntax":
            take("=")
            out.syntax = take().strip('"')
            take(";")
        elif t == "package":
            out.package = take()
            take(";")
        elif t == "option":
            k = take()
            take("=")
            out.options[k] = take().strip('"')
            take(";")
        elif t == "message":
            name = take()
            take("{")
            fields = []
            while toks[pos] != "}":
                rep = False
                ft = take()
                if ft == "repeated":
                    rep, ft = True, take()
                if ft not in SCALARS:
                    raise SyntaxError(f"unsupported field type {ft!r} in {name}")
                fname = take()
                take("=")
                num = int(take())
                take(";")
                fields.append(FieldDef(fname, ft, num, rep))
            take("}")
            out.messages[name] = fields
        elif t == "service":
            sname = take()
            take("{")
            methods = []
            while toks[pos] != "}":
                take("rpc")
                mname = take()
                take("(")
                cs = toks[pos] == "stream"
                if cs:
                    take()
                inp = take()
                take(")")
                take("returns")
                take("(")
                ss = toks[pos] == "stream"
                if ss:
                    take()
                outp = take()
                take(")")
                if toks[pos] == "{":
                    take("{")
                    take("}")
                else:
                    take(";")
                methods.append(MethodDef(mname, inp, outp, cs, ss))
            take("}")
            out.services[sname] = methods
        else:
            raise SyntaxError(f"unexpected token {t!r}")
    return out


def build_file_descriptor(defn: ProtoDef, filename: str = "serverless_learn.proto") -> descriptor_pb2.FileDescriptorProto:
    fdp = descriptor_pb2.FileDescriptorProto(name=filename, package=defn.package, syntax=defn.syntax)
    if "objc_class_prefix" in defn.options:
        fdp.options.objc_class_prefix = defn.options["objc_class_prefix"]
    for mname, fields in defn.messages.items():
        m = fdp.message_type.add(name=mname)
        for f in fields:
            m.field.add(name=f.name, number=f.number, type=SCALARS[f.type],
                        label=_FT.LABEL_REPEATED if f.repeated else _FT.LABEL_OPTIONAL,
                        json_name=_json_name(f.name))
    for sname, methods in defn.services.items():
        s = fdp.service.add(name=sname)
        for md in methods:
            s.method.add(name=md.name, input_type=f".{defn.package}.{md.input}",
                         output_type=f".{defn.package}.{md.output}",
                         client_streaming=md.client_streaming, server_streaming=md.server_streaming)
    return fdp


def _json_name(n: str) -> str:
    parts = n.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


with open(PROTO_PATH) as _f:
    PROTO = parse_proto(_f.read())
PACKAGE = PROTO.package
_pool = descriptor_pool.DescriptorPool()
FILE_DESCRIPTOR = _pool.Add(build_file_descriptor(PROTO))

_classes = {name: message_factory.GetMessageClass(_pool.FindMessageTypeByName(f"{PACKAGE}.{name}"))
            for name in PROTO.messages}

WorkerBirthInfo = _classes["WorkerBirthInfo"]
RegisterBirthAck = _classes["RegisterBirthAck"]
Push = _classes["Push"]
PushOutcome = _classes["PushOutcome"]
Chunk = _classes["Chunk"]
ReceiveFileAck = _classes["ReceiveFileAck"]
PeerList = _classes["PeerList"]
FlowFeedback = _classes["FlowFeedback"]
LoadFeedback = _classes["LoadFeedback"]
Update = _classes["Update"]
Empty = _classes["Empty"]
FileList = _classes["FileList"]


def message_class(name: str):
    return _classes[name]


def method_path(service: str, method: str) -> str:
    """Fully-qualified gRPC path, e.g. /serverless_learn.Worker/ReceiveFile."""
    for md in PROTO.services[service]:
        if md.name == method:
            return f"/{PACKAGE}.{service}/{method}"
    raise KeyError(f"{service}.{method}")


def method_def(service: str, method: str) -> MethodDef:
    for md in PROTO.services[service]:
        if md.name == method:
            return md
    raise KeyError(f"{service}.{method}")


# The seven method paths of the original protocol, byte-for-byte
# (/root/reference/src/protos/serverless_learn.proto:8-56).
REFERENCE_METHODS = (
    "/serverless_learn.Master/RegisterBirth",
    "/serverless_learn.Master/ExchangeUpdates",
    "/serverless_learn.FileServer/DoPush",
    "/serverless_learn.FileServer/CheckUp",
    "/serverless_learn.Worker/ReceiveFile",
    "/serverless_learn.Worker/CheckUp",
    "/serverless_learn.Worker/ExchangeUpdates",
)
