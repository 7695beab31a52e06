"""The reference's API types, built at import from ``api_v1.binpb`` (the FileDescriptorSet of
``determined.api.v1.Determined`` and its messages, written by ``scripts/gen_rpc_descriptors.py``
from the reference's ``proto/buf.image.bin``; reference ``proto/src/determined/api/v1/api.proto``).

No protoc in this image, and none is needed: a private ``DescriptorPool`` takes the file
descriptors, ``message_factory`` makes the Python classes, and each method's ``google.api.http``
option (extension 72295728 of ``MethodOptions``, kept as an unknown field because the stock
``descriptor_pb2`` does not know the extension) is decoded into an ``HttpRule`` of the same pool.

    GetExperimentRequest = request_class("GetExperiment")
    rule = http_rule("GetExperiment")        # ("GET", "/api/v1/experiments/{experiment_id}", "")
"""
import functools
import os
from typing import Dict, List, NamedTuple, Tuple, Type

from google.protobuf import descriptor_pb2, descriptor_pool, message, message_factory

SERVICE = "determined.api.v1.Determined"
_HTTP_EXT = 72295728  # google.api.http on google.protobuf.MethodOptions (google/api/annotations.proto)
_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "api_v1.binpb")


class Method(NamedTuple):
    name: str
    input_type: str
    output_type: str
    server_streaming: bool
    verb: str
    path: str
    body: str  # "" (query string), "*" (whole request) or a field name


@functools.lru_cache(maxsize=1)
def _files() -> Tuple[descriptor_pb2.FileDescriptorProto, ...]:
    fds = descriptor_pb2.FileDescriptorSet()
    with open(_PATH, "rb") as f:
        fds.ParseFromString(f.read())
    return tuple(fds.file)


@functools.lru_cache(maxsize=1)
def pool() -> descriptor_pool.DescriptorPool:
    p = descriptor_pool.DescriptorPool()
    for fd in _files():
        p.Add(fd)
    return p


def message_class(full_name: str) -> Type[message.Message]:
    return message_factory.GetMessageClass(pool().FindMessageTypeByName(full_name.lstrip(".")))


def _varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = val = 0
    while True:
        b = buf[i]
        i += 1
        val |= (b & 0x7F) << shift
        if not b & 0x80:
            return val, i
        shift += 7


def _extension_bytes(raw: bytes, field: int) -> bytes:
    """Payload of length-delimited field ``field`` in a serialized message (protobuf wire format)."""
    i = 0
    while i < len(raw):
        key, i = _varint(raw, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            _, i = _varint(raw, i)
        elif wt == 1:
            i += 8
        elif wt == 5:
            i += 4
        elif wt == 2:
            n, i = _varint(raw, i)
            if num == field:
                return raw[i:i + n]
            i += n
        else:
            raise ValueError(f"unsupported wire type {wt}")
    return b""


@functools.lru_cache(maxsize=1)
def methods() -> Dict[str, Method]:
    """Every method of the service with its HTTP binding, in proto order."""
    http_rule_cls = message_class("google.api.HttpRule")
    out = {}  # type: Dict[str, Method]
    for fd in _files():
        for svc in fd.service:
            if f"{fd.package}.{svc.name}" != SERVICE:
                continue
            for m in svc.method:
                rule = http_rule_cls.FromString(_extension_bytes(m.options.SerializeToString(), _HTTP_EXT))
                kind = rule.WhichOneof("pattern")
                verb, path = (kind.upper(), getattr(rule, kind)) if kind and kind != "custom" else ("", "")
                out[m.name] = Method(m.name, m.input_type.lstrip("."), m.output_type.lstrip("."),
                                     bool(m.server_streaming), verb, path, rule.body)
    return out


def request_class(method: str) -> Type[message.Message]:
    return message_class(methods()[method].input_type)


def response_class(method: str) -> Type[message.Message]:
    return message_class(methods()[method].output_type)


def method_names() -> List[str]:
    return list(methods())
