"""gRPC front end of det-master: serves ``determined.api.v1.Determined`` (every method of
``routes.ROUTES``) over HTTP/2 and answers each call through the master's ``/api/v1`` surface, the
reverse of the reference's grpc-gateway (reference ``master/internal/grpc/api.go:28,69`` registers the
service on the master's port and the REST gateway in front of it; here the REST surface is native
and the gRPC service is the adapter).

Messages are the reference's own types (``rpc/descriptors.py`` builds them from the reference's
descriptor set), so a client generated from ``api.proto`` talks to this service unchanged: a
``GetExperimentRequest`` arrives as one, is rendered to the REST call its ``google.api.http``
binding names, and the master's JSON answer is parsed into a ``GetExperimentResponse``.  The JSON
is coerced field by field against the response descriptor first (numbers/strings/enums in the
shapes proto3-JSON requires; fields the reference message lacks are dropped), so an extra or
loosely typed key in the master's JSON never fails a call.  Server streams yield one response
message per ``{"result": ...}`` line of the REST stream.  ``GetTelemetry`` (not in the reference
service) stays ``google.protobuf.Struct``-typed.  Authentication: the ``authorization: Bearer
<token>`` call metadata (from ``Login``) is forwarded as the HTTP header.

    python -m determined_1_amd.rpc.server --master 127.0.0.1:8080 --port 8090
"""
import argparse
import json
import re
import threading
from concurrent import futures
from typing import Any, Dict, Iterator, Optional, Tuple
from urllib.parse import quote

import grpc
import requests
from google.protobuf import descriptor as _desc
from google.protobuf import json_format, message as _message, struct_pb2

from determined_1_amd.rpc import descriptors
from determined_1_amd.rpc.routes import ROUTES, SERVICE, Route

_HTTP_TO_GRPC = {400: grpc.StatusCode.INVALID_ARGUMENT, 401: grpc.StatusCode.UNAUTHENTICATED,
                 403: grpc.StatusCode.PERMISSION_DENIED, 404: grpc.StatusCode.NOT_FOUND,
                 409: grpc.StatusCode.ALREADY_EXISTS, 412: grpc.StatusCode.FAILED_PRECONDITION,
                 429: grpc.StatusCode.RESOURCE_EXHAUSTED, 501: grpc.StatusCode.UNIMPLEMENTED,
                 503: grpc.StatusCode.UNAVAILABLE, 504: grpc.StatusCode.DEADLINE_EXCEEDED}


def _camel(s: str) -> str:
    head, *rest = s.split("_")
    return head + "".join(p[:1].upper() + p[1:] for p in rest)


def _lookup(d: Dict[str, Any], dotted: str) -> Tuple[Optional[str], Any]:
    """(top-level key used, value) of a dotted field path, each part in snake_case or lowerCamelCase."""
    cur: Any = d
    top = None
    for i, part in enumerate(dotted.split(".")):
        if not isinstance(cur, dict):
            return top, None
        key = part if part in cur else _camel(part)
        if key not in cur:
            return top, None
        if i == 0:
            top = key
        cur = cur[key]
    return top, cur


def _scalar(v: Any) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))  # Struct carries numbers as doubles: ids go back out as integers
    return str(v)


def _ints(obj: Any) -> Any:
    """Struct numbers are doubles: integral values go back to JSON as integers (ids, counts)."""
    if isinstance(obj, float) and obj.is_integer() and abs(obj) < 2 ** 53:
        return int(obj)
    if isinstance(obj, dict):
        return {k: _ints(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_ints(v) for v in obj]
    return obj


def http_request(route: Route, req: Dict[str, Any]):
    """(verb, path, query params, JSON body or None) of ``route`` for the request fields ``req``."""
    used = set()

    def sub(m: "re.Match") -> str:
        top, val = _lookup(req, m.group(1))
        if val is None:
            raise KeyError(m.group(1))
        if "." not in m.group(1):
            used.add(top)
        return quote(_scalar(val), safe="")

    path = re.sub(r"\{([^}]+)\}", sub, route.path)
    rest = {k: v for k, v in req.items() if k not in used}
    if route.body == "*":
        return route.verb, path, [], rest
    if route.body:
        top, body = _lookup(req, route.body)
        params = [(k, _scalar(x)) for k, v in rest.items() if k != top and not isinstance(v, dict)
                  for x in (v if isinstance(v, list) else [v])]
        return route.verb, path, params, body if body is not None else {}
    params = [(k, _scalar(x)) for k, v in rest.items() if not isinstance(v, dict)
              for x in (v if isinstance(v, list) else [v])]
    return route.verb, path, params, None


def _to_struct(obj: Any) -> struct_pb2.Struct:
    s = struct_pb2.Struct()
    if isinstance(obj, dict):
        s.update(obj)
    elif obj is not None:
        s.update({"value": obj})
    return s


_F = _desc.FieldDescriptor
_INTS = (_F.TYPE_INT32, _F.TYPE_INT64, _F.TYPE_UINT32, _F.TYPE_UINT64, _F.TYPE_SINT32, _F.TYPE_SINT64,
         _F.TYPE_FIXED32, _F.TYPE_FIXED64, _F.TYPE_SFIXED32, _F.TYPE_SFIXED64)
_FLOATS = (_F.TYPE_FLOAT, _F.TYPE_DOUBLE)
_DROP = object()


def _is_repeated(f: _desc.FieldDescriptor) -> bool:
    return bool(f.is_repeated)


def _coerce_scalar(v: Any, f: _desc.FieldDescriptor) -> Any:
    t = f.type
    if v is None:
        return _DROP
    if t in _INTS:
        if isinstance(v, bool):
            return int(v)
        if isinstance(v, (int, float)) and float(v).is_integer():
            return int(v)
        if isinstance(v, str) and re.fullmatch(r"-?\d+", v.strip()):
            return int(v)
        return _DROP
    if t in _FLOATS:
        try:
            return float(v)
        except (TypeError, ValueError):
            return _DROP
    if t == _F.TYPE_BOOL:
        return v if isinstance(v, bool) else (v.lower() == "true" if isinstance(v, str) else bool(v))
    if t == _F.TYPE_STRING:
        if isinstance(v, (dict, list)):
            return json.dumps(v)
        return v if isinstance(v, str) else _scalar(v)
    if t == _F.TYPE_BYTES:
        return v if isinstance(v, str) else _DROP
    if t == _F.TYPE_ENUM:
        names = f.enum_type.values_by_name
        if isinstance(v, str):
            for cand in (v, v.upper(), f"STATE_{v.upper()}"):
                if cand in names:
                    return cand
            prefix = re.sub(r"(?<!^)([A-Z])", r"_\1", f.enum_type.name).upper() + "_"
            return prefix + v.upper() if prefix + v.upper() in names else _DROP
        if isinstance(v, int) and v in f.enum_type.values_by_number:
            return v
        return _DROP
    return _DROP


def coerce(obj: Any, desc: _desc.Descriptor) -> Any:
    """``obj`` (the master's JSON) reshaped to what ``json_format.ParseDict`` accepts for ``desc``."""
    name = desc.full_name
    if name == "google.protobuf.Struct":
        return obj if isinstance(obj, dict) else _DROP
    if name == "google.protobuf.ListValue":
        return obj if isinstance(obj, list) else _DROP
    if name == "google.protobuf.Value":
        return obj
    if name == "google.protobuf.Timestamp":
        return obj if isinstance(obj, str) and re.match(r"\d{4}-\d\d-\d\dT", obj) else _DROP
    if name.startswith("google.protobuf.") and name.endswith("Value"):  # wrappers
        return _coerce_scalar(obj, desc.fields_by_name["value"])
    if not isinstance(obj, dict):
        return _DROP
    out = {}
    by_key = {}
    for f in desc.fields:
        by_key[f.name] = f
        by_key[f.json_name] = f
    for k, v in obj.items():
        f = by_key.get(k)
        if f is None or v is None:
            continue
        if f.message_type is not None and f.message_type.GetOptions().map_entry:
            if not isinstance(v, dict):
                continue
            vf = f.message_type.fields_by_name["value"]
            conv = {str(mk): (coerce(mv, vf.message_type) if vf.message_type is not None else _coerce_scalar(mv, vf))
                    for mk, mv in v.items()}
            out[f.name] = {mk: mv for mk, mv in conv.items() if mv is not _DROP}
            continue
        conv1 = (lambda x: coerce(x, f.message_type)) if f.message_type is not None else \
            (lambda x: _coerce_scalar(x, f))
        if _is_repeated(f):
            if not isinstance(v, list):
                v = [v]
            vals = [conv1(x) for x in v]
            out[f.name] = [x for x in vals if x is not _DROP]
        else:
            c = conv1(v)
            if c is not _DROP:
                out[f.name] = c
    return out


def parse_response(obj: Any, cls: Any) -> _message.Message:
    msg = cls()
    d = coerce(obj if isinstance(obj, dict) else {}, cls.DESCRIPTOR)
    try:
        json_format.ParseDict(d, msg, ignore_unknown_fields=True)
    except json_format.ParseError:  # a field the coercion could not fix: keep every field that parses
        msg = cls()
        for k, v in d.items():
            part = cls()
            try:
                json_format.ParseDict({k: v}, part, ignore_unknown_fields=True)
            except json_format.ParseError:
                continue
            msg.MergeFrom(part)
    return msg


def _int64_fix(obj: Any, desc: _desc.Descriptor) -> Any:
    """proto3-JSON prints 64-bit integers as strings; the REST surface takes numbers."""
    if not isinstance(obj, dict) or desc.full_name.startswith("google.protobuf."):
        return obj
    for f in desc.fields:
        key = f.name
        if key not in obj:
            continue
        v = obj[key]
        if f.message_type is not None and not f.message_type.GetOptions().map_entry:
            obj[key] = [_int64_fix(x, f.message_type) for x in v] if isinstance(v, list) else _int64_fix(v, f.message_type)
        elif f.type in _INTS:
            conv = lambda x: int(x) if isinstance(x, str) and re.fullmatch(r"-?\d+", x) else x  # noqa: E731
            obj[key] = [conv(x) for x in v] if isinstance(v, list) else conv(v)
    return obj


def request_to_json(msg: _message.Message) -> Dict[str, Any]:
    if isinstance(msg, struct_pb2.Struct):
        return _ints(json_format.MessageToDict(msg))
    return _int64_fix(json_format.MessageToDict(msg, preserving_proto_field_name=True), msg.DESCRIPTOR)


class Gateway:
    """The servicer: one HTTP session to the master, a handler per route."""

    def __init__(self, master: str, timeout: float = 60.0) -> None:
        self.base = master if "://" in master else f"http://{master}"
        self.timeout = timeout
        self._local = threading.local()

    def _session(self) -> requests.Session:
        s = getattr(self._local, "s", None)
        if s is None:
            s = self._local.s = requests.Session()
        return s

    @staticmethod
    def _headers(context: grpc.ServicerContext) -> Dict[str, str]:
        h = {}
        for k, v in context.invocation_metadata() or ():
            if k.lower() == "authorization":
                h["Authorization"] = v
        return h

    def _fail(self, context: grpc.ServicerContext, r: requests.Response) -> None:
        try:
            msg = r.json()
            msg = msg.get("message") or msg.get("error") or r.text
        except ValueError:
            msg = r.text
        context.abort(_HTTP_TO_GRPC.get(r.status_code, grpc.StatusCode.UNKNOWN), f"{r.status_code}: {msg}"[:2000])

    def _call(self, route: Route, request: _message.Message, context, stream: bool) -> requests.Response:
        req = request_to_json(request)
        try:
            verb, path, params, body = http_request(route, req)
        except KeyError as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"missing path field {e.args[0]}")
        timeout = None if stream else self.timeout
        r = self._session().request(verb, self.base + path, params=params or None,
                                    data=None if body is None else json.dumps(body),
                                    headers=dict(self._headers(context), **({"Content-Type": "application/json"}
                                                                            if body is not None else {})),
                                    stream=stream, timeout=timeout)
        if r.status_code >= 300:
            self._fail(context, r)
        return r

    @staticmethod
    def _types(route: Route) -> Tuple[Any, Any]:
        if route.method in descriptors.methods():
            return descriptors.request_class(route.method), descriptors.response_class(route.method)
        return struct_pb2.Struct, struct_pb2.Struct

    @staticmethod
    def _reply(obj: Any, out_cls: Any) -> _message.Message:
        return _to_struct(obj) if out_cls is struct_pb2.Struct else parse_response(obj, out_cls)

    def unary(self, route: Route):
        out_cls = self._types(route)[1]

        def handle(request: _message.Message, context) -> _message.Message:
            r = self._call(route, request, context, False)
            return self._reply(r.json() if r.content else {}, out_cls)

        return handle

    def streaming(self, route: Route):
        out_cls = self._types(route)[1]

        def handle(request: _message.Message, context) -> Iterator[_message.Message]:
            r = self._call(route, request, context, True)
            try:
                for line in r.iter_lines():
                    if not context.is_active():
                        break
                    if not line:
                        continue
                    msg = json.loads(line)
                    if "error" in msg and "result" not in msg:
                        err = msg["error"]
                        context.abort(grpc.StatusCode.UNKNOWN, json.dumps(err) if not isinstance(err, str) else err)
                    yield self._reply(msg.get("result", msg), out_cls)
            finally:
                r.close()

        return handle

    def handler(self) -> grpc.GenericRpcHandler:
        table = {}
        for route in ROUTES:
            in_cls, out_cls = self._types(route)
            kw = dict(request_deserializer=in_cls.FromString, response_serializer=out_cls.SerializeToString)
            if route.stream:
                table[route.method] = grpc.unary_stream_rpc_method_handler(self.streaming(route), **kw)
            else:
                table[route.method] = grpc.unary_unary_rpc_method_handler(self.unary(route), **kw)
        return grpc.method_handlers_generic_handler(SERVICE, table)


def serve(master: str, port: int = 0, host: str = "127.0.0.1", max_workers: int = 32) -> Tuple[grpc.Server, int]:
    """Start the gRPC service on ``host:port`` (0: any free port); returns (server, bound port)."""
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers))
    server.add_generic_rpc_handlers((Gateway(master).handler(),))
    bound = server.add_insecure_port(f"{host}:{port}")
    server.start()
    return server, bound


def main() -> None:
    ap = argparse.ArgumentParser(description="gRPC front end (determined.api.v1.Determined) of det-master")
    ap.add_argument("--master", default="127.0.0.1:8080")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8090)
    args = ap.parse_args()
    server, port = serve(args.master, args.port, args.host)
    print(f"gRPC {SERVICE} on {args.host}:{port} -> {args.master}", flush=True)
    server.wait_for_termination()


if __name__ == "__main__":
    main()
