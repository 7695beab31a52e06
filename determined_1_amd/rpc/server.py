"""gRPC front end of det-master: serves ``determined.api.v1.Determined`` (every method of
``routes.ROUTES``) over HTTP/2 and answers each call through the master's ``/api/v1`` surface, the
reverse of the reference's grpc-gateway (reference ``master/internal/grpc/api.go:28,69`` registers the
service on the master's port and the REST gateway in front of it; here the REST surface is native
and the gRPC service is the adapter).

Messages travel as ``google.protobuf.Struct``: a request is the reference request message in its
JSON form (field names as in the grpc-gateway JSON, lowerCamelCase or proto snake_case), a
response the reference response message's JSON (the shapes ``native/src/api_v1.cc`` emits).  Server
streams yield one Struct per ``{"result": ...}`` line of the REST stream.  Authentication: the
``authorization: Bearer <token>`` call metadata (from ``Login``) is forwarded as the HTTP header.

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
from google.protobuf import json_format, struct_pb2

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

    def _call(self, route: Route, request: struct_pb2.Struct, context, stream: bool) -> requests.Response:
        req = _ints(json_format.MessageToDict(request))
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

    def unary(self, route: Route):
        def handle(request: struct_pb2.Struct, context) -> struct_pb2.Struct:
            r = self._call(route, request, context, False)
            return _to_struct(r.json() if r.content else {})

        return handle

    def streaming(self, route: Route):
        def handle(request: struct_pb2.Struct, context) -> Iterator[struct_pb2.Struct]:
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
                    yield _to_struct(msg.get("result", msg))
            finally:
                r.close()

        return handle

    def handler(self) -> grpc.GenericRpcHandler:
        table = {}
        for route in ROUTES:
            if route.stream:
                table[route.method] = grpc.unary_stream_rpc_method_handler(
                    self.streaming(route), request_deserializer=struct_pb2.Struct.FromString,
                    response_serializer=struct_pb2.Struct.SerializeToString)
            else:
                table[route.method] = grpc.unary_unary_rpc_method_handler(
                    self.unary(route), request_deserializer=struct_pb2.Struct.FromString,
                    response_serializer=struct_pb2.Struct.SerializeToString)
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
