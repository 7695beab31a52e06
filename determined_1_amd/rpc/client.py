"""Client of the gRPC service (``rpc.server``), on the reference's message types.

    d = Determined("127.0.0.1:8090")
    d.login("determined", "")              # Login, then the token rides on every call
    d.GetExperiment(experiment_id=3)       # -> dict (proto3 JSON of GetExperimentResponse)
    for rec in d.TrialLogs(trial_id=3, follow=True): ...
    req = d.request("GetExperiment", experiment_id=3)      # a real GetExperimentRequest
    resp = d.typed("GetExperiment")(req)                   # a real GetExperimentResponse

Keyword fields are parsed into the request message with ``json_format.ParseDict`` (snake_case or
lowerCamelCase names; nested messages as dicts; Struct fields as plain dicts).
"""
from typing import Any, Dict, Iterator, Optional, Union

import grpc
from google.protobuf import json_format, message, struct_pb2

from determined_1_amd.rpc import descriptors
from determined_1_amd.rpc.routes import BY_NAME, SERVICE


def _classes(name: str):
    if name in descriptors.methods():
        return descriptors.request_class(name), descriptors.response_class(name)
    return struct_pb2.Struct, struct_pb2.Struct


class Determined:
    def __init__(self, target: str, token: Optional[str] = None, channel: Optional[grpc.Channel] = None) -> None:
        self.channel = channel or grpc.insecure_channel(target)
        self.token = token

    def close(self) -> None:
        self.channel.close()

    def login(self, username: str, password: str = "") -> str:
        self.token = self.Login(username=username, password=password)["token"]
        return self.token

    def _metadata(self):
        return (("authorization", f"Bearer {self.token}"),) if self.token else ()

    def request(self, name: str, **fields: Any) -> message.Message:
        """The request message of method ``name`` with ``fields`` set."""
        in_cls = _classes(name)[0]
        if in_cls is struct_pb2.Struct:
            req = struct_pb2.Struct()
            req.update(fields)
            return req
        return json_format.ParseDict(fields, in_cls())

    def typed(self, name: str):
        """The raw multicallable of method ``name``: request message in, response message(s) out."""
        route = BY_NAME.get(name)
        if route is None:
            raise AttributeError(name)
        in_cls, out_cls = _classes(name)
        kw = dict(request_serializer=in_cls.SerializeToString, response_deserializer=out_cls.FromString)
        path = f"/{SERVICE}/{name}"
        return self.channel.unary_stream(path, **kw) if route.stream else self.channel.unary_unary(path, **kw)

    @staticmethod
    def _to_dict(msg: message.Message) -> Dict[str, Any]:
        if isinstance(msg, struct_pb2.Struct):
            return json_format.MessageToDict(msg)
        return json_format.MessageToDict(msg, always_print_fields_with_no_presence=True)

    def __getattr__(self, name: str):
        route = BY_NAME.get(name)
        if route is None:
            raise AttributeError(name)
        rpc = self.typed(name)
        if route.stream:
            def call_stream(timeout: Optional[float] = None, **fields: Any) -> Iterator[Dict[str, Any]]:
                for msg in rpc(self.request(name, **fields), metadata=self._metadata(), timeout=timeout):
                    yield self._to_dict(msg)

            return call_stream

        def call(timeout: Optional[float] = 60.0, **fields: Any) -> Union[Dict[str, Any], Any]:
            return self._to_dict(rpc(self.request(name, **fields), metadata=self._metadata(), timeout=timeout))

        return call
