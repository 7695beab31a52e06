"""Client of the gRPC service (``rpc.server``): ``Determined(target).GetExperiments(limit=10)``
returns the response as a dict; server-streaming methods return an iterator of dicts.

    d = Determined("127.0.0.1:8090")
    d.login("determined", "")              # Login, then the token rides on every call
    for rec in d.TrialLogs(trial_id=3, follow=True): ...
"""
from typing import Any, Dict, Iterator, Optional, Union

import grpc
from google.protobuf import json_format, struct_pb2

from determined_1_amd.rpc.routes import BY_NAME, SERVICE


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

    def __getattr__(self, name: str):
        route = BY_NAME.get(name)
        if route is None:
            raise AttributeError(name)
        path = f"/{SERVICE}/{name}"
        kw = dict(request_serializer=struct_pb2.Struct.SerializeToString,
                  response_deserializer=struct_pb2.Struct.FromString)
        if route.stream:
            rpc = self.channel.unary_stream(path, **kw)

            def call_stream(timeout: Optional[float] = None, **fields: Any) -> Iterator[Dict[str, Any]]:
                req = struct_pb2.Struct()
                req.update(fields)
                for msg in rpc(req, metadata=self._metadata(), timeout=timeout):
                    yield json_format.MessageToDict(msg)

            return call_stream
        rpc = self.channel.unary_unary(path, **kw)

        def call(timeout: Optional[float] = 60.0, **fields: Any) -> Union[Dict[str, Any], Any]:
            req = struct_pb2.Struct()
            req.update(fields)
            return json_format.MessageToDict(rpc(req, metadata=self._metadata(), timeout=timeout))

        return call
