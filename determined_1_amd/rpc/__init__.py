"""gRPC wire protocol for the master API: the ``determined.api.v1.Determined`` service (reference
``proto/src/determined/api/v1/api.proto:73-785``) served over HTTP/2 by ``rpc.server`` in front of
det-master's ``/api/v1`` gateway surface, and a client (``rpc.client.Determined``)."""
from determined_1_amd.rpc.routes import ROUTES, SERVICE  # noqa: F401
