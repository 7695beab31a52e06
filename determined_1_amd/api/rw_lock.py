"""Client for the master's distributed readers-writer lock (reference yogadl's RW-coordinator client
against ``master/internal/rw_coordinator.go``; WS ``/ws/data-layer/<resource>?read_lock=``).

The lock is held while the WebSocket is open::

    with RWLock("127.0.0.1:8080", "cache/mnist/v1", read=False):
        build_cache()

Readers share a resource; a writer excludes everyone.  Waiters are granted in arrival order and a
waiting writer blocks readers that arrive after it (see ``native/include/detcore/rw_coordinator.h``).
"""
from typing import Optional
from urllib.parse import quote

from determined_1_amd.api.request import parse_master_address
from determined_1_amd.harness._ws import WebSocket


class LockError(RuntimeError):
    pass


class RWLock:
    def __init__(self, master: str, resource: str, read: bool = True, timeout: Optional[float] = None) -> None:
        self.master = master
        self.resource = resource.strip("/")
        self.read = read
        self.timeout = timeout
        self._ws: Optional[WebSocket] = None

    def acquire(self) -> None:
        if self._ws is not None:
            raise LockError("lock already held")
        host, port = parse_master_address(self.master)
        path = f"/ws/data-layer/{quote(self.resource)}?read_lock={'true' if self.read else 'false'}"
        ws = WebSocket(host, port, path)
        if self.timeout is not None:
            ws.sock.settimeout(self.timeout)
        try:
            msg = ws.recv()
        except OSError as e:
            ws.close()
            raise LockError(f"timed out waiting for the lock on {self.resource!r}") from e
        want = "read_lock_granted" if self.read else "write_lock_granted"
        if msg != want:
            ws.close()
            raise LockError(f"unexpected reply from the RW coordinator: {msg!r}")
        ws.sock.settimeout(None)
        self._ws = ws

    def release(self) -> None:
        if self._ws is not None:
            self._ws.close()
            self._ws = None

    def __enter__(self) -> "RWLock":
        self.acquire()
        return self

    def __exit__(self, *exc: object) -> None:
        self.release()

