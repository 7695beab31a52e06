"""``det tunnel``: a TCP byte stream to a task's service through the master.

Reference: ``cli/determined_cli/tunnel.py`` (stdin/stdout over a lomond WebSocket to
``/proxy/<service>/``, used as an ssh ProxyCommand).  The master side here splices the WebSocket
upgrade of ``/proxy/<task>/`` onto a raw TCP connection to the service (``native/src/master.cc``),
binary frames both ways (an empty frame is the client's EOF: the master half-closes the service
connection), so any TCP protocol reaches the task -- not only the HTTP the plain proxy forwards.
Two client modes:

* stdio (the reference's): ``python -m determined_1_amd.cli.tunnel MASTER cmd-7`` copies stdin to
  the service and the service to stdout (``ssh -o ProxyCommand=...``);
* listen: ``det tunnel cmd-7 --listen 8888`` forwards every connection to local port 8888 over its
  own WebSocket (a browser on a notebook, a database client, ...).

TLS follows the harness WebSocket client (``DET_USE_TLS`` / ``DET_MASTER_CERT_FILE`` /
``DET_MASTER_CERT_NAME``, or ``--cert-file`` / ``--cert-name``).
"""
import argparse
import os
import socket
import sys
import threading
from typing import Callable, Optional

from determined_1_amd.harness._ws import WebSocket, WebSocketError


def _split_master(master: str):
    m = master.split("://", 1)[-1].rstrip("/")
    host, _, port = m.rpartition(":")
    return (host or m), int(port or 8080)


def open_tunnel(master: str, service: str, tls: Optional[bool] = None, token: Optional[str] = None) -> WebSocket:
    """The tunnel WebSocket to ``service``.  The master gates the upgrade on the session like any
    user route (``--require-auth``): the token is the CLI's saved login for ``master`` (or
    ``DET_USER_TOKEN``) unless given."""
    from determined_1_amd.api.request import _load_token

    host, port = _split_master(master)
    svc = service if service.startswith("cmd-") else f"cmd-{service}"
    tok = token if token is not None else _load_token(master)
    headers = {"Authorization": f"Bearer {tok}"} if tok else None
    return WebSocket(host, port, f"/proxy/{svc}/", timeout=30.0, tls=tls, headers=headers)


def splice(ws: WebSocket, read: Callable[[], bytes], write: Callable[[bytes], None],
           close_local: Callable[[], None]) -> None:
    """Pump bytes local -> service on a thread and service -> local here until the service side
    ends.  Local EOF is forwarded as an empty binary frame (the master half-closes the service
    connection), so a request/response stream still gets its answer after stdin closes."""

    def up():
        try:
            while True:
                chunk = read()
                if not chunk:
                    ws.send_binary(b"")
                    return
                ws.send_binary(chunk)
        except (OSError, WebSocketError):
            ws.close()

    t = threading.Thread(target=up, daemon=True)
    t.start()
    try:
        while True:
            m = ws.recv_bytes()
            if m is None:
                break
            write(m)
    except OSError:
        pass
    finally:
        ws.close()
        close_local()
    t.join(timeout=5)


def tunnel_stdio(master: str, service: str, tls: Optional[bool] = None) -> None:
    ws = open_tunnel(master, service, tls)
    stdin = os.fdopen(sys.stdin.fileno(), "rb", buffering=0, closefd=False)
    stdout = os.fdopen(sys.stdout.fileno(), "wb", buffering=0, closefd=False)
    splice(ws, lambda: stdin.read(65536), stdout.write, lambda: None)


def tunnel_listen(master: str, service: str, port: int, host: str = "127.0.0.1", tls: Optional[bool] = None,
                  ready: Optional[threading.Event] = None, stop: Optional[threading.Event] = None) -> int:
    """Accept local connections on host:port (0 = ephemeral) and tunnel each to the service.
    Returns when ``stop`` is set (or never, from the CLI)."""
    srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    srv.bind((host, port))
    srv.listen(16)
    srv.settimeout(0.5)
    bound = srv.getsockname()[1]
    if ready is not None:
        ready.port = bound  # type: ignore[attr-defined]
        ready.set()
    else:
        print(f"tunnel to {service}: listening on {host}:{bound}", file=sys.stderr, flush=True)

    def serve(conn: socket.socket):
        try:
            ws = open_tunnel(master, service, tls)
        except (OSError, WebSocketError) as e:
            print(f"tunnel: {e}", file=sys.stderr)
            conn.close()
            return

        def close_local():
            try:
                conn.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            conn.close()

        splice(ws, lambda: conn.recv(65536), conn.sendall, close_local)

    try:
        while stop is None or not stop.is_set():
            try:
                conn, _ = srv.accept()
            except socket.timeout:
                continue
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            threading.Thread(target=serve, args=(conn,), daemon=True).start()
    finally:
        srv.close()
    return bound


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="Tunnel a TCP stream to a task service through a master")
    ap.add_argument("master_addr")
    ap.add_argument("service", help="command id or cmd-<id>")
    ap.add_argument("--listen", type=int, default=None, help="forward this local port instead of stdio")
    ap.add_argument("--cert-file")
    ap.add_argument("--cert-name")
    a = ap.parse_args(argv)
    tls = None
    if a.cert_file:
        os.environ["DET_MASTER_CERT_FILE"] = a.cert_file
        tls = True
    if a.cert_name:
        os.environ["DET_MASTER_CERT_NAME"] = a.cert_name
    if a.listen is not None:
        tunnel_listen(a.master_addr, a.service, a.listen, tls=tls)
    else:
        tunnel_stdio(a.master_addr, a.service, tls=tls)


if __name__ == "__main__":
    main()
