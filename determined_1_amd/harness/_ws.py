"""Minimal synchronous WebSocket client (RFC 6455, text + binary frames) for the harness <-> master
channel and the ``det tunnel`` byte stream.

The reference uses ``lomond`` (``harness/determined/layers/_socket_manager.py:41-69``); it is not
installed here and the protocol needs only text frames, ping/pong and close, so this is ~100 lines
of stdlib instead of a dependency.
"""
import base64
import os
import socket
import struct
import threading
from typing import Dict, Optional


class WebSocketError(RuntimeError):
    pass


class WebSocket:
    def __init__(self, host: str, port: int, path: str, timeout: Optional[float] = 30.0,
                 tls: Optional[bool] = None, headers: Optional[Dict[str, str]] = None) -> None:
        """``tls=None``: TLS iff the task/CLI environment says the master speaks it (``DET_USE_TLS``,
        ``DET_MASTER_CERT_FILE``; ``DET_MASTER_CERT_NAME`` overrides the name checked).  ``headers``:
        extra request headers of the upgrade (e.g. ``Authorization`` for auth-gated sockets)."""
        raw = socket.create_connection((host, port), timeout=timeout)
        raw.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        if tls is None:
            tls = (os.environ.get("DET_USE_TLS", "") or "").strip().lower() in ("1", "true", "yes", "on")
        if tls:
            import ssl

            ctx = ssl.create_default_context(cafile=os.environ.get("DET_MASTER_CERT_FILE") or None)
            raw = ctx.wrap_socket(raw, server_hostname=os.environ.get("DET_MASTER_CERT_NAME") or host)
        self.sock = raw
        key = base64.b64encode(os.urandom(16)).decode()
        req = (f"GET {path} HTTP/1.1\r\nHost: {host}:{port}\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
               f"Sec-WebSocket-Key: {key}\r\nSec-WebSocket-Version: 13\r\n"
               + "".join(f"{k}: {v}\r\n" for k, v in (headers or {}).items()) + "\r\n")
        self.sock.sendall(req.encode())
        self._buf = b""
        while b"\r\n\r\n" not in self._buf:
            chunk = self.sock.recv(4096)
            if not chunk:
                raise WebSocketError("connection closed during websocket handshake")
            self._buf += chunk
        head, self._buf = self._buf.split(b"\r\n\r\n", 1)
        if b" 101 " not in head.split(b"\r\n", 1)[0]:
            raise WebSocketError(f"websocket upgrade refused: {head[:200]!r}")
        self.sock.settimeout(None)
        self._send_lock = threading.Lock()
        self.closed = False

    def _read_exact(self, n: int) -> bytes:
        while len(self._buf) < n:
            chunk = self.sock.recv(max(65536, n - len(self._buf)))
            if not chunk:
                raise WebSocketError("connection closed")
            self._buf += chunk
        out, self._buf = self._buf[:n], self._buf[n:]
        return out

    def _send_frame(self, opcode: int, payload: bytes) -> None:
        header = bytearray([0x80 | opcode])
        n = len(payload)
        if n < 126:
            header.append(0x80 | n)
        elif n < 65536:
            header.append(0x80 | 126)
            header += struct.pack(">H", n)
        else:
            header.append(0x80 | 127)
            header += struct.pack(">Q", n)
        mask = os.urandom(4)
        header += mask
        # XOR-mask via int arithmetic (fast enough for control-plane messages)
        m = (mask * (n // 4 + 1))[:n]
        masked = (int.from_bytes(payload, "little") ^ int.from_bytes(m, "little")).to_bytes(n, "little") if n else b""
        with self._send_lock:
            self.sock.sendall(bytes(header) + masked)

    def send(self, text: str) -> None:
        if self.closed:
            raise WebSocketError("send on closed websocket")
        self._send_frame(0x1, text.encode())

    def send_binary(self, data: bytes) -> None:
        if self.closed:
            raise WebSocketError("send on closed websocket")
        self._send_frame(0x2, data)

    def recv(self) -> Optional[str]:
        """Next text message, or None when the peer closed the connection."""
        m = self.recv_bytes()
        return None if m is None else m.decode()

    def recv_bytes(self) -> Optional[bytes]:
        """Next text or binary message as bytes, or None when the peer closed the connection."""
        message = b""
        while True:
            try:
                b0, b1 = self._read_exact(2)
            except (WebSocketError, OSError):
                self.closed = True
                return None
            fin, opcode = b0 & 0x80, b0 & 0x0F
            n = b1 & 0x7F
            if n == 126:
                n = struct.unpack(">H", self._read_exact(2))[0]
            elif n == 127:
                n = struct.unpack(">Q", self._read_exact(8))[0]
            mask = self._read_exact(4) if b1 & 0x80 else None
            payload = self._read_exact(n)
            if mask:
                m = (mask * (n // 4 + 1))[:n]
                payload = (int.from_bytes(payload, "little") ^ int.from_bytes(m, "little")).to_bytes(n, "little") if n else b""
            if opcode == 0x8:
                self.close()
                return None
            if opcode == 0x9:
                self._send_frame(0xA, payload)
                continue
            if opcode == 0xA:
                continue
            message += payload
            if fin:
                return message

    def close(self) -> None:
        if self.closed:
            return
        self.closed = True
        try:
            self._send_frame(0x8, b"")
        except OSError:
            pass
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()
