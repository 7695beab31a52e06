"""Interactive shell task (``det shell start|open``; SURVEY M21, reference
``master/internal/command/shell_manager.go``).

The reference starts ``sshd`` in the task container with a generated key pair and the CLI runs
``ssh`` through the master's TCP proxy.  Neither sshd nor a raw TCP proxy exists here, so the
MI355X build serves the shell itself: a bash on a pseudo-terminal, exposed as a small HTTP API
that the master's ``/proxy/cmd-<id>/`` forwards, guarded by a per-shell token (the key-pair
analogue) that only the launching CLI knows:

    POST /input?token=T              raw bytes -> the pty
    GET  /output?token=T&offset=N&wait=S   long-poll: {"offset", "data" (base64), "exited", "exit_code"}
    POST /resize?token=T             {"rows", "cols"} -> TIOCSWINSZ
    GET  /status?token=T

The task reports its port with ``POST /commands/<id>/ready`` like the TensorBoard service, keeps
the last ``BUFFER`` bytes of output for reconnecting clients, and exits (ending the task) shortly
after the shell does.

    python -m determined_1_amd.exec.shell [--port 0]           (inside the task; env DET_SHELL_TOKEN)
"""
import argparse
import base64
import fcntl
import hmac
import json
import os
import pty
import select
import signal
import struct
import subprocess
import sys
import termios
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, Optional

BUFFER = 4 << 20


class Pty:
    def __init__(self, argv) -> None:
        self.master_fd, slave = pty.openpty()
        env = dict(os.environ)
        env.setdefault("TERM", "xterm-256color")
        env.pop("DET_SHELL_TOKEN", None)
        self.proc = subprocess.Popen(argv, stdin=slave, stdout=slave, stderr=slave, env=env, start_new_session=True,
                                     close_fds=True)
        os.close(slave)
        self.buf = bytearray()
        self.base = 0  # stream offset of buf[0]
        self.cv = threading.Condition()
        self.exit_code: Optional[int] = None
        threading.Thread(target=self._pump, daemon=True).start()

    def _pump(self) -> None:
        while True:
            try:
                r, _, _ = select.select([self.master_fd], [], [], 0.5)
            except (OSError, ValueError):
                break
            if r:
                try:
                    data = os.read(self.master_fd, 65536)
                except OSError:
                    data = b""
                if not data:
                    break
                with self.cv:
                    self.buf += data
                    if len(self.buf) > BUFFER:
                        drop = len(self.buf) - BUFFER
                        del self.buf[:drop]
                        self.base += drop
                    self.cv.notify_all()
            elif self.proc.poll() is not None:
                break
        rc = self.proc.wait()
        with self.cv:
            self.exit_code = rc if rc >= 0 else 128 - rc
            self.cv.notify_all()

    def read(self, offset: int, wait: float) -> Dict[str, Any]:
        deadline = time.time() + wait
        with self.cv:
            while self.base + len(self.buf) <= offset and self.exit_code is None:
                left = deadline - time.time()
                if left <= 0:
                    break
                self.cv.wait(left)
            start = max(offset, self.base)
            data = bytes(self.buf[start - self.base:])
            end = self.base + len(self.buf)
            return {"offset": end, "start": start, "data": base64.b64encode(data).decode(),
                    "exited": self.exit_code is not None and start >= end - len(data) and not data,
                    "exit_code": self.exit_code}

    def write(self, data: bytes) -> None:
        os.write(self.master_fd, data)

    def resize(self, rows: int, cols: int) -> None:
        fcntl.ioctl(self.master_fd, termios.TIOCSWINSZ, struct.pack("HHHH", rows, cols, 0, 0))


def make_handler(sh: Pty, token: str):
    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a: Any) -> None:
            pass

        def _auth(self) -> Optional[Dict[str, str]]:
            q = dict(urllib.parse.parse_qsl(urllib.parse.urlparse(self.path).query))
            if not token or not hmac.compare_digest(q.get("token", ""), token):
                self._send(403, {"error": "bad shell token"})
                return None
            return q

        def _send(self, code: int, obj: Any) -> None:
            body = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def _body(self) -> bytes:
            n = int(self.headers.get("Content-Length", "0") or 0)
            return self.rfile.read(n) if n else b""

        def do_GET(self) -> None:
            q = self._auth()
            if q is None:
                return
            path = urllib.parse.urlparse(self.path).path.rstrip("/")
            if path.endswith("/output"):
                self._send(200, sh.read(int(q.get("offset", "0")), min(float(q.get("wait", "10")), 20.0)))
            elif path.endswith("/status"):
                self._send(200, {"pid": sh.proc.pid, "exit_code": sh.exit_code})
            else:
                self._send(404, {"error": "not found"})

        def do_POST(self) -> None:
            q = self._auth()
            if q is None:
                return
            path = urllib.parse.urlparse(self.path).path.rstrip("/")
            body = self._body()
            if path.endswith("/input"):
                if sh.exit_code is None:
                    sh.write(body)
                self._send(200, {})
            elif path.endswith("/resize"):
                j = json.loads(body or b"{}")
                sh.resize(int(j.get("rows", 24)), int(j.get("cols", 80)))
                self._send(200, {})
            else:
                self._send(404, {"error": "not found"})

    return H


def serve(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--linger", type=float, default=5.0, help="seconds to keep serving output after exit")
    ap.add_argument("--shell", default=os.environ.get("SHELL", "/bin/bash"))
    args = ap.parse_args(argv)
    token = os.environ.get("DET_SHELL_TOKEN", "")
    if not token:
        print("DET_SHELL_TOKEN is not set; refusing to serve an unauthenticated shell", file=sys.stderr)
        return 2
    sh = Pty([args.shell, "-i"])
    srv = ThreadingHTTPServer((args.host, args.port), make_handler(sh, token))
    srv.daemon_threads = True
    port = srv.server_address[1]
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    master = os.environ.get("DET_MASTER")
    task = os.environ.get("DET_TASK_ID", "")
    if master and task.startswith("cmd-"):
        from determined_1_amd.api.request import MasterClient

        MasterClient(master).post(f"/commands/{task[4:]}/ready", {"port": port})
    print(f"[shell] serving pid {sh.proc.pid} on port {port}", flush=True)
    while sh.exit_code is None:
        time.sleep(0.2)
    time.sleep(args.linger)
    srv.shutdown()
    return sh.exit_code or 0


# --------------------------------------------------------------------------------- client
def open_shell(client: Any, cid: int, token: str, stdin=None, stdout=None) -> int:
    """Attach the local terminal (or the given streams) to shell task ``cid`` through the master's
    proxy; returns the shell's exit status."""
    stdin = stdin or sys.stdin
    stdout = stdout or sys.stdout
    base = f"/proxy/cmd-{cid}"
    q = urllib.parse.urlencode({"token": token})
    tty = stdin.isatty()
    old = None
    if tty:
        import tty as ttymod

        old = termios.tcgetattr(stdin.fileno())
        ttymod.setraw(stdin.fileno())
        try:
            rows, cols = os.get_terminal_size(stdin.fileno())
            client._call("POST", f"{base}/resize?{q}", {"rows": rows, "cols": cols})
        except OSError:
            pass
    stop = threading.Event()

    def pump_in() -> None:
        fd = stdin.fileno()
        while not stop.is_set():
            r, _, _ = select.select([fd], [], [], 0.2)
            if not r:
                continue
            data = os.read(fd, 4096)
            if not data:
                break
            client.session.post(client_url(client, f"{base}/input?{q}"), data=data, timeout=30)

    th = threading.Thread(target=pump_in, daemon=True)
    th.start()
    offset = 0
    out = stdout.buffer if hasattr(stdout, "buffer") else None
    try:
        while True:
            r = client._call("GET", f"{base}/output?{q}&offset={offset}&wait=10")
            data = base64.b64decode(r["data"])
            if data:
                if out is not None:
                    out.write(data)
                    out.flush()
                else:
                    stdout.write(data.decode(errors="replace"))
                    stdout.flush()
            offset = r["offset"]
            if r["exit_code"] is not None and not data:
                return int(r["exit_code"])
    finally:
        stop.set()
        if old is not None:
            termios.tcsetattr(stdin.fileno(), termios.TCSADRAIN, old)


def client_url(client: Any, path: str) -> str:
    from determined_1_amd.api.request import make_url

    return make_url(client.master, path)


if __name__ == "__main__":
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(143))
    sys.exit(serve())
