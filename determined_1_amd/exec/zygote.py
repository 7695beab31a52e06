"""Warm trial-process server ("zygote") for det-agent.

A trial container is a fresh Python process: on an MI355X box the interpreter + ``import torch`` +
the harness imports cost ~2 s of every container start (``profiles/r1_asha_16trial.json``:
``imports done`` 2.04 s of a 5.4 s container).  An ASHA search starts a container per rung, so that
cost is paid 30-40 times per 16-trial search.  The reference pays the same in a fresh Docker
container per trial (``agent/internal/container/container.go``) and has no counterpart; this is the
MI355X-first replacement.

The agent starts one zygote per node.  It imports torch and the harness modules ONCE -- without
touching the GPU (no HIP runtime init, no torch op that would start OpenMP threads) -- then serves
fork requests on a unix socket:

    request  : 4-byte big-endian length + JSON {"argv": [...], "env": {...}, "cwd": "..."},
               with the container's stdout/stderr pipe write ends attached as SCM_RIGHTS
    reply    : "pid <pid>\\n" once the child exists, "exit <code>\\n" when it ends

The child becomes its own process-group leader (the agent signals containers as ``kill(-pgid)``),
takes the pipes as fd 1/2, replaces its environment with the container's (HIP reads
``HIP_VISIBLE_DEVICES`` at its lazy init, which happens after the fork) and runs the harness module
as ``__main__``.  Only ``-m determined_1_amd.exec.*`` targets are served; anything else is refused
and the agent fork/execs it as before.  The zygote exits when its parent (the agent) goes away.
"""
import array
import json
import os
import runpy
import select
import signal
import socket
import struct
import sys
import time
from typing import Dict, List, Optional, Tuple

ALLOWED_PREFIX = "determined_1_amd.exec."


def preload() -> None:
    """Import what every trial process imports, without creating a GPU context."""
    import numpy  # noqa: F401
    import torch  # noqa: F401
    import torch.nn  # noqa: F401
    import torch.optim  # noqa: F401
    import torch.utils.data  # noqa: F401
    # torch.optim.Optimizer.__init__ imports torch._dynamo lazily: 1.5 s per trial process on a
    # fresh box (bytecode-compiling dynamo + sympy), measured in scripts/dbg/profile_trial_build.py
    import torch._dynamo  # noqa: F401

    import determined_1_amd  # noqa: F401
    import determined_1_amd.exec.harness  # noqa: F401
    import determined_1_amd.pytorch  # noqa: F401
    import determined_1_amd.harness.launcher  # noqa: F401
    try:
        import determined_1_amd.tensorboard  # noqa: F401
    except ImportError:
        pass


def _recv_request(conn: socket.socket) -> Tuple[Dict, List[int]]:
    fds = array.array("i")
    buf = b""
    while len(buf) < 4:
        msg, anc, _, _ = conn.recvmsg(65536, socket.CMSG_SPACE(8 * fds.itemsize))
        if not msg:
            raise EOFError("client closed before request")
        for level, typ, data in anc:
            if level == socket.SOL_SOCKET and typ == socket.SCM_RIGHTS:
                fds.frombytes(data[: len(data) - (len(data) % fds.itemsize)])
        buf += msg
    (n,) = struct.unpack(">I", buf[:4])
    body = buf[4:]
    while len(body) < n:
        chunk = conn.recv(n - len(body))
        if not chunk:
            raise EOFError("short request")
        body += chunk
    return json.loads(body[:n].decode()), list(fds)


def _child(req: Dict, fds: List[int], close: List[int]) -> None:
    """Runs in the forked child; never returns."""
    code = 1
    t_fork = time.time()
    try:
        os.setpgid(0, 0)
        for fd in close:
            try:
                os.close(fd)
            except OSError:
                pass
        signal.signal(signal.SIGCHLD, signal.SIG_DFL)
        signal.signal(signal.SIGTERM, signal.SIG_DFL)
        signal.signal(signal.SIGINT, signal.default_int_handler)
        signal.set_wakeup_fd(-1)
        if len(fds) >= 2:
            os.dup2(fds[0], 1)
            os.dup2(fds[1], 2)
            for fd in fds:
                if fd > 2:
                    os.close(fd)
        sys.stdout = os.fdopen(1, "w", buffering=1, closefd=False)
        sys.stderr = os.fdopen(2, "w", buffering=1, closefd=False)
        if req.get("uid") is not None and int(req["uid"]) != os.geteuid():
            # the task owner's host account (agent user group): drop privileges before any user code
            os.setgroups([int(req["gid"])])
            os.setgid(int(req["gid"]))
            os.setuid(int(req["uid"]))
        cwd = req.get("cwd") or os.getcwd()
        os.chdir(cwd)
        env = req.get("env") or {}
        os.environ.clear()
        os.environ.update({str(k): str(v) for k, v in env.items()})
        os.environ["DET_ZYGOTE_PID"] = str(os.getppid())
        os.environ["DET_PROCESS_T0"] = repr(t_fork)  # the harness timeline's origin (harness/timeline.py)
        pp = [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p]
        sys.path[:] = [cwd] + pp + [p for p in sys.path if p and p not in pp and p != cwd]
        argv = list(req["argv"])
        mod = argv[1]
        sys.argv = [mod] + argv[2:]
        import warnings

        # the target was preloaded, so runpy notes that it re-executes it as __main__
        warnings.filterwarnings("ignore", category=RuntimeWarning, module="runpy")
        try:
            runpy.run_module(mod, run_name="__main__", alter_sys=True)
            code = 0
        except SystemExit as e:
            code = e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
        except BaseException:
            import traceback

            traceback.print_exc()
            code = 1
        try:
            sys.stdout.flush()
            sys.stderr.flush()
        except Exception:
            pass
    finally:
        os._exit(code)


def serve(path: str, parent: Optional[int] = None) -> None:
    if os.path.exists(path):
        os.unlink(path)
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(path)
    os.chmod(path, 0o600)
    srv.listen(64)
    rd, wr = os.pipe()
    os.set_blocking(wr, False)
    os.set_blocking(rd, False)
    signal.set_wakeup_fd(wr)
    signal.signal(signal.SIGCHLD, lambda *_: None)
    stop = {"now": False}
    signal.signal(signal.SIGTERM, lambda *_: stop.update(now=True))
    waiting: Dict[int, socket.socket] = {}
    print(f"[zygote] ready on {path} (pid {os.getpid()})", file=sys.stderr, flush=True)
    while not stop["now"]:
        if parent is not None and os.getppid() != parent:
            break
        try:
            ready, _, _ = select.select([srv, rd], [], [], 1.0)
        except InterruptedError:
            ready = []
        if rd in ready:
            try:
                while os.read(rd, 512):
                    pass
            except BlockingIOError:
                pass
        while True:
            try:
                pid, status = os.waitpid(-1, os.WNOHANG)
            except ChildProcessError:
                break
            if pid == 0:
                break
            code = os.waitstatus_to_exitcode(status)
            code = code if code >= 0 else 128 - code
            conn = waiting.pop(pid, None)
            if conn is not None:
                try:
                    conn.sendall(f"exit {code}\n".encode())
                except OSError:
                    pass
                conn.close()
        if srv in ready:
            try:
                conn, _ = srv.accept()
            except OSError:
                continue
            fds: List[int] = []
            try:
                conn.settimeout(10)
                req, fds = _recv_request(conn)
                argv = req.get("argv") or []
                if len(argv) < 2 or argv[0] != "-m" or not str(argv[1]).startswith(ALLOWED_PREFIX):
                    conn.sendall(b"refused\n")
                    conn.close()
                    continue
                pid = os.fork()
                if pid == 0:
                    _child(req, fds, [srv.fileno(), conn.fileno(), rd, wr])
                try:
                    os.setpgid(pid, pid)
                except OSError:
                    pass
                conn.sendall(f"pid {pid}\n".encode())
                waiting[pid] = conn
            except Exception as e:  # a bad client must not take the zygote down
                print(f"[zygote] request failed: {e!r}", file=sys.stderr, flush=True)
                try:
                    conn.close()
                except OSError:
                    pass
            finally:
                for fd in fds:
                    try:
                        os.close(fd)
                    except OSError:
                        pass
    srv.close()
    try:
        os.unlink(path)
    except OSError:
        pass


class Spawned:
    """A zygote child as seen by the client: its pid and the socket its exit status arrives on."""

    def __init__(self, sock: socket.socket, reply, pid: int) -> None:
        self.sock, self.reply, self.child_pid = sock, reply, pid

    def wait(self) -> int:
        line = self.reply.readline().strip()
        self.sock.close()
        return int(line[5:]) if line.startswith("exit ") else -1


def spawn(path: str, argv: List[str], env: Dict[str, str], cwd: str, out_fd: int, err_fd: int) -> Spawned:
    """Client side of the protocol (det-agent speaks it in C++; tests use this)."""
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.connect(path)
    body = json.dumps({"argv": argv, "env": env, "cwd": cwd}).encode()
    s.sendmsg([struct.pack(">I", len(body)) + body],
              [(socket.SOL_SOCKET, socket.SCM_RIGHTS, array.array("i", [out_fd, err_fd]).tobytes())])
    f = s.makefile("r")
    line = f.readline().strip()
    if not line.startswith("pid "):
        s.close()
        raise RuntimeError(f"zygote refused: {line!r}")
    return Spawned(s, f, int(line[4:]))


def main() -> int:
    import argparse

    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--socket", required=True)
    ap.add_argument("--no-preload", action="store_true")
    args = ap.parse_args()
    parent = os.getppid()
    if not args.no_preload:
        preload()
        import threading

        import torch

        # a HIP context or extra threads would not survive the fork: refuse to serve (the agent
        # then fork/execs every container)
        if torch.cuda.is_initialized() or threading.active_count() != 1:
            print("[zygote] preload initialised the GPU or started threads; not serving", file=sys.stderr)
            return 1
    serve(args.socket, parent)
    return 0


if __name__ == "__main__":
    sys.exit(main())
