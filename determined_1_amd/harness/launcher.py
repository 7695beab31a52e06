"""Multi-process fan-out for multi-slot trials (reference ``layers/_worker_process.py:48-339``;
``horovodrun`` + ZMQ there, plain child processes + ``multiprocessing.connection`` here).

The chief harness process of each container starts one worker per local slot
(``python -m determined_1_amd.exec.worker_process``), each bound to one GPU and joined into one
``torch.distributed`` world (RCCL data group + gloo control group, rendezvous at the chief
container).  Every workload from the layer above is broadcast to all local workers and the local
rank 0 response is returned (others answer ``Skipped``).  Worker liveness is checked while waiting,
and a worker exception is re-raised in the launcher with its traceback.
"""
import logging
import os
import secrets
import subprocess
import sys
import threading
import time
from multiprocessing.connection import Client, Connection, Listener, wait
from typing import Any, Dict, List, Optional

from determined_1_amd import constants, workload
from determined_1_amd.env import EnvContext, RendezvousInfo


class WorkerFailed(RuntimeError):
    pass


def _prefix_lines(stream: Any, prefix: str) -> None:
    for raw in iter(stream.readline, b""):
        sys.stdout.write(prefix + raw.decode(errors="replace"))
        sys.stdout.flush()


class SubprocessLauncher:
    def __init__(self, env: EnvContext, stream: workload.Stream, rendezvous: RendezvousInfo, local_size: int,
                 load_path: Optional[str] = None, python: str = sys.executable,
                 extra_env: Optional[Dict[str, str]] = None) -> None:
        self.env = env
        self.stream = stream
        self.rendezvous = rendezvous
        self.local_size = local_size
        authkey = secrets.token_bytes(16)
        self.listener = Listener(("127.0.0.1", 0), authkey=authkey)
        port = self.listener.address[1]
        n_containers = max(1, rendezvous.get_size())
        cross_rank = rendezvous.get_rank()
        world = local_size * n_containers
        chief_host = rendezvous.get_ip_addresses()[0] if rendezvous.get_size() else "127.0.0.1"
        store_port = constants.DIST_STORE_PORT + int(env.det_trial_unique_port_offset)
        self.procs = []  # type: List[subprocess.Popen]
        self._log_threads = []  # type: List[threading.Thread]
        for local_rank in range(local_size):
            e = dict(os.environ)
            e.update(extra_env or {})
            e.update({
                "RANK": str(cross_rank * local_size + local_rank),
                "LOCAL_RANK": str(local_rank),
                "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(local_size),
                "DET_CROSS_RANK": str(cross_rank),
                "DET_CROSS_SIZE": str(n_containers),
                "MASTER_ADDR": chief_host,
                "MASTER_PORT": str(store_port),
                "DET_LAUNCHER_PORT": str(port),
                "DET_LAUNCHER_AUTHKEY": authkey.hex(),
                "DET_RENDEZVOUS_ADDRS": ",".join(rendezvous.get_addrs()),
                "DET_RENDEZVOUS_ADDRS2": ",".join(rendezvous.addrs2),
                "DET_RENDEZVOUS_RANK": str(cross_rank),
                "DET_LOAD_PATH": str(load_path) if load_path else "",
            })
            proc = subprocess.Popen([python, "-m", "determined_1_amd.exec.worker_process"], env=e,
                                    stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
            self.procs.append(proc)
            # rank-prefixed log lines (reference exec/worker_process_wrapper.py:15-18)
            rank = cross_rank * local_size + local_rank
            t = threading.Thread(target=_prefix_lines, args=(proc.stdout, f"[rank={rank}] "), daemon=True)
            t.start()
            self._log_threads.append(t)
        self.conns = [None] * local_size  # type: List[Optional[Connection]]
        deadline = time.time() + constants.DIST_STARTUP_TIMEOUT_SECONDS
        self.listener._listener._socket.settimeout(1.0)  # type: ignore[attr-defined]
        while any(c is None for c in self.conns):
            self._health_check()
            if time.time() > deadline:
                raise WorkerFailed("workers did not connect in time")
            try:
                c = self.listener.accept()
            except OSError:
                continue
            kind, local_rank, pid = c.recv()
            assert kind == "hello"
            self.conns[local_rank] = c
            logging.info("worker local_rank=%d pid=%d connected", local_rank, pid)

    def _health_check(self) -> None:
        for i, p in enumerate(self.procs):
            rc = p.poll()
            if rc is not None:
                raise WorkerFailed(f"worker process local_rank={i} exited with code {rc}")

    def _send_recv(self, w: workload.Workload, args: List[Any]) -> workload.Response:
        for c in self.conns:
            c.send((w, args))
        responses = [None] * self.local_size  # type: List[Any]
        pending = {c: i for i, c in enumerate(self.conns)}
        while pending:
            ready = wait(list(pending), timeout=2.0)
            if not ready:
                self._health_check()
                continue
            for c in ready:
                i = pending.pop(c)
                try:
                    kind, payload = c.recv()
                except EOFError:
                    raise WorkerFailed(f"worker local_rank={i} closed its channel")
                if kind == "error":
                    raise WorkerFailed(f"worker local_rank={i} failed:\n{payload}")
                responses[i] = payload
        chief = responses[0]
        return chief if chief is not None else workload.Skipped()

    def run(self) -> None:
        try:
            for w, args, respond in self.stream:
                resp = self._send_recv(w, [str(a) if hasattr(a, "__fspath__") else a for a in args])
                respond(resp)
                if w.kind == workload.Workload.Kind.TERMINATE:
                    break
        finally:
            self.close()

    def close(self) -> None:
        for c in self.conns:
            if c is not None:
                try:
                    c.close()
                except OSError:
                    pass
        deadline = time.time() + 30
        for p in self.procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
        for t in self._log_threads:
            t.join(timeout=5)
        self.listener.close()


class WorkerReceiver(workload.Source):
    """Worker side: yields broadcast workloads, sends this rank's response back."""

    def __init__(self, local_rank: int) -> None:
        port = int(os.environ["DET_LAUNCHER_PORT"])
        key = bytes.fromhex(os.environ["DET_LAUNCHER_AUTHKEY"])
        self.conn = Client(("127.0.0.1", port), authkey=key)
        self.conn.send(("hello", local_rank, os.getpid()))

    def __iter__(self) -> workload.Stream:
        import pathlib

        while True:
            try:
                w, args = self.conn.recv()
            except EOFError:
                return
            if w.kind == workload.Workload.Kind.CHECKPOINT_MODEL:
                args = [pathlib.Path(a) for a in args]

            def respond(r: workload.Response) -> None:
                self.conn.send(("resp", r))

            yield w, args, respond
            if w.kind == workload.Workload.Kind.TERMINATE:
                return

    def send_error(self, tb: str) -> None:
        try:
            self.conn.send(("error", tb))
        except OSError:
            pass
