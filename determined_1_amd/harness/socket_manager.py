"""Master WebSocket layer (reference ``layers/_socket_manager.py:34-207``).

Connects to ``ws://<master>/ws/trial/<e>/<t>/<c>``, blocks until ``RENDEZVOUS_INFO``, yields the
initial workload from the environment and then every ``RUN_WORKLOAD`` the master sends; each
response is sent back as ``WORKLOAD_COMPLETED`` (C-done contract).  Non-chief containers' answers
are ``Skipped`` and never sent; TERMINATE is not answered.
"""
import datetime
import json
import logging
import time
from typing import Any, Dict, Optional

from determined_1_amd import util, workload
from determined_1_amd.env import EnvContext, RendezvousInfo
from determined_1_amd.harness._ws import WebSocket, WebSocketError


def _now() -> str:
    return datetime.datetime.now(datetime.timezone.utc).isoformat().replace("+00:00", "Z")


class SocketManager(workload.Source):
    def __init__(self, env: EnvContext, connect_timeout_s: float = 120.0) -> None:
        self.env = env
        path = f"/ws/trial/{env.det_experiment_id}/{env.det_trial_id}/{env.container_id}"
        deadline = time.time() + connect_timeout_s
        last: Optional[Exception] = None
        self.ws = None
        while time.time() < deadline:
            try:
                self.ws = WebSocket(env.master_addr, int(env.master_port), path)
                break
            except (OSError, WebSocketError) as e:
                last = e
                time.sleep(0.5)
        if self.ws is None:
            raise RuntimeError(f"cannot connect to master at {env.master_addr}:{env.master_port}: {last}")
        self.current = None  # type: Optional[workload.Workload]
        from determined_1_amd.harness.profiler import HarnessProfiler

        self.profiler = HarnessProfiler() if HarnessProfiler.enabled() else None
        self.rendezvous_info = self._wait_for_rendezvous()

    def _wait_for_rendezvous(self) -> RendezvousInfo:
        while True:
            msg = self.ws.recv()
            if msg is None:
                raise RuntimeError("master closed the trial socket before RENDEZVOUS_INFO")
            m = json.loads(msg)
            if m.get("type") == "RENDEZVOUS_INFO":
                logging.info("rendezvous: rank %s of %s", m["rank"], m["addrs"])
                return RendezvousInfo(m["addrs"], m["addrs2"], int(m["rank"]))
            logging.warning("ignoring message before rendezvous: %s", m.get("type"))

    def _responder(self, w: workload.Workload, start: str):
        """``respond({"metrics": ..., "exited_reason"?: ...})`` -> WORKLOAD_COMPLETED."""

        def respond(resp: workload.Response) -> None:
            if self.profiler is not None:
                self.profiler.stop()
            if isinstance(resp, workload.Skipped) or w.kind == workload.Workload.Kind.TERMINATE:
                return
            msg: Dict[str, Any] = {
                "type": "WORKLOAD_COMPLETED",
                "workload": w.__json__(),
                "start_time": start,
                "end_time": _now(),
                "metrics": resp.get("metrics"),
            }
            if resp.get("exited_reason"):
                msg["exited_reason"] = resp["exited_reason"]
            self.ws.send(util.json_encode(msg))

        return respond

    def respond_current(self, resp: Dict[str, Any]) -> None:
        """Answer the workload in flight out-of-band (e.g. ``exited_reason: INVALID_HP``)."""
        if self.current is not None:
            self._responder(self.current, _now())(resp)

    def _profiled(self, w: workload.Workload):
        """Run the harness profiler around one workload (reference _socket_manager.py:179-207)."""
        if self.profiler is not None:
            self.profiler.start(f"step-{w.step_id}-{w.kind.name}")
        return w

    def __iter__(self) -> workload.Stream:
        w = self._profiled(self.env.initial_workload)
        self.current = w
        yield w, [], self._responder(w, _now())
        while True:
            raw = self.ws.recv()
            if raw is None:
                logging.info("master closed the trial socket")
                return
            m = json.loads(raw)
            if m.get("type") != "RUN_WORKLOAD":
                logging.warning("unexpected message from master: %s", m.get("type"))
                continue
            w = self._profiled(workload.Workload.from_json(m["workload"]))
            self.current = w
            yield w, [], self._responder(w, _now())
            if w.kind == workload.Workload.Kind.TERMINATE:
                return

    def close(self) -> None:
        if self.ws is not None:
            self.ws.close()
