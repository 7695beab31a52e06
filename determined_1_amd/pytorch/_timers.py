"""Per-batch phase timers (SURVEY §5.1 "new build": data / forward / backward / exposed
communication / optimizer), enabled with ``DET_STEP_TIMERS=1``.

Device phases are bracketed with HIP events on the compute stream, so timing adds no host
synchronisation inside the step; the events are resolved once at the end of each RUN_STEP
workload and logged as mean milliseconds per batch (and returned for the TensorBoard writer).
"""
import logging
import os
import time
from typing import Dict, List, Optional

import torch


class StepTimers:
    PHASES = ("forward", "backward", "optimizer")

    def __init__(self, device: torch.device) -> None:
        self.enabled = os.environ.get("DET_STEP_TIMERS", "") not in ("", "0") and device.type == "cuda"
        self.device = device
        self._marks = []  # type: List[Dict[str, torch.cuda.Event]]
        self._data_s = 0.0
        self._cur = None  # type: Optional[Dict[str, torch.cuda.Event]]

    def _ev(self, name: str) -> None:
        if self._cur is None:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self._cur[name] = e
        self._cur["cpu_" + name] = time.perf_counter()  # host issue time: CPU-bound phases show here

    def batch_start(self, data_seconds: float) -> None:
        if not self.enabled:
            return
        self._data_s += data_seconds
        self._cur = {}
        self._marks.append(self._cur)
        self._ev("start")

    def backward_start(self) -> None:
        if self.enabled:
            self._ev("bwd0")

    def backward_end(self) -> None:
        if self.enabled:
            self._ev("bwd1")

    def comm_start(self) -> None:
        if self.enabled:
            self._ev("comm0")

    def comm_end(self) -> None:
        """After the compute stream was made to wait for the gradient all-reduces: the device
        time between comm0 and comm1 is the EXPOSED communication (RCCL work still running after
        backward finished); the overlapped part is already inside ``backward``."""
        if self.enabled:
            self._ev("comm1")

    def step_end(self) -> None:
        if self.enabled:
            self._ev("opt1")

    def report(self, step_id: int) -> Dict[str, float]:
        if not self.enabled or not self._marks:
            return {}
        torch.cuda.synchronize(self.device)
        acc = {"forward": 0.0, "backward": 0.0, "comm_exposed": 0.0, "optimizer": 0.0, "cpu_forward": 0.0,
               "cpu_backward": 0.0, "cpu_optimizer": 0.0}
        n = 0
        for m in self._marks:
            if not all(k in m for k in ("start", "bwd0", "bwd1")):
                continue
            acc["forward"] += m["start"].elapsed_time(m["bwd0"])
            acc["backward"] += m["bwd0"].elapsed_time(m["bwd1"])
            acc["cpu_forward"] += 1000.0 * (m["cpu_bwd0"] - m["cpu_start"])
            acc["cpu_backward"] += 1000.0 * (m["cpu_bwd1"] - m["cpu_bwd0"])
            if "opt1" in m:
                opt0 = "comm1" if "comm1" in m else "bwd1"
                if "comm1" in m:
                    acc["comm_exposed"] += m["comm0"].elapsed_time(m["comm1"])
                acc["optimizer"] += m[opt0].elapsed_time(m["opt1"])
                acc["cpu_optimizer"] += 1000.0 * (m["cpu_opt1"] - m["cpu_bwd1"])
            n += 1
        out = {f"timer/{k}_ms": v / max(1, n) for k, v in acc.items()}
        out["timer/data_ms"] = 1000.0 * self._data_s / max(1, len(self._marks))
        logging.info("step %d phase timers (ms/batch): %s", step_id,
                     ", ".join(f"{k.split('/')[1]}={v:.3f}" for k, v in out.items()))
        self._marks = []
        self._data_s = 0.0
        self._cur = None
        return out
