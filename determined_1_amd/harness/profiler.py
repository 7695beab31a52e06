"""Harness profiler (reference ``layers/_harness_profiler.py:55-182``): a sampling
thread recording CPU %, RSS, disk/net/process IO (psutil) and GPU busy % / VRAM (amdgpu sysfs)
every ``interval`` seconds while a workload runs; dumps ``/tmp/step-<id>-<kind>.json``.

Enabled with ``DET_HARNESS_PROFILER=1`` (set through ``environment.environment_variables``)."""
import json
import os
import threading
import time
from typing import Any, Dict, List, Optional

from determined_1_amd import gpu


class HarnessProfiler:
    def __init__(self, interval: float = 0.1, out_dir: str = "/tmp") -> None:
        self.interval = interval
        self.out_dir = out_dir
        self._samples = []  # type: List[Dict[str, Any]]
        self._stop = threading.Event()
        self._thread = None  # type: Optional[threading.Thread]
        self._tag = ""

    @staticmethod
    def enabled() -> bool:
        return os.environ.get("DET_HARNESS_PROFILER", "") not in ("", "0", "false")

    def _sample(self) -> Dict[str, Any]:
        import psutil

        p = psutil.Process()
        rec = {"t": time.time(), "cpu_percent": psutil.cpu_percent(None), "rss": p.memory_info().rss}
        try:
            io = p.io_counters()
            rec["proc_read_bytes"], rec["proc_write_bytes"] = io.read_bytes, io.write_bytes
        except (AttributeError, OSError):
            pass
        d = psutil.disk_io_counters()
        if d:
            rec["disk_read_bytes"], rec["disk_write_bytes"] = d.read_bytes, d.write_bytes
        n = psutil.net_io_counters()
        if n:
            rec["net_sent"], rec["net_recv"] = n.bytes_sent, n.bytes_recv
        rec["gpus"] = gpu.utilization()
        return rec

    def _loop(self) -> None:
        while not self._stop.wait(self.interval):
            try:
                self._samples.append(self._sample())
            except Exception:  # noqa: BLE001 - sampling must never kill training
                pass

    def start(self, tag: str) -> None:
        self._tag = tag
        self._samples = []
        self._stop.clear()
        self._thread = threading.Thread(target=self._loop, daemon=True)
        self._thread.start()

    def stop(self) -> str:
        self._stop.set()
        if self._thread is not None:
            self._thread.join()
        path = os.path.join(self.out_dir, f"{self._tag}.json")
        with open(path, "w") as f:
            json.dump(self._samples, f)
        return path
