"""Trial-process startup/workload timeline (``DET_TIMELINE=1``): logs seconds since the process was
created at each harness milestone so per-trial overhead (interpreter + imports, HIP init, storage
probe, rendezvous, model build, each workload, exit) can be read from the trial logs.  Used by
``scripts/bench_asha.py`` to explain the ASHA trials/hr number."""
import logging
import os
import time

_T0 = None


def _start() -> float:
    global _T0
    if _T0 is None:
        try:
            import psutil

            _T0 = psutil.Process().create_time()
        except Exception:
            _T0 = time.time()
    return _T0


def enabled() -> bool:
    # read per call: a zygote-forked trial process imported this module before its env was set
    return os.environ.get("DET_TIMELINE", "0") == "1"


def mark(label: str) -> None:
    if enabled():
        logging.info("[timeline] +%.3fs %s", time.time() - _start(), label)
