"""Trial-process startup/workload timeline (``DET_TIMELINE=1``): logs seconds since the process was
created at each harness milestone so per-trial overhead (interpreter + imports, HIP init, storage
probe, rendezvous, model build, each workload, exit) can be read from the trial logs.  Used by
``scripts/bench_asha.py`` to explain the ASHA trials/hr number."""
import logging
import os
import time

_T0 = None


def _process_start_wall() -> float:
    """Wall-clock creation time of this process from /proc/self/stat (clock ticks since boot) and
    CLOCK_BOOTTIME, to ~10 ms.  (psutil's create_time adds the integer-second boot time of
    /proc/stat, a constant bias of up to 1 s that read as ~1 s of "imports" per container.)"""
    with open("/proc/self/stat") as f:
        fields = f.read().rsplit(")", 1)[1].split()
    start_ticks = int(fields[19])  # field 22 of proc(5), counted after the ")" of the command name
    since_start = time.clock_gettime(time.CLOCK_BOOTTIME) - start_ticks / os.sysconf("SC_CLK_TCK")
    return time.time() - since_start


def _start() -> float:
    global _T0
    if _T0 is None:
        t0 = os.environ.get("DET_PROCESS_T0")  # set by the zygote at the fork (exact)
        try:
            _T0 = float(t0) if t0 else _process_start_wall()
        except (OSError, ValueError, IndexError):
            _T0 = time.time()
    return _T0


def enabled() -> bool:
    # read per call: a zygote-forked trial process imported this module before its env was set
    return os.environ.get("DET_TIMELINE", "0") == "1"


def mark(label: str) -> None:
    if enabled():
        logging.info("[timeline] +%.3fs %s", time.time() - _start(), label)
