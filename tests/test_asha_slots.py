"""The ASHA benchmark's multi-slot scheduling path on CPU: ``scripts/bench_asha.py`` with 8
artificial slots runs the 16-trial adaptive_asha CIFAR-10 search (scaled down to 40 batches, fp32)
through det-master + det-agent, fills all 8 slots at once, and reports slot occupancy / scheduler
idle time (BASELINE's ASHA shape is 8 GPUs; the real-GPU runs use 1 slot per box)."""
import json
import os
import pathlib
import subprocess
import sys

import pytest

REPO = pathlib.Path(__file__).resolve().parent.parent


@pytest.mark.timeout(900)
def test_bench_asha_eight_artificial_slots(tmp_path):
    env = dict(os.environ, DET_BENCH_LOGDIR=str(tmp_path), MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, str(REPO / "scripts" / "bench_asha.py"), "--artificial-slots", "8",
                        "--max-length-batches", "16", "--max-trials", "16", "--amp", "O0", "--validation-records", "128", "--timeout", "600"],
                       capture_output=True, text=True, timeout=800, env=env, cwd=str(REPO))
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["state"] == "COMPLETED", res
    assert res["trials_completed"] == 16
    assert res["slots"] == 8
    assert res["peak_busy_slots"] == 8, res  # the scheduler ran 8 trials at once
    assert 0.0 <= res["scheduler_idle_frac"] < 1.0
    (tmp_path / "asha_8slot.json").write_text(json.dumps(res))
