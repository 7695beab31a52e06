"""RCCL (ProcessGroupNCCL) data path on the one GPU of the box.

RCCL refuses two ranks on one device, so the multi-rank path runs with WORLD_SIZE=1 and
DET_FORCE_DISTRIBUTED=1: every collective of a real data-parallel step (arena broadcast, bucketed
all-to-all + fp32 shard sum + all-gather or all-reduce, bf16 compression, aggregation windows)
executes on RCCL's stream against the compute stream.  Parameters after 8 steps must match the
plain single-process run: exactly where the world-1 reduction is a copy, within bf16 rounding where
compression rounds the gradients."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "dist_scripts", "gpu_dp_worker.py")


def _run(out: str, forced: bool, amp: str, agg: int, compress: bool, reduction: str) -> dict:
    from determined_1_amd.deploy.local import free_port

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "DET_DIST_BACKEND",
                                                             "DET_DIST_SHARE_GPU")}
    if forced:
        env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(free_port()), DET_FORCE_DISTRIBUTED="1")
    r = subprocess.run([sys.executable, WORKER, out, amp, str(agg), "1" if compress else "0", reduction],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return torch.load(out + ".pt")


@pytest.mark.parametrize("amp,agg,compress,reduction,exact", [
    ("O2", 2, False, "fp32_accum", True),    # bf16 arena: all-to-all + det_sum_rows + all-gather
    ("O0", 2, True, "fp32_accum", False),    # fp32 arena, bf16 wire (compression), fp32 shard sum
    ("O0", 1, False, "allreduce", True),     # fp32 arena: RCCL all-reduce
])
def test_rccl_world1_matches_single_process(gpu, tmp_path, amp, agg, compress, reduction, exact):
    ref = _run(str(tmp_path / "ref"), False, amp, agg, compress, reduction)
    got = _run(str(tmp_path / "dp"), True, amp, agg, compress, reduction)
    assert not ref["dist"] and got["dist"] and got["backend"] == "nccl"
    modes = {b["mode"] for bs in got["buckets"] for b in bs}
    want = "allreduce" if (amp == "O0" and not compress) or reduction == "allreduce" else "fp32_accum"
    assert modes == {want}, got["buckets"]
    if exact:
        torch.testing.assert_close(got["params"], ref["params"], rtol=0, atol=0)
    else:
        torch.testing.assert_close(got["params"], ref["params"], rtol=2e-2, atol=2e-3)
    assert not torch.equal(got["params"], torch.zeros_like(got["params"]))
