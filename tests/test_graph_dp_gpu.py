"""hipGraph capture of data-parallel and aggregation steps.

The bucketer's RCCL collectives are recorded into the train-step graph (issued from the capturing
stream's backward hooks, in bucket order), and each position of an aggregation window is its own
graph key with the host state (GradSink window, optimizer step counters) restored after a replay.
On the one GPU of the box the multi-process path runs as a world-1 RCCL group
(DET_FORCE_DISTRIBUTED=1, tests/test_rccl_gpu.py): the graph-replayed run must match the eager run
of the same trial, and most steps must have come from replays."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "dist_scripts", "gpu_dp_worker.py")


def _run(out: str, graph: bool, amp: str, agg: int, compress: bool, reduction: str) -> dict:
    from determined_1_amd.deploy.local import free_port

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "DET_DIST_BACKEND",
                                                             "DET_DIST_SHARE_GPU")}
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(free_port()), DET_FORCE_DISTRIBUTED="1", DET_HIP_GRAPH="1" if graph else "0",
               GDP_HALF_STEPS="16")
    r = subprocess.run([sys.executable, WORKER, out, amp, str(agg), "1" if compress else "0", reduction],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return torch.load(out + ".pt")


@pytest.mark.parametrize("amp,agg,compress,reduction", [
    ("O2", 1, False, "fp32_accum"),  # bf16 arena: all-to-all + det_sum_rows (side stream) + all-gather
    ("O2", 2, False, "fp32_accum"),  # a 2-batch aggregation window: two position graphs
    ("O0", 1, False, "allreduce"),   # fp32 arena: RCCL all-reduce
    ("O0", 3, True, "fp32_accum"),   # bf16 wire compression, 3-batch windows
])
def test_dp_graph_replay_matches_eager(gpu, tmp_path, amp, agg, compress, reduction):
    eager = _run(str(tmp_path / "eager"), False, amp, agg, compress, reduction)
    graph = _run(str(tmp_path / "graph"), True, amp, agg, compress, reduction)
    assert graph["dist"] and graph["backend"] == "nccl"
    st = graph["graph"]
    assert st is not None and st["disabled"] is None, st
    assert st["captures"] >= agg and st["replays"] >= 32 - 4 * agg, st
    torch.testing.assert_close(graph["params"], eager["params"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(torch.tensor(graph["losses"]), torch.tensor(eager["losses"]), rtol=1e-5, atol=1e-6)
