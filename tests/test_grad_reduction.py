"""Gradient bucket plan and reduction accuracy (CPU, gloo, up to 8 ranks).

The bf16 O2 arena is reduced with fp32 accumulation (all-to-all reduce-scatter + fp32 shard sum
+ all-gather, ``parallel/ddp.py``); these tests bound its error against the exact float64 sum
of the same bf16 inputs and show it is tighter than a plain bf16 all-reduce."""
import os
import subprocess
import sys

import pytest
import torch

from determined_1_amd.ops.arena import Arena
from determined_1_amd.parallel.ddp import MB, apply_rccl_env, auto_bucket_cap, plan_buckets

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "dist_scripts", "reduce_worker.py")


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(out: str, world: int, reduction: str, dtype: str = "bfloat16", compress: bool = False) -> list:
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, WORKER, out, reduction, dtype, "1" if compress else "0"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        o, _ = p.communicate(timeout=240)
        assert p.returncode == 0, o.decode()[-3000:]
    return [torch.load(f"{out}.{r}.pt") for r in range(world)]


def _exact_sum(world: int, numel: int, dtype: torch.dtype) -> torch.Tensor:
    tot = torch.zeros(numel, dtype=torch.float64)
    for r in range(world):
        g = torch.Generator().manual_seed(1234 + r)
        tot += (torch.randn(numel, generator=g) * (1.0 + r)).to(dtype).double()
    return tot


def test_plan_buckets_tail_first_and_cover():
    params = [torch.nn.Parameter(torch.zeros(n)) for n in [300_000, 1000, 800_000, 50_000, 700_000, 64, 900_000]]
    a = Arena(params, torch.device("cpu"))
    cap = 4 * 1024 * 1024
    bs = plan_buckets([a], cap)
    # contiguous, ordered, covering the whole arena, every param exactly once
    assert bs[0].lo == 0 and bs[-1].hi == a.numel
    for x, y in zip(bs, bs[1:]):
        assert x.hi == y.lo
    assert sorted(i for b in bs for i in b.params) == list(range(len(params)))
    # the tail bucket (first layers, reduced last and never overlapped) is the small one
    slack = 64 * 4  # arena alignment padding
    assert bs[-1].nbytes <= max(cap // 4, max(a.numels[i] for i in bs[-1].params) * 4) + slack


def test_auto_bucket_cap():
    assert auto_bucket_cap(51 * MB, 64 * MB) == 51 * MB // 8
    assert auto_bucket_cap(4 * MB, 64 * MB) == 2 * MB
    assert auto_bucket_cap(1000 * MB, 64 * MB) == 64 * MB
    assert auto_bucket_cap(1000 * MB, 25 * MB) == 25 * MB


def test_apply_rccl_env():
    env = {"NCCL_PROTO": "LL"}
    applied = apply_rccl_env({"rccl": {"algo": "Tree", "protocol": "Simple", "min_channels": 16}}, env)
    assert env["NCCL_ALGO"] == "Tree" and env["NCCL_MIN_NCHANNELS"] == "16"
    assert env["NCCL_PROTO"] == "LL" and "NCCL_PROTO" not in applied  # explicit env wins


@pytest.mark.parametrize("world", [2, 8])
def test_fp32_accum_bf16_error_bound(tmp_path, world):
    res = _run(str(tmp_path / "acc"), world, "fp32_accum")
    assert set(res[0]["modes"]) == {"fp32_accum"} and res[0]["nbuckets"] > 1
    for r in range(1, world):  # every rank ends with identical bits
        assert torch.equal(res[0]["reduced"], res[r]["reduced"])
    red = res[0]["reduced"].double()
    exact = _exact_sum(world, red.numel(), torch.bfloat16)
    # one rounding of the exact sum to bf16: |err| <= 2^-8 |exact| (half an ulp, 8 mantissa bits)
    err = (red - exact).abs()
    assert bool((err <= exact.abs() * 2.0 ** -8 + 1e-30).all()), float((err / exact.abs().clamp_min(1e-30)).max())
    if world == 8:
        ring = _run(str(tmp_path / "ring"), world, "allreduce")
        rerr = (ring[0]["reduced"].double() - exact).abs()
        assert float(err.mean()) < 0.75 * float(rerr.mean())  # strictly more accurate than a bf16 ring


def test_fp32_arena_uses_allreduce_and_compression_accumulates(tmp_path):
    res = _run(str(tmp_path / "f32"), 4, "fp32_accum", dtype="float32")
    assert set(res[0]["modes"]) == {"allreduce"}
    exact = _exact_sum(4, res[0]["reduced"].numel(), torch.float32)
    torch.testing.assert_close(res[0]["reduced"].double(), exact, rtol=1e-5, atol=1e-5)
    comp = _run(str(tmp_path / "cmp"), 4, "fp32_accum", dtype="float32", compress=True)
    assert set(comp[0]["modes"]) == {"fp32_accum"}
    err = (comp[0]["reduced"].double() - exact).abs()
    # inputs rounded to bf16 once (2^-9 relative each), the fp32 sum rounded once
    assert float((err / exact.abs().clamp_min(1e-3)).median()) < 2.0 ** -7
