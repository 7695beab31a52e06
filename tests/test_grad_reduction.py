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


def _run(out: str, world: int, reduction: str, dtype: str = "bfloat16", compress: bool = False,
         extra_env: dict = None, logs: list = None) -> list:
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   OMP_NUM_THREADS="1", **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, WORKER, out, reduction, dtype, "1" if compress else "0"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        o, _ = p.communicate(timeout=240)
        assert p.returncode == 0, o.decode()[-3000:]
        if logs is not None:
            logs.append(o.decode())
    return [torch.load(f"{out}.{r}.pt", weights_only=False) for r in range(world)]


def _abs_sum(world: int, numel: int, dtype: torch.dtype) -> torch.Tensor:
    tot = torch.zeros(numel, dtype=torch.float64)
    for r in range(world):
        g = torch.Generator().manual_seed(1234 + r)
        tot += (torch.randn(numel, generator=g) * (1.0 + r)).to(dtype).double().abs()
    return tot


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


@pytest.mark.parametrize("world", [2, 4, 8])
def test_auto_reduction_agrees_across_ranks(tmp_path, world):
    """grad_reduction: auto times both algorithms collectively; every rank must pick identical
    per-bucket modes (else the collective sequences diverge and the job hangs)."""
    res = _run(str(tmp_path / "auto"), world, "auto")
    choice0 = res[0]["auto_choice"]
    assert choice0 and all(v["mode"] in ("fp32_accum", "allreduce") for v in choice0.values())
    assert all("allreduce_ms" in v and "fp32_accum_ms" in v for v in choice0.values())
    for r in range(1, world):
        assert res[r]["auto_choice"] == choice0
        assert res[r]["modes"] == res[0]["modes"]
        assert torch.equal(res[0]["reduced"], res[r]["reduced"])
    red = res[0]["reduced"].double()
    exact = _exact_sum(world, red.numel(), torch.bfloat16)
    # either algorithm: within a bf16 ring's worst case (world-1 roundings of partial sums)
    assert bool(((red - exact).abs() <= _abs_sum(world, red.numel(), torch.bfloat16) * world * 2.0 ** -8).all())


def test_fp32_accum_downgrade_warns_at_world_3(tmp_path):
    logs = []
    res = _run(str(tmp_path / "w3"), 3, "fp32_accum", logs=logs)
    assert res[0]["downgraded"], "64-element-aligned buckets are not divisible by 3"
    assert "allreduce" in res[0]["modes"]
    assert any("fall back to a" in o and "not divisible by world size 3" in o for o in logs), logs[0][-2000:]
    n = res[0]["reduced"].numel()
    exact = _exact_sum(3, n, torch.bfloat16)
    assert bool(((res[0]["reduced"].double() - exact).abs() <= _abs_sum(3, n, torch.bfloat16) * 3 * 2.0 ** -8).all())


def test_tensor_fusion_autotune_converges_identically(tmp_path):
    """auto_tune_tensor_fusion: caps searched over the first windows, decision identical on every
    rank at the same window, CSV log written by rank 0, reduction still exact afterwards."""
    from determined_1_amd.parallel import ddp

    windows = len(ddp.AUTOTUNE_CAPS_MB) * ddp.AUTOTUNE_WINDOWS + 3
    out = str(tmp_path / "tune")
    res = _run(out, 2, "fp32_accum", extra_env={"DET_TEST_AUTOTUNE": "1", "DET_TEST_WINDOWS": str(windows)})
    assert res[0]["tuned"] and res[0]["tuned"] == res[1]["tuned"]
    assert res[0]["caps"] == res[1]["caps"]
    assert len(set(res[0]["caps"])) >= 2  # the search visited several caps
    assert res[0]["caps"][-1] == res[0]["caps"][-2]  # settled
    lines = open(out + ".autotune.csv").read().strip().splitlines()
    assert lines[0] == "cap_mb,window_ms,chosen" and sum(int(l.split(",")[2]) for l in lines[1:]) == 1
    exact = _exact_sum(2, res[0]["reduced"].numel(), torch.bfloat16)
    err = (res[0]["reduced"].double() - exact).abs()
    assert bool((err <= exact.abs() * 2.0 ** -8 + 1e-30).all())


@pytest.mark.parametrize("world", [2, 4])
def test_graph_capture_reduction_path_order_and_numerics(tmp_path, world):
    """the reduction a hipGraph capture records for fp32_accum buckets (fp32
    reduce-scatter of the widened bucket, one rounding of the shard, in-place all-gather, all on the
    capturing stream -- RCCL's all-to-all does not capture) launches the buckets in the same order as
    the eager path and reduces to the same sums: exactly at 2 ranks, within one bf16 rounding of the
    eager fp32_accum result at 4 (the fp32 sums of the two paths may round differently)."""
    eager = _run(str(tmp_path / "e"), world, "fp32_accum")
    graph = _run(str(tmp_path / "g"), world, "fp32_accum", extra_env={"DET_TEST_GRAPH_PATH": "1"})
    n = eager[0]["nbuckets"]
    for r in range(world):
        assert eager[r]["launch_log"] == graph[r]["launch_log"] == list(range(n))
        torch.testing.assert_close(graph[r]["reduced"], graph[0]["reduced"], rtol=0, atol=0)  # ranks agree
    ge, gg = eager[0]["reduced"].double(), graph[0]["reduced"].double()
    if world == 2:
        torch.testing.assert_close(gg, ge, rtol=0, atol=0)
    else:
        ulp = ge.abs() * 2.0 ** -7 + 1e-30
        assert bool(((gg - ge).abs() <= ulp).all())
    exact = _exact_sum(world, gg.numel(), torch.bfloat16)
    assert float((gg - exact).abs().max()) <= float((exact.abs() * 2.0 ** -8).max()) + 1e-6
