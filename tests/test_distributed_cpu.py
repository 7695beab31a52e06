"""Multi-process data parallelism on CPU (gloo): N ranks x per-slot batch == 1 rank x global batch."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "dist_scripts", "dp_worker.py")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(out: str, world: int, agg: int, compress: bool = False, **extra_env: str) -> None:
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, **extra_env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, WORKER, out, "XORTrial", str(agg), "1" if compress else "0"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, o.decode()[-4000:]


def test_dp2_checkpoint_inside_aggregation_window_resumes_exactly(tmp_path):
    """a checkpoint taken mid-window keeps the ranks' partial sums (summed into the
    chief's copy), so a restored 2-rank run steps on the same gradient sums as an uninterrupted one."""
    ckpt = str(tmp_path / "ckpt")
    _launch(str(tmp_path / "full"), 2, 2, MODE="full")
    _launch(str(tmp_path / "first"), 2, 2, MODE="ckpt", CKPT=ckpt)
    saved = torch.load(os.path.join(ckpt, "state_dict.pth"), weights_only=False)
    assert saved.get("accumulated_grads") is not None  # batch 3 of a 2-batch window
    _launch(str(tmp_path / "resumed"), 2, 2, MODE="resume", CKPT=ckpt)
    full, res0, res1 = (torch.load(str(tmp_path / f)) for f in ("full.0.pt", "resumed.0.pt", "resumed.1.pt"))
    torch.testing.assert_close(res0, res1, rtol=0, atol=0)
    torch.testing.assert_close(res0, full, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("agg", [1, 2])
def test_dp2_matches_single_process(tmp_path, agg):
    _launch(str(tmp_path / "single"), 1, agg)
    _launch(str(tmp_path / "dp"), 2, agg)
    ref = torch.load(str(tmp_path / "single.0.pt"))
    r0 = torch.load(str(tmp_path / "dp.0.pt"))
    r1 = torch.load(str(tmp_path / "dp.1.pt"))
    torch.testing.assert_close(r0, r1, rtol=0, atol=0)  # ranks stay bitwise in sync
    torch.testing.assert_close(r0, ref, rtol=1e-5, atol=1e-6)
    import json

    resp = json.load(open(str(tmp_path / "dp.0.json")))
    assert resp[0]["metrics"]["num_inputs"] == 32  # 4 batches x 4 per slot x 2 ranks
    assert "validation_loss" in resp[2]["metrics"]["validation_metrics"]
    assert json.load(open(str(tmp_path / "dp.1.json"))) == [None, None, None]  # non-chief: Skipped


def test_dp2_bf16_compression_close(tmp_path):
    _launch(str(tmp_path / "single"), 1, 1)
    _launch(str(tmp_path / "dpc"), 2, 1, compress=True)
    ref = torch.load(str(tmp_path / "single.0.pt"))
    r0 = torch.load(str(tmp_path / "dpc.0.pt"))
    torch.testing.assert_close(r0, ref, rtol=5e-2, atol=5e-3)


def test_bench_two_ranks_gloo_smoke(tmp_path):
    """bench.py under torch.distributed.run with 2 CPU ranks: the exact multi-GPU code path of the
    driver's scaling run (bucketer + grad sink + fused optimizer + metric gather), on gloo."""
    import subprocess
    import sys

    from determined_1_amd.deploy.local import free_port

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(repo, "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--arch", "resnet18", "--batch-per-gpu", "2",
                        "--image-size", "32", "--amp", "O0"], capture_output=True, text=True, timeout=600, cwd=repo)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["value"] > 0


def test_bench_self_launch_plain_invocation():
    """``python bench.py --gpus 2`` with no launcher env: bench.py spawns its own 2 ranks (the
    driver's SCALE invocation), joins them over gloo on CPU and prints one JSON line."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--arch", "resnet18", "--batch-per-gpu", "2", "--image-size", "32", "--amp", "O0"],
                       capture_output=True, text=True, timeout=600, cwd=repo, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["world_size_seen"] == [2, 2] and out["config"]["backend"] == "gloo"
    assert out["config"]["warmup_s"] >= 0 and out["value"] > 0
    # multi-rank runs always report per-rank step time and skew (first-contact diagnostics)
    assert len(out["config"]["rank_ms_per_step"]) == 2 and out["config"]["rank_skew_pct"] >= 0


def test_bench_collectives_cpu_two_ranks():
    """scripts/bench_collectives.py self-launches its ranks (gloo here) and prints one line per
    (size, algorithm) plus the auto-rule summary."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(repo, "scripts", "bench_collectives.py"), "--gpus", "2", "--cpu",
                        "--sizes-mb", "0.5,1", "--iters", "2"], capture_output=True, text=True, timeout=300, cwd=repo,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    algos = {(x["size_mb"], x["algo"]) for x in recs if "algo" in x}
    assert algos == {(m, a) for m in (0.5, 1.0) for a in ("allreduce_bf16", "allreduce_fp32", "fp32_accum_bf16")}
    assert all(x["ms"] > 0 and x["world"] == 2 for x in recs if "algo" in x)
    summary = [x for x in recs if "summary" in x]
    assert summary and set(summary[0]["choice_by_mb"].values()) <= {"allreduce", "fp32_accum"}


def test_miopen_db_per_rank_and_key_merge(tmp_path, monkeypatch):
    """Each local rank of a multi-rank job gets its own writable db; seeding merges by key and never
    overwrites an entry the user already tuned; a changed shipped db is merged in again."""
    import importlib

    from determined_1_amd.ops import miopen_db

    shipped = tmp_path / "shipped"
    (shipped / "db").mkdir(parents=True)
    (shipped / "cache").mkdir()
    (shipped / "db" / "x.ufdb.txt").write_text("k1=shipped1\nk2=shipped2\n")
    (shipped / "cache" / "k.ukdb").write_bytes(b"bin")
    monkeypatch.setattr(miopen_db, "SHIPPED", str(shipped))
    envs = [{"DET_MIOPEN_DIR": str(tmp_path / "run"), "WORLD_SIZE": "2", "LOCAL_RANK": str(r)} for r in range(2)]
    dbs = [miopen_db.configure(e) for e in envs]
    assert dbs[0] != dbs[1] and dbs[0].endswith("rank0/db") and dbs[1].endswith("rank1/db")
    user = tmp_path / "run" / "rank0" / "db" / "x.ufdb.txt"
    user.write_text("k1=user_tuned\n")
    (shipped / "db" / "x.ufdb.txt").write_text("k1=shipped1\nk2=shipped2\nk3=shipped3\n")
    import os as _os
    _os.utime(shipped / "db" / "x.ufdb.txt", (1, 1))  # shipped db changed -> new stamp
    e0 = {"DET_MIOPEN_DIR": str(tmp_path / "run"), "WORLD_SIZE": "2", "LOCAL_RANK": "0"}
    miopen_db.configure(e0)
    got = dict(l.split("=", 1) for l in user.read_text().splitlines())
    assert got == {"k1": "user_tuned", "k2": "shipped2", "k3": "shipped3"}
    importlib.reload(miopen_db)


def test_bench_rejects_mismatched_world():
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=repo, env=env)
    assert r.returncode == 2 and "--gpus is 2" in r.stderr


def test_partial_window_grads_with_missing_grad_on_one_rank(tmp_path):
    """one rank without a .grad for a parameter still joins the same all-reduce (zeros
    plus a presence flag), so the mid-window checkpoint neither hangs nor misaligns the sums."""
    port = _free_port()
    out = str(tmp_path / "pw.pt")
    script = os.path.join(HERE, "dist_scripts", "partial_window_worker.py")
    procs = [subprocess.Popen([sys.executable, script, out],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(2)]
    for p in procs:
        o, _ = p.communicate(timeout=120)
        assert p.returncode == 0, o.decode()[-3000:]
    got = torch.load(out)[0]
    # parameter i holds (rank + 1 + i) on each rank that has it; rank 1 has none for i = 2
    for i, g in enumerate(got):
        want = float(1 + i) + (0.0 if i == 2 else float(2 + i))
        assert torch.equal(g, torch.full_like(g, want)), (i, g)
