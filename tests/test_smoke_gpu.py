import pytest

pytestmark = pytest.mark.gpu


def test_graft_smoke(gpu):
    import __graft_entry__ as g

    g.smoke()


def test_bench_two_ranks_sharing_the_gpu(gpu, tmp_path):
    """bench.py under torch.distributed.run with 2 ranks folded onto this GPU (DET_DIST_SHARE_GPU=1)
    over gloo: the data-parallel GPU path of the driver's scaling run (GradSink landing, bucketed
    async all-reduce launched from backward hooks on CUDA tensors, fused SGD, metric gather).  RCCL
    itself refuses two ranks on one device, so the collective backend is the only difference."""
    import json
    import os
    import subprocess
    import sys

    from determined_1_amd.deploy.local import free_port

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DET_DIST_SHARE_GPU="1", DET_DIST_BACKEND="gloo", DET_STEP_TIMERS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(repo, "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "2", "--batch-per-gpu", "16", "--image-size", "64",
                        "--bucket-mb", "8", "--cudnn-benchmark", "0"],
                       capture_output=True, text=True, timeout=300, cwd=repo, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["value"] > 0
    assert out["config"]["final_avg_loss"] is not None
    ph = out["config"]["phase_ms"]  # step timers, incl. the exposed all-reduce wait after backward
    assert ph["forward_ms"] > 0 and ph["backward_ms"] > 0 and ph["optimizer_ms"] > 0 and ph["comm_exposed_ms"] >= 0


def test_bert_two_ranks_sharing_the_gpu_with_aggregation(gpu):
    """scripts/bench_bert.py with 2 ranks on this GPU over gloo and aggregation_frequency 2 under
    bf16 O2: DP bucketing + gradient landing straight into the arena + skipped-sync windows."""
    import json
    import os
    import subprocess
    import sys

    from determined_1_amd.deploy.local import free_port

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DET_DIST_SHARE_GPU="1", DET_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
                        os.path.join(repo, "scripts", "bench_bert.py"), "--steps", "4", "--warmup", "2", "--agg", "2"],
                       capture_output=True, text=True, timeout=300, cwd=repo, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["config"]["tf_fallbacks"] == 0
