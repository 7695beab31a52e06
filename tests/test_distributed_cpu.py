"""Multi-process data parallelism on CPU (gloo): N ranks x per-slot batch == 1 rank x global batch."""
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


def _launch(out: str, world: int, agg: int, compress: bool = False) -> None:
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
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
