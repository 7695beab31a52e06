"""Repro for trial containers dying with SIGSEGV in the first step after a restore (ASHA rung 2)
with hip_graph + hip_graph_batches: train 3 steps + checkpoint, then a fresh controller restores
and trains 2 more steps.  faulthandler prints the Python stack on a crash."""
import faulthandler
import os
import pathlib
import sys
import tempfile

faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from determined_1_amd.experimental import load_model_def  # noqa: E402
from tests.utils import Recorder, run  # noqa: E402

os.environ.setdefault("DET_HIP_GRAPH", "1")
os.environ.setdefault("DET_GRAPH_BATCHES", "16")
Trial = load_model_def(os.path.join(REPO, "examples", "computer_vision", "cifar10_pytorch")).CIFARTrial
bs = int(sys.argv[1]) if len(sys.argv) > 1 else 52
hp = {"learning_rate": 1e-3, "learning_rate_decay": 1e-6, "layer1_dropout": 0.3, "layer2_dropout": 0.3,
      "layer3_dropout": 0.3, "global_batch_size": bs, "amp": os.environ.get("AMP", "O2"), "validation_records": 2000}
d = pathlib.Path(tempfile.mkdtemp())
rec = Recorder().train(1, 100, 0).train(2, 100, 100).train(3, 100, 200).validate(3, 300).checkpoint(3, 300, d / "ck")
ctrl, resp = run(Trial, hp, rec, use_gpu=True, records_per_epoch=50000)
torch.cuda.synchronize()
print("phase 1 ok", ctrl._graph.stats() if ctrl._graph else None, flush=True)
del ctrl
rec = Recorder().train(4, 100, 300).train(5, 100, 400).validate(5, 500)
ctrl, resp = run(Trial, hp, rec, load_path=d / "ck", total_batches=300, use_gpu=True, records_per_epoch=50000)
torch.cuda.synchronize()
print("phase 2 ok", ctrl._graph.stats() if ctrl._graph else None, flush=True)
