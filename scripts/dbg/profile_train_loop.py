"""Host-side cost of one graph-replayed CIFAR train batch: cProfile of 2000 batches after warmup."""
import cProfile
import io
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "examples", "computer_vision", "cifar10_pytorch"))
import torch  # noqa: E402

from determined_1_amd import workload  # noqa: E402
from determined_1_amd.experimental import make_controller  # noqa: E402
import model_def  # noqa: E402

cfg = {"hyperparameters": {"global_batch_size": 32, "learning_rate": 1e-3, "learning_rate_decay": 1e-6,
                           "layer1_dropout": 0.25, "layer2_dropout": 0.25, "layer3_dropout": 0.5, "amp": "O2"},
       "searcher": {"name": "single", "metric": "validation_error", "max_length": {"batches": 100}},
       "records_per_epoch": 50000, "optimizations": {"hip_graph": True}}
prof = cProfile.Profile()
marks = {}


def mark(name):
    def f(_):
        torch.cuda.synchronize()
        marks[name] = time.time()
        if name == "warm":
            prof.enable()
        elif name == "timed":
            prof.disable()
    return f


stream = iter([(workload.train_workload(1, num_batches=200), [], mark("warm")),
               (workload.train_workload(2, num_batches=2000, total_batches_processed=200), [], mark("timed")),
               (workload.terminate_workload(2, total_batches_processed=2200), [], workload.ignore_response)])
ctrl = make_controller(model_def.CIFARTrial, cfg, stream, use_gpu=True)
ctrl.run()
print("ms/batch %.4f" % ((marks["timed"] - marks["warm"]) * 1000 / 2000), flush=True)
s = io.StringIO()
pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(40)
print(s.getvalue())
