"""cProfile of one CIFAR trial's construction (the 'trial constructed' phase of every ASHA
container) on the GPU: where do ~1.6 s go?"""
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

t0 = time.time()
torch.cuda.init()
torch.empty(1, device="cuda")
print("hip init %.3f s" % (time.time() - t0), flush=True)
cfg = {"hyperparameters": {"global_batch_size": 32, "learning_rate": 1e-3, "learning_rate_decay": 1e-6,
                           "layer1_dropout": 0.25, "layer2_dropout": 0.25, "layer3_dropout": 0.5, "amp": "O2"},
       "searcher": {"name": "single", "metric": "validation_error", "max_length": {"batches": 100}},
       "records_per_epoch": 50000, "optimizations": {"hip_graph": True}}
stream = iter([(workload.train_workload(1, num_batches=20), [], workload.ignore_response),
               (workload.terminate_workload(1, total_batches_processed=20), [], workload.ignore_response)])
pr = cProfile.Profile()
t0 = time.time()
pr.enable()
ctrl = make_controller(model_def.CIFARTrial, cfg, stream, use_gpu=True)
pr.disable()
print("controller build %.3f s" % (time.time() - t0), flush=True)
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
print(s.getvalue())
t0 = time.time()
pr2 = cProfile.Profile()
pr2.enable()
ctrl.run()
torch.cuda.synchronize()
pr2.disable()
print("20 batches incl. first-batch work %.3f s" % (time.time() - t0), flush=True)
s = io.StringIO()
pstats.Stats(pr2, stream=s).sort_stats("cumulative").print_stats(30)
print(s.getvalue())
