"""Seed the shipped MIOpen db + kernel cache (determined_1_amd/ops/miopen_db/) with every conv
problem the ASHA benchmark's CIFAR-10 trial can hit: the adaptive.yaml search space draws
global_batch_size from 16..64, and each batch size is a distinct MIOpen problem whose kernels are
JIT-compiled on first use (~4.7 s of every new trial container, scripts/dbg/profile_trial_build.py).

    python scripts/miopen_seed_cifar.py [--min 16] [--max 64] [--harvest DIR]
Runs the real CIFARTrial (bf16 O2) for 2 train batches + a short validation per batch size."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "examples", "computer_vision", "cifar10_pytorch"))

from determined_1_amd.ops import miopen_db  # noqa: E402

miopen_db.configure(os.environ)

import torch  # noqa: E402

from determined_1_amd import workload  # noqa: E402
from determined_1_amd.experimental import make_controller  # noqa: E402
import model_def  # noqa: E402


class SmallVal(model_def.CIFARTrial):
    def build_validation_data_loader(self):
        from determined_1_amd import pytorch
        from determined_1_amd.models.synthetic import SyntheticClassification

        b = self.context.get_per_slot_batch_size()
        return pytorch.DataLoader(SyntheticClassification(3 * b + 5, (3, 32, 32), seed=1), batch_size=b)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--min", type=int, default=16)
    ap.add_argument("--max", type=int, default=64)
    ap.add_argument("--harvest", default="", help="copy the db + kernel cache here (e.g. gpurun_out/miopen_db)")
    args = ap.parse_args()
    for b in range(args.min, args.max + 1):
        t0 = time.time()
        cfg = {"hyperparameters": {"global_batch_size": b, "learning_rate": 1e-3, "learning_rate_decay": 1e-6,
                                   "layer1_dropout": 0.25, "layer2_dropout": 0.25, "layer3_dropout": 0.5, "amp": "O2"},
               "searcher": {"name": "single", "metric": "validation_error", "max_length": {"batches": 4}},
               "records_per_epoch": 50000, "optimizations": {"hip_graph": True}}
        stream = iter([(workload.train_workload(1, num_batches=4), [], workload.ignore_response),
                       (workload.validation_workload(1, total_batches_processed=4), [], workload.ignore_response),
                       (workload.terminate_workload(1, total_batches_processed=4), [], workload.ignore_response)])
        make_controller(SmallVal, cfg, stream, use_gpu=True).run()
        torch.cuda.synchronize()
        print(f"batch {b}: {time.time() - t0:.2f} s", flush=True)
    if args.harvest:
        n = miopen_db.harvest(args.harvest, with_cache=True)
        print(f"harvested {n} files into {args.harvest}", flush=True)


if __name__ == "__main__":
    main()
