"""One rank of the ResNet-50 data-parallel equivalence runs (tests/test_dp_resnet_gpu.py).  Usage:
    [torch.distributed.run env + DET_DIST_SHARE_GPU=1 DET_DIST_BACKEND=gloo] \
        python resnet_dp_worker.py OUT AMP COMPRESS DATA STEPS LR MOMENTUM
The real fused ResNet-50 path of the benchmark trial (examples/computer_vision/resnet50_pytorch:
fused BN with linked shortcut gradients and deferred applies, native 1x1/3x3/stem convs, GradSink
landing, fused arena SGD, and -- with 2 ranks -- the gradient bucketer: fp32_accum for the bf16
arena, bf16 wire compression for the fp32 one) on 64x64 images, 8 per rank.  DATA picks the
per-rank batches: "seq" batch i at step i; "dup" each batch twice in a row, so with 2 ranks both
see batch i at step i; "b0"/"b1" only batch 0 / 1; "pair" batches 0, 1 (2 ranks: one each).
Writes the flat fp32 master weights (the arena's, O2) or fp32 parameters (O0) to OUT.pt."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "examples", "computer_vision", "resnet50_pytorch"))

import torch  # noqa: E402

from determined_1_amd import pytorch as det_torch  # noqa: E402
from model_def import ResNetImageNetTrial  # noqa: E402
from determined_1_amd import workload  # noqa: E402
from determined_1_amd.experimental._local import make_controller  # noqa: E402
from tests.utils import Recorder, base_config  # noqa: E402

PER_RANK, SIZE = 8, 64


class Batches(torch.utils.data.Dataset):
    def __init__(self, order):
        # batch b from its own generator: its content must not depend on how many batches the run
        # uses ("b0" alone vs "pair"), or the split-batch check compares different data
        n = max(order) + 1
        self.img = torch.empty((n, PER_RANK, SIZE, SIZE, 3), dtype=torch.uint8)
        self.lab = torch.empty((n, PER_RANK), dtype=torch.int64)
        for b in range(n):
            g = torch.Generator().manual_seed(11 + 1000 * b)
            self.img[b] = torch.randint(0, 256, (PER_RANK, SIZE, SIZE, 3), generator=g, dtype=torch.uint8)
            self.lab[b] = torch.randint(0, 10, (PER_RANK,), generator=g)
        self.order = order

    def __len__(self):
        return len(self.order) * PER_RANK

    def __getitem__(self, i):
        b = self.order[i // PER_RANK]
        return self.img[b, i % PER_RANK], self.lab[b, i % PER_RANK]


class Trial(ResNetImageNetTrial):
    def build_training_data_loader(self) -> det_torch.DataLoader:
        data, steps = os.environ["RDP_DATA"], int(os.environ["RDP_STEPS"])
        order = {"seq": list(range(steps)), "dup": [i for i in range(steps) for _ in range(2)], "b0": [0], "b1": [1],
                 "pair": [0, 1]}[data]
        return det_torch.DataLoader(Batches(order), batch_size=self.context.get_per_slot_batch_size(), shuffle=False)


if os.environ.get("RDP_DEBUG"):  # print each rank's batch labels (data-sharding checks)
    _orig_tb = Trial.train_batch

    def _tb(self, batch, epoch_idx, batch_idx):
        print("RANK", os.environ.get("RANK", "0"), "batch", batch_idx, "labels", batch[1].tolist(), flush=True)
        return _orig_tb(self, batch, epoch_idx, batch_idx)

    Trial.train_batch = _tb


def main() -> None:
    out, amp, compress, data, steps, lr, mom = sys.argv[1:8]
    # O0 runs the fp32 convolutions on MIOpen: deterministic solvers only, so that two processes on
    # the same batches agree to rounding (the weight-gradient solvers with atomics otherwise add
    # run-to-run noise the comparison would mistake for a reduction error)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    os.environ["RDP_DATA"], os.environ["RDP_STEPS"] = data, steps
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rec = Recorder().train(1, int(steps), 0)
    hp = {"global_batch_size": PER_RANK * world, "amp": amp, "num_classes": 10, "image_size": SIZE, "lr": float(lr),
          "momentum": float(mom), "weight_decay": 0.0}
    cfg = base_config(hp, resources={"slots_per_trial": world},
                      optimizations={"gradient_compression": compress == "1", "grad_reduction": "fp32_accum"})
    ctrl = make_controller(Trial, cfg, rec.stream(), trial_seed=3, use_gpu=os.environ.get("RDP_CPU") != "1",
                           initial_workload=workload.train_workload(1, num_batches=1, total_batches_processed=0))
    ctx = ctrl.context
    ctx._finalize()  # arenas (+ fp32 masters at O2) exist from here on; idempotent

    def flat():
        fused = [st.fused for st in ctx._opt_states if st.fused is not None]
        assert fused, "the benchmark trial's SGD runs on the fused arena optimizer"
        return torch.cat([(a.master if a.has_master else a.flat_param).detach().float().reshape(-1).cpu()
                          for f in fused for a in f.arenas])

    init = flat()
    ctrl.run()
    resp = rec.responses
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    import torch.distributed as dist

    from determined_1_amd.ops import conv, norm

    info = {"params": flat(), "init": init, "world": world, "dist": dist.is_initialized(),
            "buckets": json.loads(json.dumps([st.bucketer.describe() for st in ctx._opt_states if st.bucketer is not None],
                                          default=float)),
            "counts": {"fwd_apply": dict(conv.FWD_APPLY_COUNTS), "bn_bwd": dict(conv.BN_BWD_COUNTS),
                       "conv3x3": dict(conv.CONV3X3_COUNTS), "bn_apply": dict(conv.BN_APPLY_COUNTS),
                       "bn_fallbacks": norm.FALLBACKS["count"]},
            "loss": [float(m["loss"]) for r in resp if isinstance(r, dict) and "metrics" in r
                     for m in r["metrics"]["batch_metrics"]]}
    if int(os.environ.get("RANK", "0")) == 0:
        torch.save(info, out + ".pt")
    from determined_1_amd.parallel import dist as pdist

    pdist.shutdown()


if __name__ == "__main__":
    main()
