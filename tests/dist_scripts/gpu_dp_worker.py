"""One rank of a GPU data-parallel equivalence run.  Usage:
    [RANK/WORLD_SIZE/MASTER_* + DET_FORCE_DISTRIBUTED=1] python gpu_dp_worker.py OUT AMP AGG COMPRESS REDUCTION
Trains a small MLP PyTorchTrial on cuda for 8 batches and writes the final parameters plus the
bucketer layout to OUT.pt.  With DET_FORCE_DISTRIBUTED=1 and WORLD_SIZE=1 the whole multi-process
path runs over ProcessGroupNCCL (= RCCL): rank-0 broadcast of arenas/buffers/optimizer state,
GradSink landing, the gradient bucketer (all-to-all + fp32 shard sum + all-gather, or all-reduce),
bf16 compression and aggregation windows."""
import os
import sys
from typing import Any, Dict

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from determined_1_amd import pytorch  # noqa: E402
from tests.utils import Recorder, run  # noqa: E402


class MLPTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        torch.manual_seed(7)
        m = torch.nn.Sequential(torch.nn.Linear(64, 512), torch.nn.ReLU(), torch.nn.Linear(512, 512), torch.nn.ReLU(),
                                torch.nn.Linear(512, 10))
        self.model = context.wrap_model(m)
        self.opt = context.wrap_optimizer(torch.optim.SGD(self.model.parameters(), lr=0.05, momentum=0.9))
        amp = context.get_hparams()["amp"]
        if amp != "O0":
            self.model, self.opt = context.configure_apex_amp(self.model, self.opt, opt_level=amp)

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, Any]:
        x, y = batch
        loss = torch.nn.functional.cross_entropy(self.model(x).float(), y)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        x, y = batch
        return {"validation_loss": torch.nn.functional.cross_entropy(self.model(x).float(), y)}

    def build_training_data_loader(self) -> pytorch.DataLoader:
        g = torch.Generator().manual_seed(3)
        ds = torch.utils.data.TensorDataset(torch.randn(256, 64, generator=g), torch.randint(0, 10, (256,), generator=g))
        return pytorch.DataLoader(ds, batch_size=self.context.get_per_slot_batch_size(), shuffle=False)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        return self.build_training_data_loader()


def ctrl_responses(rec: Recorder):
    return [r["metrics"]["batch_metrics"] for r in rec.responses if isinstance(r, dict) and "batch_metrics" in
            r.get("metrics", {})]


def main() -> None:
    out, amp, agg, compress, reduction = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4] == "1", sys.argv[5]
    half = int(os.environ.get("GDP_HALF_STEPS", "4"))  # batches per training workload (2 workloads)
    rec = Recorder().train(1, half, 0).train(2, half, half)
    gpu = torch.cuda.is_available()
    ctrl, _ = run(MLPTrial, {"global_batch_size": 16, "amp": amp}, rec, trial_seed=5, use_gpu=gpu,
                  optimizations={"aggregation_frequency": agg, "gradient_compression": compress,
                                 "grad_reduction": reduction})
    if gpu:
        torch.cuda.synchronize()
    ctx = ctrl.context
    params = torch.cat([p.detach().reshape(-1).float().cpu() for p in ctx.models[0].parameters()])
    import torch.distributed as dist

    info = {"params": params, "dist": dist.is_initialized(),
            "backend": dist.get_backend() if dist.is_initialized() else None,
            "buckets": [st.bucketer.describe() for st in ctx._opt_states if st.bucketer is not None],
            "graph": ctrl._graph.stats() if getattr(ctrl, "_graph", None) is not None else None,
            "losses": [float(b["loss"]) for r in ctrl_responses(rec) for b in r]}
    if info["graph"] is not None:
        info["graph"] = {k: (v if isinstance(v, (int, type(None))) else str(v)) for k, v in info["graph"].items()}
    torch.save(info, out + ".pt")
    from determined_1_amd.parallel import dist as pdist

    pdist.shutdown()


if __name__ == "__main__":
    main()
