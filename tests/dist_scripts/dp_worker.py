"""One rank of a multi-process data-parallel run (gloo on CPU).  Usage:
    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p python dp_worker.py OUT TRIAL AGG [COMPRESS]
Writes the final flat parameter vector of rank r to OUT.r.pt and the validation response."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from tests.fixtures import xor  # noqa: E402
from tests.utils import Recorder, run  # noqa: E402


def main() -> None:
    out, trial_name, agg = sys.argv[1], sys.argv[2], int(sys.argv[3])
    compress = len(sys.argv) > 4 and sys.argv[4] == "1"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    trial_cls = getattr(xor, trial_name)
    # MODE (env): "" the default 4+4 batches; "full" 8 batches; "ckpt" 3 batches then a checkpoint inside
    # the aggregation window (to CKPT); "resume" the last 5 batches from CKPT
    mode = os.environ.get("MODE", "")
    import pathlib

    load_path = None
    if mode == "full":
        rec = Recorder().train(1, 8, 0)
    elif mode == "ckpt":
        rec = Recorder().train(1, 3, 0).checkpoint(1, 3, pathlib.Path(os.environ["CKPT"]))
    elif mode == "resume":
        rec, load_path = Recorder().train(2, 5, 3), pathlib.Path(os.environ["CKPT"])
    else:
        rec = Recorder().train(1, 4, 0).train(2, 4, 4).validate(2, 8)
    ctrl, resp = run(trial_cls, {"global_batch_size": 8, "optimizer": "adam", "lr": 0.05}, rec, trial_seed=11,
                     load_path=load_path, total_batches=3 if mode == "resume" else 0,
                     resources={"slots_per_trial": world},
                     optimizations={"aggregation_frequency": agg, "gradient_compression": compress,
                                    "average_training_metrics": True})
    params = torch.cat([p.detach().reshape(-1).float() for p in ctrl.context.models[0].parameters()])
    rank = int(os.environ.get("RANK", "0"))
    torch.save(params, f"{out}.{rank}.pt")
    with open(f"{out}.{rank}.json", "w") as f:
        json.dump([r if isinstance(r, dict) else None for r in resp], f, default=float)
    from determined_1_amd.parallel import dist

    dist.shutdown()


if __name__ == "__main__":
    main()
