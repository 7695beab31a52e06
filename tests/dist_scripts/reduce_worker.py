"""One rank of the gradient-reduction accuracy check (gloo on CPU).  Usage:
    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p python reduce_worker.py OUT REDUCTION DTYPE
Every rank fills a bf16 (or fp32) arena with rank-seeded gradients, runs GradientBucketer with the
given reduction and writes the reduced flat gradient to OUT.r.pt."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from determined_1_amd.ops.arena import Arena  # noqa: E402
from determined_1_amd.parallel.ddp import GradientBucketer  # noqa: E402


def main() -> None:
    out, reduction, dtype = sys.argv[1], sys.argv[2], getattr(torch, sys.argv[3])
    compress = len(sys.argv) > 4 and sys.argv[4] == "1"
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.manual_seed(0)
    shapes = [(1000, 300), (4096,), (64, 64, 3, 3), (200, 200), (17,), (512, 1024)]
    params = [torch.nn.Parameter(torch.zeros(s, dtype=dtype)) for s in shapes]
    arena = Arena(params, torch.device("cpu"))
    g = torch.Generator().manual_seed(1234 + rank)
    full = torch.randn(arena.numel, generator=g) * (1.0 + rank)
    arena.flat_grad.copy_(full.to(dtype))
    autotune = os.environ.get("DET_TEST_AUTOTUNE") == "1"
    b = GradientBucketer([arena], world_size=world, cap_mb=1.0, reduction=reduction,
                         compression=torch.bfloat16 if compress else None, autotune=autotune,
                         autotune_log=f"{out}.autotune.csv" if autotune else None)
    caps = []
    windows = int(os.environ.get("DET_TEST_WINDOWS", "1"))
    b.graph_path = os.environ.get("DET_TEST_GRAPH_PATH") == "1"  # the reduction a hipGraph capture records
    b.launch_log = []
    for _ in range(windows):
        arena.flat_grad.copy_(full.to(dtype))
        b.prepare_backward(True)
        # buckets complete in reverse arena order here (the sink/hooks would announce them as
        # backward produces them); the bucketer must still launch them in bucket order
        for bi in reversed(range(len(b.buckets))):
            b._group_ready(bi)
        b.synchronize()
        caps.append(b.cap_bytes)
    torch.save({"reduced": arena.flat_grad.clone(), "modes": [x.mode for x in b.buckets],
                "nbuckets": len(b.buckets), "auto_choice": b.auto_choice, "downgraded": b.downgraded,
                "caps": caps, "tuned": None if b._tuner is None else b._tuner.result,
                "launch_log": b.launch_log}, f"{out}.{rank}.pt")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
