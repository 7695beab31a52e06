"""Which aten op of a bf16 Linear backward replays stale from a hipGraph?  (linear_graph_repro.py:
the bias gradient is right on the first replay and wrong from the second on at batch >= 512.)
Logs the backward's aten ops, then replays each candidate op alone, 3 times on new inputs.
    python scripts/dbg/linear_graph_ops.py"""
import json

import torch
import torch.nn as nn
from torch.utils._python_dispatch import TorchDispatchMode


class _Log(TorchDispatchMode):
    def __init__(self) -> None:
        super().__init__()
        self.ops = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):  # noqa: ANN001
        desc = []
        for a in args:
            if isinstance(a, torch.Tensor):
                desc.append(f"T{tuple(a.shape)}:{str(a.dtype)[6:]}:{tuple(a.stride())}")
            else:
                desc.append(repr(a)[:40])
        self.ops.append(f"{func.name()}({', '.join(desc)}) {kwargs or ''}")
        return func(*args, **(kwargs or {}))


def trace(bs: int) -> list:
    dev = torch.device("cuda")
    fc = nn.Linear(2048, 1000).to(dev, torch.bfloat16)
    x = torch.randn(bs, 2048, device=dev, dtype=torch.bfloat16, requires_grad=True)
    y = torch.randint(0, 1000, (bs,), device=dev)
    loss = nn.functional.cross_entropy(fc(x).float(), y)
    log = _Log()
    with log:
        loss.backward()
    return log.ops


def replay_op(name: str, fn, make, replays: int = 3) -> dict:
    """fn(static inputs) captured once, replayed on `replays` fresh inputs vs eager."""
    torch.manual_seed(0)
    static = make()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(*static)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn(*static)
    res = {"op": name}
    for k in range(replays):
        new = make()
        ref = fn(*new).clone()
        for dst, src in zip(static, new):
            dst.copy_(src)
        g.replay()
        torch.cuda.synchronize()
        res[f"r{k}"] = float((out.float() - ref.float()).abs().max() / (ref.float().abs().max() + 1e-12))
    return res


def main() -> None:
    for bs in (256, 512):
        print(json.dumps({"bs": bs, "backward_ops": trace(bs)}), flush=True)
    dev = torch.device("cuda")
    bs = 512

    def mk_g():
        return [torch.randn(bs, 1000, device=dev, dtype=torch.bfloat16)]

    def mk_gx():
        return [torch.randn(bs, 1000, device=dev, dtype=torch.bfloat16),
                torch.randn(bs, 2048, device=dev, dtype=torch.bfloat16)]

    cases = [
        ("sum0", lambda g: g.sum(0), mk_g),
        ("sum0_keepdim", lambda g: g.sum(0, keepdim=True), mk_g),
        ("sum0_fp32acc", lambda g: g.sum(0, dtype=torch.float32), mk_g),
        ("mm_dw", lambda g, x: g.t().mm(x), mk_gx),
        ("mm_dw_then_sum", lambda g, x: g.t().mm(x).sum() + g.sum(0).float().sum(), mk_gx),
        ("dw_and_db", lambda g, x: torch.cat([g.t().mm(x)[:, :1].flatten(), g.sum(0)]), mk_gx),
    ]
    for name, fn, make in cases:
        print(json.dumps(replay_op(name, fn, make)), flush=True)


if __name__ == "__main__":
    main()
