"""Does a captured bf16 Linear + cross-entropy backward replay correctly on new inputs?  Plain
torch, no framework code: for each batch size, capture one step on batch A, replay on batch B and
compare every gradient with the eager step on B.  Also the bare bias-grad reduction (sum over rows)
and the bf16 row-sum variants torch can pick.   python scripts/dbg/linear_graph_repro.py"""
import json

import torch
import torch.nn as nn


def rel(a: torch.Tensor, b: torch.Tensor) -> float:
    return float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12))


def linear_case(bs: int, fin: int = 2048, fout: int = 1000, mode: str = "global", replays: int = 3) -> dict:
    torch.manual_seed(0)
    dev = torch.device("cuda")
    fc = nn.Linear(fin, fout).to(dev, torch.bfloat16)
    lossf = nn.CrossEntropyLoss()
    xa = torch.randn(bs, fin, device=dev, dtype=torch.bfloat16)
    ya = torch.randint(0, fout, (bs,), device=dev)
    batches = [(torch.randn(bs, fin, device=dev, dtype=torch.bfloat16), torch.randint(0, fout, (bs,), device=dev))
               for _ in range(replays)]

    def step(x, y):
        fc.weight.grad = None
        fc.bias.grad = None
        xx = x.detach().requires_grad_(True)
        loss = lossf(fc(xx).float(), y)
        loss.backward()
        return loss.detach(), xx.grad, fc.weight.grad, fc.bias.grad

    # eager references
    refs = [[t.clone() for t in step(x, y)] for x, y in batches]
    # warm up on a side stream as torch's docs do, then capture on A
    sx, sy = xa.clone(), ya.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step(sx, sy)
    torch.cuda.current_stream().wait_stream(s)
    fc.weight.grad = None
    fc.bias.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode=mode):
        out = step(sx, sy)
    names = ("loss", "dx", "dw", "db")
    res = {"bs": bs, "mode": mode}
    for k, ((x, y), ref) in enumerate(zip(batches, refs)):
        sx.copy_(x)
        sy.copy_(y)
        g.replay()
        torch.cuda.synchronize()
        res[f"replay{k}"] = {n: rel(o, r) for n, o, r in zip(names, out, ref)}
    return res


def rowsum_case(bs: int, n: int = 1000, replays: int = 3) -> dict:
    dev = torch.device("cuda")
    a = torch.randn(bs, n, device=dev, dtype=torch.bfloat16)
    bs_ = [torch.randn(bs, n, device=dev, dtype=torch.bfloat16) for _ in range(replays)]
    st = a.clone()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        st.sum(0)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        out = st.sum(0)
    res = {"bs": bs}
    for k, b in enumerate(bs_):
        st.copy_(b)
        g.replay()
        torch.cuda.synchronize()
        res[f"rowsum_rel{k}"] = rel(out, b.sum(0))
    return res


def main() -> None:
    res = []
    for bs in (128, 256, 512, 1024):
        for mode in ("global", "thread_local"):
            res.append(linear_case(bs, mode=mode))
            print(json.dumps(res[-1]), flush=True)
        res.append(rowsum_case(bs))
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
