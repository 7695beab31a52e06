"""Numerics of the hand-written gfx950 kernels against plain fp32 PyTorch references."""
import copy

import pytest
import torch

from determined_1_amd.ops import functional as F
from determined_1_amd.ops.optim import FusedOptimizer

pytestmark = pytest.mark.gpu

OPTS = [
    (torch.optim.SGD, dict(lr=0.1)),
    (torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-2)),
    (torch.optim.SGD, dict(lr=0.1, momentum=0.9, nesterov=True)),
    (torch.optim.Adam, dict(lr=1e-2, weight_decay=1e-2)),
    (torch.optim.Adam, dict(lr=1e-2, amsgrad=True)),
    (torch.optim.AdamW, dict(lr=1e-2, weight_decay=1e-1)),
    (torch.optim.RMSprop, dict(lr=1e-2, momentum=0.9, centered=True, weight_decay=1e-3)),
    (torch.optim.Adagrad, dict(lr=1e-1, lr_decay=0.01, initial_accumulator_value=0.1)),
    (torch.optim.Adadelta, dict(lr=1.0, weight_decay=1e-3)),
]


def _model():
    torch.manual_seed(0)
    # odd sizes exercise the vector body + scalar tail of the kernels
    return torch.nn.Sequential(torch.nn.Linear(37, 129), torch.nn.ReLU(), torch.nn.Linear(129, 11))


@pytest.mark.parametrize("cls,kw", OPTS)
def test_fused_optimizer_matches_torch(gpu, cls, kw):
    ref = _model()
    dut = copy.deepcopy(ref).to(gpu)
    o_ref = cls(ref.parameters(), **kw)
    o_dut = cls(dut.parameters(), **kw)
    fused = FusedOptimizer(o_dut, gpu)
    fused.grad_scale = 0.5
    g = torch.Generator().manual_seed(1)
    for _ in range(4):
        # identical gradients on both sides isolate the optimizer kernel's numerics
        o_ref.zero_grad()
        o_dut.zero_grad()
        for pr, pd in zip(ref.parameters(), dut.parameters()):
            gr = torch.randn(pr.shape, generator=g)
            pr.grad = gr * 0.5
            pd.grad.copy_(gr.to(gpu))
        o_ref.step()
        o_dut.step()
    for a, b in zip(ref.parameters(), dut.parameters()):
        torch.testing.assert_close(b.detach().cpu(), a.detach(), rtol=2e-5, atol=2e-6)
    # state dict layout identical to stock torch
    s_ref, s_dut = o_ref.state_dict()["state"], o_dut.state_dict()["state"]
    for k in s_ref:
        assert set(s_ref[k].keys()) == set(s_dut[k].keys())


def test_bf16_params_fp32_master(gpu):
    torch.manual_seed(0)
    ref = torch.nn.Linear(64, 33)
    dut = copy.deepcopy(ref).to(gpu).to(torch.bfloat16)
    with torch.no_grad():  # the fp32 master starts from the bf16 model weights
        for p in ref.parameters():
            p.copy_(p.bfloat16().float())
    o_ref = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    o_dut = torch.optim.SGD(dut.parameters(), lr=0.05, momentum=0.9)
    fused = FusedOptimizer(o_dut, gpu)
    assert fused.arenas[0].has_master
    for _ in range(3):
        x = torch.randn(8, 64)
        o_ref.zero_grad()
        ref(x).sum().backward()
        # feed the reference the same (bf16-rounded) gradient the device sees
        for p in ref.parameters():
            p.grad = p.grad.bfloat16().float()
        o_ref.step()
        o_dut.zero_grad()
        for pr, pd in zip(ref.parameters(), dut.parameters()):
            pd.grad.copy_(pr.grad.to(gpu, torch.bfloat16))
        o_dut.step()
    a = fused.arenas[0]
    for i, p in enumerate(a.params):
        pr = dict(ref.named_parameters())["weight" if p.dim() == 2 else "bias"]
        torch.testing.assert_close(a.view(a.master, i).cpu(), pr.detach(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(p.detach().float().cpu(), pr.detach().bfloat16().float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("n", [1, 7, 4096, 1000003])
@pytest.mark.parametrize("src_dt,dst_dt", [(torch.float32, torch.bfloat16), (torch.bfloat16, torch.float32),
                                           (torch.float32, torch.float16), (torch.float32, torch.float32)])
def test_scale_cast(gpu, n, src_dt, dst_dt):
    x = torch.randn(n, device=gpu).to(src_dt)
    y = torch.empty(n, device=gpu, dtype=dst_dt)
    F.scale_cast_(x, y, 0.25)
    torch.testing.assert_close(y.float().cpu(), (x.float().cpu() * 0.25).to(dst_dt).float())


@pytest.mark.parametrize("sizes", [[5], [1000003, 17, 4096 * 33]])
def test_global_norm_and_clip(gpu, sizes):
    segs = [torch.randn(s, device=gpu) for s in sizes]
    ws = F.NormWorkspace(segs)
    F.global_norm_(ws, pre_scale=0.5, max_norm=1.0)
    ref = torch.sqrt(sum((s.double().cpu() ** 2).sum() for s in segs)) * 0.5
    torch.testing.assert_close(ws.norm.cpu().double()[0], ref, rtol=1e-5, atol=0)
    torch.testing.assert_close(ws.clip_coef.cpu()[0], torch.tensor(min(1.0, 1.0 / (ref.item() + 1e-6))).float())
    assert int(ws.found_inf.item()) == 0
    segs[-1][3] = float("inf")
    F.global_norm_(ws)
    assert int(ws.found_inf.item()) == 1


def test_unscale_check(gpu):
    x = torch.randn(10007, device=gpu)
    ref = x.cpu() * 0.125
    flag = torch.zeros(1, dtype=torch.int32, device=gpu)
    F.unscale_check_(x, 0.125, flag)
    torch.testing.assert_close(x.cpu(), ref)
    assert flag.item() == 0
    x[77] = float("nan")
    F.unscale_check_(x, 1.0, flag)
    assert flag.item() == 1


def test_multi_tensor_copy(gpu):
    ts = [torch.randn(n, device=gpu) for n in (3, 4096, 1, 70001)]
    mt = F.MultiTensorCopy(ts, flat_dtype=torch.bfloat16)
    flat = mt.pack(2.0)
    ref = torch.cat([t.cpu() * 2.0 for t in ts]).bfloat16()
    torch.testing.assert_close(flat.cpu(), ref)
    for t in ts:
        t.zero_()
    mt.unpack(0.5)
    torch.testing.assert_close(torch.cat([t.cpu() for t in ts]), ref.float() * 0.5)


@pytest.mark.parametrize("out_dt", [torch.bfloat16, torch.float32])
def test_u8_normalize(gpu, out_dt):
    img = torch.randint(0, 256, (3, 17, 19, 3), dtype=torch.uint8)
    mean, std = (120.0, 110.0, 100.0), (50.0, 60.0, 70.0)
    ref = F.u8_normalize(img, mean, std, out_dtype=torch.float32)
    got = F.u8_normalize(img.to(gpu), mean, std, out_dtype=out_dt)
    assert got.is_contiguous(memory_format=torch.channels_last)
    tol = dict(rtol=1e-2, atol=1e-2) if out_dt == torch.bfloat16 else dict(rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(got.float().cpu(), ref, **tol)


@pytest.mark.parametrize("rows,n", [(1, 4096), (8, 1_000_003), (3, 6), (8, 2 ** 20)])
@pytest.mark.parametrize("src_dt,dst_dt", [(torch.bfloat16, torch.bfloat16), (torch.float16, torch.float16),
                                           (torch.bfloat16, torch.float32), (torch.float32, torch.float32)])
def test_sum_rows_fp32_accumulation(gpu, rows, n, src_dt, dst_dt):
    """det_sum_rows vs the fp32 reference: one rounding of the fp32 sum of the rows."""
    x = (torch.randn(rows * n, device=gpu) * 3).to(src_dt)
    y = torch.empty(n, device=gpu, dtype=dst_dt)
    F.sum_rows_(x, rows, y, scale=0.5)
    ref = (x.float().cpu().view(rows, n).sum(0) * 0.5).to(dst_dt)
    torch.testing.assert_close(y.cpu(), ref, rtol=1e-6 if dst_dt == torch.float32 else 0, atol=1e-5 if dst_dt == torch.float32 else 0)
