"""Which SDPA backend runs for the BERT shapes on ROCm, and what layouts its outputs/grads have."""
import torch
import torch.nn.functional as F

B, S, nh, hd = 12, 384, 12, 64
H = nh * hd
dev = "cuda"
qkv = torch.randn(B, S, 3 * H, device=dev, dtype=torch.bfloat16, requires_grad=True)
q, k, v = qkv.view(B, S, 3, nh, hd).permute(2, 0, 3, 1, 4).unbind(0)
print("q strides", q.stride())
mask = torch.zeros(B, 1, 1, S, device=dev, dtype=torch.bfloat16)
for name, m in (("mask", mask), ("nomask", None)):
    out = F.scaled_dot_product_attention(q, k, v, attn_mask=m, dropout_p=0.1)
    print(name, "out", out.shape, out.stride(), "grad_fn", type(out.grad_fn).__name__)
    out.sum().backward()
    print(name, "qkv.grad", qkv.grad.stride())
    qkv.grad = None
try:
    r = torch.ops.aten._scaled_dot_product_efficient_attention(q, k, v, mask.expand(B, nh, S, S), True, 0.1, False)
    print("eff fwd ok", [t.shape for t in r], r[0].stride(), r[1].dtype, r[2], r[3])
    g = torch.ops.aten._scaled_dot_product_efficient_attention_backward(
        torch.ones_like(r[0]), q, k, v, mask.expand(B, nh, S, S), r[0], r[1], r[2], r[3], 0.1, [True, True, True, False], False)
    print("eff bwd ok", [None if t is None else (t.shape, t.stride()) for t in g])
except Exception as e:
    print("eff ops failed", repr(e)[:300])
try:
    r = torch.ops.aten._scaled_dot_product_flash_attention(q, k, v, 0.1, False, True)
    print("flash fwd ok", len(r), r[0].stride())
except Exception as e:
    print("flash failed", repr(e)[:300])
for be in ("flash", "efficient", "math"):
    print("backend enabled", be, getattr(torch.backends.cuda, f"{be}_sdp_enabled")())
