"""CPU checks of ops/transformer.py dispatch logic (the GPU numerics are in test_transformer_gpu.py)."""
import torch

from determined_1_amd.ops import transformer as T


def _fake_bl_gemm(ta, tb, m, n, k, A, lda, B, ldb, D, ldd, bias=None, beta=0.0):
    """Column-major D[m, n] = A[m, k] B[k, n] (+ beta D): row-major D^T[n, m] = B^T[n, k] A^T[k, m]."""
    assert ta == 0 and tb == 0 and bias is None
    a_rm = A.reshape(-1)[:k * m].view(k, m).float()
    b_rm = B.reshape(-1)[:n * k].view(n, k).float()
    d_rm = D.view(n, m)
    d_rm.copy_(beta * d_rm.float() + b_rm @ a_rm)


def test_linked_residual_grad_kept_on_library_branch(monkeypatch):
    """a parked residual gradient that the beta = 1 branch cannot take (here: a
    non-contiguous view) is still summed into dx on the plain library-GEMM branch."""
    monkeypatch.setattr(T, "_bl_ok", lambda *ts: True)
    monkeypatch.setattr(T, "_bl_gemm", _fake_bl_gemm)
    torch.manual_seed(0)
    M, N, K = 8, 6, 4
    dz, x2, w = torch.randn(M, N), torch.randn(M, K), torch.randn(N, K)
    dr = torch.randn(K, M).t()  # [M, K], not contiguous: skips the beta = 1 branch
    assert not dr.is_contiguous()
    dx, dw, _ = T._mm_backward(dz, x2, w, True, False, None, dr)
    torch.testing.assert_close(dx, dz @ w + dr)
    assert dw is None


def test_notify_direct_grads_runs_post_accumulate_hooks():
    """gradients written in place under capture fire the post-accumulate hooks (the DP
    bucketer's per-parameter counter, user hooks) that AccumulateGrad would have run."""
    from determined_1_amd.ops.arena import notify_direct_grads

    p = torch.nn.Parameter(torch.zeros(3))
    q = torch.nn.Parameter(torch.zeros(2))
    seen = []
    p.register_post_accumulate_grad_hook(lambda t: seen.append(("p", t is p)))
    notify_direct_grads([p, q])
    assert seen == [("p", True)]
