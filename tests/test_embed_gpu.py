"""BERT embedding lookup-and-sum (ops/csrc/det_embed.hip) against torch's three nn.Embedding lookups,
and its backward under hipGraph replays with batches whose distinct-id count differs from the
captured one (torch's own backward sizes its launches from the captured batch's count and ran out
of bounds in the BERT graph replays, round-5 sessions 13/14)."""
import pytest
import torch
import torch.nn.functional as F

from determined_1_amd.ops import transformer as tf

pytestmark = pytest.mark.gpu


def _ref(ids, tt, w, t, p, pad):
    S = ids.shape[1]
    pos = torch.arange(S, device=ids.device)
    return F.embedding(ids, w, pad) + F.embedding(tt, t) + F.embedding(pos, p)


def _tables(gpu, dtype, V=1000, H=64, P=40, integer=False, seed=0):
    g = torch.Generator().manual_seed(seed)
    mk = (lambda *s: torch.randint(-3, 4, s, generator=g).float()) if integer else (lambda *s: torch.randn(*s, generator=g))
    return [mk(*s).to(gpu).to(dtype).requires_grad_(True) for s in ((V, H), (2, H), (P, H))]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_forward_and_backward_match_torch(gpu, dtype):
    B, S = 6, 32
    integer = dtype == torch.float32  # fp32: integer values, every sum exact in any order
    w, t, p = _tables(gpu, dtype, integer=integer)
    w2, t2, p2 = [x.detach().clone().requires_grad_(True) for x in (w, t, p)]
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, 40, (B, S), generator=g).to(gpu)  # few distinct ids: long runs
    ids[0, :5] = 0  # padding rows get no gradient
    tt = torch.randint(0, 2, (B, S), generator=g).to(gpu)
    out = tf.bert_embeddings(ids, tt, w, t, p, 0)
    ref = _ref(ids, tt, w2, t2, p2, 0)
    assert torch.equal(out, ref)
    dy = (torch.randint(-2, 3, (B, S, w.shape[1]), generator=g).float() if integer
          else torch.randn(B, S, w.shape[1], generator=g)).to(gpu).to(dtype)
    out.backward(dy)
    if integer:
        ref.backward(dy)
        for a, b in ((w, w2), (t, t2), (p, p2)):
            assert torch.equal(a.grad, b.grad)
        return
    # bf16: each gradient row is summed in fp32 and rounded once, so it must equal the fp32 sum of
    # the same bf16 gradient rows to bf16 rounding (torch's bf16 backward accumulates with more
    # rounding; it is not the reference here)
    w3, t3, p3 = [x.detach().float().requires_grad_(True) for x in (w, t, p)]
    _ref(ids, tt, w3, t3, p3, 0).backward(dy.float())
    for a, b in ((w, w3), (t, t3), (p, p3)):
        torch.testing.assert_close(a.grad.float(), b.grad, rtol=8e-3, atol=1e-6)


def test_backward_replays_with_varying_distinct_ids(gpu):
    """Captured forward + backward (gradients accumulated into pinned .grad buffers, as the trial's
    arena does), replayed on batches from 3 to 4000+ distinct ids: every replay equals the eager
    computation of the same batch."""
    B, S, V = 12, 384, 30522
    w, t, p = _tables(gpu, torch.float32, V=V, H=64, P=512, integer=True)
    for x in (w, t, p):
        x.grad = torch.zeros_like(x)
    ids = torch.zeros(B, S, dtype=torch.long, device=gpu)
    tt = torch.zeros(B, S, dtype=torch.long, device=gpu)
    dy = torch.ones(B, S, 64, device=gpu)

    def step():
        tf.bert_embeddings(ids, tt, w, t, p, 0).backward(dy)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    ids.fill_(5)  # captured with ONE distinct id
    with torch.cuda.graph(graph):
        step()
    gen = torch.Generator().manual_seed(3)
    for hi in (3, 50, 4000, V, 7):
        ids.copy_(torch.randint(0, hi, (B, S), generator=gen).to(gpu))
        tt.copy_(torch.randint(0, 2, (B, S), generator=gen).to(gpu))
        for x in (w, t, p):
            x.grad.zero_()
        graph.replay()
        torch.cuda.synchronize()
        got = [x.grad.clone() for x in (w, t, p)]
        w2, t2, p2 = [x.detach().clone().requires_grad_(True) for x in (w, t, p)]
        _ref(ids, tt, w2, t2, p2, 0).backward(dy)
        for a, b in zip(got, (w2.grad, t2.grad, p2.grad)):
            assert torch.equal(a, b), hi


def test_graph_probe_keeps_torch_sort_path_embedding_eager(gpu):
    """The warm-up probe of pytorch/_graph.py flags torch's own embedding backward once it takes the
    host-sized sort path (> 3072 indices), and passes the short-index form."""
    from determined_1_amd.pytorch._graph import library_conv_reason

    emb = torch.nn.Embedding(100, 8).to(gpu)
    for n, hit in ((4000, True), (1000, False)):
        ids = torch.randint(0, 100, (n,), device=gpu)

        def step():
            emb(ids).sum().backward()

        _, reason = library_conv_reason(step)
        assert (reason is not None) == hit, (n, reason)
        if hit:
            assert "embedding" in reason
