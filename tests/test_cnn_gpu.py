"""Numerics of the native CIFAR-10 CNN (ops/cnn.py, csrc/det_cnn.hip) against the fp32 PyTorch
reference of the same network (models.CIFAR10CNN's torch layers).

fp32 (O0): exact-integer tests.  Integer inputs and sparse {-1, 0, 1} weights keep every partial sum
an integer below 2^24, where fp32 arithmetic is exact in any summation order and the exact-fp32
MFMA (v_mfma_f32_16x16x4_f32) must reproduce the reference bit for bit: logits, every weight and
bias gradient, through ReLU, max-pool (argmax routing) and both dropout forms (with the kernel's own
masks applied to the reference).  bf16 (O2): the same network within bf16 rounding tolerance.
"""
import os

import pytest
import torch

from determined_1_amd.models import CIFAR10CNN

pytestmark = pytest.mark.gpu


def _int_model(dev, dtype=torch.float32, seed=0, density=0.12, ps=(0.0, 0.0, 0.0)):
    g = torch.Generator().manual_seed(seed)
    m = CIFAR10CNN(*ps)
    with torch.no_grad():
        for p in m.parameters():
            keep = torch.rand(p.shape, generator=g) < density
            p.copy_(torch.randint(-1, 2, p.shape, generator=g).float() * keep)
    return m.to(dev).to(memory_format=torch.channels_last).to(dtype)


def _int_input(dev, n, dtype=torch.float32, seed=1):
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(-3, 4, (n, 3, 32, 32), generator=g).float()
    return x.to(dev).to(dtype).contiguous(memory_format=torch.channels_last)


def _reference(model, x, masks=None):
    """fp32 torch forward of the module's layers, dropout replaced by the given factor tensors."""
    net = model.net
    h = x.float()
    for i, layer in enumerate(net):
        if isinstance(layer, torch.nn.modules.dropout._DropoutNd):
            if masks is None or not model.training:
                continue
            m = masks[{5: 0, 11: 1, 15: 2}[i]]
            if m is None:
                continue
            h = h * (m.view(h.shape[0], -1, 1, 1) if h.dim() == 4 else m.view(h.shape[0], -1))
            continue
        if isinstance(layer, (torch.nn.Conv2d, torch.nn.Linear)):
            w, b = layer.weight.float(), layer.bias.float()
            h = torch.nn.functional.conv2d(h, w, b, padding=layer.padding) if isinstance(layer, torch.nn.Conv2d) \
                else torch.nn.functional.linear(h, w, b)
            continue
        h = layer(h)
    return h


def _grads(model):
    return [p.grad.detach().float().clone() for p in model.parameters()]


@pytest.mark.parametrize("n", [32, 16, 7])
@pytest.mark.parametrize("train", [False, True])
def test_fp32_forward_backward_exact(gpu, n, train):
    from determined_1_amd.ops import cnn

    # 1/(1-p) = 2 and 4: the dropout scale keeps every product an integer, so exactness holds
    ps = (0.5, 0.5, 0.75) if train else (0.0, 0.0, 0.0)
    model = _int_model(gpu, ps=ps)
    model.train(train)
    x = _int_input(gpu, n)
    cnn.DEBUG["keep_masks"] = True
    try:
        out = model(x)  # native path
        masks = cnn.DEBUG["masks"]
    finally:
        cnn.DEBUG["keep_masks"] = False
    assert out.dtype == torch.float32 and out.shape == (n, 10)
    if train:
        for m, p, cols in zip(masks, ps, (32, 64, 512)):
            assert m is not None and m.numel() == n * cols
            vals = set(torch.unique(m).tolist())
            assert vals <= {0.0, float(torch.tensor(1.0 / (1.0 - p), dtype=torch.float32))}
    ref_model = _int_model(gpu, ps=ps)
    ref_model.load_state_dict(model.state_dict())
    ref_model.train(train)
    ref = _reference(ref_model, x, masks)
    assert ref.abs().max() < 2 ** 24
    assert torch.equal(out, ref), (out - ref).abs().max()
    g = torch.Generator().manual_seed(5)
    dl = torch.randint(-2, 3, (n, 10), generator=g).float().to(gpu)
    out.backward(dl)
    ref.backward(dl)
    for (name, p), q in zip(model.named_parameters(), ref_model.parameters()):
        assert p.grad is not None, name
        assert q.grad.abs().max() < 2 ** 24
        assert torch.equal(p.grad.float(), q.grad.float()), (name, (p.grad.float() - q.grad.float()).abs().max())


def test_bf16_close_to_fp32_reference(gpu, monkeypatch):
    """bf16 (O2) storage: the native network's error against fp32 stays within that of torch's own
    bf16 layers on the same weights and input (both round activations and gradients to bf16)."""
    torch.manual_seed(0)
    model = CIFAR10CNN(0.0, 0.0, 0.0).to(gpu).to(memory_format=torch.channels_last).to(torch.bfloat16)
    ref_model = CIFAR10CNN(0.0, 0.0, 0.0).to(gpu).to(memory_format=torch.channels_last)
    ref_model.load_state_dict({k: v.float() for k, v in model.state_dict().items()})
    torch_bf16 = CIFAR10CNN(0.0, 0.0, 0.0).to(gpu).to(memory_format=torch.channels_last).to(torch.bfloat16)
    torch_bf16.load_state_dict(model.state_dict())
    torch_bf16.native = False
    x = torch.randn(32, 3, 32, 32, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dl = torch.randn(32, 10, device=gpu)
    out = model(x)
    ref = _reference(ref_model, x.float())
    tb = torch_bf16(x).float()
    err = float((out - ref).abs().max() / ref.abs().max())
    err_t = float((tb - ref).abs().max() / ref.abs().max())
    assert err < max(3e-2, 2 * err_t), (err, err_t)
    out.backward(dl)
    ref.backward(dl)
    tb.backward(dl)
    for (name, p), q, t in zip(model.named_parameters(), ref_model.parameters(), torch_bf16.parameters()):
        e = float((p.grad.float() - q.grad).norm() / q.grad.norm().clamp_min(1e-12))
        e_t = float((t.grad.float() - q.grad).norm() / q.grad.norm().clamp_min(1e-12))
        assert e < max(5e-2, 2 * e_t), (name, e, e_t)


def test_dropout_masks_fresh_per_call_and_rate(gpu):
    from determined_1_amd.ops import cnn

    model = _int_model(gpu, ps=(0.25, 0.25, 0.5))
    model.train()
    x = _int_input(gpu, 64)
    cnn.DEBUG["keep_masks"] = True
    try:
        model(x)
        a = [m.clone() for m in cnn.DEBUG["masks"]]
        model(x)
        b = cnn.DEBUG["masks"]
    finally:
        cnn.DEBUG["keep_masks"] = False
    for ma, mb, p in zip(a, b, (0.25, 0.25, 0.5)):
        assert not torch.equal(ma, mb)
        rate = float((ma == 0).float().mean())
        assert abs(rate - p) < 0.06, rate


def test_cross_entropy_matches_torch(gpu):
    from determined_1_amd.ops.cnn import cross_entropy

    torch.manual_seed(3)
    z = torch.randn(48, 10, device=gpu, requires_grad=True)
    y = torch.randint(0, 10, (48,), device=gpu)
    loss, acc, err = cross_entropy(z, y, with_accuracy=True, with_error=True)
    z2 = z.detach().clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(z2, y)
    assert torch.allclose(loss, ref, rtol=1e-6, atol=1e-6)
    assert float(acc) == float((z.argmax(1) == y).float().mean())
    assert abs(float(err) - (1.0 - float(acc))) < 1e-6
    loss.backward()
    ref.backward()
    assert torch.allclose(z.grad, z2.grad, rtol=1e-5, atol=1e-7)


def test_cross_entropy_unit_seed_gradient_from_the_forward_launch(gpu):
    """With the shared unit seed (ops.seed_grad, what the trial context passes) the backward hands
    over the gradient the forward launch already wrote: bit-equal to the backward kernel's for a seed
    of 1 from a private tensor, and any other seed still scales through the backward kernel."""
    from determined_1_amd.ops import cnn, seed_grad
    from determined_1_amd.ops.cnn import cross_entropy

    torch.manual_seed(4)
    z0 = torch.randn(32, 10, device=gpu)
    y = torch.randint(0, 10, (32,), device=gpu)
    grads = []
    for seed in ("unit", 1.0, 2.5):
        z = z0.clone().requires_grad_(True)
        loss = cross_entropy(z, y)
        g = seed_grad.unit_for(loss) if seed == "unit" else torch.full((), seed, device=gpu)
        assert seed_grad.is_unit(g) == (seed == "unit")
        before = cnn.XENT_FROM_FORWARD["count"]
        loss.backward(g)
        assert cnn.XENT_FROM_FORWARD["count"] == before + (seed == "unit"), seed  # no backward launch for it
        grads.append(z.grad)
    assert torch.equal(grads[0], grads[1])
    torch.testing.assert_close(grads[2], 2.5 * grads[1], rtol=1e-6, atol=1e-8)


def test_graph_replays_train_the_native_cnn(gpu, monkeypatch):
    """The whole native step (masks, GEMMs, finishes, RMSprop) captured and replayed: finite, learning,
    fresh masks per replay (the device offset counter), grads landing in the arena in place."""
    import sys

    ex = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "computer_vision",
                      "cifar10_pytorch")
    from determined_1_amd import workload
    from determined_1_amd.experimental import load_model_def, make_controller

    model_def = load_model_def(ex)  # uniquely named: other examples' model_def modules may be loaded

    cfg = {"hyperparameters": {"global_batch_size": 32, "learning_rate": 1e-3, "train_records": 6400, "amp": "O2"},
           "searcher": {"name": "single", "metric": "validation_error", "max_length": {"batches": 400}},
           "records_per_epoch": 6400, "scheduling_unit": 100,
           "optimizations": {"hip_graph": True, "hip_graph_batches": 20}}
    res = []

    def stream():
        for s in range(4):
            yield workload.train_workload(s + 1, num_batches=100, total_batches_processed=100 * s), [], res.append
        yield workload.terminate_workload(), [], workload.ignore_response

    ctrl = make_controller(model_def.CIFARTrial, cfg, stream(), use_gpu=True, trial_seed=3)
    ctrl.run()
    losses = [r["metrics"]["avg_metrics"]["loss"] for r in res]
    assert all(l == l and abs(l) < 1e3 for l in losses), losses
    assert losses[-1] < losses[0], losses
    st = ctrl._graph.stats()
    assert st["disabled"] is None and st["chunk_replays"] > 0, st


def test_graph_replay_update_matches_fp32_same_mask_recompute(gpu):
    """A captured native training step (masks, forward, cross entropy, backward, SGD update) replayed
    several times: every replay draws fresh masks, and each replay's parameter update equals the fp32
    torch recomputation of that step with that replay's own masks (replay vs same-mask
    recomputation)."""
    from determined_1_amd.ops import cnn
    from determined_1_amd.ops import transformer as tf

    torch.manual_seed(11)
    model = CIFAR10CNN(0.25, 0.25, 0.5).to(gpu).to(memory_format=torch.channels_last)
    model.train()
    params = list(model.parameters())
    x = torch.randn(16, 3, 32, 32, device=gpu).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device=gpu)
    lr = 0.05

    def step():
        out = model(x)
        loss = cnn.cross_entropy(out, y)
        loss.backward()
        with torch.no_grad():
            for p in params:
                p.sub_(lr * p.grad)
                p.grad.zero_()
        return loss

    tf.rng_base(gpu)  # the device offset counter exists before the capture
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    cnn.DEBUG["keep_masks"] = True
    try:
        with torch.cuda.graph(g):
            tf.bump_rng_base()
            static_loss = step()
        masks = cnn.DEBUG["masks"]
    finally:
        cnn.DEBUG["keep_masks"] = False
    seen = []
    for _ in range(4):
        before = [p.detach().clone() for p in params]
        g.replay()
        torch.cuda.synchronize()
        assert torch.isfinite(static_loss)
        cur = [m.clone() for m in masks]
        assert not any(all(torch.equal(a, b) for a, b in zip(cur, prev)) for prev in seen)
        seen.append(cur)
        ref = _int_model(gpu, ps=(0.25, 0.25, 0.5))
        with torch.no_grad():
            for q, b in zip(ref.parameters(), before):
                q.copy_(b)
        ref.train()
        out = _reference(ref, x, cur)
        torch.nn.functional.cross_entropy(out, y).backward()
        for (name, p), q, b in zip(model.named_parameters(), ref.parameters(), before):
            expect = b - lr * q.grad
            torch.testing.assert_close(p.detach(), expect, rtol=1e-4, atol=1e-5, msg=name)
