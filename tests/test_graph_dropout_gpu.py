"""torch's own dropout under the trial's hipGraph capture (pytorch/_graph.py): every replay must draw
a fresh mask (the default generator's Philox offset advances per replay), for the element-wise
(``nn.Dropout``) and channel (``nn.Dropout2d``) forms, in bf16 and fp32, with the graph captured in
a shared private pool after eager warm-up steps -- the CIFAR trial's layers (reference
examples/computer_vision/cifar10_pytorch/model_def.py:64-78)."""
import pytest
import torch
import torch.nn as nn


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("layer", ["dropout", "dropout2d"])
def test_graph_replays_draw_fresh_torch_dropout_masks(gpu, dtype, layer):
    torch.manual_seed(0)
    mod = nn.Dropout(0.5) if layer == "dropout" else nn.Dropout2d(0.5)
    x = torch.ones(32, 64, 8, 8, device=gpu, dtype=dtype).to(memory_format=torch.channels_last)
    for _ in range(2):  # eager warm-up, as the trial does before capturing
        mod(x)
    pool = torch.cuda.graph_pool_handle()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, pool=pool):
            y = mod(x)
    torch.cuda.current_stream().wait_stream(s)
    outs = []
    for _ in range(4):
        g.replay()
        outs.append(y.clone())
        mod(x)  # an eager step between replays (tail batches run eagerly)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.isfinite(o.float()).all()
        kept = (o != 0).float().mean().item()
        assert 0.35 < kept < 0.65
        assert torch.all((o == 0) | (o.float() == 2.0))
    for i in range(len(outs)):
        for j in range(i):
            assert not torch.equal(outs[i], outs[j]), f"replays {j} and {i} drew the same mask"


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_two_dropout_layers_per_step_and_eager_steps_draw_distinct_masks(gpu, dtype):
    """Two dropout layers in ONE captured step (module and functional form) and eager steps between
    replays: every mask drawn -- per layer, per replay, per eager step -- is distinct, i.e. no two
    draws share a Philox offset."""
    torch.manual_seed(1)
    mod = nn.Dropout(0.5)
    x = torch.ones(16, 4096, device=gpu, dtype=dtype)

    def step():
        return mod(x), nn.functional.dropout(x, 0.5, training=True)

    for _ in range(2):
        step()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            ya, yb = step()
    torch.cuda.current_stream().wait_stream(s)
    masks = []
    for _ in range(3):
        g.replay()
        masks += [ya.clone(), yb.clone()]
        masks += [m.clone() for m in step()]
    torch.cuda.synchronize()
    for m in masks:
        kept = (m != 0).float().mean().item()
        assert 0.45 < kept < 0.55
    for i in range(len(masks)):
        for j in range(i):
            assert not torch.equal(masks[i], masks[j]), f"draws {j} and {i} share a mask"
