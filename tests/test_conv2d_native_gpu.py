"""The detection backbones' convolutions on the hand-written kernels (ops.conv.conv2d_native,
VERDICT r5 item 7): every ResNet-50 / FPN conv kind at batch 2 and non-square detection-sized
inputs, forward and both gradients, against a plain fp32 PyTorch conv of the same op.  Integer-valued
operands keep every product and fp32 sum exact, so the only rounding is the bf16 store of an output,
and the kernels must match the reference rounded to bf16 bit for bit."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ints(shape, lo, hi, g, dev, cl=False):
    t = torch.randint(lo, hi + 1, shape, generator=g).float().to(dev)
    return t.contiguous(memory_format=torch.channels_last) if cl else t


CASES = [  # (cin, cout, k, stride, pad, h, w)
    (64, 128, 1, 1, 0, 13, 17),    # lateral / conv1 / conv3 1x1
    (256, 512, 1, 2, 0, 14, 10),   # stride-2 projection shortcut
    (128, 128, 3, 1, 1, 15, 11),   # 3x3 stride 1 (and the FPN output convs)
    (256, 256, 3, 2, 1, 13, 9),    # 3x3 stride 2 (layer2-4 first block, RetinaNet P6/P7)
    (3, 64, 7, 2, 3, 37, 53),      # stem
]


@pytest.mark.parametrize("cin,cout,k,stride,pad,h,w", CASES)
def test_conv2d_native_matches_fp32_reference(gpu, cin, cout, k, stride, pad, h, w):
    from determined_1_amd.ops import conv

    g = torch.Generator().manual_seed(cin * 7 + k)
    x = _ints((2, cin, h, w), -2, 2, g, gpu, cl=True)
    wt = _ints((cout, cin, k, k), -2, 2, g, gpu).contiguous(memory_format=torch.channels_last)
    xb = x.to(torch.bfloat16).requires_grad_(k != 7)
    wp = wt.clone().requires_grad_(True)  # fp32 parameter: gradient summed in fp32
    before = dict(conv.CONV2D_COUNTS)
    y = conv.conv2d_native(xb, wp, stride, pad)
    assert y is not None and conv.CONV2D_COUNTS["native"] == before["native"] + 1
    xr = x.clone().requires_grad_(k != 7)
    wr = wt.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, stride, pad)
    assert y.shape == yr.shape and y.dtype == torch.bfloat16
    torch.testing.assert_close(y.float(), yr.to(torch.bfloat16).float(), rtol=0, atol=0)
    dy = _ints(tuple(yr.shape), -1, 1, g, gpu, cl=True)
    y.backward(dy.to(torch.bfloat16))
    yr.backward(dy)
    torch.testing.assert_close(wp.grad, wr.grad, rtol=0, atol=0)
    if k != 7:
        torch.testing.assert_close(xb.grad.float(), xr.grad.to(torch.bfloat16).float(), rtol=0, atol=0)


def test_conv2d_native_declines_uncovered_shapes(gpu):
    from determined_1_amd.ops import conv

    x = torch.randn(2, 256, 8, 8, device=gpu, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert conv.conv2d_native(x, torch.randn(12, 256, 1, 1, device=gpu), 1, 0) is None  # RPN box head
    assert conv.conv2d_native(x.contiguous(), torch.randn(256, 256, 3, 3, device=gpu), 1, 1) is None  # NCHW
    assert conv.conv2d_native(x.float(), torch.randn(256, 256, 3, 3, device=gpu), 1, 1) is None  # fp32, no autocast


def test_faster_rcnn_backbone_and_fpn_run_native(gpu):
    """A bf16 Faster R-CNN training step: every backbone / FPN / RPN conv of 64-multiple channels
    runs natively (only the 1x1 RPN heads stay on the library), and the losses match the all-library
    run of the same weights and images."""
    from determined_1_amd.models.faster_rcnn import FasterRCNN
    from determined_1_amd.ops import conv

    torch.manual_seed(0)
    model = FasterRCNN(num_classes=3, min_size=256, max_size=320).to(gpu).to(torch.bfloat16)
    model.train()
    g = torch.Generator().manual_seed(1)
    imgs = [torch.rand(3, 240, 300, generator=g).to(gpu).to(torch.bfloat16) for _ in range(2)]
    tgts = [{"boxes": torch.tensor([[20.0, 30.0, 120.0, 160.0]], device=gpu),
             "labels": torch.tensor([1], device=gpu)} for _ in range(2)]
    losses = {}
    for native in (True, False):
        conv.NATIVE_CONV2D = native
        try:
            c0 = dict(conv.CONV2D_COUNTS)
            torch.manual_seed(5)
            out = model(imgs, tgts)
            loss = sum(v.float() for v in out.values())
            loss.backward()
            losses[native] = {k: float(v) for k, v in out.items()}
            if native:
                n = conv.CONV2D_COUNTS["native"] - c0["native"]
                assert n >= 53 + 8, conv.CONV2D_COUNTS  # 53 backbone convs + 4 lateral + 4 output FPN convs
        finally:
            conv.NATIVE_CONV2D = True
        model.zero_grad(set_to_none=True)
    for k in losses[True]:
        a, b = losses[True][k], losses[False][k]
        assert abs(a - b) <= 0.05 * max(1.0, abs(b)), (k, a, b)
