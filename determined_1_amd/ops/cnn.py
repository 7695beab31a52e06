"""The CIFAR-10 CNN (the ASHA benchmark's trial) on ``csrc/det_cnn.hip``: forward, backward, dropout
and cross entropy as ~20 launches per training batch instead of ~130 library kernels.

    logits = cifar_cnn(x, params, (p1, p2, p3), training)      # x: [N, 3, 32, 32] channels_last
    loss, acc = cross_entropy(logits, y, with_accuracy=True)

``params`` are the 12 tensors of ``models.CIFAR10CNN`` (conv1..conv4, fc1, fc2 weight + bias) in any
memory format (weights are read through their strides).  Reference network:
``examples/computer_vision/cifar10_pytorch/model_def.py:47-65`` (Dropout2d after both pools, element
dropout on the fc1 output, RMSprop).

Gradients: in a hipGraph capture (``optimizations.hip_graph``) the weight gradients are accumulated
straight into the parameters' ``.grad`` arena views by the finishing kernels (no AccumulateGrad add
per parameter); elsewhere they are produced into ``arena.landing_buffer`` slots or fresh tensors and
returned to autograd.  CPU tensors and unsupported shapes use the torch module (``supported``).
"""
import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import torch

from determined_1_amd.ops import _lib, seed_grad
from determined_1_amd.ops import transformer as _tf

c_void_p, c_i32, c_i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64

# det_cnn.hip enums
S_ACT_CONV, S_ACT_FLAT, S_ACT_ROWS, S_GRAD_ROWS, S_GRAD_CONV_T, S_WGT_CONV, S_WGT_CONV_T, S_WGT_FC, S_WGT_FC_T = range(9)
(E_BIAS_RELU, E_BIAS_RELU_POOL, E_BIAS_RELU_DROP, E_BIAS, E_MASK_POS, E_DROP_POS, E_DROP_POS_FLAT, E_GRAD_FC,
 E_GRAD_CONV) = range(9)
# split-K sizing: at least this many workgroups per launch where K allows.  Every pass here is
# latency-bound (each K tile of a block costs a global round trip, ~2.4 us measured), so the K loop
# is cut short and spread over more blocks; the finish launch that sums the slabs costs ~5 us.
# 512: O2 batch-32 trial 0.269 ms/batch vs 0.296 (1024), 0.281 (768), 0.275 (384), r5s19.
BLOCKS_TARGET = int(os.environ.get("DET_CNN_BLOCKS", "512"))
DEBUG = {"keep_masks": False, "masks": None}  # tests: the dropout factors of the last forward
XENT_FROM_FORWARD = {"count": 0}  # cross-entropy backwards served by the forward launch (unit seed)


class Operand(ctypes.Structure):
    _fields_ = [("p", c_void_p)] + [(n, c_i32) for n in ("dt", "src", "H", "W", "C", "R", "S", "pad", "OH", "OW",
                                                           "pool", "transpose")] + \
               [("idx", c_void_p)] + [(n, c_i64) for n in ("so", "sc", "sr", "ss")]


class Job(ctypes.Structure):
    _fields_ = [("a", Operand), ("b", Operand), ("M", c_i64), ("N", c_i64), ("K", c_i64)] + \
               [(n, c_i32) for n in ("splits", "epi", "out_dt", "bias_dt", "drop_cols", "HW", "C", "PW", "PH", "gC",
                                     "gS", "accumulate")] + \
               [(n, c_void_p) for n in ("out", "bias", "drop", "act", "idx")] + \
               [(n, c_i64) for n in ("gso", "gsc", "gsr", "gss")] + [("gbias", c_void_p), ("slab", c_void_p)]


SIGNATURES = {
    "det_cnn_gemm": ([c_void_p, c_i32, ctypes.POINTER(Job), ctypes.POINTER(Job)], ctypes.c_int),
    "det_cnn_finish": ([c_void_p, ctypes.POINTER(Job), c_i32], ctypes.c_int),
    "det_cnn_splits": ([c_i64, c_i32], ctypes.c_int),
    "det_cnn_masks": ([c_void_p, c_void_p, c_i64, ctypes.c_float, c_void_p, c_i64, ctypes.c_float, c_void_p, c_i64,
                       ctypes.c_float, ctypes.c_uint64, ctypes.c_uint64, c_void_p], ctypes.c_int),
    "det_cnn_xent_fwd": ([c_void_p, c_void_p, c_void_p, c_i32, c_i32, c_void_p, c_void_p, c_void_p], ctypes.c_int),
    "det_cnn_xent_bwd": ([c_void_p, c_void_p, c_void_p, c_void_p, c_i32, c_i32, c_void_p], ctypes.c_int),
}

_DT = {torch.float32: 0, torch.bfloat16: 1}
LAYERS = ((3, 32, 32, 0), (32, 32, 30, 0), (32, 64, 14, 1), (64, 64, 14, 0))  # (Cin, Cout, H in, pad)


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


# largest per-image tensor of the network (conv1's activation / gradient, 30 x 30 x 32): det_cnn.hip's
# index math is 32-bit, so a batch is native only while N * this < 2^31
_MAX_ELEMS_PER_IMAGE = 30 * 30 * 32


def supported(x: torch.Tensor, params: Sequence[torch.Tensor]) -> bool:
    if not (x.is_cuda and x.dim() == 4 and tuple(x.shape[1:]) == (3, 32, 32) and x.dtype in _DT):
        return False
    if x.shape[0] * _MAX_ELEMS_PER_IMAGE >= (1 << 31):
        return False  # det_cnn.hip indexes with 32-bit math: the torch layers take oversized batches
    if any(p.device != x.device or p.dtype != x.dtype for p in params):
        return False
    shapes = [(32, 3, 3, 3), (32,), (32, 32, 3, 3), (32,), (64, 32, 3, 3), (64,), (64, 64, 3, 3), (64,), (512, 2304),
              (512,), (10, 512), (10,)]
    return len(params) == 12 and all(tuple(p.shape) == s for p, s in zip(params, shapes)) and _lib.lib_available()


def _conv_act(t: torch.Tensor, dt: int, H: int, C: int, pad: int, OH: int, pool: int = 0) -> Operand:
    return Operand(p=t.data_ptr(), dt=dt, src=S_ACT_CONV, H=H, W=H, C=C, R=3, S=3, pad=pad, OH=OH, OW=OH, pool=pool)


def _wgt(w: torch.Tensor, dt: int, src: int, C: int) -> Operand:
    st = w.stride()
    if w.dim() == 4:
        return Operand(p=w.data_ptr(), dt=dt, src=src, C=C, R=3, S=3, so=st[0], sc=st[1], sr=st[2], ss=st[3])
    return Operand(p=w.data_ptr(), dt=dt, src=src, C=C, so=st[0], sc=st[1])


def _splits(lib, K: int, blocks: int) -> int:
    want = max(1, min(BLOCKS_TARGET // max(1, blocks), K // 64))
    return int(lib.det_cnn_splits(K, want))


def _tiles(M: int, N: int) -> int:
    return ((M + 63) // 64) * ((N + 63) // 64)


class _Runner:
    """Issues the jobs of one pass; owns the split-K slabs of the pass (freed with it)."""

    def __init__(self, ref: torch.Tensor) -> None:
        self.lib = _lib.get_lib()
        self.st = _stream(ref)
        self.dev = ref.device
        self.bf16 = 1 if ref.dtype == torch.bfloat16 else 0
        self.keep = []  # type: List[torch.Tensor]

    def prepare(self, job: Job, split: bool = True) -> Job:
        if split:
            s = _splits(self.lib, int(job.K), _tiles(int(job.M), int(job.N)))
        else:
            s = 1
        job.splits = s
        if s > 1:
            slab = torch.empty(s * int(job.M) * int(job.N), dtype=torch.float32, device=self.dev)
            self.keep.append(slab)
            job.slab = slab.data_ptr()
        return job

    def gemm(self, j0: Job, j1: Optional[Job] = None) -> List[Job]:
        _lib.check(self.lib.det_cnn_gemm(self.st, self.bf16, ctypes.byref(j0), ctypes.byref(j1) if j1 is not None else None),
                   "det_cnn_gemm")
        return [j for j in (j0, j1) if j is not None and j.splits > 1]

    def finish(self, jobs: List[Job]) -> None:
        for i in range(0, len(jobs), 4):
            chunk = jobs[i:i + 4]
            arr = (Job * len(chunk))(*chunk)
            _lib.check(self.lib.det_cnn_finish(self.st, arr, len(chunk)), "det_cnn_finish")


def _masks(x: torch.Tensor, n: int, ps: Tuple[float, float, float], training: bool):
    """Dropout factors (0 or 1/(1-p)) for the two Dropout2d layers ([N, 32], [N, 64]) and the element
    dropout on fc1 ([N, 512]); None where the layer is inactive."""
    if not training or all(p <= 0 for p in ps):
        return None, None, None
    lib = _lib.get_lib()
    sizes = (n * 32, n * 64, n * 512)
    outs = [torch.empty(sz, dtype=torch.float32, device=x.device) if p > 0 else None for sz, p in zip(sizes, ps)]
    seed, off = _tf.next_rng()
    base = _tf.rng_base(x.device)
    _lib.check(lib.det_cnn_masks(_stream(x), _p(outs[0]), sizes[0], float(ps[0]), _p(outs[1]), sizes[1], float(ps[1]),
                                 _p(outs[2]), sizes[2], float(ps[2]), seed, off, base), "det_cnn_masks")
    return tuple(outs)


def _forward(x: torch.Tensor, params: Sequence[torch.Tensor], ps, training: bool):
    w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, w6, b6 = params
    n = x.shape[0]
    dt = _DT[x.dtype]
    xh = x.permute(0, 2, 3, 1)
    if not xh.is_contiguous():
        xh = xh.contiguous()
    R = _Runner(x)
    m2, m4, m5 = _masks(x, n, ps, training)
    if DEBUG["keep_masks"]:
        DEBUG["masks"] = (m2, m4, m5)
    kw = dict(dtype=x.dtype, device=x.device)
    a1 = torch.empty(n, 30, 30, 32, **kw)
    a2 = torch.empty(n, 14, 14, 32, **kw)
    a3 = torch.empty(n, 14, 14, 64, **kw)
    a4 = torch.empty(n, 6, 6, 64, **kw)
    a5 = torch.empty(n, 512, **kw)
    idx2 = torch.empty(n, 14, 14, 32, dtype=torch.uint8, device=x.device)
    idx4 = torch.empty(n, 6, 6, 64, dtype=torch.uint8, device=x.device)
    logits = torch.empty(n, 10, dtype=torch.float32, device=x.device)
    # conv1 3->32 (valid) + bias + relu
    R.gemm(R.prepare(Job(a=_conv_act(xh, dt, 32, 3, 0, 30), b=_wgt(w1, dt, S_WGT_CONV, 3), M=n * 900, N=32, K=27,
                         epi=E_BIAS_RELU, out=a1.data_ptr(), out_dt=dt, bias=b1.data_ptr(), bias_dt=dt), split=False))
    # conv2 32->32 + bias + relu + maxpool + dropout2d (window-ordered rows)
    # (not split: 784 tiles already fill the chip; split + finish measured 30 vs 19 us)
    R.finish(R.gemm(R.prepare(Job(a=_conv_act(a1, dt, 30, 32, 0, 28, pool=1), b=_wgt(w2, dt, S_WGT_CONV, 32), M=n * 784,
                                  N=32, K=288, epi=E_BIAS_RELU_POOL, out=a2.data_ptr(), out_dt=dt, bias=b2.data_ptr(),
                                  bias_dt=dt, drop=_p(m2), drop_cols=32, idx=idx2.data_ptr(), PH=14, PW=14),
                              split=n * 784 < 16384)))
    # conv3 32->64 pad 1 + bias + relu
    R.finish(R.gemm(R.prepare(Job(a=_conv_act(a2, dt, 14, 32, 1, 14), b=_wgt(w3, dt, S_WGT_CONV, 32), M=n * 196, N=64,
                                  K=288, epi=E_BIAS_RELU, out=a3.data_ptr(), out_dt=dt, bias=b3.data_ptr(), bias_dt=dt))))
    # conv4 64->64 + bias + relu + maxpool + dropout2d
    R.finish(R.gemm(R.prepare(Job(a=_conv_act(a3, dt, 14, 64, 0, 12, pool=1), b=_wgt(w4, dt, S_WGT_CONV, 64), M=n * 144,
                                  N=64, K=576, epi=E_BIAS_RELU_POOL, out=a4.data_ptr(), out_dt=dt, bias=b4.data_ptr(),
                                  bias_dt=dt, drop=_p(m4), drop_cols=64, idx=idx4.data_ptr(), PH=6, PW=6))))
    # fc1 2304->512 (torch's NCHW flatten order) + bias + relu + dropout: split-K, finished by a launch
    fin = R.gemm(R.prepare(Job(a=Operand(p=a4.data_ptr(), dt=dt, src=S_ACT_FLAT, H=6, W=6, C=64),
                               b=_wgt(w5, dt, S_WGT_FC, 2304), M=n, N=512, K=2304, epi=E_BIAS_RELU_DROP,
                               out=a5.data_ptr(), out_dt=dt, bias=b5.data_ptr(), bias_dt=dt, drop=_p(m5),
                               drop_cols=512)))
    R.finish(fin)
    # fc2 512->10 + bias -> fp32 logits (split-K: one block would walk K serially)
    fin = R.gemm(R.prepare(Job(a=Operand(p=a5.data_ptr(), dt=dt, src=S_ACT_ROWS, C=512), b=_wgt(w6, dt, S_WGT_FC, 512),
                         M=n, N=10, K=512, epi=E_BIAS, out=logits.data_ptr(), out_dt=dt, bias=b6.data_ptr(),
                         bias_dt=dt)))
    R.finish(fin)
    saved = (xh, a1, a2, a3, a4, a5, idx2, idx4, m2, m4, m5)
    return logits, saved


def _grad_targets(w: torch.Tensor, b: torch.Tensor, direct: bool):
    """Where the kernels write a (weight, bias) pair's gradients: [(tensor, returned-to-autograd)] x 2
    and the accumulate flag the pair shares.  In a capture with both ``.grad`` pinned (arena views)
    they accumulate in place; otherwise fresh gradients (arena landing slots when the GradSink offers
    them) go back to autograd."""
    if direct and all(p.grad is not None and p.grad.stride() == p.stride() for p in (w, b)):
        return [(w.grad, False), (b.grad, False)], 1
    from determined_1_amd.ops.arena import landing_buffer

    out = []
    for p in (w, b):
        buf = landing_buffer(p)
        if buf is None or buf.stride() != p.stride():
            buf = torch.empty_strided(p.shape, p.stride(), dtype=p.dtype, device=p.device)
        out.append((buf, True))
    return out, 0


def _backward(dlogits: torch.Tensor, params: Sequence[torch.Tensor], saved):
    w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, w6, b6 = params
    xh, a1, a2, a3, a4, a5, idx2, idx4, m2, m4, m5 = saved
    n = xh.shape[0]
    dt = _DT[xh.dtype]
    R = _Runner(xh)
    direct = torch.cuda.is_current_stream_capturing()
    targets, acc = [], []
    for i in range(0, 12, 2):
        pair, a = _grad_targets(params[i], params[i + 1], direct)
        targets += pair
        acc += [a, a]
    g = [t[0] for t in targets]
    kw = dict(dtype=xh.dtype, device=xh.device)
    dl = dlogits.contiguous().float()
    dz5 = torch.empty(n, 512, **kw)
    g4 = torch.empty(n, 12, 12, 64, **kw)  # conv4's output gradient: dp4 routed through the max-pool
    dy3 = torch.empty(n, 14, 14, 64, **kw)
    g2 = torch.empty(n, 28, 28, 32, **kw)  # conv2's output gradient (unpooled dp2)
    dy1 = torch.empty(n, 30, 30, 32, **kw)

    def gfc(i: int, K: int) -> dict:
        st = g[i].stride()
        return dict(epi=E_GRAD_FC, out=g[i].data_ptr(), out_dt=dt, gso=st[0], gsc=st[1], gbias=g[i + 1].data_ptr(),
                    accumulate=acc[i])

    def gconv(i: int, cin: int) -> dict:
        st = g[i].stride()
        return dict(epi=E_GRAD_CONV, out=g[i].data_ptr(), out_dt=dt, gso=st[0], gsc=st[1], gsr=st[2], gss=st[3],
                    gC=cin, gS=3, gbias=g[i + 1].data_ptr(), accumulate=acc[i])

    deferred = []  # type: List[Job]

    def step(j0: Job, j1: Optional[Job] = None) -> None:
        """Launch a (weight grad, input grad) pair; a split input gradient is finished before the
        next layer reads it, split weight gradients are finished together at the end."""
        split = R.gemm(j0, j1)
        deferred.extend(j for j in split if j.epi in (E_GRAD_FC, E_GRAD_CONV))
        R.finish([j for j in split if j.epi not in (E_GRAD_FC, E_GRAD_CONV)])

    # fc2: weight grad (K = batch) || input grad -> dz5 = d(a5) * drop * (a5 > 0)
    step(R.prepare(Job(a=Operand(p=dl.data_ptr(), dt=0, src=S_GRAD_ROWS, C=10, transpose=1),
                       b=Operand(p=a5.data_ptr(), dt=dt, src=S_ACT_ROWS, C=512), M=10, N=513, K=n, **gfc(10, n))),
         R.prepare(Job(a=Operand(p=dl.data_ptr(), dt=0, src=S_GRAD_ROWS, C=10), b=_wgt(w6, dt, S_WGT_FC_T, 0),
                       M=n, N=512, K=10, epi=E_DROP_POS, out=dz5.data_ptr(), out_dt=dt, act=a5.data_ptr(),
                       drop=_p(m5), drop_cols=512, HW=1)))
    # fc1: weight grad || input grad -> d(a4) * drop2d * (a4 > 0), written unpooled (the argmax of each
    # 2x2 window, zeros elsewhere) as conv4's output gradient g4
    step(R.prepare(Job(a=Operand(p=dz5.data_ptr(), dt=dt, src=S_GRAD_ROWS, C=512, transpose=1),
                       b=Operand(p=a4.data_ptr(), dt=dt, src=S_ACT_FLAT, H=6, W=6, C=64), M=512, N=2305, K=n,
                       **gfc(8, n))),
         R.prepare(Job(a=Operand(p=dz5.data_ptr(), dt=dt, src=S_GRAD_ROWS, C=512), b=_wgt(w5, dt, S_WGT_FC_T, 0),
                       M=n, N=2304, K=512, epi=E_DROP_POS_FLAT, out=g4.data_ptr(), out_dt=dt,
                       act=a4.data_ptr(), drop=_p(m4), drop_cols=64, HW=36, C=64, idx=idx4.data_ptr(), PH=6, PW=6)))
    # conv4: weight grad || input grad -> dy3 = d(a3) * (a3 > 0)
    step(R.prepare(Job(a=Operand(p=g4.data_ptr(), dt=dt, src=S_GRAD_CONV_T, C=64, OH=12, OW=12, transpose=1),
                       b=_conv_act(a3, dt, 14, 64, 0, 12), M=64, N=577, K=n * 144, **gconv(6, 64))),
         R.prepare(Job(a=Operand(p=g4.data_ptr(), dt=dt, src=S_GRAD_CONV_T, H=12, W=12, C=64, R=3, S=3, pad=0,
                                 OH=14, OW=14),
                       b=_wgt(w4, dt, S_WGT_CONV_T, 64), M=n * 196, N=64, K=576, epi=E_MASK_POS,
                       out=dy3.data_ptr(), out_dt=dt, act=a3.data_ptr())))
    # conv3 (pad 1): weight grad || input grad -> d(a2) * drop2d * (a2 > 0), unpooled: conv2's g2
    step(R.prepare(Job(a=Operand(p=dy3.data_ptr(), dt=dt, src=S_GRAD_CONV_T, C=64, OH=14, OW=14, transpose=1),
                       b=_conv_act(a2, dt, 14, 32, 1, 14), M=64, N=289, K=n * 196, **gconv(4, 32))),
         R.prepare(Job(a=Operand(p=dy3.data_ptr(), dt=dt, src=S_GRAD_CONV_T, H=14, W=14, C=64, R=3, S=3, pad=1,
                                 OH=14, OW=14),
                       b=_wgt(w3, dt, S_WGT_CONV_T, 64), M=n * 196, N=32, K=576, epi=E_DROP_POS,
                       out=g2.data_ptr(), out_dt=dt, act=a2.data_ptr(), drop=_p(m2), drop_cols=32, HW=196,
                       idx=idx2.data_ptr(), PH=14, PW=14)))
    # conv2: weight grad || input grad -> dy1 = d(a1) * (a1 > 0)
    step(R.prepare(Job(a=Operand(p=g2.data_ptr(), dt=dt, src=S_GRAD_CONV_T, C=32, OH=28, OW=28, transpose=1),
                       b=_conv_act(a1, dt, 30, 32, 0, 28), M=32, N=289, K=n * 784, **gconv(2, 32))),
         R.prepare(Job(a=Operand(p=g2.data_ptr(), dt=dt, src=S_GRAD_CONV_T, H=28, W=28, C=32, R=3, S=3, pad=0,
                                 OH=30, OW=30),
                       b=_wgt(w2, dt, S_WGT_CONV_T, 32), M=n * 900, N=32, K=288, epi=E_MASK_POS,
                       out=dy1.data_ptr(), out_dt=dt, act=a1.data_ptr())))
    # conv1: weight grad only (no input gradient)
    step(R.prepare(Job(a=Operand(p=dy1.data_ptr(), dt=dt, src=S_GRAD_CONV_T, C=32, OH=30, OW=30, transpose=1),
                        b=_conv_act(xh, dt, 32, 3, 0, 30), M=32, N=28, K=n * 900, **gconv(0, 3))))
    R.finish(deferred)
    from determined_1_amd.ops.arena import notify_direct_grads

    notify_direct_grads([p for p, t in zip(params, targets) if not t[1]])  # written in place: no AccumulateGrad
    return [t[0] if t[1] else None for t in targets]


class _CifarCNN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ps, training, *params):  # type: ignore[override]
        logits, saved = _forward(x, params, ps, training)
        ctx.saved = saved
        ctx.params = params
        return logits

    @staticmethod
    def backward(ctx, dlogits):  # type: ignore[override]
        grads = _backward(dlogits, ctx.params, ctx.saved)
        ctx.saved = None
        return (None, None, None, *grads)


def cifar_cnn(x: torch.Tensor, params: Sequence[torch.Tensor], ps: Tuple[float, float, float],
              training: bool) -> torch.Tensor:
    """fp32 logits [N, 10] of the CIFAR-10 CNN on the native kernels (see ``supported``)."""
    return _CifarCNN.apply(x, tuple(float(p) for p in ps), bool(training), *params)


class _XEnt(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, y):  # type: ignore[override]
        n, c = logits.shape
        z = logits.contiguous().float()
        yy = y.contiguous().long()
        out = torch.empty(3, dtype=torch.float32, device=logits.device)  # loss, accuracy, error
        # the gradient for a unit seed comes out of the same launch when a backward is coming
        dz1 = torch.empty_like(z) if ctx.needs_input_grad[0] else None  # (grad mode is off in here)
        _lib.check(_lib.get_lib().det_cnn_xent_fwd(_stream(z), z.data_ptr(), yy.data_ptr(), n, c, out.data_ptr(),
                                                   out.data_ptr() + 4, None if dz1 is None else dz1.data_ptr()),
                   "det_cnn_xent_fwd")
        ctx.dz1 = dz1
        ctx.save_for_backward(z, yy)
        ctx.dtype = logits.dtype
        loss, acc, err = out[0], out[1], out[2]
        ctx.mark_non_differentiable(acc, err)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the metrics (two fill launches)
        return loss, acc, err

    @staticmethod
    def backward(ctx, gloss, gacc, gerr):  # type: ignore[override]
        z, yy = ctx.saved_tensors
        if gloss is None:
            return None, None
        if ctx.dz1 is not None and seed_grad.is_unit(gloss):
            dz1, ctx.dz1 = ctx.dz1, None
            XENT_FROM_FORWARD["count"] += 1
            return dz1.to(ctx.dtype), None
        n, c = z.shape
        dz = torch.empty_like(z)
        g = gloss.reshape(1).float().contiguous()
        _lib.check(_lib.get_lib().det_cnn_xent_bwd(_stream(z), z.data_ptr(), yy.data_ptr(), g.data_ptr(), n, c,
                                                   dz.data_ptr()), "det_cnn_xent_bwd")
        return dz.to(ctx.dtype), None


def cross_entropy(logits: torch.Tensor, y: torch.Tensor, with_accuracy: bool = False, with_error: bool = False):
    """Mean cross entropy (torch.nn.functional.cross_entropy semantics) in one launch, with the
    batch accuracy (first-maximum argmax, as torch.argmax) as a second output and the error rate
    (1 - accuracy) as a third if asked -- all from the same launch."""
    if not (logits.is_cuda and logits.dim() == 2) or not _lib.lib_available():
        loss = torch.nn.functional.cross_entropy(logits.float(), y)
        acc = (logits.argmax(1) == y).float().mean()
        outs = (loss,) + ((acc,) if with_accuracy else ()) + ((1.0 - acc,) if with_error else ())
        return outs if len(outs) > 1 else loss
    loss, acc, err = _XEnt.apply(logits, y)
    outs = (loss,) + ((acc,) if with_accuracy else ()) + ((err,) if with_error else ())
    return outs if len(outs) > 1 else loss
