"""Loader for the hand-written gfx950 kernel library (``libdetkernels.so``).

The library is a plain C ABI built by ``hipcc --offload-arch=gfx950 -shared`` (see
``determined_1_amd/ops/build.py``) and loaded with ctypes.  Kernels are launched on the caller's
current HIP stream (``torch.cuda.current_stream().cuda_stream``) so they order correctly with
PyTorch work and are capturable into hipGraphs.

Policy: on a GPU tensor the HIP library MUST be used.  If it is missing we raise instead of
silently falling back to eager PyTorch (the harness's "native code loaded" check depends on
that).  CPU tensors (unit tests on the build host) use the pure-PyTorch reference
implementations in ``functional.py``.
"""
import ctypes
import os
import pathlib
import threading
from typing import Optional

_HERE = pathlib.Path(__file__).resolve().parent
LIB_NAME = "libdetkernels.so"
LIB_PATH = _HERE / LIB_NAME
ABI_VERSION = 21

_lock = threading.Lock()
_lib = None  # type: Optional[ctypes.CDLL]

F32, BF16, F16 = 0, 1, 2

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_float = ctypes.c_float

_SIGNATURES = {
    "det_abi_version": ([], c_int),
    # stream, g_dtype, out_dtype, p, g, buf, out_model, n, lr, momentum, dampening, wd,
    # nesterov, first_step, g_scale, g_scale_dev, found_inf
    "det_sgd_step": (
        [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_i64]
        + [c_float] * 4
        + [c_int, c_int, c_float, c_void_p, c_void_p],
        c_int,
    ),
    # stream, g_dtype, out_dtype, p, g, m, v, vmax, out_model, n, lr, b1, b2, eps, wd, adamw,
    # amsgrad, bias_c1, bias_c2_sqrt, g_scale, g_scale_dev, found_inf
    "det_adam_step": (
        [c_void_p, c_int, c_int] + [c_void_p] * 6 + [c_i64] + [c_float] * 5
        + [c_int, c_int, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p],
        c_int,
    ),
    # stream, g_dtype, out_dtype, p, g, square_avg, momentum_buf, grad_avg, out_model, n, lr,
    # alpha, eps, wd, momentum, centered, g_scale, g_scale_dev, found_inf
    "det_rmsprop_step": (
        [c_void_p, c_int, c_int] + [c_void_p] * 6 + [c_i64] + [c_float] * 5
        + [c_int, c_float, c_void_p, c_void_p],
        c_int,
    ),
    # stream, g_dtype, out_dtype, p, g, sum, out_model, n, clr, eps, wd, g_scale, g_scale_dev,
    # found_inf
    "det_adagrad_step": (
        [c_void_p, c_int, c_int] + [c_void_p] * 4 + [c_i64] + [c_float] * 3
        + [c_float, c_void_p, c_void_p],
        c_int,
    ),
    # stream, g_dtype, out_dtype, p, g, square_avg, acc_delta, out_model, n, lr, rho, eps, wd,
    # g_scale, g_scale_dev, found_inf
    "det_adadelta_step": (
        [c_void_p, c_int, c_int] + [c_void_p] * 5 + [c_i64] + [c_float] * 4
        + [c_float, c_void_p, c_void_p],
        c_int,
    ),
    "det_scale_cast": ([c_void_p, c_void_p, c_int, c_void_p, c_int, c_i64, c_float, c_void_p], c_int),
    # stream, in, in_dtype, out, out_dtype, rows, n, scale
    "det_sum_rows": ([c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_i64, c_float], c_int),
    "det_sumsq_num_partials": ([c_i64], c_int),
    "det_sumsq_partials": ([c_void_p, c_void_p, c_int, c_i64, c_void_p], c_int),
    "det_norm_finalize": (
        [c_void_p, c_void_p, c_int, c_float, c_float, c_void_p, c_void_p, c_void_p],
        c_int,
    ),
    "det_unscale_check": ([c_void_p, c_void_p, c_int, c_i64, c_float, c_void_p], c_int),
    "det_mt_copy": ([c_void_p, c_void_p, c_int, c_int, c_int, c_i64, c_float], c_int),
    # hipGraph_t, mode (0 count, 1 replace memset nodes by fill-kernel nodes) -> memsets found
    "det_graph_fix_memsets": ([c_void_p, c_int], c_int),
    # stream, A, B, C, bias, bias_dt, M, N, K, lda, ldb, ldc, mode, C2, epi
    "det_gemm8": ([c_void_p] * 5 + [c_int, c_i64] + [c_int] * 6 + [c_void_p, c_int], c_int),
    "det_u8_normalize": (
        [c_void_p, c_void_p, c_void_p, c_int, c_i64, c_int, c_void_p, c_void_p],
        c_int,
    ),
    # det_norm.hip: fused BatchNorm(+add)(+ReLU), channels_last
    # stream, dtype, d, x, M, C, gamma, mean, rstd, psum, psumx, nrb, rpb, dx, dgamma, dbeta, coef
    "det_bn_bwd_from_partials": ([c_void_p, c_int, c_void_p, c_void_p, c_i64, c_int] + [c_void_p] * 5 + [c_int, c_i64]
                                 + [c_void_p] * 5, c_int),
    "det_bn_bwd_scratch_elems": ([c_int], c_i64),
    "det_bn_bwd_finalize_partials": ([c_void_p, c_i64, c_int] + [c_void_p] * 5 + [c_int, c_i64] + [c_void_p] * 4, c_int),
    "det_bn_bwd_apply_coef": ([c_void_p, c_int, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p], c_int),
    "det_bn_apply_res_mbits": ([c_void_p] * 3 + [c_void_p, c_i64, c_int] + [c_void_p] * 5, c_int),
    "det_bn_ws_elems": ([c_i64, c_int], c_i64),
    "det_bn_fin_ws_elems": ([c_int], c_i64),
    # stream, dtype, x, res, y, M, C, gamma, beta, running_mean, running_var, nbt, momentum, eps,
    # relu, save_mean, save_rstd, scale, shift, ws, mask_bits
    "det_bn_fwd_train": (
        [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_i64, c_int] + [c_void_p] * 5
        + [c_float, c_float, c_int] + [c_void_p] * 6,
        c_int,
    ),
    # stream, dtype, x, M, C, gamma, beta, running_mean, running_var, nbt, momentum, eps,
    # save_mean, save_rstd, scale, shift, ws
    # stream, kind, src, dst, nbytes, blocks, unroll, value, sink  (det_stream.hip yardsticks)
    "det_stream": ([c_void_p, c_int, c_void_p, c_void_p, c_i64, c_int, c_int, ctypes.c_uint32, c_void_p], c_int),
    "det_bn_stats_train": (
        [c_void_p, c_int, c_void_p, c_i64, c_int] + [c_void_p] * 5 + [c_float, c_float] + [c_void_p] * 5,
        c_int,
    ),
    # stream, dtype, x, y, idx(u8), N, H, W, C
    # ... + bn_scale, bn_shift (nullable: the pooled tensor's BN + ReLU applied in the pool)
    "det_maxpool3s2_fwd": ([c_void_p, c_int, c_void_p, c_void_p, c_void_p] + [c_int] * 4 + [c_void_p] * 2, c_int),
    # stream, dtype, dy, idx(u8), dx, N, H, W, C
    # ... + bn_x, bn_mean, bn_scale, bn_shift, psum, psumx (nullable BN-backward epilogue)
    "det_maxpool3s2_bwd": ([c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 4 + [c_void_p] * 6,
                           c_int),
    "det_maxpool3s2_bwd_rows_per_block": ([], c_int),
    "det_maxpool3s2_bwd_partial_rows": ([c_int] * 4, c_i64),
    "det_maxpool3s2_set_fwd_rows": ([c_int], None),
    # stream, dtype, x|dy, y|dx, N, HW, C (global average pooling, channels_last)
    "det_gap_fwd": ([c_void_p, c_int, c_void_p, c_void_p] + [c_int] * 3, c_int),
    "det_gap_bwd": ([c_void_p, c_int, c_void_p, c_void_p] + [c_int] * 3, c_int),
    "det_bn_apply": ([c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p, c_int], c_int),
    # stream, dtype, dy, x, mask_bits, M, C, mask_mode, gamma, save_mean, save_rstd, scale, shift, dx, dres,
    # dgamma, dbeta, ws
    # stream, dtype, dy, dy2, x, mbits, M, C, mask_mode, gamma, mean, rstd, scale, shift, dx, dres,
    # dgamma, dbeta, ws
    "det_bn_bwd": (
        [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_int] + [c_void_p] * 10 + [c_int],
        c_int,
    ),
    "det_bn_bwd_coef_offset": ([c_i64, c_int], c_i64),
    # stream, dtype, x, res, y, M, C, rpb, nrb, pmean, pm2, gamma, beta, rmean, rvar, nbt, momentum, eps, relu,
    # apply, save_mean, save_rstd, scale, shift, mbits, ws, res_scale, res_shift
    "det_bn_fwd_from_partials": (
        [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_int, c_int] + [c_void_p] * 7
        + [c_float, c_float, c_int, c_int] + [c_void_p] * 8,
        c_int,
    ),
    # det_detect.hip: multi-level RoIAlign (NHWC) and device NMS
    # stream, dtype, rois, level, K, n_levels, feats**, hs*, ws*, scales*, C, PH, PW, sampling, out
    "det_roi_align_fwd": ([c_void_p, c_int, c_void_p, c_void_p, c_int, c_int] + [c_void_p] * 4 + [c_int] * 4
                          + [c_void_p], c_int),
    # stream, dtype, rois, level, K, n_levels, grads**, hs*, ws*, scales*, C, PH, PW, sampling, dy
    "det_roi_align_bwd": ([c_void_p, c_int, c_void_p, c_void_p, c_int, c_int] + [c_void_p] * 4 + [c_int] * 4
                          + [c_void_p], c_int),
    "det_nms_mask_words": ([c_int], c_int),
    "det_nms_max_boxes": ([], c_int),
    # stream, boxes, n, thr, mask, keep
    "det_nms": ([c_void_p, c_void_p, c_int, c_float, c_void_p, c_void_p], c_int),
    # det_conv.hip: 1x1-conv GEMMs (MFMA) with fused BN statistics / BN-apply+ReLU prologue
    "det_conv_nt_rows_per_block": ([c_int], c_int),
    "det_conv_nt_set_wide": ([c_int], c_int),
    "det_conv_nt_set_pf": ([c_int], c_int),
    # stream, X, W, bias (nullable), Y, M, N, K
    "det_linear_fwd": ([c_void_p] * 5 + [c_i64, c_int, c_int], c_int),
    # det_blaslt.hip: hipBLASLt with cached per-shape plans (path of torch's libhipblaslt)
    "det_blaslt_init": ([ctypes.c_char_p], c_int),
    # stream, transa, transb, m, n, k, A, lda, B, ldb, D, ldd, bias, beta, dtype, ws, ws_bytes
    "det_blaslt_gemm": ([c_void_p, c_int, c_int, c_i64, c_i64, c_i64, c_void_p, c_i64, c_void_p, c_i64, c_void_p, c_i64,
                         c_void_p, ctypes.c_float, c_int, c_void_p, c_i64, c_int], c_int),
    # stream, A, B, C, M, N, K, scale, shift, pmean, pm2, Ho, Wo, Hi, Wi
    # ... + res, aout, abits, res_scale, res_shift
    "det_conv_nt": ([c_void_p] * 4 + [c_i64, c_int, c_int] + [c_void_p] * 4 + [c_int] * 4 + [c_void_p] * 5, c_int),
    "det_conv_tn_ws_elems": ([c_i64, c_int, c_int], c_i64),
    # stream, A, B, C, M, N, K, x, mean, scale, shift, mbits, add, psum, psumx, mode
    "det_conv_nt_bnbwd": ([c_void_p] * 4 + [c_i64, c_int, c_int] + [c_void_p] * 8 + [c_int, c_int] + [c_void_p] * 3
                          + [c_int] * 4, c_int),
    "det_conv_dgrad": ([c_void_p] * 4 + [c_i64, c_int, c_int] + [c_void_p] * 3, c_int),
    # det_igemm.hip: pipelined implicit-GEMM conv (LDS-DMA ring)
    "det_igemm_rows_per_block": ([], c_int),
    # stream, X, W, Y, zero, M, N, Cin, Hi, Wi, Ho, Wo, R, S, stride, pad, pmean, pm2
    "det_igemm_conv": ([c_void_p] * 5 + [c_i64] + [c_int] * 10 + [c_void_p] * 2, c_int),
    "det_igemm_rows_per_block_cfg": ([c_int, c_int], c_int),
    # stream, W (KRSC), in_dtype (0 fp32 / 1 bf16), out [C, R*S*K] bf16, K, C, R, S
    "det_conv_dgrad_weight": ([c_void_p, c_void_p, c_int, c_void_p] + [c_int] * 4, c_int),
    # stream, n, w ptrs (int64[n]), out ptrs (int64[n]), dims (int32[n][5]: K, C, R, S, bf16)
    "det_conv_dgrad_weight_multi": ([c_void_p, c_int, c_void_p, c_void_p, c_void_p], c_int),
    # ... + cfg (0 = automatic per shape)
    "det_igemm_conv_cfg": ([c_void_p] * 5 + [c_i64] + [c_int] * 10 + [c_void_p] * 2 + [c_int], c_int),
    "det_igemm_conv_bnbwd": ([c_void_p] * 5 + [c_i64] + [c_int] * 10 + [c_void_p] * 6 + [c_int], c_int),
    # stream, dY, Wd [Cin][9*Cout], dX, zero, Nb, Ho, Wo, Cout, Cin, bn_x, bn_mean, bn_scale, bn_shift,
    # psum, psumx (nullable BNB epilogue), cfg
    "det_igemm_dgrad_s2": ([c_void_p] * 5 + [c_int] * 5 + [c_void_p] * 6 + [c_int], c_int),
    "det_igemm_dgrad_s2_rows_per_block": ([c_int, c_int], c_int),
    # stream, X, W [N][9][Cin], Y, Nb, H, W, Cin, N, pro_scale, pro_shift, pmean, pm2, bn_x, bn_mean,
    # bn_scale, bn_shift, psum, psumx, grid (0 = one persistent block per CU)
    "det_conv3p": ([c_void_p] * 4 + [c_int] * 5 + [c_void_p] * 10 + [c_int], c_int),
    "det_conv3p_wgrad_ws_elems": ([c_i64, c_int, c_int], c_i64),
    "det_stemp_wgrad_ws_elems": ([c_i64], c_i64),
    # stream, dY, X4, out, out_dtype, M, Hi, Wi, Ho, Wo, ws, out_scale, bn_x, coef (nullable deferred BN apply)
    "det_stemp_fwd": ([c_void_p] * 4 + [c_i64] + [c_int] * 4 + [c_void_p] * 2, c_int),
    "det_stemp_fwd_rows_per_block": ([], c_int),
    "det_stemp_wgrad": ([c_void_p] * 4 + [c_int, c_i64] + [c_int] * 4 + [c_void_p, c_float] + [c_void_p] * 2, c_int),
    # stream, dY, X, out, out_dtype, Nb, H, W, Cin, N, ws, out_scale
    "det_conv3p_wgrad": ([c_void_p] * 4 + [c_int] * 6 + [c_void_p, c_float], c_int),
    # stream, dY, X, out, out_dtype, M, N, Cin, Hi, Wi, Ho, Wo, R, S, stride, pad, ws, out_scale
    "det_conv_wgrad": ([c_void_p] * 4 + [c_int, c_i64] + [c_int] * 10 + [c_void_p, c_float], c_int),
    "det_igemm_wgrad_ws_elems": ([c_i64, c_int, c_int, c_int], c_i64),
    "det_igemm_wgrad": ([c_void_p] * 4 + [c_int, c_i64] + [c_int] * 10 + [c_void_p, c_float, c_int], c_int),
    # stream, dY, X, out, out_dtype, M, N, K, scale_x, shift_x, ws, out_scale, Ho, Wo, Hi, Wi
    "det_conv_tn": ([c_void_p] * 4 + [c_int, c_i64, c_int, c_int] + [c_void_p] * 3 + [c_float] + [c_int] * 4, c_int),
    # stream, X, W, Y, M, Hi, Wi, Ho, Wo, pmean, pm2
    "det_stem_conv_fwd": ([c_void_p] * 4 + [c_i64] + [c_int] * 4 + [c_void_p] * 2, c_int),
    "det_stem_conv_wgrad_ws_elems": ([c_i64], c_i64),
    # stream, dY, X, out, out_dtype, M, Hi, Wi, Ho, Wo, ws, out_scale
    "det_stem_conv_wgrad": ([c_void_p] * 4 + [c_int, c_i64] + [c_int] * 4 + [c_void_p, c_float], c_int),
    # stream, in(u8 NHWC C<=3), out(NHWC 4), out_dtype, npix, C, mean, std
    "det_u8_normalize_pad4": ([c_void_p, c_void_p, c_void_p, c_int, c_i64, c_int, c_void_p, c_void_p], c_int),
    # det_transformer.hip: fused LayerNorm / dropout / residual / GELU / bias-grad epilogues
    "det_tf_ln_max_hidden": ([], c_int),
    "det_tf_ln_ws_elems": ([c_i64, c_int], c_i64),
    # stream, dtype, h, r, y, rows, H, gamma, beta, eps, p, seed, offset, mean, rstd, offset base
    "det_tf_ln_fwd": (
        [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p, c_float, c_float,
         ctypes.c_uint64, ctypes.c_uint64, c_void_p, c_void_p, c_void_p],
        c_int,
    ),
    # stream, dtype, dy, h, r, mean, rstd, gamma, rows, H, p, seed, offset, dr, dh, dgamma, dbeta, dbias, ws,
    # offset base
    "det_tf_ln_bwd": (
        [c_void_p, c_int] + [c_void_p] * 6 + [c_i64, c_int, c_float, ctypes.c_uint64, ctypes.c_uint64]
        + [c_void_p] * 7,
        c_int,
    ),
    "det_tf_col_ws_elems": ([c_i64, c_int], c_i64),
    "det_tf_gelu_fwd": ([c_void_p, c_int, c_void_p, c_void_p, c_i64, c_int], c_int),
    # stream, dtype, da, z, dz, rows, C, dbias, ws
    "det_tf_gelu_bwd": ([c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p, c_int], c_int),
    # stream, dtype, x, rows, C, out, ws
    "det_tf_colsum": ([c_void_p, c_int, c_void_p, c_i64, c_int, c_void_p, c_void_p], c_int),
    # det_attention.hip: MFMA flash attention (bf16 head_dim 32/64/128, fp32 32/64, any length)
    # dtype (0 bf16, 1 fp32), head_dim, Lq, Lk
    "det_attn_supported": ([c_int, c_int, c_int, c_int], c_int),
    # stream, const DetAttnParams* (transformer._AttnParams)
    "det_attn_forward": ([c_void_p, c_void_p], c_int),
    "det_attn_backward": ([c_void_p, c_void_p], c_int),
    "det_attn_set_bwd_merged": ([c_int], c_int),
    # stream, B, nh, Lq, Lk, p, seed, offset, out, offset base
    "det_attn_dropout_mask": ([c_void_p, c_int, c_int, c_int, c_int, c_float, ctypes.c_uint64, ctypes.c_uint64,
                               c_void_p, c_void_p], c_int),
    "det_tf_dropout_mask": ([c_void_p, c_i64, c_float, ctypes.c_uint64, ctypes.c_uint64, c_void_p, c_void_p], c_int),
    "det_tf_rng_bump": ([c_void_p, c_void_p], c_int),
    "det_embed_fwd": ([c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int],
                      c_int),
    "det_embed_ws_floats": ([c_int, c_int, c_int], ctypes.c_int64),
    "det_embed_bwd": ([c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                       c_int, ctypes.c_int64, c_void_p, c_int], c_int),
}


class KernelLibraryMissing(RuntimeError):
    pass


def lib_available() -> bool:
    try:
        get_lib()
        return True
    except (KernelLibraryMissing, OSError):
        return False


def get_lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = os.environ.get("DET_KERNELS_LIB", str(LIB_PATH))
        if not os.path.exists(path):
            raise KernelLibraryMissing(
                f"{path} not found: build it with `python -m determined_1_amd.ops.build` "
                "(hipcc --offload-arch=gfx950).  GPU tensors never fall back to eager PyTorch."
            )
        lib = ctypes.CDLL(path)
        from determined_1_amd.ops.cnn import SIGNATURES as _CNN_SIGS

        for name, (argtypes, restype) in list(_SIGNATURES.items()) + list(_CNN_SIGS.items()):
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = restype
        ver = lib.det_abi_version()
        if ver != ABI_VERSION:
            raise KernelLibraryMissing(
                f"{path} has ABI {ver}, expected {ABI_VERSION}; rebuild the kernels"
            )
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"HIP kernel {what} failed with hipError {rc}")
