// det_kernels.hip — hand-written CDNA4 (gfx950) kernels for the training hot path.
//
// Everything here is bandwidth-bound streaming work, so the design rules are the HBM ones
// (cdna_hip_programming.md Guideline 11/13, Appendix B "Element-wise" / "Reduction"):
//   * wave64 blocks of 256 threads, 16-byte vector loads/stores per lane (float4 / 8x bf16),
//   * grid = min(work/256, 256 CUs x 8) and grid-stride the rest,
//   * reductions: wave shuffle -> LDS -> one partial per block -> tiny finalize launch
//     (no float atomics, so results are bitwise reproducible run-to-run),
//   * no host syncs anywhere: AMP overflow, grad-norm clipping and the optimizer skip decision
//     are carried in device scalars so an entire optimizer step can be captured in a hipGraph.
//
// The parameter "arena" design (see determined_1_amd/ops/arena.py): every trainable parameter of
// a wrapped model lives inside one flat fp32 buffer per param group, and every gradient inside a
// matching flat buffer.  That makes the reference's Horovod tensor-fusion pack/unpack
// (harness/determined/pytorch/_pytorch_context.py:192-198) unnecessary: a gradient
// bucket *is* a contiguous slice of the arena, the optimizer is ONE launch per param group, and
// gradient averaging / aggregation_frequency division / AMP unscale / clip coefficient are all
// folded into that launch as a scale.
//
// C ABI only (loaded with ctypes from determined_1_amd/ops/_lib.py) so the library builds with a
// bare `hipcc --offload-arch=gfx950 -shared` in seconds and has no torch-header dependency.

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

namespace {

constexpr int kBlock = 256;
constexpr int kMaxGrid = 256 * 8;  // 256 CUs x 8 resident blocks

enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(__hip_bfloat16 x) { return __bfloat162float(x); }
__device__ __forceinline__ float to_f(__half x) { return __half2float(x); }

template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ __hip_bfloat16 from_f<__hip_bfloat16>(float x) {
  return __float2bfloat16(x);
}
template <> __device__ __forceinline__ __half from_f<__half>(float x) { return __float2half(x); }

// 4-element vector load/store in any of the three dtypes.  f32: one dwordx4; bf16/f16: one dwordx2.
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  static __device__ __forceinline__ float4 load(const float* p, int64_t i) {
    return reinterpret_cast<const float4*>(p)[i];
  }
  static __device__ __forceinline__ void store(float* p, int64_t i, float4 v) {
    reinterpret_cast<float4*>(p)[i] = v;
  }
};
template <typename H> struct Vec4Half {
  static __device__ __forceinline__ float4 load(const H* p, int64_t i) {
    uint2 raw = reinterpret_cast<const uint2*>(p)[i];
    H h[4];
    *reinterpret_cast<uint2*>(h) = raw;
    return make_float4(to_f(h[0]), to_f(h[1]), to_f(h[2]), to_f(h[3]));
  }
  static __device__ __forceinline__ void store(H* p, int64_t i, float4 v) {
    H h[4] = {from_f<H>(v.x), from_f<H>(v.y), from_f<H>(v.z), from_f<H>(v.w)};
    reinterpret_cast<uint2*>(p)[i] = *reinterpret_cast<uint2*>(h);
  }
};
template <> struct Vec4<__hip_bfloat16> : Vec4Half<__hip_bfloat16> {};
template <> struct Vec4<__half> : Vec4Half<__half> {};

inline int grid_for(int64_t work_items) {
  int64_t g = (work_items + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > kMaxGrid) g = kMaxGrid;
  return static_cast<int>(g);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Block-wide sum of one float per thread; result valid in thread 0.
__device__ __forceinline__ float block_sum(float v) {
  __shared__ float red[kBlock / 64];
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) s += red[w];
  }
  return s;
}

// ------------------------------------------------------------------------------------------
// Fused optimizers over a flat fp32 master arena.
//
// Each functor sees ONE element: p (fp32 master value, in/out), g (already fully scaled fp32
// gradient) and its state slots.  Semantics match torch.optim.* (torch 2.x, foreach=False,
// maximize=False) so optimizer.state_dict() round-trips with the stock classes, which is what
// the reference's checkpoint format stores (_pytorch_trial.py:722-755).
// ------------------------------------------------------------------------------------------
struct SgdArgs {
  float lr, momentum, dampening, wd;
  int nesterov, first_step;
};
struct AdamArgs {
  float lr, beta1, beta2, eps, wd;
  int adamw, amsgrad;
  float bias_c1, bias_c2_sqrt;  // 1-b1^t, sqrt(1-b2^t)
  // nullable: [lr, bias_c1, bias_c2_sqrt] read from device memory at run time instead of the values
  // above -- a hipGraph replays its kernel arguments, and these three change every step
  const float* hyper;
};
struct RmsArgs {
  float lr, alpha, eps, wd, momentum;
  int centered;
};
struct AdagradArgs {
  float clr, eps, wd;  // clr = lr / (1 + (step-1)*lr_decay)
};
struct AdadeltaArgs {
  float lr, rho, eps, wd;
};

struct SgdOp {
  SgdArgs a;
  __device__ __forceinline__ void operator()(float& p, float g, float* s0, float*, float*) const {
    float d = g;
    if (a.wd != 0.f) d = fmaf(a.wd, p, d);
    if (a.momentum != 0.f) {
      float buf = a.first_step ? d : fmaf(a.momentum, *s0, (1.f - a.dampening) * d);
      *s0 = buf;
      d = a.nesterov ? fmaf(a.momentum, buf, d) : buf;
    }
    p = fmaf(-a.lr, d, p);
  }
};

struct AdamOp {
  AdamArgs a;
  __device__ __forceinline__ void operator()(float& p, float g, float* m, float* v,
                                             float* vmax) const {
    const float lr = a.hyper ? a.hyper[0] : a.lr;
    const float bc1 = a.hyper ? a.hyper[1] : a.bias_c1;
    const float bc2s = a.hyper ? a.hyper[2] : a.bias_c2_sqrt;
    if (a.wd != 0.f) {
      if (a.adamw)
        p = p * (1.f - lr * a.wd);
      else
        g = fmaf(a.wd, p, g);
    }
    float mm = fmaf(a.beta1, *m - g, g);  // lerp(g, m, beta1) == b1*m + (1-b1)*g
    float vv = fmaf(a.beta2, *v, (1.f - a.beta2) * g * g);
    *m = mm;
    *v = vv;
    float vd = vv;
    if (a.amsgrad) {
      vd = fmaxf(*vmax, vv);
      *vmax = vd;
    }
    float denom = sqrtf(vd) / bc2s + a.eps;
    p = p - (lr / bc1) * (mm / denom);
  }
};

struct RmsOp {
  RmsArgs a;
  __device__ __forceinline__ void operator()(float& p, float g, float* sq, float* buf,
                                             float* gavg) const {
    if (a.wd != 0.f) g = fmaf(a.wd, p, g);
    float s = fmaf(a.alpha, *sq, (1.f - a.alpha) * g * g);
    *sq = s;
    float avg;
    if (a.centered) {
      float ga = fmaf(a.alpha, *gavg, (1.f - a.alpha) * g);
      *gavg = ga;
      avg = sqrtf(fmaf(-ga, ga, s)) + a.eps;
    } else {
      avg = sqrtf(s) + a.eps;
    }
    if (a.momentum > 0.f) {
      float b = fmaf(a.momentum, *buf, g / avg);
      *buf = b;
      p = fmaf(-a.lr, b, p);
    } else {
      p = fmaf(-a.lr, g / avg, p);
    }
  }
};

struct AdagradOp {
  AdagradArgs a;
  __device__ __forceinline__ void operator()(float& p, float g, float* sum, float*, float*) const {
    if (a.wd != 0.f) g = fmaf(a.wd, p, g);
    float s = fmaf(g, g, *sum);
    *sum = s;
    p = p - a.clr * g / (sqrtf(s) + a.eps);
  }
};

struct AdadeltaOp {
  AdadeltaArgs a;
  __device__ __forceinline__ void operator()(float& p, float g, float* sq, float* acc,
                                             float*) const {
    if (a.wd != 0.f) g = fmaf(a.wd, p, g);
    float s = fmaf(a.rho, *sq, (1.f - a.rho) * g * g);
    *sq = s;
    float delta = sqrtf(*acc + a.eps) / sqrtf(s + a.eps) * g;
    *acc = fmaf(a.rho, *acc, (1.f - a.rho) * delta * delta);
    p = fmaf(-a.lr, delta, p);
  }
};

// One generic streaming kernel: 4 elements / lane / iteration, grid-stride.
//   g_scale_host * (*g_scale_dev) is the combined gradient scale (1/world * 1/agg * 1/loss_scale
//   * clip_coef); found_inf (device int) skips the update entirely (AMP overflow) without a host
//   round trip; out_model (optional) receives a low-precision copy of the updated master params
//   (O2-style bf16 model weights).
template <typename TG, typename TO, typename Op, int NS>
__global__ void __launch_bounds__(kBlock)
opt_kernel(float* __restrict__ p, const TG* __restrict__ g, float* __restrict__ s0,
           float* __restrict__ s1, float* __restrict__ s2, TO* __restrict__ out_model, int64_t n,
           float g_scale_host, const float* __restrict__ g_scale_dev,
           const int* __restrict__ found_inf, Op op) {
  if (found_inf != nullptr && *found_inf != 0) return;
  float gs = g_scale_host;
  if (g_scale_dev != nullptr) gs *= *g_scale_dev;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = Vec4<float>::load(p, i);
    float4 gv = Vec4<TG>::load(g, i);
    float4 a0 = make_float4(0, 0, 0, 0), a1 = a0, a2 = a0;
    if (NS > 0) a0 = Vec4<float>::load(s0, i);
    if (NS > 1) a1 = Vec4<float>::load(s1, i);
    if (NS > 2) a2 = Vec4<float>::load(s2, i);
    op(pv.x, gv.x * gs, &a0.x, &a1.x, &a2.x);
    op(pv.y, gv.y * gs, &a0.y, &a1.y, &a2.y);
    op(pv.z, gv.z * gs, &a0.z, &a1.z, &a2.z);
    op(pv.w, gv.w * gs, &a0.w, &a1.w, &a2.w);
    Vec4<float>::store(p, i, pv);
    if (NS > 0) Vec4<float>::store(s0, i, a0);
    if (NS > 1) Vec4<float>::store(s1, i, a1);
    if (NS > 2) Vec4<float>::store(s2, i, a2);
    if (out_model != nullptr) Vec4<TO>::store(out_model, i, pv);
  }
  // scalar tail (n % 4 elements) handled by the first threads of block 0
  if (blockIdx.x == 0) {
    int64_t t = (n4 << 2) + threadIdx.x;
    if (t < n) {
      float pv = p[t];
      float a0 = NS > 0 ? s0[t] : 0.f, a1 = NS > 1 ? s1[t] : 0.f, a2 = NS > 2 ? s2[t] : 0.f;
      op(pv, to_f(g[t]) * gs, &a0, &a1, &a2);
      p[t] = pv;
      if (NS > 0) s0[t] = a0;
      if (NS > 1) s1[t] = a1;
      if (NS > 2) s2[t] = a2;
      if (out_model != nullptr) out_model[t] = from_f<TO>(pv);
    }
  }
}

template <typename Op, int NS>
int launch_opt(hipStream_t st, int g_dtype, int out_dtype, float* p, const void* g, float* s0,
               float* s1, float* s2, void* out_model, int64_t n, float gsh, const float* gsd,
               const int* found_inf, Op op) {
  if (n <= 0) return 0;
  int grid = grid_for((n + 3) / 4);
#define DET_OPT_LAUNCH(TG, TO)                                                                  \
  hipLaunchKernelGGL((opt_kernel<TG, TO, Op, NS>), dim3(grid), dim3(kBlock), 0, st, p,         \
                     static_cast<const TG*>(g), s0, s1, s2, static_cast<TO*>(out_model), n, gsh, \
                     gsd, found_inf, op)
  // out_model dtype only matters when out_model != nullptr
  if (out_dtype == kF16) {
    if (g_dtype == kF32) DET_OPT_LAUNCH(float, __half);
    else if (g_dtype == kBF16) DET_OPT_LAUNCH(__hip_bfloat16, __half);
    else DET_OPT_LAUNCH(__half, __half);
  } else {
    if (g_dtype == kF32) DET_OPT_LAUNCH(float, __hip_bfloat16);
    else if (g_dtype == kBF16) DET_OPT_LAUNCH(__hip_bfloat16, __hip_bfloat16);
    else DET_OPT_LAUNCH(__half, __hip_bfloat16);
  }
#undef DET_OPT_LAUNCH
  return static_cast<int>(hipGetLastError());
}

// ------------------------------------------------------------------------------------------
// scale + cast (gradient compression pack/unpack, K1/K2; aggregation divide K5)
// ------------------------------------------------------------------------------------------
template <typename TI, typename TO>
__global__ void __launch_bounds__(kBlock)
scale_cast_kernel(const TI* __restrict__ in, TO* __restrict__ out, int64_t n, float scale,
                  const float* __restrict__ scale_dev) {
  float s = scale;
  if (scale_dev != nullptr) s *= *scale_dev;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = Vec4<TI>::load(in, i);
    v.x *= s; v.y *= s; v.z *= s; v.w *= s;
    Vec4<TO>::store(out, i, v);
  }
  if (blockIdx.x == 0) {
    int64_t t = (n4 << 2) + threadIdx.x;
    if (t < n) out[t] = from_f<TO>(to_f(in[t]) * s);
  }
}

// ------------------------------------------------------------------------------------------
// sum-of-squares partials (grad-norm clipping K6 and AMP non-finite detection K3)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(kBlock)
sumsq_kernel(const T* __restrict__ x, int64_t n, float* __restrict__ partials) {
  float acc = 0.f;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = Vec4<T>::load(x, i);
    acc = fmaf(v.x, v.x, acc);
    acc = fmaf(v.y, v.y, acc);
    acc = fmaf(v.z, v.z, acc);
    acc = fmaf(v.w, v.w, acc);
  }
  if (blockIdx.x == 0) {
    int64_t t = (n4 << 2) + threadIdx.x;
    if (t < n) {
      float v = to_f(x[t]);
      acc = fmaf(v, v, acc);
    }
  }
  float s = block_sum(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// Single-block finalize: norm = sqrt(sum(partials)) * pre_scale;
// found_inf |= !finite(norm); clip_coef = min(1, max_norm / (norm + 1e-6)) (1 if max_norm <= 0).
__global__ void __launch_bounds__(kBlock)
norm_finalize_kernel(const float* __restrict__ partials, int nparts, float pre_scale,
                     float max_norm, float* __restrict__ norm_out, int* __restrict__ found_inf,
                     float* __restrict__ clip_coef) {
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += partials[i];
  float s = block_sum(acc);
  if (threadIdx.x == 0) {
    float norm = sqrtf(s) * pre_scale;
    bool bad = !isfinite(norm);
    if (norm_out != nullptr) norm_out[0] = norm;
    if (found_inf != nullptr && bad) found_inf[0] = 1;
    if (clip_coef != nullptr) {
      float c = 1.f;
      if (max_norm > 0.f && !bad) c = fminf(1.f, max_norm / (norm + 1e-6f));
      clip_coef[0] = c;
    }
  }
}

// In-place scale with non-finite detection (AMP unscale before a user clip function).
template <typename T>
__global__ void __launch_bounds__(kBlock)
unscale_check_kernel(T* __restrict__ x, int64_t n, float scale, int* __restrict__ found_inf) {
  bool bad = false;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = Vec4<T>::load(x, i);
    v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
    bad |= !isfinite(v.x) | !isfinite(v.y) | !isfinite(v.z) | !isfinite(v.w);
    Vec4<T>::store(x, i, v);
  }
  if (blockIdx.x == 0) {
    int64_t t = (n4 << 2) + threadIdx.x;
    if (t < n) {
      float v = to_f(x[t]) * scale;
      bad |= !isfinite(v);
      x[t] = from_f<T>(v);
    }
  }
  // one store per wave that saw a non-finite value (benign race: all writers store 1)
  if (__any(bad) && (threadIdx.x & 63) == 0) found_inf[0] = 1;
}

// ------------------------------------------------------------------------------------------
// Multi-tensor copy (+scale, +cast) through a device-resident pointer table.
// table layout (int64): [src_ptr, dst_ptr, numel] x ntensors.  blockIdx.y = tensor.
// Used for coalescing buffers / state for broadcast (SURVEY C-2, C-3) and for parameters that
// could not be placed in an arena.
// ------------------------------------------------------------------------------------------
template <typename TI, typename TO>
__global__ void __launch_bounds__(kBlock)
mt_copy_kernel(const int64_t* __restrict__ table, float scale) {
  const int64_t* row = table + 3 * blockIdx.y;
  const TI* src = reinterpret_cast<const TI*>(row[0]);
  TO* dst = reinterpret_cast<TO*>(row[1]);
  const int64_t n = row[2];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // vector path only if both ends are 16-byte aligned for 4 elements of each type
  const bool aligned = ((row[0] % (4 * sizeof(TI))) == 0) && ((row[1] % (4 * sizeof(TO))) == 0);
  int64_t start = 0;
  if (aligned) {
    const int64_t n4 = n >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
      float4 v = Vec4<TI>::load(src, i);
      v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
      Vec4<TO>::store(dst, i, v);
    }
    start = n4 << 2;
  }
  for (int64_t i = start + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = from_f<TO>(to_f(src[i]) * scale);
}

// ------------------------------------------------------------------------------------------
// Input pipeline: uint8 NHWC images -> normalized bf16/f32 NHWC (== channels_last NCHW).
// 16 bytes of u8 per lane per iteration.  mean/inv_std are per-channel (C <= 4), in __constant__
// -like kernel args.
// ------------------------------------------------------------------------------------------
struct ChanParams {
  float mean[4];
  float inv_std[4];
};

// uint8 NHWC (C <= 3) -> bf16 NHWC with the channels padded to 4 (zero 4th channel): one 8-B store
// per pixel, the layout the ResNet stem implicit GEMM (det_conv.hip GM_STEM) reads.
__global__ void __launch_bounds__(kBlock)
u8_normalize_pad4_kernel(const uint8_t* __restrict__ in, ushort4* __restrict__ out, int64_t npix, int C,
                         ChanParams cp) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += stride) {
    float f[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < C; ++c) f[c] = (static_cast<float>(in[p * C + c]) - cp.mean[c]) * cp.inv_std[c];
    ushort4 o;
    o.x = __builtin_bit_cast(unsigned short, static_cast<__bf16>(f[0]));
    o.y = __builtin_bit_cast(unsigned short, static_cast<__bf16>(f[1]));
    o.z = __builtin_bit_cast(unsigned short, static_cast<__bf16>(f[2]));
    o.w = __builtin_bit_cast(unsigned short, static_cast<__bf16>(f[3]));
    out[p] = o;
  }
}

// C == 3, npix % 4 == 0: four pixels per thread -- their 12 input bytes as three aligned 32-bit loads
// and their 32 output bytes as two 16-B stores (the per-pixel kernel issues three byte loads and an
// 8-B store per pixel: 2.2 TB/s at the ResNet-50 batch, profiles/r5_resnet50_steady.csv).  Same
// arithmetic per element, so bit-equal to it.
__global__ void __launch_bounds__(kBlock)
u8_normalize_pad4_c3x4_kernel(const uint32_t* __restrict__ in, uint4* __restrict__ out, int64_t nquad, ChanParams cp) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nquad; q += stride) {
    const uint32_t w[3] = {in[3 * q], in[3 * q + 1], in[3 * q + 2]};
    uint32_t o[8];
#pragma unroll
    for (int px = 0; px < 4; ++px) {
      unsigned short h[4];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int b = px * 3 + c;
        const float v = static_cast<float>((w[b >> 2] >> (8 * (b & 3))) & 0xffu);
        h[c] = __builtin_bit_cast(unsigned short, static_cast<__bf16>((v - cp.mean[c]) * cp.inv_std[c]));
      }
      h[3] = __builtin_bit_cast(unsigned short, static_cast<__bf16>(0.f));
      o[2 * px] = static_cast<uint32_t>(h[0]) | (static_cast<uint32_t>(h[1]) << 16);
      o[2 * px + 1] = static_cast<uint32_t>(h[2]) | (static_cast<uint32_t>(h[3]) << 16);
    }
    out[2 * q] = make_uint4(o[0], o[1], o[2], o[3]);
    out[2 * q + 1] = make_uint4(o[4], o[5], o[6], o[7]);
  }
}

template <typename TO>
__global__ void __launch_bounds__(kBlock)
u8_normalize_kernel(const uint8_t* __restrict__ in, TO* __restrict__ out, int64_t n, int C,
                    ChanParams cp) {
  const int64_t n16 = n >> 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    uint4 raw = reinterpret_cast<const uint4*>(in)[i];
    const uint8_t* b = reinterpret_cast<const uint8_t*>(&raw);
    int c = static_cast<int>((i * 16) % C);
    float f[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      f[j] = (static_cast<float>(b[j]) - cp.mean[c]) * cp.inv_std[c];
      c = (c + 1 == C) ? 0 : c + 1;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      Vec4<TO>::store(out, i * 4 + q, make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]));
  }
  if (blockIdx.x == 0) {
    int64_t t = (n16 << 4) + threadIdx.x;
    if (t < n) {
      int c = static_cast<int>(t % C);
      out[t] = from_f<TO>((static_cast<float>(in[t]) - cp.mean[c]) * cp.inv_std[c]);
    }
  }
}


// ------------------------------------------------------------------------------------------
// Shard reduction for the fp32-accumulating gradient reduce-scatter (parallel/ddp.py): after an
// all-to-all over xGMI each rank holds `rows` low-precision copies of its own 1/rows shard of a
// gradient bucket, one per peer.  out[i] = scale * sum_r in[r * n + i], accumulated in fp32 and
// rounded ONCE (a ring all-reduce in bf16 rounds after every hop).  4 elements per lane per
// row; rows (= world size) is small, so the row loop is fully in registers.
// ------------------------------------------------------------------------------------------
template <typename TI, typename TO>
__global__ void __launch_bounds__(kBlock)
sum_rows_kernel(const TI* __restrict__ in, TO* __restrict__ out, int rows, int64_t n, float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = 0; r < rows; ++r) {
      float4 v = Vec4<TI>::load(in + r * n, i);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    acc.x *= scale; acc.y *= scale; acc.z *= scale; acc.w *= scale;
    Vec4<TO>::store(out, i, acc);
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int r = 0; r < rows; ++r) acc += to_f(in[r * n + i]);
    out[i] = from_f<TO>(acc * scale);
  }
}

}  // namespace

// ============================================================================================
// C ABI
// ============================================================================================
extern "C" {

int det_abi_version() { return 21; }

int det_sgd_step(void* stream, int g_dtype, int out_dtype, float* p, const void* g, float* buf,
                 void* out_model, int64_t n, float lr, float momentum, float dampening, float wd,
                 int nesterov, int first_step, float g_scale, const float* g_scale_dev,
                 const int* found_inf) {
  SgdOp op{{lr, momentum, dampening, wd, nesterov, first_step}};
  if (momentum != 0.f)
    return launch_opt<SgdOp, 1>((hipStream_t)stream, g_dtype, out_dtype, p, g, buf, nullptr,
                                nullptr, out_model, n, g_scale, g_scale_dev, found_inf, op);
  return launch_opt<SgdOp, 0>((hipStream_t)stream, g_dtype, out_dtype, p, g, nullptr, nullptr,
                              nullptr, out_model, n, g_scale, g_scale_dev, found_inf, op);
}

int det_adam_step(void* stream, int g_dtype, int out_dtype, float* p, const void* g, float* m,
                  float* v, float* vmax, void* out_model, int64_t n, float lr, float beta1,
                  float beta2, float eps, float wd, int adamw, int amsgrad, float bias_c1,
                  float bias_c2_sqrt, float g_scale, const float* g_scale_dev,
                  const int* found_inf, const float* hyper) {
  AdamOp op{{lr, beta1, beta2, eps, wd, adamw, amsgrad, bias_c1, bias_c2_sqrt, hyper}};
  if (amsgrad)
    return launch_opt<AdamOp, 3>((hipStream_t)stream, g_dtype, out_dtype, p, g, m, v, vmax,
                                 out_model, n, g_scale, g_scale_dev, found_inf, op);
  return launch_opt<AdamOp, 2>((hipStream_t)stream, g_dtype, out_dtype, p, g, m, v, nullptr,
                               out_model, n, g_scale, g_scale_dev, found_inf, op);
}

int det_rmsprop_step(void* stream, int g_dtype, int out_dtype, float* p, const void* g,
                     float* square_avg, float* momentum_buf, float* grad_avg, void* out_model,
                     int64_t n, float lr, float alpha, float eps, float wd, float momentum,
                     int centered, float g_scale, const float* g_scale_dev,
                     const int* found_inf) {
  RmsOp op{{lr, alpha, eps, wd, momentum, centered}};
  return launch_opt<RmsOp, 3>((hipStream_t)stream, g_dtype, out_dtype, p, g, square_avg,
                              momentum_buf, grad_avg, out_model, n, g_scale, g_scale_dev,
                              found_inf, op);
}

int det_adagrad_step(void* stream, int g_dtype, int out_dtype, float* p, const void* g,
                     float* sum, void* out_model, int64_t n, float clr, float eps, float wd,
                     float g_scale, const float* g_scale_dev, const int* found_inf) {
  AdagradOp op{{clr, eps, wd}};
  return launch_opt<AdagradOp, 1>((hipStream_t)stream, g_dtype, out_dtype, p, g, sum, nullptr,
                                  nullptr, out_model, n, g_scale, g_scale_dev, found_inf, op);
}

int det_adadelta_step(void* stream, int g_dtype, int out_dtype, float* p, const void* g,
                      float* square_avg, float* acc_delta, void* out_model, int64_t n, float lr,
                      float rho, float eps, float wd, float g_scale, const float* g_scale_dev,
                      const int* found_inf) {
  AdadeltaOp op{{lr, rho, eps, wd}};
  return launch_opt<AdadeltaOp, 2>((hipStream_t)stream, g_dtype, out_dtype, p, g, square_avg,
                                   acc_delta, nullptr, out_model, n, g_scale, g_scale_dev,
                                   found_inf, op);
}

int det_scale_cast(void* stream, const void* in, int in_dtype, void* out, int out_dtype,
                   int64_t n, float scale, const float* scale_dev) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  int grid = grid_for((n + 3) / 4);
#define DET_SC(TI, TO)                                                                       \
  hipLaunchKernelGGL((scale_cast_kernel<TI, TO>), dim3(grid), dim3(kBlock), 0, st,            \
                     static_cast<const TI*>(in), static_cast<TO*>(out), n, scale, scale_dev)
#define DET_SC_OUT(TI)                          \
  if (out_dtype == kF32) DET_SC(TI, float);     \
  else if (out_dtype == kBF16) DET_SC(TI, __hip_bfloat16); \
  else DET_SC(TI, __half);
  if (in_dtype == kF32) { DET_SC_OUT(float) }
  else if (in_dtype == kBF16) { DET_SC_OUT(__hip_bfloat16) }
  else { DET_SC_OUT(__half) }
#undef DET_SC_OUT
#undef DET_SC
  return static_cast<int>(hipGetLastError());
}

// out[0:n] = scale * sum_{r<rows} in[r*n : (r+1)*n]  (fp32 accumulation).  n % 4 == 0 is the
// fast path; `in` rows must be 8-byte aligned for 16-bit types (callers pass arena slices).
int det_sum_rows(void* stream, const void* in, int in_dtype, void* out, int out_dtype, int rows,
                 int64_t n, float scale) {
  if (n <= 0 || rows <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  int grid = grid_for((n + 3) / 4);
#define DET_SR(TI, TO)                                                                       \
  hipLaunchKernelGGL((sum_rows_kernel<TI, TO>), dim3(grid), dim3(kBlock), 0, st,              \
                     static_cast<const TI*>(in), static_cast<TO*>(out), rows, n, scale)
#define DET_SR_OUT(TI)                          \
  if (out_dtype == kF32) DET_SR(TI, float);     \
  else if (out_dtype == kBF16) DET_SR(TI, __hip_bfloat16); \
  else DET_SR(TI, __half);
  if (in_dtype == kF32) { DET_SR_OUT(float) }
  else if (in_dtype == kBF16) { DET_SR_OUT(__hip_bfloat16) }
  else { DET_SR_OUT(__half) }
#undef DET_SR_OUT
#undef DET_SR
  return static_cast<int>(hipGetLastError());
}

// Number of partial slots det_sumsq_partials writes for n elements.
int det_sumsq_num_partials(int64_t n) { return grid_for((n + 3) / 4); }

int det_sumsq_partials(void* stream, const void* x, int dtype, int64_t n, float* partials) {
  hipStream_t st = (hipStream_t)stream;
  int grid = grid_for((n + 3) / 4);
  if (dtype == kF32)
    hipLaunchKernelGGL(sumsq_kernel<float>, dim3(grid), dim3(kBlock), 0, st,
                       static_cast<const float*>(x), n, partials);
  else if (dtype == kBF16)
    hipLaunchKernelGGL(sumsq_kernel<__hip_bfloat16>, dim3(grid), dim3(kBlock), 0, st,
                       static_cast<const __hip_bfloat16*>(x), n, partials);
  else
    hipLaunchKernelGGL(sumsq_kernel<__half>, dim3(grid), dim3(kBlock), 0, st,
                       static_cast<const __half*>(x), n, partials);
  return static_cast<int>(hipGetLastError());
}

int det_norm_finalize(void* stream, const float* partials, int nparts, float pre_scale,
                      float max_norm, float* norm_out, int* found_inf, float* clip_coef) {
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(1), dim3(kBlock), 0, (hipStream_t)stream,
                     partials, nparts, pre_scale, max_norm, norm_out, found_inf, clip_coef);
  return static_cast<int>(hipGetLastError());
}

int det_unscale_check(void* stream, void* x, int dtype, int64_t n, float scale, int* found_inf) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  int grid = grid_for((n + 3) / 4);
  if (dtype == kF32)
    hipLaunchKernelGGL(unscale_check_kernel<float>, dim3(grid), dim3(kBlock), 0, st,
                       static_cast<float*>(x), n, scale, found_inf);
  else if (dtype == kBF16)
    hipLaunchKernelGGL(unscale_check_kernel<__hip_bfloat16>, dim3(grid), dim3(kBlock), 0, st,
                       static_cast<__hip_bfloat16*>(x), n, scale, found_inf);
  else
    hipLaunchKernelGGL(unscale_check_kernel<__half>, dim3(grid), dim3(kBlock), 0, st,
                       static_cast<__half*>(x), n, scale, found_inf);
  return static_cast<int>(hipGetLastError());
}

int det_mt_copy(void* stream, const int64_t* table_dev, int ntensors, int in_dtype,
                int out_dtype, int64_t max_numel, float scale) {
  if (ntensors <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  int64_t gx = (max_numel / 4 + kBlock - 1) / kBlock;
  if (gx < 1) gx = 1;
  if (gx > 64) gx = 64;
  dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(ntensors));
#define DET_MT(TI, TO) \
  hipLaunchKernelGGL((mt_copy_kernel<TI, TO>), grid, dim3(kBlock), 0, st, table_dev, scale)
#define DET_MT_OUT(TI)                          \
  if (out_dtype == kF32) DET_MT(TI, float);     \
  else if (out_dtype == kBF16) DET_MT(TI, __hip_bfloat16); \
  else DET_MT(TI, __half);
  if (in_dtype == kF32) { DET_MT_OUT(float) }
  else if (in_dtype == kBF16) { DET_MT_OUT(__hip_bfloat16) }
  else { DET_MT_OUT(__half) }
#undef DET_MT_OUT
#undef DET_MT
  return static_cast<int>(hipGetLastError());
}

int det_u8_normalize(void* stream, const uint8_t* in, void* out, int out_dtype, int64_t n, int C,
                     const float* mean, const float* stdv) {
  if (n <= 0) return 0;
  if (C < 1 || C > 4) return -1;
  ChanParams cp;
  for (int c = 0; c < 4; ++c) {
    cp.mean[c] = c < C ? mean[c] : 0.f;
    cp.inv_std[c] = c < C ? 1.f / stdv[c] : 1.f;
  }
  hipStream_t st = (hipStream_t)stream;
  int grid = grid_for((n + 15) / 16);
  if (out_dtype == kBF16)
    hipLaunchKernelGGL(u8_normalize_kernel<__hip_bfloat16>, dim3(grid), dim3(kBlock), 0, st, in,
                       static_cast<__hip_bfloat16*>(out), n, C, cp);
  else if (out_dtype == kF16)
    hipLaunchKernelGGL(u8_normalize_kernel<__half>, dim3(grid), dim3(kBlock), 0, st, in,
                       static_cast<__half*>(out), n, C, cp);
  else
    hipLaunchKernelGGL(u8_normalize_kernel<float>, dim3(grid), dim3(kBlock), 0, st, in,
                       static_cast<float*>(out), n, C, cp);
  return static_cast<int>(hipGetLastError());
}


int det_u8_normalize_pad4(void* stream, const uint8_t* in, void* out, int out_dtype, int64_t npix, int C,
                          const float* mean, const float* stdv) {
  if (npix <= 0) return 0;
  if (C < 1 || C > 3 || out_dtype != kBF16) return -1;
  ChanParams cp;
  for (int c = 0; c < 4; ++c) {
    cp.mean[c] = c < C ? mean[c] : 0.f;
    cp.inv_std[c] = c < C ? 1.f / stdv[c] : 1.f;
  }
  hipStream_t st = (hipStream_t)stream;
  if (C == 3 && npix % 4 == 0 && (reinterpret_cast<uintptr_t>(in) & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
    const int64_t nquad = npix / 4;
    hipLaunchKernelGGL(u8_normalize_pad4_c3x4_kernel, dim3(grid_for(nquad)), dim3(kBlock), 0, st,
                       reinterpret_cast<const uint32_t*>(in), static_cast<uint4*>(out), nquad, cp);
    return static_cast<int>(hipGetLastError());
  }
  hipLaunchKernelGGL(u8_normalize_pad4_kernel, dim3(grid_for(npix)), dim3(kBlock), 0, st, in,
                     static_cast<ushort4*>(out), npix, C, cp);
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
