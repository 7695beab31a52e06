// det_pool.hip — 3x3 / stride-2 / pad-1 max pooling (the ResNet stem) for channels_last bf16/fp32.
//
// Why this exists: torch's NHWC max_pool2d stores an int64 argmax per output element (8 B next to
// a 2-B bf16 value) and its backward zero-fills the input gradient and scatters into it: 1.7 ms per
// ResNet-50 step at batch 512 (profiles/r1_resnet50_bs512_o2_steady.csv, 'max_pool_*_nhwc'), at
// 1.2-2.9 TB/s.  Here:
//   forward  one thread = 8 channels of one output pixel: 9 x 16-B loads, per-channel max and the
//            winning window slot (0..8) as ONE byte;
//   backward one thread = 8 channels of one INPUT pixel: it gathers the (at most 2 x 2) windows
//            that contain it and adds dy where the window's argmax byte names it — no zero fill,
//            no atomics, every input-gradient element written exactly once.
// Tie-breaking matches torch (first maximum in row-major window order wins; NaN propagates).
//
// Reference parity: torchvision ResNet stem nn.MaxPool2d(3, 2, 1) used by the reference's
// examples/computer_vision (SURVEY §6 north-star model).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float bf2f(unsigned short u) { return __uint_as_float(static_cast<uint32_t>(u) << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));
}

typedef unsigned char uc8 __attribute__((ext_vector_type(8)));

template <typename T> struct Vec8;
template <> struct Vec8<unsigned short> {  // 16 B as four 32-bit words (two bf16 each)
  static __device__ __forceinline__ void load(const unsigned short* p, float (&v)[8]) {
    const uint4 r = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(w[k] << 16);
      v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void store(unsigned short* p, const float (&v)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = static_cast<uint32_t>(f2bf(v[2 * k])) | (static_cast<uint32_t>(f2bf(v[2 * k + 1])) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

struct PoolGeom {
  int N, H, W, C, Ho, Wo;
};

// BNP: x is the input of the training BatchNorm + ReLU whose output is pooled (the ResNet stem); the
// pool applies relu(x * scale + shift), rounded to bf16 exactly like det_norm.hip's apply, to each
// window value, so that activation is never written to HBM or read back.
template <typename T, bool BNP = false>
__global__ void __launch_bounds__(kThreads) maxpool_fwd(const T* __restrict__ x, T* __restrict__ y,
                                                        uint8_t* __restrict__ idx, PoolGeom g, int nvec,
                                                        const float* __restrict__ bn_scale = nullptr,
                                                        const float* __restrict__ bn_shift = nullptr) {
  const int cv = g.C / 8;
  // 32-bit index math (nvec < 2^31, checked by the host): 64-bit division is a long software sequence
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < nvec; i += gridDim.x * kThreads) {
    int t = i;
    const int c8 = t % cv; t /= cv;
    const int ow = t % g.Wo; t /= g.Wo;
    const int oh = t % g.Ho;
    const int n = t / g.Ho;
    // torch semantics: start from -inf with the window's first valid slot, take v if v > max
    // or v is NaN (the first NaN then sticks)
    const uint8_t slot0 = static_cast<uint8_t>(3 * (oh == 0 ? 1 : 0) + (ow == 0 ? 1 : 0));
    float bsc[8], bsh[8];
    if constexpr (BNP) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bsc[j] = bn_scale[8 * c8 + j];
        bsh[j] = bn_shift[8 * c8 + j];
      }
    }
    float m[8];
    uint8_t a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = -INFINITY;
      a[j] = slot0;
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int h = 2 * oh - 1 + kh;
      if (h < 0 || h >= g.H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int w = 2 * ow - 1 + kw;
        if (w < 0 || w >= g.W) continue;
        float v[8];
        Vec8<T>::load(x + ((static_cast<int64_t>(n) * g.H + h) * g.W + w) * g.C + 8 * c8, v);
        if constexpr (BNP) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[j] = __uint_as_float(static_cast<uint32_t>(f2bf(fmaxf(__fmaf_rn(v[j], bsc[j], bsh[j]), 0.f))) << 16);
        }
        const uint8_t slot = static_cast<uint8_t>(3 * kh + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (v[j] > m[j] || (__builtin_isnan(v[j]) && !__builtin_isnan(m[j]))) {
            m[j] = v[j];
            a[j] = slot;
          }
        }
      }
    }
    Vec8<T>::store(y + static_cast<int64_t>(i) * 8, m);
    uc8 av;
#pragma unroll
    for (int j = 0; j < 8; ++j) av[j] = a[j];
    *reinterpret_cast<uc8*>(idx + static_cast<int64_t>(i) * 8) = av;
  }
}

// Row-staged forward (the default where three input rows fit LDS): one block = pooled row oh of one
// image; the input rows 2 oh - 1 .. 2 oh + 1 are staged once into LDS (BNP: normalised + ReLU'd
// and rounded while staging, once per element instead of once per window that reads it), then each
// output vector takes its nine window values from LDS in maxpool_fwd's order (same max, same argmax
// byte, same tie and NaN handling).  The gather above re-fetches every input vector ~2.25 times
// through the texture path.  Consecutive pooled rows (sharing an input row) run on one XCD.
template <typename T, bool BNP>
__global__ void __launch_bounds__(kThreads) maxpool_fwd_rows(const T* __restrict__ x, T* __restrict__ y,
                                                             uint8_t* __restrict__ idx, PoolGeom g, int nblk,
                                                             const float* __restrict__ bn_scale,
                                                             const float* __restrict__ bn_shift) {
  extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
  T* xs = reinterpret_cast<T*>(psm);  // [3][W][C]
  const int cv = g.C / 8, rowv = g.W * cv;
  const int b = blockIdx.x, per = nblk / 8, rem = nblk % 8, xcd = b % 8, bi = b / 8;
  const int blk = xcd < rem ? xcd * (per + 1) + bi : rem * (per + 1) + (xcd - rem) * per + bi;
  const int n = blk / g.Ho, oh = blk - n * g.Ho;
  const int hlo = max(0, 2 * oh - 1), hhi = min(g.H - 1, 2 * oh + 1);  // valid input rows
  const int nv = (hhi - hlo + 1) * rowv;
  const int64_t xbase = static_cast<int64_t>(n * g.H + hlo) * g.W * g.C;
  const int c8s = threadIdx.x % cv;  // the staging thread's channel group is fixed (kThreads % cv == 0)
  float bsc[8], bsh[8];
  if constexpr (BNP) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bsc[j] = bn_scale[8 * c8s + j];
      bsh[j] = bn_shift[8 * c8s + j];
    }
  }
  // LDS row r holds input row 2 oh - 1 + r
  const int r0 = hlo - (2 * oh - 1);
#pragma unroll 4
  for (int v = threadIdx.x; v < nv; v += kThreads) {
    float val[8];
    Vec8<T>::load(x + xbase + static_cast<int64_t>(v) * 8, val);
    if constexpr (BNP) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        val[j] = __uint_as_float(static_cast<uint32_t>(f2bf(fmaxf(__fmaf_rn(val[j], bsc[j], bsh[j]), 0.f))) << 16);
    }
    Vec8<T>::store(xs + (static_cast<int64_t>(r0) * rowv + v) * 8, val);
  }
  __syncthreads();
  const int nout = g.Wo * cv;
  for (int i = threadIdx.x; i < nout; i += kThreads) {
    const int ow = i / cv, c8 = i - ow * cv;
    const uint8_t slot0 = static_cast<uint8_t>(3 * (oh == 0 ? 1 : 0) + (ow == 0 ? 1 : 0));
    float m[8];
    uint8_t a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = -INFINITY;
      a[j] = slot0;
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int h = 2 * oh - 1 + kh;
      if (h < 0 || h >= g.H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int w = 2 * ow - 1 + kw;
        if (w < 0 || w >= g.W) continue;
        float v[8];
        Vec8<T>::load(xs + (static_cast<int64_t>(kh) * rowv + w * cv + c8) * 8, v);
        const uint8_t slot = static_cast<uint8_t>(3 * kh + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (v[j] > m[j] || (__builtin_isnan(v[j]) && !__builtin_isnan(m[j]))) {
            m[j] = v[j];
            a[j] = slot;
          }
        }
      }
    }
    const int64_t o = (static_cast<int64_t>(n * g.Ho + oh) * g.Wo + ow) * g.C + 8 * c8;
    Vec8<T>::store(y + o, m);
    uc8 av;
#pragma unroll
    for (int j = 0; j < 8; ++j) av[j] = a[j];
    *reinterpret_cast<uc8*>(idx + o) = av;
  }
}

// One block = kBwdRows consecutive INPUT pixels (all channels); thread t owns channel group
// t % (C/8) of pixels t / (C/8), + 256 / (C/8), ...  Pixel coordinates in 32-bit math (the input has
// < 2^31 pixels; 64-bit division is a long software sequence per element).
// kTwo: a second upstream gradient dy2 of the pooled output (a linked projection shortcut that also
// reads it, ops/norm.py linked_conv2d) is summed in the gather instead of by a separate add pass.
// BNB: the pooled tensor is the output of a training BatchNorm + ReLU (the ResNet stem): the gathered
// gradient is masked with relu'(x * scale + shift) (x = the BN input) and each block writes the BN
// backward's partial sums psum = sum d, psumx = sum d (x - mean) over its pixels -- the BN backward
// is then a finalize and an apply (ops/norm.py fused_bwd), with no partial pass over the tensor.
constexpr int kBwdRows = 512;

struct BnbArgs {
  const unsigned short* x;  // BN input [pixels, C]
  const float* mean;
  const float* scale;
  const float* shift;
  float* psum;   // [blocks, C]
  float* psumx;  // [blocks, C]
};

template <typename T, bool kTwo, bool BNB>
__global__ void __launch_bounds__(kThreads) maxpool_bwd(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                        const uint8_t* __restrict__ idx, T* __restrict__ dx, PoolGeom g,
                                                        BnbArgs bn) {
  const int cv = g.C / 8;
  const int c8 = threadIdx.x % cv, lanes = kThreads / cv;
  const int npix = g.N * g.H * g.W;
  const int p0 = blockIdx.x * kBwdRows;
  const int p1 = min(npix, p0 + kBwdRows);
  float mu[8], sc[8], sh[8], s1[8], s2[8];
  if constexpr (BNB) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mu[j] = bn.mean[8 * c8 + j];
      sc[j] = bn.scale[8 * c8 + j];
      sh[j] = bn.shift[8 * c8 + j];
      s1[j] = 0.f;
      s2[j] = 0.f;
    }
  }
  for (int p = p0 + static_cast<int>(threadIdx.x) / cv; p < p1; p += lanes) {
    const int w = p % g.W;
    const int t = p / g.W;
    const int h = t % g.H;
    const int n = t / g.H;
    const int64_t e = static_cast<int64_t>(p) * g.C + 8 * c8;
    // every operand of the (at most 2 x 2) windows that contain this pixel is loaded up front, with no
    // branch on loaded data (an argmax test before the dy load made each window two dependent
    // round trips): windows oh with 2*oh-1 <= h <= 2*oh+1 -> oh in {(h+1)/2 - d : d = 0,1}
    int64_t off[4];
    bool ok[4];
    uint8_t me[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oh = (h + 1) / 2 - (q >> 1), kh = h - (2 * oh - 1);
      const int ow = (w + 1) / 2 - (q & 1), kw = w - (2 * ow - 1);
      ok[q] = oh >= 0 && oh < g.Ho && kh >= 0 && kh <= 2 && ow >= 0 && ow < g.Wo && kw >= 0 && kw <= 2;
      off[q] = ok[q] ? (static_cast<int64_t>(n * g.Ho + oh) * g.Wo + ow) * g.C + 8 * c8 : 0;
      me[q] = static_cast<uint8_t>(3 * kh + kw);
    }
    uc8 av[4];
    float d[4][8];
    float xv[8];
    if constexpr (BNB) Vec8<unsigned short>::load(bn.x + e, xv);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (ok[q]) {
        av[q] = *reinterpret_cast<const uc8*>(idx + off[q]);
        Vec8<T>::load(dy + off[q], d[q]);
        if constexpr (kTwo) {
          float d2[8];
          Vec8<T>::load(dy2 + off[q], d2);
#pragma unroll
          for (int j = 0; j < 8; ++j) d[q][j] += d2[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          av[q][j] = 0xff;
          d[q][j] = 0.f;
        }
      }
    }
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) a += av[q][j] == me[q] ? d[q][j] : 0.f;
      acc[j] = a;
    }
    if constexpr (BNB) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float dm = __fmaf_rn(xv[j], sc[j], sh[j]) > 0.f ? acc[j] : 0.f;
        const float dr = __uint_as_float(static_cast<uint32_t>(f2bf(dm)) << 16);  // what the apply reads back
        acc[j] = dr;
        s1[j] += dr;
        s2[j] += dr * (xv[j] - mu[j]);
      }
    }
    Vec8<T>::store(dx + e, acc);
  }
  if constexpr (BNB) {
    __shared__ float red[kThreads][17];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[threadIdx.x][j] = s1[j];
      red[threadIdx.x][8 + j] = s2[j];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < g.C; c += kThreads) {  // channel c = 8 * group + j
      const int grp = c / 8, j = c % 8;
      float t1 = 0.f, t2 = 0.f;
      for (int l = 0; l < lanes; ++l) {
        t1 += red[l * cv + grp][j];
        t2 += red[l * cv + grp][8 + j];
      }
      bn.psum[static_cast<int64_t>(blockIdx.x) * g.C + c] = t1;
      bn.psumx[static_cast<int64_t>(blockIdx.x) * g.C + c] = t2;
    }
  }
}

// Row-staged variant (the default where the window rows fit LDS): one block = one pooled row oh of
// one image, i.e. the input rows 2 oh and 2 oh + 1, which read only the window rows oh and oh + 1.
// Those two rows of dy (+ dy2, summed in fp32) and of the argmax bytes are staged once into LDS with
// coalesced 16-B loads; each input pixel then gathers its (at most 2 x 2) windows from LDS.  The
// per-pixel gather above issues ~12 vector-memory instructions per 8 input pixels (8-B argmax and
// 16-B gradient pieces of up to four windows, re-fetched by the neighbouring pixels through the
// texture path) -- 2.2 TB/s at the ResNet stem; here a block issues ~3 per 8 pixels, the rest is LDS.
// Summation order per element is the gather kernel's (bit-identical results).  Blocks are mapped so
// that consecutive pooled rows (which share a window row) run on the same XCD (its own L2).
// BN partial sums are per block: [N * Ho, C].
template <typename T, bool kTwo, bool BNB>
__global__ void __launch_bounds__(kThreads) maxpool_bwd_rows(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                             const uint8_t* __restrict__ idx, T* __restrict__ dx,
                                                             PoolGeom g, BnbArgs bn, int nblk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
  const int cv = g.C / 8, rowv = g.Wo * cv;  // 8-channel vectors per window row
  float* ds = reinterpret_cast<float*>(psm);                               // [2][Wo][C] fp32
  uint8_t* is = psm + static_cast<size_t>(2) * g.Wo * g.C * sizeof(float);  // [2][Wo][C]
  const int b = blockIdx.x, per = nblk / 8, rem = nblk % 8, xcd = b % 8, bi = b / 8;
  const int blk = xcd < rem ? xcd * (per + 1) + bi : rem * (per + 1) + (xcd - rem) * per + bi;
  const int n = blk / g.Ho, oh = blk - n * g.Ho;
  const int nrows = oh + 1 < g.Ho ? 2 : 1;
  const int nv = nrows * rowv;
  const int64_t wbase = static_cast<int64_t>(n * g.Ho + oh) * g.Wo * g.C;
#pragma unroll 4
  for (int v = threadIdx.x; v < nv; v += kThreads) {
    const int64_t off = wbase + static_cast<int64_t>(v) * 8;
    float d[8];
    Vec8<T>::load(dy + off, d);
    if constexpr (kTwo) {
      float d2[8];
      Vec8<T>::load(dy2 + off, d2);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] += d2[j];
    }
    const uc8 av = *reinterpret_cast<const uc8*>(idx + off);
    float4* dst = reinterpret_cast<float4*>(ds + static_cast<int64_t>(v) * 8);
    dst[0] = make_float4(d[0], d[1], d[2], d[3]);
    dst[1] = make_float4(d[4], d[5], d[6], d[7]);
    *reinterpret_cast<uc8*>(is + static_cast<int64_t>(v) * 8) = av;
  }
  const int c8 = threadIdx.x % cv, lanes = kThreads / cv;
  float mu[8], sc[8], sh[8], s1[8], s2[8];
  if constexpr (BNB) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mu[j] = bn.mean[8 * c8 + j];
      sc[j] = bn.scale[8 * c8 + j];
      sh[j] = bn.shift[8 * c8 + j];
      s1[j] = 0.f;
      s2[j] = 0.f;
    }
  }
  const int h0 = 2 * oh, hrows = min(2, g.H - h0), npx = hrows * g.W;
  // the BN input of the block's input rows is contiguous: element offset of pixel p = xbase + p * C;
  // its loads run one item ahead (the first under the staging barrier)
  const int64_t xbase = static_cast<int64_t>(n * g.H + h0) * g.W * g.C + 8 * c8;
  uint4 xnext = make_uint4(0u, 0u, 0u, 0u);
  if constexpr (BNB) {
    const int p = static_cast<int>(threadIdx.x) / cv;
    if (p < npx) xnext = *reinterpret_cast<const uint4*>(bn.x + xbase + static_cast<int64_t>(p) * g.C);
  }
  __syncthreads();
  for (int p = static_cast<int>(threadIdx.x) / cv; p < npx; p += lanes) {
    const int hr = p >= g.W ? 1 : 0, w = p - hr * g.W, h = h0 + hr;
    const int64_t e = xbase + static_cast<int64_t>(p) * g.C;
    float xv[8];
    if constexpr (BNB) {
      const uint32_t wd[4] = {xnext.x, xnext.y, xnext.z, xnext.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xv[2 * k] = __uint_as_float(wd[k] << 16);
        xv[2 * k + 1] = __uint_as_float(wd[k] & 0xffff0000u);
      }
      if (p + lanes < npx) xnext = *reinterpret_cast<const uint4*>(bn.x + e + static_cast<int64_t>(lanes) * g.C);
    }
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // the gather kernel's window order
      const int ohq = (h + 1) / 2 - (q >> 1), kh = h - (2 * ohq - 1);
      const int owq = (w + 1) / 2 - (q & 1), kw = w - (2 * owq - 1);
      if (ohq >= 0 && ohq < g.Ho && kh >= 0 && kh <= 2 && owq >= 0 && owq < g.Wo && kw >= 0 && kw <= 2) {
        const int li = ((ohq - oh) * g.Wo + owq) * g.C + 8 * c8;
        const float4 lo = *reinterpret_cast<const float4*>(ds + li), hi = *reinterpret_cast<const float4*>(ds + li + 4);
        const float dv[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        const uc8 av = *reinterpret_cast<const uc8*>(is + li);
        const uint8_t me = static_cast<uint8_t>(3 * kh + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += av[j] == me ? dv[j] : 0.f;
      }
    }
    if constexpr (BNB) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float dm = __fmaf_rn(xv[j], sc[j], sh[j]) > 0.f ? acc[j] : 0.f;
        const float dr = __uint_as_float(static_cast<uint32_t>(f2bf(dm)) << 16);
        acc[j] = dr;
        s1[j] += dr;
        s2[j] += dr * (xv[j] - mu[j]);
      }
    }
    Vec8<T>::store(dx + e, acc);
  }
  if constexpr (BNB) {
    __syncthreads();  // the staged rows are dead: the reduction reuses the LDS
    float* red = ds;  // [kThreads][17]
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[threadIdx.x * 17 + j] = s1[j];
      red[threadIdx.x * 17 + 8 + j] = s2[j];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < g.C; c += kThreads) {
      const int grp = c / 8, j = c % 8;
      float t1 = 0.f, t2 = 0.f;
      for (int l = 0; l < lanes; ++l) {
        t1 += red[(l * cv + grp) * 17 + j];
        t2 += red[(l * cv + grp) * 17 + 8 + j];
      }
      bn.psum[static_cast<int64_t>(blk) * g.C + c] = t1;
      bn.psumx[static_cast<int64_t>(blk) * g.C + c] = t2;
    }
  }
}

// LDS bytes of maxpool_bwd_rows (two window rows, fp32 gradient + argmax byte; >= the BN reduction)
size_t rows_lds(const PoolGeom& g) {
  size_t b = static_cast<size_t>(2) * g.Wo * g.C * 5;
  const size_t red = static_cast<size_t>(kThreads) * 17 * sizeof(float);
  return b > red ? b : red;
}
constexpr size_t kRowsLdsMax = 64 * 1024;

int grid_for(int64_t work) {
  int64_t b = (work + kThreads - 1) / kThreads;
  if (b > 16384) b = 16384;
  return static_cast<int>(b < 1 ? 1 : b);
}

// ---- global average pooling (the ResNet head: [N, H, W, C] -> [N, C]) ----
// torch lowers AdaptiveAvgPool2d((1, 1)) to a mean whose backward is grad.expand(N, C, H, W) / HW
// (a strided elementwise kernel) followed by a channels_last copy for the consuming BN backward: two
// non-vectorised passes over the 102-MB ResNet-50 layer-4 activation at batch 512
// (profiles/r5_resnet50_steady.csv, 'elementwise_kernel_manual_unroll' x2, 0.16 ms/step).
// forward: a block owns kGapVec 8-channel vectors of one image; its kGapPix pixel lanes each sum every
// kGapPix-th pixel in fp32 and the lanes combine in a fixed order through LDS (deterministic).
constexpr int kGapVec = 32, kGapPix = kThreads / kGapVec;
template <typename T>
__global__ void __launch_bounds__(kThreads) gap_fwd(const T* __restrict__ x, T* __restrict__ y, int HW, int C,
                                                    float inv_hw) {
  __shared__ float part[kGapPix][kGapVec][8];
  const int vpi = C / 8 / kGapVec;  // blocks per image
  const int n = blockIdx.x / vpi, cb = blockIdx.x - n * vpi;
  const int v = threadIdx.x % kGapVec, pl = threadIdx.x / kGapVec;
  const int c0 = (cb * kGapVec + v) * 8;
  const T* base = x + static_cast<int64_t>(n) * HW * C + c0;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int p = pl; p < HW; p += kGapPix) {
    float f[8];
    Vec8<T>::load(base + static_cast<int64_t>(p) * C, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += f[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[pl][v][j] = acc[j];
  __syncthreads();
  if (pl != 0) return;
  for (int q = 1; q < kGapPix; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += part[q][v][j];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= inv_hw;
  Vec8<T>::store(y + static_cast<int64_t>(n) * C + c0, acc);
}

// backward: dx[n, p, c] = dy[n, c] / HW, one 16-B vector of one pixel per thread (grid-stride); the
// dy row is L2-resident, so this is a pure write stream
// (32-bit index math: nvec < 2^31, checked by the host -- a 64-bit division is a long software sequence)
template <typename T>
__global__ void __launch_bounds__(kThreads) gap_bwd(const T* __restrict__ dy, T* __restrict__ dx, int HW, int C,
                                                    float hw, int nvec) {
  const uint32_t cv = static_cast<uint32_t>(C) / 8;
  for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < static_cast<uint32_t>(nvec); i += gridDim.x * kThreads) {
    const uint32_t np = i / cv;  // n * HW + p
    const uint32_t c = (i - np * cv) * 8;
    const uint32_t n = np / static_cast<uint32_t>(HW);
    float f[8];
    Vec8<T>::load(dy + static_cast<int64_t>(n) * C + c, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = f[j] / hw;  // as torch's MeanBackward: grad / HW, one rounding
    Vec8<T>::store(dx + static_cast<int64_t>(i) * 8, f);
  }
}

}  // namespace

int g_fwd_rows = -1;  // -1: DET_POOL_FWD_ROWS decides on first use

extern "C" {

// 1: the row-staged forward (maxpool_fwd_rows) where it fits, 0: the per-output gather.
void det_maxpool3s2_set_fwd_rows(int on) { g_fwd_rows = on ? 1 : 0; }

// x [N, H, W, C] (channels_last) -> y [N, Ho, Wo, C], idx [N, Ho, Wo, C] uint8 (window slot 0..8).
// dtype 0 = fp32, 1 = bf16; C % 8 == 0.  Ho = (H - 1) / 2 + 1 (kernel 3, stride 2, pad 1).
// bn_scale / bn_shift (nullable, bf16 only): x is the input of a BatchNorm + ReLU and the pool reads
// relu(x * scale + shift) (the BN's apply deferred into the pool, maxpool_fwd BNP).
int det_maxpool3s2_fwd(void* stream, int dtype, const void* x, void* y, uint8_t* idx, int N, int H, int W, int C,
                       const float* bn_scale, const float* bn_shift) {
  if (C % 8 != 0 || N <= 0 || H <= 0 || W <= 0) return -1;
  if ((bn_scale == nullptr) != (bn_shift == nullptr) || (bn_scale && dtype != 1)) return -2;
  PoolGeom g{N, H, W, C, (H - 1) / 2 + 1, (W - 1) / 2 + 1};
  const int64_t nvec = static_cast<int64_t>(N) * g.Ho * g.Wo * (C / 8);
  if (nvec >= (static_cast<int64_t>(1) << 31)) return -3;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t flds = static_cast<size_t>(3) * W * C * (dtype == 1 ? 2 : 4);
  // the row-staged forward is opt-in (DET_POOL_FWD_ROWS=1): at the ResNet stem it ran 0.55 ms against
  // the gather's 0.33 (LDS-bound occupancy of 3 blocks / CU and a load-all-then-compute block)
  if (g_fwd_rows < 0) {
    const char* e = std::getenv("DET_POOL_FWD_ROWS");
    g_fwd_rows = e != nullptr && e[0] == '1' ? 1 : 0;
  }
  if (g_fwd_rows == 1 && flds <= kRowsLdsMax && kThreads % (C / 8) == 0 && static_cast<int64_t>(N) * g.Ho < (static_cast<int64_t>(1) << 31)) {
    const int nblk = N * g.Ho;
    const dim3 grid(static_cast<unsigned>(nblk)), block(kThreads);
    if (dtype == 1 && bn_scale)
      hipLaunchKernelGGL((maxpool_fwd_rows<unsigned short, true>), grid, block, flds, st,
                         static_cast<const unsigned short*>(x), static_cast<unsigned short*>(y), idx, g, nblk, bn_scale,
                         bn_shift);
    else if (dtype == 1)
      hipLaunchKernelGGL((maxpool_fwd_rows<unsigned short, false>), grid, block, flds, st,
                         static_cast<const unsigned short*>(x), static_cast<unsigned short*>(y), idx, g, nblk, nullptr,
                         nullptr);
    else
      hipLaunchKernelGGL((maxpool_fwd_rows<float, false>), grid, block, flds, st, static_cast<const float*>(x),
                         static_cast<float*>(y), idx, g, nblk, nullptr, nullptr);
    return static_cast<int>(hipGetLastError());
  }
  if (dtype == 1 && bn_scale)
    hipLaunchKernelGGL((maxpool_fwd<unsigned short, true>), dim3(grid_for(nvec)), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), static_cast<unsigned short*>(y), idx, g,
                       static_cast<int>(nvec), bn_scale, bn_shift);
  else if (dtype == 1)
    hipLaunchKernelGGL(maxpool_fwd<unsigned short>, dim3(grid_for(nvec)), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), static_cast<unsigned short*>(y), idx, g,
                       static_cast<int>(nvec));
  else
    hipLaunchKernelGGL(maxpool_fwd<float>, dim3(grid_for(nvec)), dim3(kThreads), 0, st, static_cast<const float*>(x),
                       static_cast<float*>(y), idx, g, static_cast<int>(nvec));
  return static_cast<int>(hipGetLastError());
}

// Input pixels per partial-sum block of the per-pixel gather kernel's BN-backward epilogue.
int det_maxpool3s2_bwd_rows_per_block() { return kBwdRows; }

// Rows of the BN partial sums det_maxpool3s2_bwd writes for this shape (psum / psumx [rows, C]):
// N * Ho with the row-staged kernel, ceil(N*H*W / det_maxpool3s2_bwd_rows_per_block()) otherwise.
int64_t det_maxpool3s2_bwd_partial_rows(int N, int H, int W, int C) {
  const PoolGeom g{N, H, W, C, (H - 1) / 2 + 1, (W - 1) / 2 + 1};
  if (rows_lds(g) <= kRowsLdsMax && static_cast<int64_t>(N) * g.Ho < (static_cast<int64_t>(1) << 31))
    return static_cast<int64_t>(N) * g.Ho;
  return (static_cast<int64_t>(N) * H * W + kBwdRows - 1) / kBwdRows;
}

// dy [N, Ho, Wo, C] (+ optional dy2 of the same shape, summed), idx from the forward -> dx [N, H, W, C]
// (fully overwritten).  C % 8 == 0 and 256 % (C / 8) == 0; N*H*W < 2^31.
// bn_x (nullable, bf16 only): with bn_mean/scale/shift [C] and psum/psumx
// [det_maxpool3s2_bwd_partial_rows(N, H, W, C), C],
// dx = relu'(bn_x * scale + shift) * gradient and the BN-backward partials (see maxpool_bwd BNB).
int det_maxpool3s2_bwd(void* stream, int dtype, const void* dy, const void* dy2, const uint8_t* idx, void* dx, int N,
                       int H, int W, int C, const void* bn_x, const float* bn_mean, const float* bn_scale,
                       const float* bn_shift, float* psum, float* psumx) {
  if (C % 8 != 0 || N <= 0 || H <= 0 || W <= 0 || kThreads % (C / 8) != 0) return -1;
  if (static_cast<int64_t>(N) * H * W >= (static_cast<int64_t>(1) << 31)) return -3;
  if (bn_x && (dtype != 1 || !bn_mean || !bn_scale || !bn_shift || !psum || !psumx)) return -2;
  PoolGeom g{N, H, W, C, (H - 1) / 2 + 1, (W - 1) / 2 + 1};
  const int64_t npix = static_cast<int64_t>(N) * H * W;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const BnbArgs bn{static_cast<const unsigned short*>(bn_x), bn_mean, bn_scale, bn_shift, psum, psumx};
  if (rows_lds(g) <= kRowsLdsMax && static_cast<int64_t>(N) * g.Ho < (static_cast<int64_t>(1) << 31)) {
    const int nblk = N * g.Ho;
    const dim3 grid(static_cast<unsigned>(nblk)), block(kThreads);
    const size_t lds = rows_lds(g);
    if (dtype == 1) {
      auto* a = static_cast<const unsigned short*>(dy);
      auto* b = static_cast<const unsigned short*>(dy2);
      auto* o = static_cast<unsigned short*>(dx);
      if (bn_x) {
        if (dy2) hipLaunchKernelGGL((maxpool_bwd_rows<unsigned short, true, true>), grid, block, lds, st, a, b, idx, o, g, bn, nblk);
        else hipLaunchKernelGGL((maxpool_bwd_rows<unsigned short, false, true>), grid, block, lds, st, a, b, idx, o, g, bn, nblk);
      } else {
        if (dy2) hipLaunchKernelGGL((maxpool_bwd_rows<unsigned short, true, false>), grid, block, lds, st, a, b, idx, o, g, bn, nblk);
        else hipLaunchKernelGGL((maxpool_bwd_rows<unsigned short, false, false>), grid, block, lds, st, a, b, idx, o, g, bn, nblk);
      }
    } else {
      auto* a = static_cast<const float*>(dy);
      auto* b = static_cast<const float*>(dy2);
      auto* o = static_cast<float*>(dx);
      if (dy2) hipLaunchKernelGGL((maxpool_bwd_rows<float, true, false>), grid, block, lds, st, a, b, idx, o, g, bn, nblk);
      else hipLaunchKernelGGL((maxpool_bwd_rows<float, false, false>), grid, block, lds, st, a, b, idx, o, g, bn, nblk);
    }
    return static_cast<int>(hipGetLastError());
  }
  const dim3 grid(static_cast<unsigned>((npix + kBwdRows - 1) / kBwdRows)), block(kThreads);
  if (dtype == 1) {
    auto* a = static_cast<const unsigned short*>(dy);
    auto* b = static_cast<const unsigned short*>(dy2);
    auto* o = static_cast<unsigned short*>(dx);
    if (bn_x) {
      if (dy2) hipLaunchKernelGGL((maxpool_bwd<unsigned short, true, true>), grid, block, 0, st, a, b, idx, o, g, bn);
      else hipLaunchKernelGGL((maxpool_bwd<unsigned short, false, true>), grid, block, 0, st, a, b, idx, o, g, bn);
    } else {
      if (dy2) hipLaunchKernelGGL((maxpool_bwd<unsigned short, true, false>), grid, block, 0, st, a, b, idx, o, g, bn);
      else hipLaunchKernelGGL((maxpool_bwd<unsigned short, false, false>), grid, block, 0, st, a, b, idx, o, g, bn);
    }
  } else {
    auto* a = static_cast<const float*>(dy);
    auto* b = static_cast<const float*>(dy2);
    auto* o = static_cast<float*>(dx);
    if (dy2)
      hipLaunchKernelGGL((maxpool_bwd<float, true, false>), grid, block, 0, st, a, b, idx, o, g, bn);
    else
      hipLaunchKernelGGL((maxpool_bwd<float, false, false>), grid, block, 0, st, a, b, idx, o, g, bn);
  }
  return static_cast<int>(hipGetLastError());
}

// Global average pooling of channels_last x [N, H, W, C] -> y [N, C]; dtype 0 = fp32, 1 = bf16.
// C % 256 == 0 (32 vectors of 8 channels per workgroup).
int det_gap_fwd(void* stream, int dtype, const void* x, void* y, int N, int HW, int C) {
  if (N <= 0 || HW <= 0 || C <= 0 || C % (8 * kGapVec) != 0) return -1;
  const int64_t nblk = static_cast<int64_t>(N) * (C / 8 / kGapVec);
  if (nblk >= (static_cast<int64_t>(1) << 31)) return -3;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const float inv = 1.f / static_cast<float>(HW);
  if (dtype == 1)
    hipLaunchKernelGGL(gap_fwd<unsigned short>, dim3(static_cast<unsigned>(nblk)), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), static_cast<unsigned short*>(y), HW, C, inv);
  else
    hipLaunchKernelGGL(gap_fwd<float>, dim3(static_cast<unsigned>(nblk)), dim3(kThreads), 0, st,
                       static_cast<const float*>(x), static_cast<float*>(y), HW, C, inv);
  return static_cast<int>(hipGetLastError());
}

// dy [N, C] -> dx [N, H, W, C] (channels_last, fully overwritten) = dy / HW.  C % 8 == 0.
int det_gap_bwd(void* stream, int dtype, const void* dy, void* dx, int N, int HW, int C) {
  if (N <= 0 || HW <= 0 || C <= 0 || C % 8 != 0) return -1;
  const int64_t nvec = static_cast<int64_t>(N) * HW * (C / 8);
  if (nvec >= (static_cast<int64_t>(1) << 31)) return -3;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const float hw = static_cast<float>(HW);
  if (dtype == 1)
    hipLaunchKernelGGL(gap_bwd<unsigned short>, dim3(grid_for(nvec)), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(dy), static_cast<unsigned short*>(dx), HW, C, hw, static_cast<int>(nvec));
  else
    hipLaunchKernelGGL(gap_bwd<float>, dim3(grid_for(nvec)), dim3(kThreads), 0, st, static_cast<const float*>(dy),
                       static_cast<float*>(dx), HW, C, hw, static_cast<int>(nvec));
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
