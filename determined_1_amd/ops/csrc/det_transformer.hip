// det_transformer.hip — fused transformer-encoder epilogues for CDNA4 (gfx950, wave64).
//
// Why this exists: in the BERT-base SQuAD-shape step (profiles/r1_bert_base_bs12_o2_steady.csv,
// 12.7 ms of GPU time per step) ~3.9 ms go to HBM-bound glue around the GEMMs: torch's
// LayerNorm fwd/bwd (4 launches per LN), dropout + masked-scale, residual adds, GELU fwd/bwd and
// 73 bias-gradient column reductions at ~17 us each.  These kernels fold that glue into the
// minimum number of passes:
//
//   ln_fwd        y = LayerNorm(dropout(h) + r)         one pass: reads h, r; writes y, mean, rstd
//   ln_bwd        dz = LN'(dy); dr = dz; dh = dropout'(dz) and per-block partial sums of
//                 dgamma = sum(dy * xhat), dbeta = sum(dy), dbias = sum(dh)   (one pass)
//   ln_finalize   reduces the partials -> dgamma, dbeta and the preceding Linear's bias grad
//   gelu_fwd      a = gelu(z) (erf form, as BERT; tanh form for ALBERT's gelu_new)
//   gelu_bwd      dz = da * gelu'(z) with the bias-grad partials of the producing Linear fused
//   colsum        bias grad of a plain Linear (QKV) without torch's generic reduction
//
// Dropout masks are never stored: a counter-based Philox4x32-10 stream keyed by (seed, offset)
// and indexed by element/4 regenerates the identical mask in the backward pass, so a lane draws
// exactly one Philox block for its 4 consecutive elements.
//
// Row kernels (LN): forward = one workgroup per row (128/256/512 threads x 8 columns, block
// reductions); backward = one wavefront per row up to H = 2048 (lane owns 4 consecutive elements at
// 4*(lane + 64*i), i < K = ceil(H/256)), a workgroup per row above.  The two-pass mean/variance
// is exact in registers.  Column reductions use two levels (LDS per block, then a finalize launch) and no
// float atomics, so every gradient is bitwise reproducible.  No host syncs anywhere.
//
// Reference parity: the reference runs BERT through HuggingFace modules on torch/cuDNN
// (examples/nlp/bert_squad_pytorch/model_def.py:39-75); these kernels implement the same math
// (LayerNorm eps, dropout-before-residual, erf GELU) for determined_1_amd/models/bert.py.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>
#include <cstring>

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kFinThreads = 1024;
constexpr int kMaxH = 8192;        // LayerNorm width limit (workgroup-per-row kernels above 2048)
constexpr int kMaxNarrowH = 2048;  // wave-per-row kernels up to here
constexpr int kFinCols = 64;

__device__ __forceinline__ float bf2f(unsigned short u) { return __uint_as_float(static_cast<uint32_t>(u) << 16); }
// RNE; adjacent conversions pair into gfx950's v_cvt_pk_bf16_f32
__device__ __forceinline__ unsigned short f2bf(float f) {
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));
}

typedef unsigned short us4 __attribute__((ext_vector_type(4)));
typedef unsigned short us8 __attribute__((ext_vector_type(8)));

template <typename T> struct V4;
template <> struct V4<unsigned short> {
  static __device__ __forceinline__ void load(const unsigned short* p, float (&v)[4]) {
    us4 r = *reinterpret_cast<const us4*>(p);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = bf2f(r[j]);
  }
  static __device__ __forceinline__ void store(unsigned short* p, const float (&v)[4]) {
    us4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = f2bf(v[j]);
    *reinterpret_cast<us4*>(p) = r;
  }
};
template <> struct V4<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[4]) {
    float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};

template <typename T> struct V8;
template <> struct V8<unsigned short> {
  static __device__ __forceinline__ void load(const unsigned short* p, float (&v)[8]) {
    us8 r = *reinterpret_cast<const us8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f(r[j]);
  }
  static __device__ __forceinline__ void store(unsigned short* p, const float (&v)[8]) {
    us8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = f2bf(v[j]);
    *reinterpret_cast<us8*>(p) = r;
  }
};
template <> struct V8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    float4 a = reinterpret_cast<const float4*>(p)[0];
    float4 b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

template <typename T> __device__ __forceinline__ T from_float(float f);
template <> __device__ __forceinline__ float from_float<float>(float f) { return f; }
template <> __device__ __forceinline__ unsigned short from_float<unsigned short>(float f) { return f2bf(f); }

// ---- Philox4x32-10 (counter-based; Salmon et al. 2011) --------------------------------------
struct Rng {
  uint32_t k0, k1, o0, o1;  // key = seed, counter words 2/3 = offset
  uint32_t thresh;          // drop if u < thresh  (thresh = p * 2^32)
  float scale;              // 1 / (1 - p)
  // nullable: device counter added to counter word 3 when the kernel runs.  A hipGraph replays the
  // (seed, offset) kernel arguments it captured; the captured step bumps this counter first, so every
  // replay draws fresh masks (ops/transformer.py rng_base / bump_rng_base)
  const uint32_t* obase;
};

__device__ __forceinline__ void philox(uint64_t idx, const Rng& g, uint32_t (&u)[4]) {
  uint32_t c0 = static_cast<uint32_t>(idx), c1 = static_cast<uint32_t>(idx >> 32), c2 = g.o0,
           c3 = g.o1 + (g.obase != nullptr ? *g.obase : 0u);
  uint32_t k0 = g.k0, k1 = g.k1;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  u[0] = c0; u[1] = c1; u[2] = c2; u[3] = c3;
}

// mask * scale for the 4 elements of element-group `grp`
__device__ __forceinline__ void drop_factors(uint64_t grp, const Rng& g, float (&m)[4]) {
  uint32_t u[4];
  philox(grp, g, u);
#pragma unroll
  for (int j = 0; j < 4; ++j) m[j] = u[j] >= g.thresh ? g.scale : 0.f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

struct LnArgs {
  const void* h;      // [rows, H] input of the dropout (output of the preceding Linear)
  const void* r;      // [rows, H] residual (nullable)
  void* y;            // [rows, H]
  const void* gamma;  // [H]
  const void* beta;   // [H]
  float* mean;        // [rows]
  float* rstd;        // [rows]
  int64_t rows;
  int H;
  float eps;
  int dropout;        // 0: identity
  Rng rng;
};

// ---------------------------------------------------------------------------------------------
// y = LN(dropout(h) + r): one wave per row, grid-stride over rows.
// ---------------------------------------------------------------------------------------------
template <typename T, int K, int R = 1>
__global__ void __launch_bounds__(kThreads) ln_fwd_kernel(LnArgs a) {
  // R rows per wave per iteration: their loads are all in flight before the first reduction (a row
  // of BERT-base is 3 loads per lane, too little to cover the memory latency on its own)
  const int lane = threadIdx.x & 63;
  const int H4 = a.H >> 2;
  const T* h = static_cast<const T*>(a.h);
  const T* r = static_cast<const T*>(a.r);
  T* y = static_cast<T*>(a.y);
  float g[K][4], b[K][4];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int c4 = lane + 64 * i;
    if (c4 < H4) {
      V4<T>::load(static_cast<const T*>(a.gamma) + 4 * c4, g[i]);
      V4<T>::load(static_cast<const T*>(a.beta) + 4 * c4, b[i]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) g[i][j] = b[i][j] = 0.f;
    }
  }
  const float inv_h = 1.f / static_cast<float>(a.H);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kWaves;
  for (int64_t row0 = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6); row0 < a.rows;
       row0 += stride * R) {
    float v[R][K][4];
    float s[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int64_t row = row0 + q * stride;
      const bool ok = row < a.rows;
      const int64_t base = (ok ? row : 0) * a.H;
      s[q] = 0.f;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const int c4 = lane + 64 * i;
        if (ok && c4 < H4) {
          V4<T>::load(h + base + 4 * c4, v[q][i]);
          if (a.dropout) {
            float m[4];
            drop_factors(static_cast<uint64_t>(row) * H4 + c4, a.rng, m);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[q][i][j] *= m[j];
          }
          if (r) {
            float t[4];
            V4<T>::load(r + base + 4 * c4, t);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[q][i][j] += t[j];
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[q][i][j] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) s[q] += v[q][i][j];
      }
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int64_t row = row0 + q * stride;
      const float mean = wave_sum(s[q]) * inv_h;
      float s2 = 0.f;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        if (lane + 64 * i < H4) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = v[q][i][j] - mean;
            s2 += d * d;
          }
        }
      }
      const float rstd = rsqrtf(wave_sum(s2) * inv_h + a.eps);
      if (row >= a.rows) continue;
      const int64_t base = row * a.H;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const int c4 = lane + 64 * i;
        if (c4 < H4) {
          float o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = (v[q][i][j] - mean) * rstd * g[i][j] + b[i][j];
          V4<T>::store(y + base + 4 * c4, o);
        }
      }
      if (lane == 0) {
        a.mean[row] = mean;
        a.rstd[row] = rstd;
      }
    }
  }
}

struct LnBwdArgs {
  const void* dy;
  const void* h;
  const void* r;      // nullable (then z = dropout(h))
  const float* mean;
  const float* rstd;
  const void* gamma;
  void* dr;           // grad of the residual (= dz), nullable
  void* dh;           // grad of h (= dropout'(dz)), nullable
  float* ws;          // [gridDim.x][3][H] partials: dgamma, dbeta, dbias
  int64_t rows;
  int H;
  int dropout;
  Rng rng;
};

template <typename T, int K, int R = 1>
__global__ void __launch_bounds__(kThreads) ln_bwd_kernel(LnBwdArgs a) {
  // H <= 2048 (K <= 8): dy, xhat and the dropout factors of the row stay in registers between the
  // two passes; wider rows use ln_bwd_wide.  R rows per wave per iteration, their loads all issued
  // before the first reduction.
  extern __shared__ float red[];  // [kWaves][H]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int H4 = a.H >> 2;
  const T* dy = static_cast<const T*>(a.dy);
  const T* h = static_cast<const T*>(a.h);
  const T* r = static_cast<const T*>(a.r);
  T* dr = static_cast<T*>(a.dr);
  T* dh = static_cast<T*>(a.dh);
  float g[K][4], adg[K][4], adb[K][4], adh[K][4];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int c4 = lane + 64 * i;
    if (c4 < H4) V4<T>::load(static_cast<const T*>(a.gamma) + 4 * c4, g[i]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (c4 >= H4) g[i][j] = 0.f;
      adg[i][j] = adb[i][j] = adh[i][j] = 0.f;
    }
  }
  const float inv_h = 1.f / static_cast<float>(a.H);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kWaves;
  for (int64_t row0 = static_cast<int64_t>(blockIdx.x) * kWaves + wave; row0 < a.rows; row0 += stride * R) {
    float d[R][K][4], hv[R][K][4], rv[R][K][4];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int64_t row = row0 + q * stride;
      const bool ok = row < a.rows;
      const int64_t base = (ok ? row : 0) * a.H;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const int c4 = lane + 64 * i;
        if (ok && c4 < H4) {
          V4<T>::load(dy + base + 4 * c4, d[q][i]);
          V4<T>::load(h + base + 4 * c4, hv[q][i]);
          if (r) V4<T>::load(r + base + 4 * c4, rv[q][i]);
          else {
#pragma unroll
            for (int j = 0; j < 4; ++j) rv[q][i][j] = 0.f;
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) d[q][i][j] = hv[q][i][j] = rv[q][i][j] = 0.f;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int64_t row = row0 + q * stride;
      if (row >= a.rows) continue;  // uniform across the wave
      const int64_t base = row * a.H;
      const float mean = a.mean[row], rstd = a.rstd[row];
      float xh[K][4], m[K][4];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const int c4 = lane + 64 * i;
        if (c4 < H4) {
          if (a.dropout) {
            drop_factors(static_cast<uint64_t>(row) * H4 + c4, a.rng, m[i]);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) m[i][j] = 1.f;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float z = hv[q][i][j] * m[i][j] + rv[q][i][j];  // z = dropout(h) + r
            xh[i][j] = (z - mean) * rstd;
            const float dx = d[q][i][j] * g[i][j];
            s1 += dx;
            s2 += dx * xh[i][j];
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) xh[i][j] = m[i][j] = 0.f;
        }
      }
      s1 = wave_sum(s1) * inv_h;
      s2 = wave_sum(s2) * inv_h;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const int c4 = lane + 64 * i;
        if (c4 < H4) {
          float dz[4], dhv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            dz[j] = rstd * (d[q][i][j] * g[i][j] - s1 - xh[i][j] * s2);
            dhv[j] = dz[j] * m[i][j];
            adg[i][j] += d[q][i][j] * xh[i][j];
            adb[i][j] += d[q][i][j];
            adh[i][j] += dhv[j];
          }
          if (dr) V4<T>::store(dr + base + 4 * c4, dz);
          if (dh) V4<T>::store(dh + base + 4 * c4, dhv);
        }
      }
    }
  }
  // block merge of the per-lane column partials (one quantity at a time: LDS = kWaves * H floats),
  // then one partial row per block
  const int H = a.H;
  float* out = a.ws + static_cast<int64_t>(blockIdx.x) * 3 * H;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < H4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) red[wave * H + 4 * c4 + j] = q == 0 ? adg[i][j] : q == 1 ? adb[i][j] : adh[i][j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < H; c += kThreads) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) s += red[w * H + c];
      out[q * H + c] = s;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Wide rows (H > 2048: ALBERT-xxlarge's 4096): one 512-thread workgroup per row, a thread owns
// 8 consecutive columns per 4096 (16-B vectors), block reductions through LDS.  The wave-per-row
// kernels above would keep 64+ columns per lane at one wave per SIMD (measured 1.4 TB/s fwd,
// profiles/r1_albert_xxlarge_bs8_o2_per_step.txt); here every lane has one 16-B load per tensor
// in flight per row and the register footprint is small.  The backward keeps its dgamma / dbeta /
// dbias partials in registers across a grid-stride row loop and writes one partial row per
// workgroup for colsum_finalize.
// ---------------------------------------------------------------------------------------------
constexpr int kWideThreads = 512;     // workgroup of the widest rows (H > 2048)
constexpr int kWideMaxWaves = kWideThreads / 64;

template <int NT>
__device__ __forceinline__ float block_sum_wide(float v, float* red) {  // red: NT/64 floats
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) t += red[w];
  __syncthreads();
  return t;
}

template <int NT>
__device__ __forceinline__ void block_sum2_wide(float& a, float& b, float* red) {  // red: 2 x NT/64
  a = wave_sum(a);
  b = wave_sum(b);
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = a;
    red[NT / 64 + (threadIdx.x >> 6)] = b;
  }
  __syncthreads();
  float ta = 0.f, tb = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    ta += red[w];
    tb += red[NT / 64 + w];
  }
  __syncthreads();
  a = ta;
  b = tb;
}

// dropout factors of the 8 columns starting at 8*c8 of `row` (two Philox groups of 4, the same
// group indexing as the wave-per-row kernels)
__device__ __forceinline__ void wide_drop(int64_t row, int H, int c8, const Rng& g, float (&m)[8]) {
  float m0[4], m1[4];
  const uint64_t grp = static_cast<uint64_t>(row) * (H >> 2) + 2 * c8;
  drop_factors(grp, g, m0);
  drop_factors(grp + 1, g, m1);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m[j] = m0[j];
    m[4 + j] = m1[j];
  }
}

template <typename T, int V, int NT>
__global__ void __launch_bounds__(NT) ln_fwd_wide(LnArgs a) {
  __shared__ float red[2 * kWideMaxWaves];
  const int H8 = a.H >> 3;
  const T* h = static_cast<const T*>(a.h);
  const T* r = static_cast<const T*>(a.r);
  T* y = static_cast<T*>(a.y);
  const float inv_h = 1.f / static_cast<float>(a.H);
  for (int64_t row = blockIdx.x; row < a.rows; row += gridDim.x) {
    const int64_t base = row * a.H;
    float v[V][8];
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const int c8 = threadIdx.x + NT * q;
      if (c8 < H8) {
        V8<T>::load(h + base + 8 * c8, v[q]);
        if (a.dropout) {
          float m[8];
          wide_drop(row, a.H, c8, a.rng, m);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[q][j] *= m[j];
        }
        if (r) {
          float t[8];
          V8<T>::load(r + base + 8 * c8, t);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[q][j] += t[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[q][j];
      }
    }
    const float mean = block_sum_wide<NT>(s, red) * inv_h;
    float s2 = 0.f;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      if (threadIdx.x + NT * q < H8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[q][j] - mean;
          s2 += d * d;
        }
      }
    }
    const float rstd = rsqrtf(block_sum_wide<NT>(s2, red + NT / 64) * inv_h + a.eps);
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const int c8 = threadIdx.x + NT * q;
      if (c8 < H8) {
        float g[8], b[8], o[8];
        V8<T>::load(static_cast<const T*>(a.gamma) + 8 * c8, g);
        V8<T>::load(static_cast<const T*>(a.beta) + 8 * c8, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[q][j] - mean) * rstd * g[j] + b[j];
        V8<T>::store(y + base + 8 * c8, o);
      }
    }
    if (threadIdx.x == 0) {
      a.mean[row] = mean;
      a.rstd[row] = rstd;
    }
  }
}

template <typename T, int V, int NT>
__global__ void __launch_bounds__(NT) ln_bwd_wide(LnBwdArgs a) {
  __shared__ float red[2 * kWideMaxWaves];
  const int H = a.H, H8 = H >> 3;
  const T* dy = static_cast<const T*>(a.dy);
  const T* h = static_cast<const T*>(a.h);
  const T* r = static_cast<const T*>(a.r);
  T* dr = static_cast<T*>(a.dr);
  T* dh = static_cast<T*>(a.dh);
  float g[V][8], adg[V][8], adb[V][8], adh[V][8];
#pragma unroll
  for (int q = 0; q < V; ++q) {
    const int c8 = threadIdx.x + NT * q;
    if (c8 < H8) V8<T>::load(static_cast<const T*>(a.gamma) + 8 * c8, g[q]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (c8 >= H8) g[q][j] = 0.f;
      adg[q][j] = adb[q][j] = adh[q][j] = 0.f;
    }
  }
  const float inv_h = 1.f / static_cast<float>(H);
  for (int64_t row = blockIdx.x; row < a.rows; row += gridDim.x) {
    const int64_t base = row * H;
    const float mean = a.mean[row], rstd = a.rstd[row];
    float d[V][8], xh[V][8], m[V][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const int c8 = threadIdx.x + NT * q;
      if (c8 < H8) {
        float z[8];
        V8<T>::load(dy + base + 8 * c8, d[q]);
        V8<T>::load(h + base + 8 * c8, z);
        if (a.dropout) {
          wide_drop(row, H, c8, a.rng, m[q]);
#pragma unroll
          for (int j = 0; j < 8; ++j) z[j] *= m[q][j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) m[q][j] = 1.f;
        }
        if (r) {
          float t[8];
          V8<T>::load(r + base + 8 * c8, t);
#pragma unroll
          for (int j = 0; j < 8; ++j) z[j] += t[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[q][j] = (z[j] - mean) * rstd;
          const float dx = d[q][j] * g[q][j];
          s1 += dx;
          s2 += dx * xh[q][j];
        }
      }
    }
    block_sum2_wide<NT>(s1, s2, red);
    s1 *= inv_h;
    s2 *= inv_h;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const int c8 = threadIdx.x + NT * q;
      if (c8 < H8) {
        float dz[8], dhv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          dz[j] = rstd * (d[q][j] * g[q][j] - s1 - xh[q][j] * s2);
          dhv[j] = dz[j] * m[q][j];
          adg[q][j] += d[q][j] * xh[q][j];
          adb[q][j] += d[q][j];
          adh[q][j] += dhv[j];
        }
        if (dr) V8<T>::store(dr + base + 8 * c8, dz);
        if (dh) V8<T>::store(dh + base + 8 * c8, dhv);
      }
    }
  }
  float* out = a.ws + static_cast<int64_t>(blockIdx.x) * 3 * H;
#pragma unroll
  for (int q = 0; q < V; ++q) {
    const int c8 = threadIdx.x + NT * q;
    if (c8 < H8) {
      V8<float>::store(out + 8 * c8, adg[q]);
      V8<float>::store(out + H + 8 * c8, adb[q]);
      V8<float>::store(out + 2 * H + 8 * c8, adh[q]);
    }
  }
}

// Sum `parts` partial rows of width W (fp32) -> up to 3 outputs of width W/3 each (or one of W).
// COLS columns per block (kFinThreads / COLS lanes split each column's rows); DET_FIN_COLS=16|32|64
// picks it (32 by default: twice the blocks of 64 and half the serial rows per lane)
template <typename T, int COLS = kFinCols>
__global__ void __launch_bounds__(kFinThreads)
colsum_finalize(const float* __restrict__ ws, int parts, int W, int seg, T* __restrict__ o0, T* __restrict__ o1,
                T* __restrict__ o2) {
  constexpr int kFinLanes = kFinThreads / COLS;
  __shared__ float red[kFinLanes][COLS];
  const int cl = threadIdx.x % COLS, ln = threadIdx.x / COLS;
  const int col = blockIdx.x * COLS + cl;
  float s = 0.f;
  if (col < W) {
    int p = ln;
    for (; p + 3 * kFinLanes < parts; p += 4 * kFinLanes) {
      const float a = ws[static_cast<int64_t>(p) * W + col];
      const float b = ws[static_cast<int64_t>(p + kFinLanes) * W + col];
      const float c = ws[static_cast<int64_t>(p + 2 * kFinLanes) * W + col];
      const float d = ws[static_cast<int64_t>(p + 3 * kFinLanes) * W + col];
      s += (a + b) + (c + d);
    }
    for (; p < parts; p += kFinLanes) s += ws[static_cast<int64_t>(p) * W + col];
  }
  red[ln][cl] = s;
  __syncthreads();
  if (ln == 0 && col < W) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < kFinLanes; ++l) t += red[l][cl];
    const int which = col / seg, c = col - which * seg;
    T* o = which == 0 ? o0 : which == 1 ? o1 : o2;
    if (o) o[c] = from_float<T>(t);
  }
}

int fin_cols() {
  static const int c = [] {
    const char* e = std::getenv("DET_FIN_COLS");
    const int v = e != nullptr ? std::atoi(e) : 0;
    return v == 16 || v == 64 ? v : 32;  // 32: LN backward 19.1 vs 20.4 us, BERT graph +0.56 % (r6s73)
  }();
  return c;
}
template <typename T>
void launch_colsum_finalize(hipStream_t st, const float* ws, int parts, int W, int seg, T* o0, T* o1, T* o2) {
  const int cols = fin_cols();
  if (cols == 16)
    hipLaunchKernelGGL((colsum_finalize<T, 16>), dim3((W + 15) / 16), dim3(kFinThreads), 0, st, ws, parts, W, seg, o0, o1, o2);
  else if (cols == 32)
    hipLaunchKernelGGL((colsum_finalize<T, 32>), dim3((W + 31) / 32), dim3(kFinThreads), 0, st, ws, parts, W, seg, o0, o1, o2);
  else
    hipLaunchKernelGGL((colsum_finalize<T, kFinCols>), dim3((W + kFinCols - 1) / kFinCols), dim3(kFinThreads), 0, st, ws,
                       parts, W, seg, o0, o1, o2);
}

// ---------------------------------------------------------------------------------------------
// Column-tiled elementwise + bias-grad partials over a [rows, C] matrix (C % 8 == 0):
// a lane owns 8 consecutive columns, a block covers tpr column groups x R rows per iteration and
// one row-block; partial column sums land in ws[row_block][C].
// ---------------------------------------------------------------------------------------------
struct ColGeom {
  int64_t rows;
  int C;
  int tpr;
  int R;
  int64_t rpb;
  int nrb;
};

ColGeom make_col_geom(int64_t rows, int C) {
  ColGeom g;
  g.rows = rows;
  g.C = C;
  const int groups = C / 8;
  int tpr = 1;
  while (tpr * 2 <= kThreads && groups % (tpr * 2) == 0) tpr *= 2;
  g.tpr = tpr;
  g.R = kThreads / tpr;
  const int gy = groups / tpr;
  // ~1024 blocks in total, >= 4 row iterations per thread so the partial traffic stays small
  int64_t nrb = (1024 + gy - 1) / gy;
  const int64_t max_rb = (rows + 4 * g.R - 1) / (4 * g.R);
  if (nrb > max_rb) nrb = max_rb;
  if (nrb < 1) nrb = 1;
  int64_t rpb = (rows + nrb - 1) / nrb;
  rpb = (rpb + g.R - 1) / g.R * g.R;
  g.rpb = rpb;
  g.nrb = static_cast<int>((rows + rpb - 1) / rpb);
  return g;
}

// ACT 0: erf GELU (BERT);  ACT 1: tanh GELU ("gelu_new": ALBERT, GPT-2)
template <int ACT> __device__ __forceinline__ float gelu_f(float z) {
  if (ACT == 0) return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
  const float u = 0.7978845608028654f * (z + 0.044715f * z * z * z);
  return 0.5f * z * (1.f + tanhf(u));
}
template <int ACT> __device__ __forceinline__ float gelu_grad(float z) {
  if (ACT == 0) {
    const float cdf = 0.5f * (1.f + erff(z * 0.70710678118654752f));
    const float pdf = 0.39894228040143268f * __expf(-0.5f * z * z);
    return cdf + z * pdf;
  }
  const float z2 = z * z;
  const float t = tanhf(0.7978845608028654f * z * (1.f + 0.044715f * z2));
  return 0.5f * (1.f + t) + 0.5f * z * (1.f - t * t) * 0.7978845608028654f * (1.f + 3.f * 0.044715f * z2);
}

// MODE 0: colsum(x) only;  MODE 1: dz = da * gelu'(z) (stored) and colsum(dz);  MODE 2: as 1, tanh GELU
template <typename T, int MODE>
__global__ void __launch_bounds__(kThreads)
col_kernel(const T* __restrict__ a, const T* __restrict__ z, T* __restrict__ dz, ColGeom g, float* __restrict__ ws) {
  __shared__ float red[kThreads * 8];
  const int tx = threadIdx.x % g.tpr, ty = threadIdx.x / g.tpr;
  const int cg = blockIdx.y * g.tpr + tx;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * g.rpb;
  const int64_t r1 = min(g.rows, r0 + g.rpb);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const int64_t C = g.C;
  for (int64_t r = r0 + ty; r < r1; r += g.R) {
    const int64_t off = r * C + cg * 8;
    float v[8];
    V8<T>::load(a + off, v);
    if (MODE >= 1) {
      float zz[8];
      V8<T>::load(z + off, zz);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= gelu_grad<MODE - 1>(zz[j]);
      V8<T>::store(dz + off, v);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  if (!ws) return;  // gelu backward without a bias (uniform across the block)
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = acc[j];
  __syncthreads();
  if (ty == 0) {
    for (int k = 1; k < g.R; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += red[(k * g.tpr + tx) * 8 + j];
    float* out = ws + static_cast<int64_t>(blockIdx.x) * C + cg * 8;
    reinterpret_cast<float4*>(out)[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    reinterpret_cast<float4*>(out)[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
}

template <typename T, int ACT>
__global__ void __launch_bounds__(kThreads) gelu_fwd_kernel(const T* __restrict__ z, T* __restrict__ a, int64_t nvec) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < nvec;
       i += static_cast<int64_t>(gridDim.x) * kThreads) {
    float v[8];
    V8<T>::load(z + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_f<ACT>(v[j]);
    V8<T>::store(a + i * 8, v);
  }
}

__global__ void __launch_bounds__(kThreads) dropout_mask_kernel(int64_t ngroups, Rng g, uint8_t* __restrict__ out) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < ngroups;
       i += static_cast<int64_t>(gridDim.x) * kThreads) {
    float m[4];
    drop_factors(static_cast<uint64_t>(i), g, m);
#pragma unroll
    for (int j = 0; j < 4; ++j) out[i * 4 + j] = m[j] != 0.f;
  }
}

__global__ void rng_bump_kernel(uint32_t* counter) {
  if (threadIdx.x == 0) counter[threadIdx.x] += 1u;
}

Rng make_rng(float p, uint64_t seed, uint64_t offset, const uint32_t* obase) {
  Rng g;
  g.obase = obase;
  g.k0 = static_cast<uint32_t>(seed);
  g.k1 = static_cast<uint32_t>(seed >> 32);
  g.o0 = static_cast<uint32_t>(offset);
  g.o1 = static_cast<uint32_t>(offset >> 32);
  double t = static_cast<double>(p) * 4294967296.0;
  g.thresh = t >= 4294967295.0 ? 0xffffffffu : static_cast<uint32_t>(t);
  g.scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  return g;
}

int ln_k(int H) { return (H / 4 + 63) / 64; }

// rows per wave per iteration of the wave-per-row LayerNorm kernels (DET_LN_ROWS, 1 or 2) and
// whether H % 8 == 0 rows up to 2048 take them for the forward instead of a workgroup per row
// (DET_LN_FWD=narrow|wide)
int ln_rows_per_wave() {
  static const int r = [] {
    const char* e = std::getenv("DET_LN_ROWS");
    return (e != nullptr && std::atoi(e) == 1) ? 1 : 2;
  }();
  return r;
}
bool ln_bwd_wide_rows() {  // DET_LN_BWD=wide: workgroup-per-row backward for H % 8 == 0 rows up to 2048 too
  static const bool w = [] {
    const char* e = std::getenv("DET_LN_BWD");
    return e != nullptr && std::strcmp(e, "wide") == 0;
  }();
  return w;
}
bool ln_fwd_narrow() {
  static const bool n = [] {
    const char* e = std::getenv("DET_LN_FWD");
    return e != nullptr && std::strcmp(e, "narrow") == 0;
  }();
  return n;
}

// workgroups of the LayerNorm backward (each writes one partial row of dgamma / dbeta / dbias):
// at most DET_LN_BWD_BLOCKS (default 512)
int64_t ln_bwd_blocks(int64_t rows) {
  static const int64_t cap = [] {
    const char* e = std::getenv("DET_LN_BWD_BLOCKS");
    const int64_t v = e != nullptr ? std::atoll(e) : 0;
    return v > 0 ? v : int64_t{512};
  }();
  int64_t b = (rows + kWaves - 1) / kWaves;
  return b < cap ? b : cap;
}

int grid_for(int64_t work, int per_block) {
  int64_t b = (work + per_block - 1) / per_block;
  if (b > 8192) b = 8192;
  return static_cast<int>(b < 1 ? 1 : b);
}

}  // namespace

extern "C" {

// Max hidden size of the LayerNorm kernels (K <= 16 register groups of 256 columns).
int det_tf_ln_max_hidden() { return kMaxH; }

int64_t det_tf_ln_ws_elems(int64_t rows, int H) { return ln_bwd_blocks(rows) * 3 * static_cast<int64_t>(H); }

// dtype: 0 = fp32, 1 = bf16 (x, r, y, gamma, beta all of that dtype).  p = dropout probability
// applied to h (0 disables).  Writes y, mean[rows], rstd[rows].
int det_tf_ln_fwd(void* stream, int dtype, const void* h, const void* r, void* y, int64_t rows, int H,
                  const void* gamma, const void* beta, float eps, float p, uint64_t seed, uint64_t offset,
                  float* mean, float* rstd, const uint32_t* obase) {
  if (H % 4 != 0 || H > kMaxH || rows <= 0) return -1;
  LnArgs a{h, r, y, gamma, beta, mean, rstd, rows, H, eps, p > 0.f, make_rng(p, seed, offset, obase)};
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int R = ln_rows_per_wave();
  if (H % 8 == 0 && !(ln_fwd_narrow() && H <= kMaxNarrowH)) {  // workgroup per row (128 / 256 / 512 threads of 8 columns each)
    const dim3 wg(static_cast<unsigned>(rows < 65536 ? rows : 65536));
#define DET_LNFW(T, VV, NT) hipLaunchKernelGGL((ln_fwd_wide<T, VV, NT>), wg, dim3(NT), 0, st, a)
#define DET_LNFW_T(T)                                   \
    if (H <= 8 * 128) DET_LNFW(T, 1, 128);              \
    else if (H <= 8 * 256) DET_LNFW(T, 1, 256);         \
    else if (H <= 8 * kWideThreads) DET_LNFW(T, 1, 512); \
    else DET_LNFW(T, 2, 512);
    if (dtype == 1) {
      DET_LNFW_T(unsigned short)
    } else {
      DET_LNFW_T(float)
    }
#undef DET_LNFW_T
#undef DET_LNFW
    return static_cast<int>(hipGetLastError());
  }
  if (H > kMaxNarrowH) return -1;
  const int grid = grid_for(rows, kWaves);
  const int K = ln_k(H);
#define DET_LNF(T, KK)                                                                        \
  if (R == 2) hipLaunchKernelGGL((ln_fwd_kernel<T, KK, 2>), dim3(grid), dim3(kThreads), 0, st, a); \
  else hipLaunchKernelGGL((ln_fwd_kernel<T, KK, 1>), dim3(grid), dim3(kThreads), 0, st, a)
#define DET_LNF_K(T)                                                              \
  switch (K) {                                                                    \
    case 1: DET_LNF(T, 1); break;                                                 \
    case 2: DET_LNF(T, 2); break;                                                 \
    case 3: DET_LNF(T, 3); break;                                                 \
    case 4: DET_LNF(T, 4); break;                                                 \
    case 5: case 6: DET_LNF(T, 6); break;                                         \
    default: DET_LNF(T, 8); break;                                                \
  }
  if (dtype == 1) {
    DET_LNF_K(unsigned short)
  } else {
    DET_LNF_K(float)
  }
  return static_cast<int>(hipGetLastError());
}

// Backward of det_tf_ln_fwd.  Outputs (each nullable): dr = dL/dz (the residual's grad),
// dh = dropout'(dz), dgamma, dbeta, dbias = column sums of dh (bias grad of the Linear that
// produced h).  ws: det_tf_ln_ws_elems(rows, H) fp32.
int det_tf_ln_bwd(void* stream, int dtype, const void* dy, const void* h, const void* r, const float* mean,
                  const float* rstd, const void* gamma, int64_t rows, int H, float p, uint64_t seed,
                  uint64_t offset, void* dr, void* dh, void* dgamma, void* dbeta, void* dbias, float* ws,
                  const uint32_t* obase) {
  if (H % 4 != 0 || H > kMaxH || rows <= 0) return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  int blocks = static_cast<int>(ln_bwd_blocks(rows));
  LnBwdArgs a{dy, h, r, mean, rstd, gamma, dr, dh, ws, rows, H, p > 0.f, make_rng(p, seed, offset, obase)};
  if (H > kMaxNarrowH || (ln_bwd_wide_rows() && H % 8 == 0)) {
    if (H % 8 != 0) return -1;
    const bool small = H <= 8 * 128;  // 128-thread rows (DET_LN_BWD=wide at BERT widths)
    if (!small && blocks > 256) blocks = 256;  // <= ln_bwd_blocks(rows): fits det_tf_ln_ws_elems
    const bool v1 = H <= 8 * kWideThreads;
    if (dtype == 1) {
      if (small) hipLaunchKernelGGL((ln_bwd_wide<unsigned short, 1, 128>), dim3(blocks), dim3(128), 0, st, a);
      else if (v1) hipLaunchKernelGGL((ln_bwd_wide<unsigned short, 1, kWideThreads>), dim3(blocks), dim3(kWideThreads), 0, st, a);
      else hipLaunchKernelGGL((ln_bwd_wide<unsigned short, 2, kWideThreads>), dim3(blocks), dim3(kWideThreads), 0, st, a);
      launch_colsum_finalize<unsigned short>(st, ws, blocks, 3 * H, H, static_cast<unsigned short*>(dgamma),
                         static_cast<unsigned short*>(dbeta), static_cast<unsigned short*>(dbias));
    } else {
      if (small) hipLaunchKernelGGL((ln_bwd_wide<float, 1, 128>), dim3(blocks), dim3(128), 0, st, a);
      else if (v1) hipLaunchKernelGGL((ln_bwd_wide<float, 1, kWideThreads>), dim3(blocks), dim3(kWideThreads), 0, st, a);
      else hipLaunchKernelGGL((ln_bwd_wide<float, 2, kWideThreads>), dim3(blocks), dim3(kWideThreads), 0, st, a);
      launch_colsum_finalize<float>(st, ws, blocks, 3 * H, H, static_cast<float*>(dgamma), static_cast<float*>(dbeta),
                         static_cast<float*>(dbias));
    }
    return static_cast<int>(hipGetLastError());
  }
  const size_t lds = static_cast<size_t>(kWaves) * H * sizeof(float);
  const int K = ln_k(H);
  const int R = ln_rows_per_wave();
#define DET_LNB(T, KK)                                                                                  \
  if (R == 2) hipLaunchKernelGGL((ln_bwd_kernel<T, KK, 2>), dim3(blocks), dim3(kThreads), lds, st, a);     \
  else hipLaunchKernelGGL((ln_bwd_kernel<T, KK, 1>), dim3(blocks), dim3(kThreads), lds, st, a)
#define DET_LNB_K(T)                                                              \
  switch (K) {                                                                    \
    case 1: DET_LNB(T, 1); break;                                                 \
    case 2: DET_LNB(T, 2); break;                                                 \
    case 3: DET_LNB(T, 3); break;                                                 \
    case 4: DET_LNB(T, 4); break;                                                 \
    case 5: case 6: DET_LNB(T, 6); break;                                         \
    default: DET_LNB(T, 8); break;                                                \
  }
  if (dtype == 1) {
    DET_LNB_K(unsigned short)
    launch_colsum_finalize<unsigned short>(st, ws, blocks, 3 * H, H, static_cast<unsigned short*>(dgamma),
                       static_cast<unsigned short*>(dbeta), static_cast<unsigned short*>(dbias));
  } else {
    DET_LNB_K(float)
    launch_colsum_finalize<float>(st, ws, blocks, 3 * H, H, static_cast<float*>(dgamma), static_cast<float*>(dbeta),
                       static_cast<float*>(dbias));
  }
  return static_cast<int>(hipGetLastError());
}

int64_t det_tf_col_ws_elems(int64_t rows, int C) {
  ColGeom g = make_col_geom(rows, C);
  return static_cast<int64_t>(g.nrb) * C;
}

// a = gelu(z), elementwise over n elements (n % 8 == 0); approx = 1 selects the tanh form.
int det_tf_gelu_fwd(void* stream, int dtype, const void* z, void* a, int64_t n, int approx) {
  if (n % 8 != 0 || n <= 0) return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t nvec = n / 8;
  const int grid = grid_for(nvec, kThreads * 4);
#define DET_GELUF(T, ACT)                                                                          \
  hipLaunchKernelGGL((gelu_fwd_kernel<T, ACT>), dim3(grid), dim3(kThreads), 0, st, static_cast<const T*>(z), \
                     static_cast<T*>(a), nvec)
  if (dtype == 1) {
    if (approx) DET_GELUF(unsigned short, 1); else DET_GELUF(unsigned short, 0);
  } else {
    if (approx) DET_GELUF(float, 1); else DET_GELUF(float, 0);
  }
#undef DET_GELUF
  return static_cast<int>(hipGetLastError());
}

// dz = da * gelu'(z) over [rows, C]; dbias (nullable) = column sums of dz.  approx = 1: tanh form.
int det_tf_gelu_bwd(void* stream, int dtype, const void* da, const void* z, void* dz, int64_t rows, int C,
                    void* dbias, float* ws, int approx) {
  if (C % 8 != 0 || rows <= 0) return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  ColGeom g = make_col_geom(rows, C);
  dim3 grid(g.nrb, C / 8 / g.tpr);
  float* w = dbias ? ws : nullptr;
  if (dtype == 1) {
    if (approx)
      hipLaunchKernelGGL((col_kernel<unsigned short, 2>), grid, dim3(kThreads), 0, st,
                         static_cast<const unsigned short*>(da), static_cast<const unsigned short*>(z),
                         static_cast<unsigned short*>(dz), g, w);
    else
      hipLaunchKernelGGL((col_kernel<unsigned short, 1>), grid, dim3(kThreads), 0, st,
                         static_cast<const unsigned short*>(da), static_cast<const unsigned short*>(z),
                         static_cast<unsigned short*>(dz), g, w);
    if (dbias)
      launch_colsum_finalize<unsigned short>(st, ws, g.nrb, C, C, static_cast<unsigned short*>(dbias), static_cast<unsigned short*>(nullptr), static_cast<unsigned short*>(nullptr));
  } else {
    if (approx)
      hipLaunchKernelGGL((col_kernel<float, 2>), grid, dim3(kThreads), 0, st, static_cast<const float*>(da),
                         static_cast<const float*>(z), static_cast<float*>(dz), g, w);
    else
      hipLaunchKernelGGL((col_kernel<float, 1>), grid, dim3(kThreads), 0, st, static_cast<const float*>(da),
                         static_cast<const float*>(z), static_cast<float*>(dz), g, w);
    if (dbias)
      launch_colsum_finalize<float>(st, ws,
                         g.nrb, C, C, static_cast<float*>(dbias), static_cast<float*>(nullptr), static_cast<float*>(nullptr));
  }
  return static_cast<int>(hipGetLastError());
}

// out[C] = column sums of x[rows, C] (the bias grad of a Linear), deterministic two-level.
int det_tf_colsum(void* stream, int dtype, const void* x, int64_t rows, int C, void* out, float* ws) {
  if (C % 8 != 0 || rows <= 0) return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  ColGeom g = make_col_geom(rows, C);
  dim3 grid(g.nrb, C / 8 / g.tpr);
  if (dtype == 1) {
    hipLaunchKernelGGL((col_kernel<unsigned short, 0>), grid, dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), nullptr, nullptr, g, ws);
    launch_colsum_finalize<unsigned short>(st, ws, g.nrb, C, C, static_cast<unsigned short*>(out), nullptr, nullptr);
  } else {
    hipLaunchKernelGGL((col_kernel<float, 0>), grid, dim3(kThreads), 0, st, static_cast<const float*>(x), nullptr,
                       nullptr, g, ws);
    launch_colsum_finalize<float>(st, ws,
                       g.nrb, C, C, static_cast<float*>(out), nullptr, nullptr);
  }
  return static_cast<int>(hipGetLastError());
}

// One increment of a dropout offset counter (Rng::obase), stream-ordered: a captured train step
// starts with it, so each replay of the graph draws new masks.
int det_tf_rng_bump(void* stream, uint32_t* counter) {
  if (!counter) return -1;
  hipLaunchKernelGGL(rng_bump_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), counter);
  return static_cast<int>(hipGetLastError());
}

// Materialise the keep-mask (1 = kept) the LN kernels use for [n] elements (n % 4 == 0); tests only.
int det_tf_dropout_mask(void* stream, int64_t n, float p, uint64_t seed, uint64_t offset, uint8_t* out,
                        const uint32_t* obase) {
  if (n % 4 != 0 || n <= 0) return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(grid_for(n / 4, kThreads)), dim3(kThreads), 0, st, n / 4,
                     make_rng(p, seed, offset, obase), out);
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
