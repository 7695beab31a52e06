// det_attention.hip — MFMA self-attention for encoder shapes (head_dim 64, seq <= 512) on gfx950.
//
// Why this exists: BERT-base SQuAD-shape (B 12, S 384, 12 heads x 64) spends 2.2 ms/step in the
// AOTriton attention kernels (profiles/r1_bert_native_bs12_o2_steady.csv), ~105 TFLOP/s — 4 % of
// the bf16 MFMA roof.  At S <= 512 a whole head's K and V fit on-chip, so each wave can hold a
// 32-query x S-key score block in accumulators: exact softmax, no online rescaling, no S x S
// matrix in memory.
//
// Forward (one workgroup = 4 waves = 128 queries of one (batch, head); wave = 32 queries):
//   1. stage V^T of the head into LDS ([d][key], row stride S+4 bf16: conflict-free 8-byte
//      fragment reads) and the key bias (log2 units) — the only barrier of the kernel;
//   2. S^T = K . Q^T with v_mfma_f32_32x32x16_bf16: A = K (16-B rows straight from global/L2),
//      B = Q^T (the lane's query row, loaded once), so every lane owns ONE query and its S keys
//      sit in the accumulator registers (T = S/32 tiles x 16);
//   3. softmax along the registers: max/sum in-lane + one lane^32 exchange; LSE = ln sum exp;
//   4. dropout: keep mask from a keyed 32-bit hash of the (b, h, q, key/2) index (two 16-bit
//      draws per hash) — regenerable bit-exactly in the backward pass;
//   5. O^T = V^T . P^T: the P accumulators are converted to bf16 in place and used as the B
//      operand (k = key rows), A = V^T fragments from LDS; O = O^T / l written as [B, S, nh, 64].
//
// Inputs are the fused QKV GEMM output [B, S, 3, nh, 64] (row stride 3H) and an additive per-key
// bias [B, S] (BERT's padding mask); outputs O [B, S, nh*64] and LSE [B, nh, S] (fp32, natural log
// of the scaled scores), which the backward kernels (below) consume.
//
// Reference parity: the reference runs attention inside HuggingFace BERT on torch
// (examples/nlp/bert_squad_pytorch/model_def.py); semantics = softmax(QK^T/sqrt(d) + bias) with
// dropout on the probabilities, as torch.nn.functional.scaled_dot_product_attention.

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kHD = 64;        // head dim
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kQB = 32 * kWaves;  // queries per workgroup

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned short us4;
typedef __attribute__((ext_vector_type(8))) unsigned short us8;

__device__ __forceinline__ float bf2f(unsigned short u) { return __uint_as_float(static_cast<uint32_t>(u) << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<unsigned short>((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<unsigned short>(u >> 16);
}

// keyed 32-bit mixer (lowbias32, C. Wellons) — dropout draws, 2 x 16 bits per call
__device__ __forceinline__ uint32_t mix32(uint32_t x, uint32_t key) {
  x ^= key;
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

struct AttnArgs {
  const unsigned short* qkv;  // [B, S, 3, nh, 64] bf16
  const float* bias;          // [B, S] additive key bias (natural units) or null
  unsigned short* out;        // [B, S, nh, 64] bf16
  float* lse;                 // [B, nh, S]
  int B, S, nh;
  float scale_log2;           // log2(e) / sqrt(64)
  uint32_t drop_thr;          // drop if 16-bit draw < thr (0: no dropout)
  float drop_scale;           // 65536 / (65536 - thr)
  uint32_t rng_key;
};

__device__ __forceinline__ uint32_t rng_key_for(uint32_t base_key, int b, int head) {
  return base_key ^ (static_cast<uint32_t>(b * 977 + head) * 0x9E3779B9u);
}

template <int T>  // T = S / 32 key tiles
__global__ void __launch_bounds__(kThreads, 1) attn_fwd_kernel(AttnArgs a) {
  extern __shared__ unsigned char smem[];
  const int S = a.S;
  const int vstride = S + 4;  // bf16 elements per V^T row
  unsigned short* vt = reinterpret_cast<unsigned short*>(smem);
  float* biasl = reinterpret_cast<float*>(smem + static_cast<size_t>(kHD) * vstride * 2);
  const int b = blockIdx.z, head = blockIdx.y;
  const int H = a.nh * kHD;
  const int64_t tok = 3LL * H;  // elements between consecutive tokens
  const unsigned short* base = a.qkv + static_cast<int64_t>(b) * S * tok + head * kHD;
  const unsigned short* kbase = base + H;
  const unsigned short* vbase = base + 2 * H;

  // ---- stage V^T and the bias -------------------------------------------------------------
  for (int i = threadIdx.x; i < (S / 2) * 8; i += kThreads) {
    const int kp = i >> 3, dg = i & 7;
    const us8 v0 = *reinterpret_cast<const us8*>(vbase + static_cast<int64_t>(2 * kp) * tok + dg * 8);
    const us8 v1 = *reinterpret_cast<const us8*>(vbase + static_cast<int64_t>(2 * kp + 1) * tok + dg * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t w = static_cast<uint32_t>(v0[e]) | (static_cast<uint32_t>(v1[e]) << 16);
      *reinterpret_cast<uint32_t*>(vt + (dg * 8 + e) * vstride + 2 * kp) = w;
    }
  }
  for (int i = threadIdx.x; i < S; i += kThreads) {
    float bv = a.bias ? a.bias[static_cast<int64_t>(b) * S + i] * 1.4426950408889634f : 0.f;
    biasl[i] = fmaxf(bv, -1e30f);  // finite: fully masked rows degrade to uniform, like fp32 torch
  }
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQB + wave * 32;
  if (q0 >= S) return;
  const int q = q0 + r;

  // ---- Q^T fragments (B operand): Q[q][16s + 8h + j] ---------------------------------------
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qf[s] = *reinterpret_cast<const bf16x8*>(base + static_cast<int64_t>(q) * tok + 16 * s + 8 * hh);

  // ---- S^T = K . Q^T -----------------------------------------------------------------------
  f32x16 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    acc[t] = f32x16{0};
    const unsigned short* krow = kbase + static_cast<int64_t>(32 * t + r) * tok + 8 * hh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(krow + 16 * s);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], acc[t], 0, 0, 0);
    }
  }

  // ---- softmax over the lane's keys (log2 domain) -------------------------------------------
  float m = -3.0e38f;
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 bv = *reinterpret_cast<const float4*>(biasl + 32 * t + 8 * g + 4 * hh);
      const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = fmaf(acc[t][4 * g + e], a.scale_log2, bb[e]);
        acc[t][4 * g + e] = x;
        m = fmaxf(m, x);
      }
    }
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float l = 0.f;
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = exp2f(acc[t][i] - m);
      acc[t][i] = p;
      l += p;
    }
  l += __shfl_xor(l, 32, 64);
  if (hh == 0) a.lse[(static_cast<int64_t>(b) * a.nh + head) * S + q] = (m + log2f(l)) * 0.6931471805599453f;

  // ---- dropout on P (keys 4g..4g+3 of each tile = 2 hashes) ---------------------------------
  if (a.drop_thr) {
    const uint32_t key = rng_key_for(a.rng_key, b, head);
    const uint32_t row = static_cast<uint32_t>(q) * static_cast<uint32_t>(S);
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t k0 = 32 * t + 8 * g + 4 * hh;
        const uint32_t h0 = mix32((row + k0) >> 1, key), h1 = mix32((row + k0 + 2) >> 1, key);
        const uint32_t d4[4] = {h0 & 0xffffu, h0 >> 16, h1 & 0xffffu, h1 >> 16};
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[t][4 * g + e] *= d4[e] < a.drop_thr ? 0.f : a.drop_scale;
      }
  }

  // ---- O^T = V^T . P^T -----------------------------------------------------------------------
  f32x16 o[2] = {f32x16{0}, f32x16{0}};
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[j] = static_cast<short>(f2bf(acc[t][8 * s + j]));
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const unsigned short* vrow = vt + (32 * u + r) * vstride + 32 * t + 16 * s + 4 * hh;
        const us4 lo = *reinterpret_cast<const us4*>(vrow);
        const us4 hi = *reinterpret_cast<const us4*>(vrow + 8);
        bf16x8 vf;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          vf[j] = static_cast<short>(lo[j]);
          vf[4 + j] = static_cast<short>(hi[j]);
        }
        o[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[u], 0, 0, 0);
      }
    }

  // ---- O = O^T / l -> [B, S, nh, 64] ---------------------------------------------------------
  const float inv_l = 1.f / l;
  unsigned short* orow = a.out + ((static_cast<int64_t>(b) * S + q) * a.nh + head) * kHD;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      us4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = f2bf(o[u][4 * g + e] * inv_l);
      *reinterpret_cast<us4*>(orow + 32 * u + 8 * g + 4 * hh) = w;
    }
}


// =============================================================================================
// Backward.  With Pd = P o Z/(1-p) (dropout keep mask Z), D_q = sum_d dO o O (= sum_k Pd dPd):
//   dV = Pd^T dO,  dPd = dO V^T,  dS = P o (dPd o Z/(1-p) - D),  dQ = dS K / 8,  dK = dS^T Q / 8.
// Two kernels so that no gradient needs a cross-workgroup sum:
//   attn_bwd_dq  (query on the lane, like the forward): S^T, dPd^T per key tile, dQ^T += K^T dS^T
//                with a K^T LDS image; also writes D (consumed by the next kernel);
//   attn_bwd_dkv (key on the lane): S, dPd per query tile, dV^T += dO^T Pd and dK^T += Q^T dS with
//                Q^T / dO^T LDS images of the whole head.
// Both write straight into the packed dQKV [B, S, 3, nh, 64] gradient of the fused QKV GEMM.
// =============================================================================================
struct BwdArgs {
  const unsigned short* qkv;   // [B, S, 3, nh, 64]
  const float* bias;           // [B, S] or null
  const unsigned short* out;   // O  [B, S, nh, 64]
  const unsigned short* dout;  // dO [B, S, nh, 64]
  const float* lse;            // [B, nh, S]
  float* delta;                // [B, nh, S]
  unsigned short* dqkv;        // [B, S, 3, nh, 64]
  int B, S, nh;
  float scale_log2;
  uint32_t drop_thr;
  float drop_scale;
  uint32_t rng_key;
};

// stage X^T ([64][S+4] bf16) of a [S, 64]-row operand whose token stride is `tok` elements
__device__ __forceinline__ void stage_transposed(unsigned short* dst, const unsigned short* src, int64_t tok, int S,
                                                 int stride) {
  for (int i = threadIdx.x; i < (S / 2) * 8; i += kThreads) {
    const int kp = i >> 3, dg = i & 7;
    const us8 v0 = *reinterpret_cast<const us8*>(src + static_cast<int64_t>(2 * kp) * tok + dg * 8);
    const us8 v1 = *reinterpret_cast<const us8*>(src + static_cast<int64_t>(2 * kp + 1) * tok + dg * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t w = static_cast<uint32_t>(v0[e]) | (static_cast<uint32_t>(v1[e]) << 16);
      *reinterpret_cast<uint32_t*>(dst + (dg * 8 + e) * stride + 2 * kp) = w;
    }
  }
}

// A operand of an X^T image: lane (r, h) elements j = X[k0 + 8(j>>2) + 4h + (j&3)][row] (k-permuted)
__device__ __forceinline__ bf16x8 frag_from_image(const unsigned short* img, int stride, int row, int k0, int hh) {
  const unsigned short* p = img + row * stride + k0 + 4 * hh;
  const us4 lo = *reinterpret_cast<const us4*>(p);
  const us4 hi = *reinterpret_cast<const us4*>(p + 8);
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[j] = static_cast<short>(lo[j]);
    f[4 + j] = static_cast<short>(hi[j]);
  }
  return f;
}

__device__ __forceinline__ bf16x8 pack_frag(const f32x16& x, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = static_cast<short>(f2bf(x[8 * s + j]));
  return f;
}

template <int T>
__global__ void __launch_bounds__(kThreads, 1) attn_bwd_dq_kernel(BwdArgs a) {
  extern __shared__ unsigned char smem[];
  const int S = a.S, stride = S + 4;
  unsigned short* kt = reinterpret_cast<unsigned short*>(smem);
  float* biasl = reinterpret_cast<float*>(smem + static_cast<size_t>(kHD) * stride * 2);
  const int b = blockIdx.z, head = blockIdx.y;
  const int H = a.nh * kHD;
  const int64_t tok = 3LL * H;
  const unsigned short* base = a.qkv + static_cast<int64_t>(b) * S * tok + head * kHD;
  const unsigned short* kbase = base + H;
  const unsigned short* vbase = base + 2 * H;
  stage_transposed(kt, kbase, tok, S, stride);
  for (int i = threadIdx.x; i < S; i += kThreads) {
    float bv = a.bias ? a.bias[static_cast<int64_t>(b) * S + i] * 1.4426950408889634f : 0.f;
    biasl[i] = fmaxf(bv, -1e30f);
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQB + wave * 32;
  if (q0 >= S) return;
  const int q = q0 + r;
  const int64_t orow = ((static_cast<int64_t>(b) * S + q) * a.nh + head) * kHD;
  bf16x8 qf[4], df[4];
  float dsum = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = *reinterpret_cast<const bf16x8*>(base + static_cast<int64_t>(q) * tok + 16 * s + 8 * hh);
    df[s] = *reinterpret_cast<const bf16x8*>(a.dout + orow + 16 * s + 8 * hh);
    const us8 ov = *reinterpret_cast<const us8*>(a.out + orow + 16 * s + 8 * hh);
#pragma unroll
    for (int j = 0; j < 8; ++j) dsum = fmaf(bf2f(static_cast<unsigned short>(df[s][j])), bf2f(ov[j]), dsum);
  }
  const float D = dsum + __shfl_xor(dsum, 32, 64);
  const int64_t li = (static_cast<int64_t>(b) * a.nh + head) * S + q;
  if (hh == 0) a.delta[li] = D;
  const float lse2 = a.lse[li] * 1.4426950408889634f;
  const uint32_t key = rng_key_for(a.rng_key, b, head);
  const uint32_t rowidx = static_cast<uint32_t>(q) * static_cast<uint32_t>(S);
  f32x16 dqt[2] = {f32x16{0}, f32x16{0}};
#pragma unroll 2
  for (int t = 0; t < T; ++t) {
    f32x16 sa = f32x16{0}, dp = f32x16{0};
    const unsigned short* krow = kbase + static_cast<int64_t>(32 * t + r) * tok + 8 * hh;
    const unsigned short* vrow = vbase + static_cast<int64_t>(32 * t + r) * tok + 8 * hh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(krow + 16 * s), qf[s], sa, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(vrow + 16 * s), df[s], dp, 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int k0 = 32 * t + 8 * g + 4 * hh;
      const float4 bv = *reinterpret_cast<const float4*>(biasl + k0);
      const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
      float z[4] = {1.f, 1.f, 1.f, 1.f};
      if (a.drop_thr) {
        const uint32_t h0 = mix32((rowidx + k0) >> 1, key), h1 = mix32((rowidx + k0 + 2) >> 1, key);
        const uint32_t d4[4] = {h0 & 0xffffu, h0 >> 16, h1 & 0xffffu, h1 >> 16};
#pragma unroll
        for (int e = 0; e < 4; ++e) z[e] = d4[e] < a.drop_thr ? 0.f : a.drop_scale;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g + e;
        const float p = exp2f(fmaf(sa[i], a.scale_log2, bb[e]) - lse2);
        sa[i] = p * fmaf(dp[i], z[e], -D);  // dS^T
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 dsf = pack_frag(sa, s);
#pragma unroll
      for (int u = 0; u < 2; ++u)
        dqt[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_from_image(kt, stride, 32 * u + r, 32 * t + 16 * s, hh),
                                                         dsf, dqt[u], 0, 0, 0);
    }
  }
  unsigned short* dq = a.dqkv + (static_cast<int64_t>(b) * S + q) * tok + head * kHD;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      us4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = f2bf(dqt[u][4 * g + e] * 0.125f);
      *reinterpret_cast<us4*>(dq + 32 * u + 8 * g + 4 * hh) = w;
    }
}

template <int T>
__global__ void __launch_bounds__(kThreads, 1) attn_bwd_dkv_kernel(BwdArgs a) {
  extern __shared__ unsigned char smem[];
  const int S = a.S, stride = S + 4;
  unsigned short* qt = reinterpret_cast<unsigned short*>(smem);
  unsigned short* dot = qt + kHD * stride;
  float* lse2 = reinterpret_cast<float*>(dot + kHD * stride);
  float* dl = lse2 + S;
  const int b = blockIdx.z, head = blockIdx.y;
  const int H = a.nh * kHD;
  const int64_t tok = 3LL * H;
  const unsigned short* base = a.qkv + static_cast<int64_t>(b) * S * tok + head * kHD;
  const unsigned short* dobase = a.dout + static_cast<int64_t>(b) * S * H + head * kHD;
  stage_transposed(qt, base, tok, S, stride);
  stage_transposed(dot, dobase, H, S, stride);
  const int64_t lrow = (static_cast<int64_t>(b) * a.nh + head) * S;
  for (int i = threadIdx.x; i < S; i += kThreads) {
    lse2[i] = a.lse[lrow + i] * 1.4426950408889634f;
    dl[i] = a.delta[lrow + i];
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int k0w = blockIdx.x * kQB + wave * 32;
  if (k0w >= S) return;
  const int kk = k0w + r;  // this lane's key
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(base + H + static_cast<int64_t>(kk) * tok + 16 * s + 8 * hh);
    vf[s] = *reinterpret_cast<const bf16x8*>(base + 2 * H + static_cast<int64_t>(kk) * tok + 16 * s + 8 * hh);
  }
  float bk = a.bias ? fmaxf(a.bias[static_cast<int64_t>(b) * S + kk] * 1.4426950408889634f, -1e30f) : 0.f;
  const uint32_t key = rng_key_for(a.rng_key, b, head);
  f32x16 dkt[2] = {f32x16{0}, f32x16{0}}, dvt[2] = {f32x16{0}, f32x16{0}};
#pragma unroll 2
  for (int tq = 0; tq < T; ++tq) {
    f32x16 sa = f32x16{0}, dp = f32x16{0};
    const unsigned short* qrow = base + static_cast<int64_t>(32 * tq + r) * tok + 8 * hh;
    const unsigned short* drow = dobase + static_cast<int64_t>(32 * tq + r) * H + 8 * hh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(qrow + 16 * s), kf[s], sa, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(drow + 16 * s), vf[s], dp, 0, 0, 0);
    }
    f32x16 pd;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int qb = 32 * tq + 8 * g + 4 * hh;
      const float4 lv = *reinterpret_cast<const float4*>(lse2 + qb);
      const float4 dv = *reinterpret_cast<const float4*>(dl + qb);
      const float ll[4] = {lv.x, lv.y, lv.z, lv.w}, dd[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g + e;
        float z = 1.f;
        if (a.drop_thr) {
          const uint32_t idx = static_cast<uint32_t>(qb + e) * static_cast<uint32_t>(S) + kk;
          const uint32_t hsh = mix32(idx >> 1, key);
          z = ((kk & 1) ? (hsh >> 16) : (hsh & 0xffffu)) < a.drop_thr ? 0.f : a.drop_scale;
        }
        const float p = exp2f(fmaf(sa[i], a.scale_log2, bk) - ll[e]);
        pd[i] = p * z;
        sa[i] = p * fmaf(dp[i], z, -dd[e]);  // dS
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pf = pack_frag(pd, s), dsf = pack_frag(sa, s);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        dvt[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_from_image(dot, stride, 32 * u + r, 32 * tq + 16 * s, hh),
                                                         pf, dvt[u], 0, 0, 0);
        dkt[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_from_image(qt, stride, 32 * u + r, 32 * tq + 16 * s, hh),
                                                         dsf, dkt[u], 0, 0, 0);
      }
    }
  }
  unsigned short* dk = a.dqkv + (static_cast<int64_t>(b) * S + kk) * tok + H + head * kHD;
  unsigned short* dv = dk + H;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      us4 wk, wv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        wk[e] = f2bf(dkt[u][4 * g + e] * 0.125f);
        wv[e] = f2bf(dvt[u][4 * g + e]);
      }
      *reinterpret_cast<us4*>(dk + 32 * u + 8 * g + 4 * hh) = wk;
      *reinterpret_cast<us4*>(dv + 32 * u + 8 * g + 4 * hh) = wv;
    }
}

__global__ void attn_mask_kernel(int B, int nh, int S, uint32_t thr, uint32_t base_key, uint8_t* out) {
  const int64_t n = static_cast<int64_t>(B) * nh * S * S;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int key = static_cast<int>(i % S);
    const int q = static_cast<int>((i / S) % S);
    const int head = static_cast<int>((i / S / S) % nh);
    const int b = static_cast<int>(i / S / S / nh);
    const uint32_t idx = static_cast<uint32_t>(q) * static_cast<uint32_t>(S) + key;
    const uint32_t h = mix32(idx >> 1, rng_key_for(base_key, b, head));
    const uint32_t d = (idx & 1) ? (h >> 16) : (h & 0xffffu);
    out[i] = d >= thr;
  }
}

void fill_args(AttnArgs& a, const void* qkv, const float* bias, void* out, float* lse, int B, int S, int nh,
               float p, uint64_t seed, uint64_t offset) {
  a.qkv = static_cast<const unsigned short*>(qkv);
  a.bias = bias;
  a.out = static_cast<unsigned short*>(out);
  a.lse = lse;
  a.B = B;
  a.S = S;
  a.nh = nh;
  a.scale_log2 = 1.4426950408889634f * 0.125f;
  uint32_t thr = p > 0.f ? static_cast<uint32_t>(p * 65536.0f + 0.5f) : 0u;
  if (thr > 65535u) thr = 65535u;
  a.drop_thr = thr;
  a.drop_scale = thr ? 65536.0f / static_cast<float>(65536u - thr) : 1.f;
  a.rng_key = static_cast<uint32_t>(seed) ^ static_cast<uint32_t>(seed >> 32) * 0x85ebca6bu ^
              static_cast<uint32_t>(offset) * 0xc2b2ae35u ^ static_cast<uint32_t>(offset >> 32);
}

size_t fwd_lds(int S) { return static_cast<size_t>(kHD) * (S + 4) * 2 + static_cast<size_t>(S) * 4; }

}  // namespace

extern "C" {

// Shapes the MFMA path covers: head_dim 64, S in {128, 256, 384, 512}.
int det_attn_supported(int S, int head_dim) {
  return head_dim == kHD && (S == 128 || S == 256 || S == 384 || S == 512);
}

// qkv [B, S, 3, nh, 64] bf16; bias [B, S] fp32 (nullable); out [B, S, nh*64] bf16; lse [B, nh, S].
int det_attn_fwd(void* stream, const void* qkv, const float* bias, void* out, float* lse, int B, int S, int nh,
                 float p, uint64_t seed, uint64_t offset) {
  if (!det_attn_supported(S, kHD) || B <= 0 || nh <= 0) return -1;
  AttnArgs a;
  fill_args(a, qkv, bias, out, lse, B, S, nh, p, seed, offset);
  hipStream_t st = static_cast<hipStream_t>(stream);
  dim3 grid((S + kQB - 1) / kQB, nh, B);
  const size_t lds = fwd_lds(S);
  switch (S / 32) {
    case 4: hipLaunchKernelGGL(attn_fwd_kernel<4>, grid, dim3(kThreads), lds, st, a); break;
    case 8: hipLaunchKernelGGL(attn_fwd_kernel<8>, grid, dim3(kThreads), lds, st, a); break;
    case 12: hipLaunchKernelGGL(attn_fwd_kernel<12>, grid, dim3(kThreads), lds, st, a); break;
    default: hipLaunchKernelGGL(attn_fwd_kernel<16>, grid, dim3(kThreads), lds, st, a); break;
  }
  return static_cast<int>(hipGetLastError());
}

// Backward: dqkv [B, S, 3, nh, 64] (fully overwritten); delta: [B, nh, S] fp32 workspace.
int det_attn_bwd(void* stream, const void* qkv, const float* bias, const void* out, const void* dout, const float* lse,
                 float* delta, void* dqkv, int B, int S, int nh, float p, uint64_t seed, uint64_t offset) {
  if (!det_attn_supported(S, kHD) || B <= 0 || nh <= 0) return -1;
  AttnArgs f;
  fill_args(f, qkv, bias, nullptr, nullptr, B, S, nh, p, seed, offset);
  BwdArgs a;
  a.qkv = static_cast<const unsigned short*>(qkv);
  a.bias = bias;
  a.out = static_cast<const unsigned short*>(out);
  a.dout = static_cast<const unsigned short*>(dout);
  a.lse = lse;
  a.delta = delta;
  a.dqkv = static_cast<unsigned short*>(dqkv);
  a.B = B;
  a.S = S;
  a.nh = nh;
  a.scale_log2 = f.scale_log2;
  a.drop_thr = f.drop_thr;
  a.drop_scale = f.drop_scale;
  a.rng_key = f.rng_key;
  hipStream_t st = static_cast<hipStream_t>(stream);
  dim3 grid((S + kQB - 1) / kQB, nh, B);
  const size_t lds_dq = static_cast<size_t>(kHD) * (S + 4) * 2 + static_cast<size_t>(S) * 4;
  const size_t lds_dkv = 2 * static_cast<size_t>(kHD) * (S + 4) * 2 + 2 * static_cast<size_t>(S) * 4;
#define DET_ATTN_BWD(TT)                                                                         \
  hipLaunchKernelGGL(attn_bwd_dq_kernel<TT>, grid, dim3(kThreads), lds_dq, st, a);              \
  hipLaunchKernelGGL(attn_bwd_dkv_kernel<TT>, grid, dim3(kThreads), lds_dkv, st, a)
  switch (S / 32) {
    case 4: DET_ATTN_BWD(4); break;
    case 8: DET_ATTN_BWD(8); break;
    case 12: DET_ATTN_BWD(12); break;
    default: DET_ATTN_BWD(16); break;
  }
#undef DET_ATTN_BWD
  return static_cast<int>(hipGetLastError());
}

// The keep mask (1 = kept) the kernels derive for (p, seed, offset): [B, nh, S, S] uint8 (tests).
int det_attn_dropout_mask(void* stream, int B, int nh, int S, float p, uint64_t seed, uint64_t offset, uint8_t* out) {
  AttnArgs a;
  fill_args(a, nullptr, nullptr, nullptr, nullptr, B, S, nh, p, seed, offset);
  hipLaunchKernelGGL(attn_mask_kernel, dim3(2048), dim3(256), 0, static_cast<hipStream_t>(stream), B, nh, S,
                     a.drop_thr, a.rng_key, out);
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
