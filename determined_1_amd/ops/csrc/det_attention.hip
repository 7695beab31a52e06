// det_attention.hip — MFMA self-attention for encoder shapes (head_dim 64, S % 64 == 0, S <= 2048)
// on gfx950, forward and backward, with regenerable dropout on the probabilities.
//
// Why this exists: BERT-base SQuAD-shape (B 12, S 384, 12 heads x 64) spent 2.2 ms/step in the
// AOTriton attention kernels (profiles/r1_bert_native_bs12_o2_steady.csv), ~105 TFLOP/s; these
// kernels take 0.99 ms (profiles/r1_bert_native_fa_bs12_o2_per_step.txt).
//
// Layout: Q/K/V are read straight from the fused QKV GEMM output [B, S, 3, nh, 64] (token stride
// 3H) and dQ/dK/dV written straight into its gradient, so no split/pack copies exist; the key bias
// is an additive per-key row [B, S] (BERT's padding mask).  O is [B, S, nh*64]; LSE [B, nh, S] is
// the natural-log normaliser the backward recomputes P from.
//
// All three kernels share one structure: a workgroup = 4 waves = 128 rows (queries, or keys for
// dK/dV) of one (batch, head), one row per lane (v_mfma_f32_32x32x16_bf16 with the row on the
// accumulator COLUMN, i.e. S^T = K . Q^T, so softmax reductions are in-lane plus one lane^32
// exchange), and the other operand streamed in 64-token blocks that are double-buffered in LDS:
// the next block is loaded into registers before the current block's MFMAs and written to the
// other buffer after them (one barrier per block).  Row-major tiles use an XOR-swizzled 16-B chunk
// layout (conflict-free A-fragment reads); operands consumed along the token axis get a
// transposed [64][64+4] image written in the same pass.  An accumulator converted to bf16 in
// registers is directly the B operand of the next product (k order permuted to match,
// frag_from_image / pack_frag).
//   forward : per key block S^T, online softmax (running max/sum in the log2 domain), O^T += V^T P^T
//   dQ      : per key block S^T, dP^T, dS^T = P o (dP^T o Z/(1-p) - D), dQ^T += K^T dS^T; writes D
//   dK, dV  : per query block S, dP, dV^T += dO^T Pd, dK^T += Q^T dS (no cross-workgroup sums)
// Dropout keep masks come from a keyed 32-bit hash of (b, h, q*S + key) (two 16-bit draws per
// hash), regenerated bit-exactly in the backward pass.
//
// Reference parity: the reference runs attention inside HuggingFace BERT/ALBERT on torch
// (examples/nlp/bert_squad_pytorch/model_def.py, examples/nlp/albert_squad_pytorch/model_def.py);
// semantics = softmax(QK^T/sqrt(d) + bias) with dropout on the probabilities, as
// torch.nn.functional.scaled_dot_product_attention.

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
// RNE conversion; the compiler pairs adjacent conversions into gfx950's v_cvt_pk_bf16_f32 (one VALU
// op per two elements instead of the ~6-op bit-twiddling sequence, which made the softmax/P packing
// phases VALU-bound at one wave per SIMD)
__device__ __forceinline__ unsigned short f2bf(float f) {
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));
}
// v_exp_f32 directly (exp2f adds a denormal range-reduction sequence; softmax arguments are <= 0)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

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

// ---- forward tiles: 64 keys per block, double-buffered in LDS -----------------------------------
constexpr int kKB = 64;                                     // keys per block
constexpr int kVtStride = kKB + 4;                          // V^T tile row stride (bf16): 136 B
constexpr int kKTileBytes = kKB * kHD * 2;                  // K tile [64 keys][64 d], 128-B rows
constexpr int kVTileBytes = kHD * kVtStride * 2;            // V^T tile [64 d][64 keys + 4]
constexpr int kFwdBufBytes = kKTileBytes + kVTileBytes;

// byte offset of 16-B chunk `ch` (0..7) of K-tile row `row`: XOR swizzle so that the 32 rows an
// MFMA A-fragment read touches (same chunk, consecutive rows) spread over all LDS banks
__device__ __forceinline__ int kswz(int row, int ch) { return row * 128 + 16 * (ch ^ (row & 7)); }

struct TileRegs {
  us8 k[2], v[2];
};

// thread i: K chunk (i & 7) of keys i>>3 and (i>>3)+32; V d-group (i & 7) of the key pair 2(i>>3), 2(i>>3)+1
__device__ __forceinline__ void load_tile(TileRegs& t, const unsigned short* kbase, const unsigned short* vbase,
                                          int64_t tok, int key0) {
  const int c = threadIdx.x & 7, kr = threadIdx.x >> 3;
  t.k[0] = *reinterpret_cast<const us8*>(kbase + static_cast<int64_t>(key0 + kr) * tok + 8 * c);
  t.k[1] = *reinterpret_cast<const us8*>(kbase + static_cast<int64_t>(key0 + kr + 32) * tok + 8 * c);
  t.v[0] = *reinterpret_cast<const us8*>(vbase + static_cast<int64_t>(key0 + 2 * kr) * tok + 8 * c);
  t.v[1] = *reinterpret_cast<const us8*>(vbase + static_cast<int64_t>(key0 + 2 * kr + 1) * tok + 8 * c);
}

__device__ __forceinline__ void store_tile(const TileRegs& t, unsigned char* buf) {
  const int c = threadIdx.x & 7, kr = threadIdx.x >> 3;
  *reinterpret_cast<us8*>(buf + kswz(kr, c)) = t.k[0];
  *reinterpret_cast<us8*>(buf + kswz(kr + 32, c)) = t.k[1];
  unsigned short* vt = reinterpret_cast<unsigned short*>(buf + kKTileBytes);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t w = static_cast<uint32_t>(t.v[0][e]) | (static_cast<uint32_t>(t.v[1][e]) << 16);
    *reinterpret_cast<uint32_t*>(vt + (8 * c + e) * kVtStride + 2 * kr) = w;
  }
}

// A operand of an X^T image: lane (r, h) elements j = X[k0 + 8(j>>2) + 4h + (j&3)][row] (k-permuted
// to match an accumulator packed as a B operand, see pack_frag)
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

// Flash-style forward: one workgroup = 4 waves = 128 queries of one (batch, head), wave = 32
// queries, lane = one query (its 32 keys of a 64-key block in two S^T accumulators).  Per key block:
//   S^T = K . Q^T (8 MFMA 32x32x16, K fragments from the swizzled LDS tile, Q^T in registers),
//   online softmax in the log2 domain (running max m / partial sum l per lane, one lane^32 max
//   exchange per block), O^T = O^T * alpha + V^T . P^T (8 MFMA, P packed to bf16 in registers).
// The next block's K/V are loaded into registers before the current block's MFMAs and written to
// the other LDS buffer after them: one barrier per block, global latency behind the math.
// Register footprint is independent of S (~110 VGPR): two workgroups per CU-SIMD pair.
__global__ void __launch_bounds__(kThreads, 2) attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = a.S;
  float* biasl = reinterpret_cast<float*>(smem + 2 * kFwdBufBytes);
  const int b = blockIdx.z, head = blockIdx.y;
  const int H = a.nh * kHD;
  const int64_t tok = 3LL * H;  // elements between consecutive tokens
  const unsigned short* base = a.qkv + static_cast<int64_t>(b) * S * tok + head * kHD;
  const unsigned short* kbase = base + H;
  const unsigned short* vbase = base + 2 * H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQB + wave * 32;
  const bool active = q0 < S;  // inactive waves still stage tiles (no early return: barriers below)
  const int q = active ? q0 + r : S - 1;

  TileRegs tr;
  load_tile(tr, kbase, vbase, tok, 0);
  for (int i = threadIdx.x; i < S; i += kThreads) {
    const float bv = a.bias ? a.bias[static_cast<int64_t>(b) * S + i] * 1.4426950408889634f : 0.f;
    biasl[i] = fmaxf(bv, -1e30f);  // finite: fully masked rows degrade to uniform, like fp32 torch
  }
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qf[s] = *reinterpret_cast<const bf16x8*>(base + static_cast<int64_t>(q) * tok + 16 * s + 8 * hh);
  store_tile(tr, smem);
  __syncthreads();

  const uint32_t key = rng_key_for(a.rng_key, b, head);
  const uint32_t rowidx = static_cast<uint32_t>(q) * static_cast<uint32_t>(S);
  float m = -INFINITY, l = 0.f;
  f32x16 o[2] = {f32x16{0}, f32x16{0}};
  const int nkb = S / kKB;
  for (int kb = 0; kb < nkb; ++kb) {
    const unsigned char* buf = smem + (kb & 1) * kFwdBufBytes;
    const unsigned short* vt = reinterpret_cast<const unsigned short*>(buf + kKTileBytes);
    if (kb + 1 < nkb) load_tile(tr, kbase, vbase, tok, (kb + 1) * kKB);

    f32x16 sc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sc[t] = f32x16{0};
#pragma unroll
      for (int s = 0; s < 4; ++s)
        sc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            *reinterpret_cast<const bf16x8*>(buf + kswz(32 * t + r, 2 * s + hh)), qf[s], sc[t], 0, 0, 0);
    }
    // scores in log2 units + key bias; block max over the lane pair (q, q^32)
    float mb = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 bv = *reinterpret_cast<const float4*>(biasl + kb * kKB + 32 * t + 8 * g + 4 * hh);
        const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = fmaf(sc[t][4 * g + e], a.scale_log2, bb[e]);
          sc[t][4 * g + e] = x;
          mb = fmaxf(mb, x);
        }
      }
    mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
    const float mn = fmaxf(m, mb);
    const float alpha = fast_exp2(m - mn);
    m = mn;
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = fast_exp2(sc[t][i] - mn);
        sc[t][i] = p;
        ls += p;
      }
    l = fmaf(l, alpha, ls);
    if (__any(alpha != 1.f)) {  // no lane's running max moved: the rescale is an exact no-op
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[u][i] *= alpha;
    }
    if (a.drop_thr) {  // keys 4g..4g+3 of each 32-key tile = 2 hashes (same draws as the backward)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t k0 = kb * kKB + 32 * t + 8 * g + 4 * hh;
          const uint32_t h0 = mix32((rowidx + k0) >> 1, key), h1 = mix32((rowidx + k0 + 2) >> 1, key);
          const uint32_t d4[4] = {h0 & 0xffffu, h0 >> 16, h1 & 0xffffu, h1 >> 16};
#pragma unroll
          for (int e = 0; e < 4; ++e) sc[t][4 * g + e] *= d4[e] < a.drop_thr ? 0.f : a.drop_scale;
        }
    }
    // O^T += V^T . P^T
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = pack_frag(sc[t], s);
#pragma unroll
        for (int u = 0; u < 2; ++u)
          o[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_from_image(vt, kVtStride, 32 * u + r, 32 * t + 16 * s, hh),
                                                         pf, o[u], 0, 0, 0);
      }
    if (kb + 1 < nkb) store_tile(tr, smem + ((kb + 1) & 1) * kFwdBufBytes);
    __syncthreads();
  }
  l += __shfl_xor(l, 32, 64);
  if (!active) return;
  if (hh == 0) a.lse[(static_cast<int64_t>(b) * a.nh + head) * S + q] = (m + log2f(l)) * 0.6931471805599453f;
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

// ---- backward tiles: 64 tokens x 64 dims, rows (swizzled) and/or a transposed image -------------
// thread i holds chunk (i & 7) of the token pair 2(i>>3), 2(i>>3)+1 of the block
__device__ __forceinline__ void load_pair(us8 (&x)[2], const unsigned short* src, int64_t tok, int row0) {
  const int c = threadIdx.x & 7, kp = threadIdx.x >> 3;
  x[0] = *reinterpret_cast<const us8*>(src + static_cast<int64_t>(row0 + 2 * kp) * tok + 8 * c);
  x[1] = *reinterpret_cast<const us8*>(src + static_cast<int64_t>(row0 + 2 * kp + 1) * tok + 8 * c);
}
__device__ __forceinline__ void store_rows(const us8 (&x)[2], unsigned char* dst) {
  const int c = threadIdx.x & 7, kp = threadIdx.x >> 3;
  *reinterpret_cast<us8*>(dst + kswz(2 * kp, c)) = x[0];
  *reinterpret_cast<us8*>(dst + kswz(2 * kp + 1, c)) = x[1];
}
__device__ __forceinline__ void store_t(const us8 (&x)[2], unsigned short* dst) {  // [64 dims][64 tokens + 4]
  const int c = threadIdx.x & 7, kp = threadIdx.x >> 3;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t w = static_cast<uint32_t>(x[0][e]) | (static_cast<uint32_t>(x[1][e]) << 16);
    *reinterpret_cast<uint32_t*>(dst + (8 * c + e) * kVtStride + 2 * kp) = w;
  }
}
__device__ __forceinline__ bf16x8 row_frag(const unsigned char* img, int row, int s, int hh) {
  return *reinterpret_cast<const bf16x8*>(img + kswz(row, 2 * s + hh));
}

// dQ (query on the lane, like the forward).  Per 64-key block (double-buffered: K rows, V rows,
// K^T image): S^T = K.Q^T, dPd^T = V.dO^T, dS^T = P o (dPd^T o Z/(1-p) - D), dQ^T += K^T . dS^T.
// Also writes D = rowsum(dO o O) for the dK/dV kernel.
constexpr int kDqBuf = 2 * kKTileBytes + kVTileBytes;
__global__ void __launch_bounds__(kThreads, 2) attn_bwd_dq_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = a.S;
  float* biasl = reinterpret_cast<float*>(smem + 2 * kDqBuf);
  const int b = blockIdx.z, head = blockIdx.y;
  const int H = a.nh * kHD;
  const int64_t tok = 3LL * H;
  const unsigned short* base = a.qkv + static_cast<int64_t>(b) * S * tok + head * kHD;
  const unsigned short* kbase = base + H;
  const unsigned short* vbase = base + 2 * H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQB + wave * 32;
  const bool active = q0 < S;
  const int q = active ? q0 + r : S - 1;

  us8 kx[2], vx[2];
  load_pair(kx, kbase, tok, 0);
  load_pair(vx, vbase, tok, 0);
  for (int i = threadIdx.x; i < S; i += kThreads) {
    const float bv = a.bias ? a.bias[static_cast<int64_t>(b) * S + i] * 1.4426950408889634f : 0.f;
    biasl[i] = fmaxf(bv, -1e30f);
  }
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
  if (active && hh == 0) a.delta[li] = D;
  const float lse2 = a.lse[li] * 1.4426950408889634f;
  const uint32_t key = rng_key_for(a.rng_key, b, head);
  const uint32_t rowidx = static_cast<uint32_t>(q) * static_cast<uint32_t>(S);
  store_rows(kx, smem);
  store_rows(vx, smem + kKTileBytes);
  store_t(kx, reinterpret_cast<unsigned short*>(smem + 2 * kKTileBytes));
  __syncthreads();

  f32x16 dqt[2] = {f32x16{0}, f32x16{0}};
  const int nkb = S / kKB;
  for (int kb = 0; kb < nkb; ++kb) {
    const unsigned char* buf = smem + (kb & 1) * kDqBuf;
    const unsigned short* kt = reinterpret_cast<const unsigned short*>(buf + 2 * kKTileBytes);
    if (kb + 1 < nkb) {
      load_pair(kx, kbase, tok, (kb + 1) * kKB);
      load_pair(vx, vbase, tok, (kb + 1) * kKB);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 sa = f32x16{0}, dp = f32x16{0};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(buf, 32 * t + r, s, hh), qf[s], sa, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(buf + kKTileBytes, 32 * t + r, s, hh), df[s], dp, 0, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int k0 = kb * kKB + 32 * t + 8 * g + 4 * hh;
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
          const float pr = fast_exp2(fmaf(sa[i], a.scale_log2, bb[e]) - lse2);
          sa[i] = pr * fmaf(dp[i], z[e], -D);  // dS^T
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 dsf = pack_frag(sa, s);
#pragma unroll
        for (int u = 0; u < 2; ++u)
          dqt[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_from_image(kt, kVtStride, 32 * u + r, 32 * t + 16 * s, hh),
                                                           dsf, dqt[u], 0, 0, 0);
      }
    }
    if (kb + 1 < nkb) {
      unsigned char* nb = smem + ((kb + 1) & 1) * kDqBuf;
      store_rows(kx, nb);
      store_rows(vx, nb + kKTileBytes);
      store_t(kx, reinterpret_cast<unsigned short*>(nb + 2 * kKTileBytes));
    }
    __syncthreads();
  }
  if (!active) return;
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

// dK, dV (key on the lane).  Per 64-query block (double-buffered: Q rows, Q^T, dO rows, dO^T):
// S = Q.K^T, dPd = dO.V^T (accumulator column = the lane's key), Pd = P o Z/(1-p),
// dS = P o (dPd o Z/(1-p) - D), dV^T += dO^T . Pd, dK^T += Q^T . dS.
constexpr int kDkvBuf = 2 * (kKTileBytes + kVTileBytes);
__global__ void __launch_bounds__(kThreads, 2) attn_bwd_dkv_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = a.S;
  float* lse2 = reinterpret_cast<float*>(smem + 2 * kDkvBuf);
  float* dl = lse2 + S;
  const int b = blockIdx.z, head = blockIdx.y;
  const int H = a.nh * kHD;
  const int64_t tok = 3LL * H;
  const unsigned short* base = a.qkv + static_cast<int64_t>(b) * S * tok + head * kHD;
  const unsigned short* dobase = a.dout + static_cast<int64_t>(b) * S * H + head * kHD;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int k0w = blockIdx.x * kQB + wave * 32;
  const bool active = k0w < S;
  const int kk = active ? k0w + r : S - 1;  // this lane's key

  us8 qx[2], dx[2];
  load_pair(qx, base, tok, 0);
  load_pair(dx, dobase, H, 0);
  const int64_t lrow = (static_cast<int64_t>(b) * a.nh + head) * S;
  for (int i = threadIdx.x; i < S; i += kThreads) {
    lse2[i] = a.lse[lrow + i] * 1.4426950408889634f;
    dl[i] = a.delta[lrow + i];
  }
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(base + H + static_cast<int64_t>(kk) * tok + 16 * s + 8 * hh);
    vf[s] = *reinterpret_cast<const bf16x8*>(base + 2 * H + static_cast<int64_t>(kk) * tok + 16 * s + 8 * hh);
  }
  const float bk = a.bias ? fmaxf(a.bias[static_cast<int64_t>(b) * S + kk] * 1.4426950408889634f, -1e30f) : 0.f;
  const uint32_t key = rng_key_for(a.rng_key, b, head);
  store_rows(qx, smem);
  store_t(qx, reinterpret_cast<unsigned short*>(smem + kKTileBytes));
  store_rows(dx, smem + kKTileBytes + kVTileBytes);
  store_t(dx, reinterpret_cast<unsigned short*>(smem + 2 * kKTileBytes + kVTileBytes));
  __syncthreads();

  f32x16 dkt[2] = {f32x16{0}, f32x16{0}}, dvt[2] = {f32x16{0}, f32x16{0}};
  const int nqb = S / kKB;
  for (int qb = 0; qb < nqb; ++qb) {
    const unsigned char* buf = smem + (qb & 1) * kDkvBuf;
    const unsigned short* qt = reinterpret_cast<const unsigned short*>(buf + kKTileBytes);
    const unsigned char* dorows = buf + kKTileBytes + kVTileBytes;
    const unsigned short* dot = reinterpret_cast<const unsigned short*>(buf + 2 * kKTileBytes + kVTileBytes);
    if (qb + 1 < nqb) {
      load_pair(qx, base, tok, (qb + 1) * kKB);
      load_pair(dx, dobase, H, (qb + 1) * kKB);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 sa = f32x16{0}, dp = f32x16{0};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(buf, 32 * t + r, s, hh), kf[s], sa, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(dorows, 32 * t + r, s, hh), vf[s], dp, 0, 0, 0);
      }
      f32x16 pd;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int qq = qb * kKB + 32 * t + 8 * g + 4 * hh;
        const float4 lv = *reinterpret_cast<const float4*>(lse2 + qq);
        const float4 dv = *reinterpret_cast<const float4*>(dl + qq);
        const float ll[4] = {lv.x, lv.y, lv.z, lv.w}, dd[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e;
          float z = 1.f;
          if (a.drop_thr) {
            const uint32_t idx = static_cast<uint32_t>(qq + e) * static_cast<uint32_t>(S) + kk;
            const uint32_t hsh = mix32(idx >> 1, key);
            z = ((kk & 1) ? (hsh >> 16) : (hsh & 0xffffu)) < a.drop_thr ? 0.f : a.drop_scale;
          }
          const float pr = fast_exp2(fmaf(sa[i], a.scale_log2, bk) - ll[e]);
          pd[i] = pr * z;
          sa[i] = pr * fmaf(dp[i], z, -dd[e]);  // dS
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = pack_frag(pd, s), dsf = pack_frag(sa, s);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          dvt[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_from_image(dot, kVtStride, 32 * u + r, 32 * t + 16 * s, hh),
                                                           pf, dvt[u], 0, 0, 0);
          dkt[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_from_image(qt, kVtStride, 32 * u + r, 32 * t + 16 * s, hh),
                                                           dsf, dkt[u], 0, 0, 0);
        }
      }
    }
    if (qb + 1 < nqb) {
      unsigned char* nb = smem + ((qb + 1) & 1) * kDkvBuf;
      store_rows(qx, nb);
      store_t(qx, reinterpret_cast<unsigned short*>(nb + kKTileBytes));
      store_rows(dx, nb + kKTileBytes + kVTileBytes);
      store_t(dx, reinterpret_cast<unsigned short*>(nb + 2 * kKTileBytes + kVTileBytes));
    }
    __syncthreads();
  }
  if (!active) return;
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

size_t fwd_lds(int S) { return 2 * static_cast<size_t>(kFwdBufBytes) + static_cast<size_t>(S) * 4; }

}  // namespace

extern "C" {

// Shapes the MFMA path covers: head_dim 64, S a multiple of 64 up to 2048 (the per-head key bias /
// LSE / delta rows live in LDS next to the double-buffered tiles).
int det_attn_supported(int S, int head_dim) {
  return head_dim == kHD && S >= 64 && S % kKB == 0 && S <= 2048;
}

// qkv [B, S, 3, nh, 64] bf16; bias [B, S] fp32 (nullable); out [B, S, nh*64] bf16; lse [B, nh, S].
int det_attn_fwd(void* stream, const void* qkv, const float* bias, void* out, float* lse, int B, int S, int nh,
                 float p, uint64_t seed, uint64_t offset) {
  if (!det_attn_supported(S, kHD) || B <= 0 || nh <= 0) return -1;
  AttnArgs a;
  fill_args(a, qkv, bias, out, lse, B, S, nh, p, seed, offset);
  hipStream_t st = static_cast<hipStream_t>(stream);
  dim3 grid((S + kQB - 1) / kQB, nh, B);
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(kThreads), fwd_lds(S), st, a);
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
  const size_t lds_dq = 2 * static_cast<size_t>(kDqBuf) + static_cast<size_t>(S) * 4;
  const size_t lds_dkv = 2 * static_cast<size_t>(kDkvBuf) + 2 * static_cast<size_t>(S) * 4;
  hipLaunchKernelGGL(attn_bwd_dq_kernel, grid, dim3(kThreads), lds_dq, st, a);
  hipLaunchKernelGGL(attn_bwd_dkv_kernel, grid, dim3(kThreads), lds_dkv, st, a);
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
