// det_attention.hip — MFMA flash attention on gfx950, forward and backward, for every attention the
// framework's models run: bf16 head_dim 32/64/128 and fp32 head_dim 32/64, any query/key length
// (masked tail blocks), separate query/key lengths (cross-attention), an additive per-key bias
// ([B, Lk], BERT/DETR padding masks) and/or a full additive bias with arbitrary broadcast strides
// ([B|1, nh|1, Lq, Lk]), and regenerable dropout on the probabilities.
//
// Why this exists: BERT-base SQuAD-shape (B 12, S 384, 12 heads x 64) spent 2.2 ms/step in the
// AOTriton attention kernels (profiles/r1_bert_native_bs12_o2_steady.csv), ~105 TFLOP/s; the
// bf16/64 instance takes 0.99 ms (profiles/r1_bert_native_fa_bs12_o2_per_step.txt).  Round 3 made
// the kernels generic so no example falls back to AOTriton or a composite SDPA (DETR: fp32,
// head_dim 32, S = feature-map pixels; ALBERT fp32 reference config: head_dim 64).
//
// Layout: Q/K/V are token-major strided views — element (b, token, head, d) at
// base + b*sb + token*st + head*HD + d — so the fused [B, S, 3, nh, HD] QKV GEMM output is read in
// place (token stride 3H) and dQ/dK/dV are written straight into its gradient; DETR's separate
// projections are the same with token stride H.  O/dO are [B, Lq, nh, HD] views the same way.
// LSE [B, nh, Lq] is the natural-log normaliser the backward recomputes P from.
//
// All three kernels share one structure: a workgroup = 4 waves = 128 rows (queries, or keys for
// dK/dV) of one (batch, head), one row per lane (32x32 MFMA with the row on the accumulator COLUMN,
// i.e. S^T = K . Q^T, so softmax reductions are in-lane plus one lane^32 exchange), and the other
// operand streamed in 64-token blocks double-buffered in LDS: the next block is loaded into
// registers before the current block's MFMAs and written to the other buffer after them (one
// barrier per block).  Row-major tiles use an XOR-swizzled 16-B chunk layout (conflict-free
// A-fragment reads); operands consumed along the token axis get a transposed [HD][64+4] image
// written in the same pass.  An accumulator (converted to bf16 in registers on the bf16 path) is
// directly the B operand of the next product with the k order permuted to match (Elt::mma_img).
// bf16 uses v_mfma_f32_32x32x16_bf16 (one 16-B chunk per lane per MFMA); fp32 uses
// v_mfma_f32_32x32x2_f32 over the same chunks (4 MFMAs per chunk), so the fp32 path keeps fp32
// operands end to end rather than rounding through bf16.
//   forward : per key block S^T, online softmax (running max/sum in the log2 domain), O^T += V^T P^T
//   dQ      : per key block S^T, dP^T, dS^T = P o (dP^T o Z/(1-p) - D), dQ^T += K^T dS^T; writes D
//   dK, dV  : per query block S, dP, dV^T += dO^T Pd, dK^T += Q^T dS (no cross-workgroup sums)
// Tails: key rows past Lk are clamped loads whose scores get a -inf bias (P = 0 exactly); query rows
// past Lq are clamped loads with LSE = +inf in the dK/dV kernel (P = 0) and are never stored.
// Dropout keep masks come from a keyed 32-bit hash of (b, h, q*LkE + key), LkE = Lk rounded up to
// a multiple of 4 (two 16-bit draws per hash), regenerated bit-exactly in the backward pass.
//
// Reference parity: the reference runs attention inside HuggingFace BERT/ALBERT and DETR's
// nn.MultiheadAttention on torch (examples/nlp/bert_squad_pytorch/model_def.py,
// examples/nlp/albert_squad_pytorch/model_def.py, examples/computer_vision/detr_coco_pytorch/
// model.py); semantics = softmax(QK^T * scale + bias) V with dropout on the probabilities, as
// torch.nn.functional.scaled_dot_product_attention.

#include <hip/hip_runtime.h>
#include <cstdlib>
#include <math.h>
#include <stdint.h>

namespace {

#ifndef DET_ATTN_WAVES
#define DET_ATTN_WAVES 4
#endif
constexpr int kWaves = DET_ATTN_WAVES;  // 32 query (or key) rows per wave
constexpr int kThreads = 64 * kWaves;
constexpr int kQB = 32 * kWaves;  // rows (queries, or keys for dK/dV) per workgroup
constexpr int kKB = 64;           // streamed tokens per block
constexpr int kTS = kKB + 4;      // transposed-image row stride (elements)
constexpr float kLog2e = 1.4426950408889634f;
constexpr int kMaxLds = 160 * 1024;

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned short us4;
typedef __attribute__((ext_vector_type(8))) unsigned short us8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
// 16-B chunk in registers (an ext vector, not HIP's uint4 union, so SROA keeps tile arrays in VGPRs)
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

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

struct Args {
  const void *q, *k, *v;        // token-major views, see header
  const void* dout;             // dO (backward)
  void* out;                    // O (written by the forward, read by the backward)
  void *dq, *dk, *dv;           // gradients (backward)
  float* lse;                   // [B, nh, Lq]
  float* delta;                 // [B, nh, Lq] (backward workspace)
  const float* kbias;           // [B, Lk] additive per-key bias (natural units) or null
  const float* mbias;           // full additive bias, element (b, h, q, k) at b*mbb + h*mbh + q*mbq + k
  int64_t qsb, qst, ksb, kst, vsb, vst, osb, ost, dosb, dost, dqsb, dqst, dksb, dkst, dvsb, dvst;
  int64_t mbb, mbh, mbq;
  int B, Lq, Lk, nh;
  float scale, scale_log2;      // softmax scale (natural) and scale * log2(e)
  uint32_t drop_thr;            // drop if 16-bit draw < thr (0: no dropout)
  float drop_scale;             // 65536 / (65536 - thr)
  uint32_t rng_key;
  // nullable: device counter folded into the key when the kernel runs (a hipGraph replays its
  // captured key; the captured step bumps the counter first -- ops/transformer.py rng_base)
  const uint32_t* rng_base;
};

// The replay counter enters the key through the mixer, not by XOR: a linear fold (key ^ base * C
// with key itself linear in the offset) lets whole families of (offset, counter) pairs land on one
// key, i.e. one mask; mixed, distinct pairs share a 32-bit key only by chance.
__device__ __forceinline__ uint32_t fold_base(uint32_t key, const uint32_t* rng_base) {
  return rng_base != nullptr ? mix32(*rng_base * 0x2545F491u + 0x632BE5ABu, key) : key;
}
__device__ __forceinline__ uint32_t run_key(const Args& a) { return fold_base(a.rng_key, a.rng_base); }

__device__ __forceinline__ uint32_t rng_key_for(uint32_t base_key, int b, int head) {
  return base_key ^ (static_cast<uint32_t>(b * 977 + head) * 0x9E3779B9u);
}
__host__ __device__ __forceinline__ int lk_even4(int Lk) { return (Lk + 3) & ~3; }

// ---- element traits: the two MFMA shapes -------------------------------------------------------
template <typename E>
struct Elt;

template <>
struct Elt<unsigned short> {  // bf16
  // acc += A . B over one 16-B chunk per lane: lane half hh holds k = 8hh..8hh+7
  __device__ static __forceinline__ void mma_chunk(f32x16& acc, const u32x4& a, const u32x4& b) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                  acc, 0, 0, 0);
  }
  // acc += Img[row][k0 .. k0+32) . P^T, P an accumulator over those 32 tokens (lane half hh holds
  // tokens 8g + 4hh + e): bf16 pack of elements 8s..8s+7 = tokens 8(2s + j/4) + 4hh + j%4, and the
  // image fragment read with the same permutation
  __device__ static __forceinline__ void mma_img(f32x16& acc, const unsigned short* img, int row, int k0,
                                                 const f32x16& p, int hh) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const unsigned short* src = img + row * kTS + k0 + 16 * s + 4 * hh;
      const us4 lo = *reinterpret_cast<const us4*>(src);
      const us4 hi = *reinterpret_cast<const us4*>(src + 8);
      bf16x8 af, bf;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        af[j] = static_cast<short>(lo[j]);
        af[4 + j] = static_cast<short>(hi[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) bf[j] = static_cast<short>(f2bf(p[8 * s + j]));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc, 0, 0, 0);
    }
  }
  __device__ static __forceinline__ void store4(unsigned short* dst, float v0, float v1, float v2, float v3) {
    us4 w;
    w[0] = f2bf(v0);
    w[1] = f2bf(v1);
    w[2] = f2bf(v2);
    w[3] = f2bf(v3);
    *reinterpret_cast<us4*>(dst) = w;
  }
  __device__ static __forceinline__ float chunk_dot(const u32x4& a, const u32x4& b) {
    const us8 x = __builtin_bit_cast(us8, a), y = __builtin_bit_cast(us8, b);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s = fmaf(bf2f(x[j]), bf2f(y[j]), s);
    return s;
  }
};

template <>
struct Elt<float> {  // fp32: 4 MFMAs 32x32x2 per 16-B chunk; lane half hh holds k column 4c + e
  __device__ static __forceinline__ void mma_chunk(f32x16& acc, const u32x4& a, const u32x4& b) {
    const f32x4 x = __builtin_bit_cast(f32x4, a), y = __builtin_bit_cast(f32x4, b);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[e], y[e], acc, 0, 0, 0);
  }
  __device__ static __forceinline__ void mma_img(f32x16& acc, const float* img, int row, int k0, const f32x16& p,
                                                 int hh) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(img + row * kTS + k0 + 8 * g + 4 * hh);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[e], p[4 * g + e], acc, 0, 0, 0);
    }
  }
  __device__ static __forceinline__ void store4(float* dst, float v0, float v1, float v2, float v3) {
    *reinterpret_cast<f32x4*>(dst) = f32x4{v0, v1, v2, v3};
  }
  __device__ static __forceinline__ float chunk_dot(const u32x4& a, const u32x4& b) {
    const f32x4 x = __builtin_bit_cast(f32x4, a), y = __builtin_bit_cast(f32x4, b);
    return x[0] * y[0] + x[1] * y[1] + x[2] * y[2] + x[3] * y[3];
  }
};

// ---- streamed 64-token tiles --------------------------------------------------------------------
// Work unit = 16-B chunk c of the token pair (2kp, 2kp+1); the row image is XOR-swizzled by chunk,
// the transposed image [HD][64 + 4] gets token pairs as one 32-bit (bf16) or 64-bit (fp32) store.
template <typename E, int HD>
struct Tile {
  static constexpr int RB = HD * static_cast<int>(sizeof(E));  // bytes per token row
  static constexpr int NCH = RB / 16;
  static constexpr int CH = 16 / static_cast<int>(sizeof(E));
  static constexpr int UNITS = 32 * NCH;
  static constexpr int NP = (UNITS + kThreads - 1) / kThreads;
  static constexpr int SWM = (NCH < 16 ? NCH : 16) - 1;
  static constexpr int ROW_BYTES = kKB * RB;
  static constexpr int T_BYTES = HD * kTS * static_cast<int>(sizeof(E));
  static_assert(RB % 16 == 0 && NCH >= 4, "head_dim too small");

  u32x4 x[NP][2];

  __device__ static __forceinline__ int off(int row, int ch) { return row * RB + 16 * (ch ^ (row & SWM)); }
  __device__ static __forceinline__ bool live(int w) { return UNITS % kThreads == 0 || w < UNITS; }

  // rows row0 .. row0+63 of src (row stride `tok` elements), rows >= nrows clamped to nrows-1
  __device__ __forceinline__ void load(const E* src, int64_t tok, int row0, int nrows) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int w = threadIdx.x + p * kThreads;
      if (!live(w)) continue;
      const int kp = w / NCH, c = w % NCH;
      const int r0 = min(row0 + 2 * kp, nrows - 1), r1 = min(row0 + 2 * kp + 1, nrows - 1);
      x[p][0] = *reinterpret_cast<const u32x4*>(src + static_cast<int64_t>(r0) * tok + c * CH);
      x[p][1] = *reinterpret_cast<const u32x4*>(src + static_cast<int64_t>(r1) * tok + c * CH);
    }
  }
  __device__ __forceinline__ void store_rows(unsigned char* dst) const {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int w = threadIdx.x + p * kThreads;
      if (!live(w)) continue;
      const int kp = w / NCH, c = w % NCH;
      *reinterpret_cast<u32x4*>(dst + off(2 * kp, c)) = x[p][0];
      *reinterpret_cast<u32x4*>(dst + off(2 * kp + 1, c)) = x[p][1];
    }
  }
  __device__ __forceinline__ void store_t(E* dst) const {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int w = threadIdx.x + p * kThreads;
      if (!live(w)) continue;
      const int kp = w / NCH, c = w % NCH;
      if constexpr (sizeof(E) == 2) {
        const us8 a = __builtin_bit_cast(us8, x[p][0]), b = __builtin_bit_cast(us8, x[p][1]);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          *reinterpret_cast<uint32_t*>(dst + (c * CH + e) * kTS + 2 * kp) =
              static_cast<uint32_t>(a[e]) | (static_cast<uint32_t>(b[e]) << 16);
      } else {
        const f32x4 a = __builtin_bit_cast(f32x4, x[p][0]), b = __builtin_bit_cast(f32x4, x[p][1]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          typedef __attribute__((ext_vector_type(2))) float f32x2;
          *reinterpret_cast<f32x2*>(dst + (c * CH + e) * kTS + 2 * kp) = f32x2{a[e], b[e]};
        }
      }
    }
  }
  __device__ static __forceinline__ u32x4 frag(const unsigned char* img, int row, int ch) {
    return *reinterpret_cast<const u32x4*>(img + off(row, ch));
  }
};

// per-key bias row in LDS, log2 units: real keys clamped finite (fully masked rows degrade to
// uniform like fp32 torch), tail keys -inf
__device__ __forceinline__ void fill_key_bias(float* dst, const float* kbias, int Lk, int LkP) {
  for (int i = threadIdx.x; i < LkP; i += kThreads)
    dst[i] = i < Lk ? (kbias ? fmaxf(kbias[i] * kLog2e, -1e30f) : 0.f) : -INFINITY;
}
__device__ __forceinline__ float mbias_log2(const float* m, int64_t i) { return fmaxf(m[i] * kLog2e, -1e30f); }

// dropout keep factors for tokens k0..k0+3 (k0 % 4 == 0) of the row with index base rowidx
__device__ __forceinline__ void drop4(float z[4], uint32_t rowidx, int k0, uint32_t key, uint32_t thr, float dscale) {
  const uint32_t h0 = mix32((rowidx + k0) >> 1, key), h1 = mix32((rowidx + k0 + 2) >> 1, key);
  const uint32_t d4[4] = {h0 & 0xffffu, h0 >> 16, h1 & 0xffffu, h1 >> 16};
#pragma unroll
  for (int e = 0; e < 4; ++e) z[e] = d4[e] < thr ? 0.f : dscale;
}

// =============================================================================================
// Forward: one workgroup = 128 queries of one (batch, head), wave = 32 queries, lane = one query
// (its 32 keys of a 64-key block in two S^T accumulators).  Per key block: S^T = K . Q^T (K
// fragments from the swizzled LDS tile, Q^T in registers), online softmax in the log2 domain (one
// lane^32 max exchange), O^T = O^T * alpha + V^T . P^T.
// =============================================================================================
template <typename E, int HD, bool MB>
__global__ void __launch_bounds__(kThreads, (HD * sizeof(E) >= 256 ? 1 : 2)) attn_fwd_kernel(Args a) {
  using TL = Tile<E, HD>;
  using EL = Elt<E>;
  constexpr int QCH = TL::NCH / 2, NU = HD / 32;
  constexpr int BUF = TL::ROW_BYTES + TL::T_BYTES;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Lq = a.Lq, Lk = a.Lk, nkb = (Lk + kKB - 1) / kKB;
  float* biasl = reinterpret_cast<float*>(smem + 2 * BUF);
  const int b = blockIdx.z, head = blockIdx.y;
  const E* qbase = static_cast<const E*>(a.q) + b * a.qsb + head * HD;
  const E* kbase = static_cast<const E*>(a.k) + b * a.ksb + head * HD;
  const E* vbase = static_cast<const E*>(a.v) + b * a.vsb + head * HD;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int qv = blockIdx.x * kQB + wave * 32 + r;
  const int q = qv < Lq ? qv : Lq - 1;  // past-the-end lanes compute a clamped row, store nothing

  TL kt, vt;
  kt.load(kbase, a.kst, 0, Lk);
  vt.load(vbase, a.vst, 0, Lk);
  fill_key_bias(biasl, a.kbias ? a.kbias + static_cast<int64_t>(b) * Lk : nullptr, Lk, nkb * kKB);
  u32x4 qf[QCH];
#pragma unroll
  for (int j = 0; j < QCH; ++j)
    qf[j] = *reinterpret_cast<const u32x4*>(qbase + static_cast<int64_t>(q) * a.qst + (2 * j + hh) * TL::CH);
  const float* mrow = MB ? a.mbias + b * a.mbb + head * a.mbh + static_cast<int64_t>(q) * a.mbq : nullptr;
  kt.store_rows(smem);
  vt.store_t(reinterpret_cast<E*>(smem + TL::ROW_BYTES));
  __syncthreads();

  const uint32_t key = rng_key_for(run_key(a), b, head);
  const uint32_t rowidx = static_cast<uint32_t>(q) * static_cast<uint32_t>(lk_even4(Lk));
  float m = -INFINITY, l = 0.f;
  f32x16 o[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) o[u] = f32x16{0};
  for (int kb = 0; kb < nkb; ++kb) {
    const unsigned char* buf = smem + (kb & 1) * BUF;
    const E* vti = reinterpret_cast<const E*>(buf + TL::ROW_BYTES);
    if (kb + 1 < nkb) {
      kt.load(kbase, a.kst, (kb + 1) * kKB, Lk);
      vt.load(vbase, a.vst, (kb + 1) * kKB, Lk);
    }
    float mb[2][16];
    if constexpr (MB) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kk = kb * kKB + 32 * t + 8 * (i >> 2) + 4 * hh + (i & 3);
          mb[t][i] = kk < Lk ? mbias_log2(mrow, kk) : 0.f;
        }
    }
    f32x16 sc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sc[t] = f32x16{0};
#pragma unroll
      for (int j = 0; j < QCH; ++j) EL::mma_chunk(sc[t], TL::frag(buf, 32 * t + r, 2 * j + hh), qf[j]);
    }
    // scores in log2 units + biases; block max over the lane pair (q, q^32)
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 bv = *reinterpret_cast<const float4*>(biasl + kb * kKB + 32 * t + 8 * g + 4 * hh);
        const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = fmaf(sc[t][4 * g + e], a.scale_log2, bb[e]);
          if constexpr (MB) x += mb[t][4 * g + e];
          sc[t][4 * g + e] = x;
          mx = fmaxf(mx, x);
        }
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
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
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[u][i] *= alpha;
    }
    if (a.drop_thr) {  // same draws as the backward
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float z[4];
          drop4(z, rowidx, kb * kKB + 32 * t + 8 * g + 4 * hh, key, a.drop_thr, a.drop_scale);
#pragma unroll
          for (int e = 0; e < 4; ++e) sc[t][4 * g + e] *= z[e];
        }
    }
    // O^T += V^T . P^T
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < NU; ++u) EL::mma_img(o[u], vti, 32 * u + r, 32 * t, sc[t], hh);
    if (kb + 1 < nkb) {
      unsigned char* nb = smem + ((kb + 1) & 1) * BUF;
      kt.store_rows(nb);
      vt.store_t(reinterpret_cast<E*>(nb + TL::ROW_BYTES));
    }
    __syncthreads();
  }
  l += __shfl_xor(l, 32, 64);
  if (qv >= Lq) return;
  if (hh == 0) a.lse[(static_cast<int64_t>(b) * a.nh + head) * Lq + qv] = (m + log2f(l)) * 0.6931471805599453f;
  const float inv_l = 1.f / l;
  E* orow = static_cast<E*>(a.out) + b * a.osb + static_cast<int64_t>(qv) * a.ost + head * HD;
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      EL::store4(orow + 32 * u + 8 * g + 4 * hh, o[u][4 * g] * inv_l, o[u][4 * g + 1] * inv_l,
                 o[u][4 * g + 2] * inv_l, o[u][4 * g + 3] * inv_l);
}

// =============================================================================================
// Backward.  With Pd = P o Z/(1-p) (dropout keep mask Z), D_q = sum_d dO o O (= sum_k Pd dPd):
//   dV = Pd^T dO,  dPd = dO V^T,  dS = P o (dPd o Z/(1-p) - D),  dQ = dS K * scale,  dK = dS^T Q * scale.
// Two kernels so that no gradient needs a cross-workgroup sum:
//   attn_bwd_dq  (query on the lane, like the forward): S^T, dPd^T per key tile, dQ^T += K^T dS^T
//                with a K^T LDS image; also writes D (consumed by the next kernel);
//   attn_bwd_dkv (key on the lane): S, dPd per query tile, dV^T += dO^T Pd and dK^T += Q^T dS with
//                Q^T / dO^T LDS images.
// =============================================================================================
// bx: the workgroup's row-tile index (blockIdx.x in the two-launch form; see attn_bwd_kernel).
// WRITE_D: this pass also writes D for the dK/dV pass (the merged form has attn_delta_kernel do it).
template <typename E, int HD, bool MB, bool WRITE_D>
__device__ __forceinline__ void attn_bwd_dq_body(const Args& a, int bx, unsigned char* smem) {
  using TL = Tile<E, HD>;
  using EL = Elt<E>;
  constexpr int QCH = TL::NCH / 2, NU = HD / 32;
  constexpr int BUF = 2 * TL::ROW_BYTES + TL::T_BYTES;  // K rows, V rows, K^T
  const int Lq = a.Lq, Lk = a.Lk, nkb = (Lk + kKB - 1) / kKB;
  float* biasl = reinterpret_cast<float*>(smem + 2 * BUF);
  const int b = blockIdx.z, head = blockIdx.y;
  const E* qbase = static_cast<const E*>(a.q) + b * a.qsb + head * HD;
  const E* kbase = static_cast<const E*>(a.k) + b * a.ksb + head * HD;
  const E* vbase = static_cast<const E*>(a.v) + b * a.vsb + head * HD;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int qv = bx * kQB + wave * 32 + r;
  const int q = qv < Lq ? qv : Lq - 1;

  TL kt, vt;
  kt.load(kbase, a.kst, 0, Lk);
  vt.load(vbase, a.vst, 0, Lk);
  fill_key_bias(biasl, a.kbias ? a.kbias + static_cast<int64_t>(b) * Lk : nullptr, Lk, nkb * kKB);
  const E* orow = static_cast<const E*>(a.out) + b * a.osb + static_cast<int64_t>(q) * a.ost + head * HD;
  const E* dorow = static_cast<const E*>(a.dout) + b * a.dosb + static_cast<int64_t>(q) * a.dost + head * HD;
  u32x4 qf[QCH], df[QCH];
  float dsum = 0.f;
#pragma unroll
  for (int j = 0; j < QCH; ++j) {
    const int c = (2 * j + hh) * TL::CH;
    qf[j] = *reinterpret_cast<const u32x4*>(qbase + static_cast<int64_t>(q) * a.qst + c);
    df[j] = *reinterpret_cast<const u32x4*>(dorow + c);
    dsum += EL::chunk_dot(df[j], *reinterpret_cast<const u32x4*>(orow + c));
  }
  const float D = dsum + __shfl_xor(dsum, 32, 64);
  const int64_t li = (static_cast<int64_t>(b) * a.nh + head) * Lq + q;
  if (WRITE_D && qv < Lq && hh == 0) a.delta[li] = D;
  const float lse2 = a.lse[li] * kLog2e;
  const float* mrow = MB ? a.mbias + b * a.mbb + head * a.mbh + static_cast<int64_t>(q) * a.mbq : nullptr;
  const uint32_t key = rng_key_for(run_key(a), b, head);
  const uint32_t rowidx = static_cast<uint32_t>(q) * static_cast<uint32_t>(lk_even4(Lk));
  kt.store_rows(smem);
  vt.store_rows(smem + TL::ROW_BYTES);
  kt.store_t(reinterpret_cast<E*>(smem + 2 * TL::ROW_BYTES));
  __syncthreads();

  f32x16 dqt[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) dqt[u] = f32x16{0};
  for (int kb = 0; kb < nkb; ++kb) {
    const unsigned char* buf = smem + (kb & 1) * BUF;
    const E* kti = reinterpret_cast<const E*>(buf + 2 * TL::ROW_BYTES);
    if (kb + 1 < nkb) {
      kt.load(kbase, a.kst, (kb + 1) * kKB, Lk);
      vt.load(vbase, a.vst, (kb + 1) * kKB, Lk);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float mb[16];
      if constexpr (MB) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kk = kb * kKB + 32 * t + 8 * (i >> 2) + 4 * hh + (i & 3);
          mb[i] = kk < Lk ? mbias_log2(mrow, kk) : 0.f;
        }
      }
      f32x16 sa = f32x16{0}, dp = f32x16{0};
#pragma unroll
      for (int j = 0; j < QCH; ++j) {
        EL::mma_chunk(sa, TL::frag(buf, 32 * t + r, 2 * j + hh), qf[j]);
        EL::mma_chunk(dp, TL::frag(buf + TL::ROW_BYTES, 32 * t + r, 2 * j + hh), df[j]);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int k0 = kb * kKB + 32 * t + 8 * g + 4 * hh;
        const float4 bv = *reinterpret_cast<const float4*>(biasl + k0);
        const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
        float z[4] = {1.f, 1.f, 1.f, 1.f};
        if (a.drop_thr) drop4(z, rowidx, k0, key, a.drop_thr, a.drop_scale);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e;
          float x = fmaf(sa[i], a.scale_log2, bb[e]);
          if constexpr (MB) x += mb[i];
          const float pr = fast_exp2(x - lse2);
          sa[i] = pr * fmaf(dp[i], z[e], -D);  // dS^T
        }
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) EL::mma_img(dqt[u], kti, 32 * u + r, 32 * t, sa, hh);
    }
    if (kb + 1 < nkb) {
      unsigned char* nb = smem + ((kb + 1) & 1) * BUF;
      kt.store_rows(nb);
      vt.store_rows(nb + TL::ROW_BYTES);
      kt.store_t(reinterpret_cast<E*>(nb + 2 * TL::ROW_BYTES));
    }
    __syncthreads();
  }
  if (qv >= Lq) return;
  E* dq = static_cast<E*>(a.dq) + b * a.dqsb + static_cast<int64_t>(qv) * a.dqst + head * HD;
  const float sc = a.scale;
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      EL::store4(dq + 32 * u + 8 * g + 4 * hh, dqt[u][4 * g] * sc, dqt[u][4 * g + 1] * sc, dqt[u][4 * g + 2] * sc,
                 dqt[u][4 * g + 3] * sc);
}

template <typename E, int HD, bool MB>
__global__ void __launch_bounds__(kThreads, (HD * sizeof(E) >= 256 ? 1 : 2)) attn_bwd_dq_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  attn_bwd_dq_body<E, HD, MB, true>(a, blockIdx.x, smem);
}

template <typename E, int HD, bool MB>
__device__ __forceinline__ void attn_bwd_dkv_body(const Args& a, int bx, unsigned char* smem) {
  using TL = Tile<E, HD>;
  using EL = Elt<E>;
  constexpr int QCH = TL::NCH / 2, NU = HD / 32;
  constexpr int BUF = 2 * (TL::ROW_BYTES + TL::T_BYTES);  // Q rows, Q^T, dO rows, dO^T
  const int Lq = a.Lq, Lk = a.Lk, nqb = (Lq + kKB - 1) / kKB;
  float* lse2 = reinterpret_cast<float*>(smem + 2 * BUF);
  float* dl = lse2 + nqb * kKB;
  const int b = blockIdx.z, head = blockIdx.y;
  const E* qbase = static_cast<const E*>(a.q) + b * a.qsb + head * HD;
  const E* dobase = static_cast<const E*>(a.dout) + b * a.dosb + head * HD;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int kv = bx * kQB + wave * 32 + r;
  const int kk = kv < Lk ? kv : Lk - 1;  // this lane's key

  TL qt, dt;
  qt.load(qbase, a.qst, 0, Lq);
  dt.load(dobase, a.dost, 0, Lq);
  const int64_t lrow = (static_cast<int64_t>(b) * a.nh + head) * Lq;
  for (int i = threadIdx.x; i < nqb * kKB; i += kThreads) {
    lse2[i] = i < Lq ? a.lse[lrow + i] * kLog2e : INFINITY;  // tail queries: P = 0
    dl[i] = i < Lq ? a.delta[lrow + i] : 0.f;
  }
  const E* krow = static_cast<const E*>(a.k) + b * a.ksb + static_cast<int64_t>(kk) * a.kst + head * HD;
  const E* vrow = static_cast<const E*>(a.v) + b * a.vsb + static_cast<int64_t>(kk) * a.vst + head * HD;
  u32x4 kf[QCH], vf[QCH];
#pragma unroll
  for (int j = 0; j < QCH; ++j) {
    kf[j] = *reinterpret_cast<const u32x4*>(krow + (2 * j + hh) * TL::CH);
    vf[j] = *reinterpret_cast<const u32x4*>(vrow + (2 * j + hh) * TL::CH);
  }
  const float bk = a.kbias ? fmaxf(a.kbias[static_cast<int64_t>(b) * Lk + kk] * kLog2e, -1e30f) : 0.f;
  const float* mcol = MB ? a.mbias + b * a.mbb + head * a.mbh + kk : nullptr;
  const uint32_t key = rng_key_for(run_key(a), b, head);
  const uint32_t lke = static_cast<uint32_t>(lk_even4(Lk));
  qt.store_rows(smem);
  qt.store_t(reinterpret_cast<E*>(smem + TL::ROW_BYTES));
  dt.store_rows(smem + TL::ROW_BYTES + TL::T_BYTES);
  dt.store_t(reinterpret_cast<E*>(smem + 2 * TL::ROW_BYTES + TL::T_BYTES));
  __syncthreads();

  f32x16 dkt[NU], dvt[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) dkt[u] = dvt[u] = f32x16{0};
  for (int qb = 0; qb < nqb; ++qb) {
    const unsigned char* buf = smem + (qb & 1) * BUF;
    const E* qti = reinterpret_cast<const E*>(buf + TL::ROW_BYTES);
    const unsigned char* dorows = buf + TL::ROW_BYTES + TL::T_BYTES;
    const E* doti = reinterpret_cast<const E*>(buf + 2 * TL::ROW_BYTES + TL::T_BYTES);
    if (qb + 1 < nqb) {
      qt.load(qbase, a.qst, (qb + 1) * kKB, Lq);
      dt.load(dobase, a.dost, (qb + 1) * kKB, Lq);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float mb[16];
      if constexpr (MB) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qq = qb * kKB + 32 * t + 8 * (i >> 2) + 4 * hh + (i & 3);
          mb[i] = qq < Lq ? mbias_log2(mcol, static_cast<int64_t>(qq) * a.mbq) : 0.f;
        }
      }
      f32x16 sa = f32x16{0}, dp = f32x16{0};
#pragma unroll
      for (int j = 0; j < QCH; ++j) {
        EL::mma_chunk(sa, TL::frag(buf, 32 * t + r, 2 * j + hh), kf[j]);
        EL::mma_chunk(dp, TL::frag(dorows, 32 * t + r, 2 * j + hh), vf[j]);
      }
      f32x16 pd;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int q0 = qb * kKB + 32 * t + 8 * g + 4 * hh;
        const float4 lv = *reinterpret_cast<const float4*>(lse2 + q0);
        const float4 dv = *reinterpret_cast<const float4*>(dl + q0);
        const float ll[4] = {lv.x, lv.y, lv.z, lv.w}, dd[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e;
          float z = 1.f;
          if (a.drop_thr) {
            const uint32_t idx = static_cast<uint32_t>(q0 + e) * lke + static_cast<uint32_t>(kk);
            const uint32_t hsh = mix32(idx >> 1, key);
            z = ((idx & 1) ? (hsh >> 16) : (hsh & 0xffffu)) < a.drop_thr ? 0.f : a.drop_scale;
          }
          float x = fmaf(sa[i], a.scale_log2, bk);
          if constexpr (MB) x += mb[i];
          const float pr = fast_exp2(x - ll[e]);
          pd[i] = pr * z;
          sa[i] = pr * fmaf(dp[i], z, -dd[e]);  // dS
        }
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        EL::mma_img(dvt[u], doti, 32 * u + r, 32 * t, pd, hh);
        EL::mma_img(dkt[u], qti, 32 * u + r, 32 * t, sa, hh);
      }
    }
    if (qb + 1 < nqb) {
      unsigned char* nb = smem + ((qb + 1) & 1) * BUF;
      qt.store_rows(nb);
      qt.store_t(reinterpret_cast<E*>(nb + TL::ROW_BYTES));
      dt.store_rows(nb + TL::ROW_BYTES + TL::T_BYTES);
      dt.store_t(reinterpret_cast<E*>(nb + 2 * TL::ROW_BYTES + TL::T_BYTES));
    }
    __syncthreads();
  }
  if (kv >= Lk) return;
  E* dk = static_cast<E*>(a.dk) + b * a.dksb + static_cast<int64_t>(kv) * a.dkst + head * HD;
  E* dv = static_cast<E*>(a.dv) + b * a.dvsb + static_cast<int64_t>(kv) * a.dvst + head * HD;
  const float sc = a.scale;
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      EL::store4(dk + 32 * u + 8 * g + 4 * hh, dkt[u][4 * g] * sc, dkt[u][4 * g + 1] * sc, dkt[u][4 * g + 2] * sc,
                 dkt[u][4 * g + 3] * sc);
      EL::store4(dv + 32 * u + 8 * g + 4 * hh, dvt[u][4 * g], dvt[u][4 * g + 1], dvt[u][4 * g + 2], dvt[u][4 * g + 3]);
    }
}

template <typename E, int HD, bool MB>  // a full bias adds a per-element load row: one wave per SIMD
__global__ void __launch_bounds__(kThreads, (MB || HD * sizeof(E) >= 256 ? 1 : 2)) attn_bwd_dkv_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  attn_bwd_dkv_body<E, HD, MB>(a, blockIdx.x, smem);
}

// D[b, h, q] = sum_d dO o O, summed exactly as attn_bwd_dq_body does (chunk-sequential fmaf per lane
// half, halves added): the pre-pass of the merged backward.  One 64-lane wave per 32 rows.
template <typename E, int HD>
__global__ void __launch_bounds__(kThreads) attn_delta_kernel(Args a) {
  using TL = Tile<E, HD>;
  using EL = Elt<E>;
  constexpr int QCH = TL::NCH / 2;
  const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int64_t rows = static_cast<int64_t>(a.B) * a.nh * a.Lq;
  for (int64_t row0 = (static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6)) * 32; row0 < rows;
       row0 += static_cast<int64_t>(gridDim.x) * kWaves * 32) {
    const int64_t li = row0 + r;
    const int64_t lc = li < rows ? li : rows - 1;
    const int q = static_cast<int>(lc % a.Lq);
    const int head = static_cast<int>((lc / a.Lq) % a.nh);
    const int b = static_cast<int>(lc / a.Lq / a.nh);
    const E* orow = static_cast<const E*>(a.out) + b * a.osb + static_cast<int64_t>(q) * a.ost + head * HD;
    const E* dorow = static_cast<const E*>(a.dout) + b * a.dosb + static_cast<int64_t>(q) * a.dost + head * HD;
    float dsum = 0.f;
#pragma unroll
    for (int j = 0; j < QCH; ++j) {
      const int c = (2 * j + hh) * TL::CH;
      dsum += EL::chunk_dot(*reinterpret_cast<const u32x4*>(dorow + c), *reinterpret_cast<const u32x4*>(orow + c));
    }
    const float D = dsum + __shfl_xor(dsum, 32, 64);
    if (li < rows && hh == 0) a.delta[li] = D;
  }
}

// The whole backward in one grid: the first nqt row tiles run the dQ pass, the rest the dK/dV pass
// (no dependency between them once D exists), so the two passes share the chip instead of running
// back to back -- at BERT shape (B 12, S 384, 12 heads) each pass alone is 432 workgroups, under two
// per CU at one wave per SIMD, latency-bound.
template <typename E, int HD, bool MB>
__global__ void __launch_bounds__(kThreads, (MB || HD * sizeof(E) >= 256 ? 1 : 2)) attn_bwd_kernel(Args a, int nqt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (static_cast<int>(blockIdx.x) < nqt) attn_bwd_dq_body<E, HD, MB, false>(a, blockIdx.x, smem);
  else attn_bwd_dkv_body<E, HD, MB>(a, blockIdx.x - nqt, smem);
}

// -1 auto, 0 two launches, 1 merged (det_attn_set_bwd_merged, else DET_ATTN_BWD_MERGED=0/1).
// auto: merged when the two passes together have at most two workgroups per CU (measured, graph
// replays, profiles/r4_attention_graph.jsonl: DETR fp32 encoder 0.139 vs 0.191 ms fwd+bwd, cross-
// attention 0.110 vs 0.121; at BERT shape, 864 workgroups, the merged grid is 6 % slower).
int g_bwd_mode = -2;
bool bwd_merged(int64_t workgroups) {
  static const int env = [] {
    const char* e = std::getenv("DET_ATTN_BWD_MERGED");
    return e ? (e[0] == '0' ? 0 : 1) : -1;
  }();
  const int mode = g_bwd_mode >= -1 ? g_bwd_mode : env;
  if (mode >= 0) return mode == 1;
  return workgroups <= 2 * 256;
}

__global__ void attn_mask_kernel(int B, int nh, int Lq, int Lk, uint32_t thr, uint32_t key0, const uint32_t* rng_base,
                                 uint8_t* out) {
  const uint32_t base_key = fold_base(key0, rng_base);  // = run_key of the attention kernels
  const int64_t n = static_cast<int64_t>(B) * nh * Lq * Lk;
  const uint32_t lke = static_cast<uint32_t>(lk_even4(Lk));
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int key = static_cast<int>(i % Lk);
    const int q = static_cast<int>((i / Lk) % Lq);
    const int head = static_cast<int>((i / Lk / Lq) % nh);
    const int b = static_cast<int>(i / Lk / Lq / nh);
    const uint32_t idx = static_cast<uint32_t>(q) * lke + static_cast<uint32_t>(key);
    const uint32_t h = mix32(idx >> 1, rng_key_for(base_key, b, head));
    const uint32_t d = (idx & 1) ? (h >> 16) : (h & 0xffffu);
    out[i] = d >= thr;
  }
}

// ---- host side ----------------------------------------------------------------------------------
template <typename E, int HD>
struct Cfg {
  using TL = Tile<E, HD>;
  static size_t fwd(int Lk) {
    return 2 * static_cast<size_t>(TL::ROW_BYTES + TL::T_BYTES) + 4 * static_cast<size_t>((Lk + kKB - 1) / kKB * kKB);
  }
  static size_t dq(int Lk) {
    return 2 * static_cast<size_t>(2 * TL::ROW_BYTES + TL::T_BYTES) +
           4 * static_cast<size_t>((Lk + kKB - 1) / kKB * kKB);
  }
  static size_t dkv(int Lq) {
    return 2 * static_cast<size_t>(2 * (TL::ROW_BYTES + TL::T_BYTES)) +
           8 * static_cast<size_t>((Lq + kKB - 1) / kKB * kKB);
  }
  static bool fits(int Lq, int Lk) {
    return fwd(Lk) <= kMaxLds && dq(Lk) <= kMaxLds && dkv(Lq) <= kMaxLds;
  }
  static void launch_fwd(hipStream_t st, const Args& a) {
    dim3 grid((a.Lq + kQB - 1) / kQB, a.nh, a.B);
    if (a.mbias)
      hipLaunchKernelGGL((attn_fwd_kernel<E, HD, true>), grid, dim3(kThreads), fwd(a.Lk), st, a);
    else
      hipLaunchKernelGGL((attn_fwd_kernel<E, HD, false>), grid, dim3(kThreads), fwd(a.Lk), st, a);
  }
  static void launch_bwd(hipStream_t st, const Args& a) {
    dim3 gq((a.Lq + kQB - 1) / kQB, a.nh, a.B), gk((a.Lk + kQB - 1) / kQB, a.nh, a.B);
    if (bwd_merged(static_cast<int64_t>(gq.x + gk.x) * a.nh * a.B)) {
      const int64_t rows = static_cast<int64_t>(a.B) * a.nh * a.Lq;
      const int64_t dgrid = (rows + kWaves * 32 - 1) / (kWaves * 32);
      hipLaunchKernelGGL((attn_delta_kernel<E, HD>), dim3(static_cast<unsigned>(dgrid < 65536 ? dgrid : 65536)),
                         dim3(kThreads), 0, st, a);
      const int nqt = static_cast<int>(gq.x);
      const dim3 g(gq.x + gk.x, a.nh, a.B);
      const size_t lds = dq(a.Lk) > dkv(a.Lq) ? dq(a.Lk) : dkv(a.Lq);
      if (a.mbias) hipLaunchKernelGGL((attn_bwd_kernel<E, HD, true>), g, dim3(kThreads), lds, st, a, nqt);
      else hipLaunchKernelGGL((attn_bwd_kernel<E, HD, false>), g, dim3(kThreads), lds, st, a, nqt);
      return;
    }
    if (a.mbias) {
      hipLaunchKernelGGL((attn_bwd_dq_kernel<E, HD, true>), gq, dim3(kThreads), dq(a.Lk), st, a);
      hipLaunchKernelGGL((attn_bwd_dkv_kernel<E, HD, true>), gk, dim3(kThreads), dkv(a.Lq), st, a);
    } else {
      hipLaunchKernelGGL((attn_bwd_dq_kernel<E, HD, false>), gq, dim3(kThreads), dq(a.Lk), st, a);
      hipLaunchKernelGGL((attn_bwd_dkv_kernel<E, HD, false>), gk, dim3(kThreads), dkv(a.Lq), st, a);
    }
  }
};

// dtype 0 = bf16, 1 = fp32
template <typename F>
bool dispatch(int dtype, int hd, F&& f) {
  if (dtype == 0 && hd == 32) return f(Cfg<unsigned short, 32>{}), true;
  if (dtype == 0 && hd == 64) return f(Cfg<unsigned short, 64>{}), true;
  if (dtype == 0 && hd == 128) return f(Cfg<unsigned short, 128>{}), true;
  if (dtype == 1 && hd == 32) return f(Cfg<float, 32>{}), true;
  if (dtype == 1 && hd == 64) return f(Cfg<float, 64>{}), true;
  return false;
}

uint32_t drop_threshold(float p) {
  uint32_t thr = p > 0.f ? static_cast<uint32_t>(p * 65536.0f + 0.5f) : 0u;
  return thr > 65535u ? 65535u : thr;
}
uint32_t host_mix32(uint32_t x, uint32_t key) {  // = mix32, for the host
  x ^= key;
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
uint32_t mix_key(uint64_t seed, uint64_t offset) {  // all 128 bits through the mixer
  uint32_t k = host_mix32(static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32) ^ 0x85ebca6bu);
  k = host_mix32(static_cast<uint32_t>(offset), k);
  return host_mix32(static_cast<uint32_t>(offset >> 32), k ^ 0xc2b2ae35u);
}

}  // namespace

extern "C" {

// mirrored by determined_1_amd/ops/transformer.py:_AttnParams (field order matters)
struct DetAttnParams {
  const void *q, *k, *v, *dout;
  void *out, *dq, *dk, *dv;
  float *lse, *delta;
  const float *kbias, *mbias;
  int64_t qsb, qst, ksb, kst, vsb, vst, osb, ost, dosb, dost, dqsb, dqst, dksb, dkst, dvsb, dvst;
  int64_t mbb, mbh, mbq;
  int32_t B, Lq, Lk, nh, hd, dtype;
  float p, scale;
  uint64_t seed, offset;
  const uint32_t* rng_base;  // nullable (Args::rng_base)
};

// Which (dtype, head_dim, Lq, Lk) the MFMA kernels cover (LDS holds the double-buffered tiles plus
// the key-bias / LSE / delta rows).
int det_attn_supported(int dtype, int hd, int Lq, int Lk) {
  if (Lq <= 0 || Lk <= 0) return 0;
  bool ok = false;
  dispatch(dtype, hd, [&](auto cfg) { ok = decltype(cfg)::fits(Lq, Lk); });
  return ok ? 1 : 0;
}

static int fill(Args& a, const DetAttnParams* P) {
  if (!P || P->B <= 0 || P->nh <= 0 || !det_attn_supported(P->dtype, P->hd, P->Lq, P->Lk)) return -1;
  a.q = P->q;
  a.k = P->k;
  a.v = P->v;
  a.dout = P->dout;
  a.out = P->out;
  a.dq = P->dq;
  a.dk = P->dk;
  a.dv = P->dv;
  a.lse = P->lse;
  a.delta = P->delta;
  a.kbias = P->kbias;
  a.mbias = P->mbias;
  a.qsb = P->qsb, a.qst = P->qst, a.ksb = P->ksb, a.kst = P->kst, a.vsb = P->vsb, a.vst = P->vst;
  a.osb = P->osb, a.ost = P->ost, a.dosb = P->dosb, a.dost = P->dost;
  a.dqsb = P->dqsb, a.dqst = P->dqst, a.dksb = P->dksb, a.dkst = P->dkst, a.dvsb = P->dvsb, a.dvst = P->dvst;
  a.mbb = P->mbb, a.mbh = P->mbh, a.mbq = P->mbq;
  a.B = P->B, a.Lq = P->Lq, a.Lk = P->Lk, a.nh = P->nh;
  a.scale = P->scale;
  a.scale_log2 = P->scale * kLog2e;
  a.drop_thr = drop_threshold(P->p);
  a.drop_scale = a.drop_thr ? 65536.0f / static_cast<float>(65536u - a.drop_thr) : 1.f;
  a.rng_key = mix_key(P->seed, P->offset);
  a.rng_base = P->rng_base;
  return 0;
}

// out = softmax(q k^T * scale + bias) v (dropout p), lse [B, nh, Lq] fp32.
int det_attn_forward(void* stream, const DetAttnParams* P) {
  Args a;
  if (fill(a, P) || !a.out || !a.lse) return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  dispatch(P->dtype, P->hd, [&](auto cfg) { decltype(cfg)::launch_fwd(st, a); });
  return static_cast<int>(hipGetLastError());
}

// dq/dk/dv fully overwritten (rows < Lq / Lk); delta [B, nh, Lq] fp32 workspace.
int det_attn_backward(void* stream, const DetAttnParams* P) {
  Args a;
  if (fill(a, P) || !a.dout || !a.dq || !a.dk || !a.dv || !a.delta) return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  dispatch(P->dtype, P->hd, [&](auto cfg) { decltype(cfg)::launch_bwd(st, a); });
  return static_cast<int>(hipGetLastError());
}

// Backward as one merged grid after a D pre-pass (1) or as the dQ and dK/dV launches back to back
// (0); -1 picks by grid size (auto, the default), < -1 restores DET_ATTN_BWD_MERGED.  For benchmarks
// and tests.  Returns the previous override.
int det_attn_set_bwd_merged(int on) {
  const int old = g_bwd_mode;
  g_bwd_mode = on < -1 ? -2 : (on > 1 ? 1 : on);
  return old;
}

// The keep mask (1 = kept) the kernels derive for (p, seed, offset): [B, nh, Lq, Lk] uint8 (tests).
int det_attn_dropout_mask(void* stream, int B, int nh, int Lq, int Lk, float p, uint64_t seed, uint64_t offset,
                          uint8_t* out, const uint32_t* rng_base) {
  hipLaunchKernelGGL(attn_mask_kernel, dim3(2048), dim3(256), 0, static_cast<hipStream_t>(stream), B, nh, Lq, Lk,
                     drop_threshold(p), mix_key(seed, offset), rng_base, out);
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
