// det_conv.hip — hand-written bf16 MFMA GEMMs for ResNet's 1x1 convolutions in NHWC, with the
// BatchNorm work that surrounds them folded into the GEMM passes.
//
// A 1x1 convolution over a channels_last activation is a plain GEMM on [rows = N*H*W, channels]:
//   forward  Y[M, Cout]   = X[M, Cin] . W[Cout, Cin]^T            (gemm_nt, "NT": both K-contiguous)
//   dgrad    dX[M, Cin]   = dY[M, Cout] . W^T[Cin, Cout]^T         (gemm_nt with the transposed weight)
//   wgrad    dW[Cout,Cin] = dY[M, Cout]^T . X[M, Cin]             (gemm_tn: reduction over the M rows)
// At ResNet-50 / bs512 shapes these are HBM-bound (layer1: K = 64 input channels, arithmetic
// intensity ~50 FLOP/B), so what matters is touching each activation byte once:
//   * forward epilogue computes the BatchNorm batch statistics of Y from the accumulators
//     (per-(row-block, channel) mean and M2 = sum of squared deviations, Chan-mergeable), which
//     removes the separate stats pass over Y (det_norm.hip bn_stats_partial);
//   * optional prologue: the A operand is relu(X * scale[k] + shift[k]) applied while staging, i.e.
//     the preceding BatchNorm-apply + ReLU is fused into the GEMM load and that activation is never
//     written to HBM (forward of conv3 over bn2's input; wgrad recomputes it the same way);
//   * 1x1 stride-2 (projection shortcut) convolutions gather their input rows in the A load.
//
// CDNA4 mapping (cdna_hip_programming.md §3, §5):
//   * v_mfma_f32_16x16x32_bf16; 4 waves (256 threads) per workgroup, wave tile 64x64 (4x4 MFMA tiles,
//     64 fp32 accumulators per lane) for the 128x128 block tile;
//   * K tile 64 (128-B LDS rows), double-buffered LDS, register staging with the next tile's global
//     loads in flight during the MFMAs and ONE barrier per K tile; XOR-swizzled 16-B chunks
//     (chunk ^ (row & 7)) so the 16 rows of an A/B fragment read spread over the banks;
//   * wgrad stages [m][n] / [m][k] row tiles as they come from HBM and reads both MFMA operands
//     with ds_read_b64_tr_b16 (hardware transpose) from an XOR-swizzled image;
//   * workgroup -> tile mapping is XCD-aware and bijective (8 XCDs, private L2 each): the blocks that
//     share an A row-panel run on one XCD;
//   * no float atomics: split-K wgrad writes fp32 slabs reduced by a second launch (deterministic).
//
// Reference parity: the reference leaves convolutions to cuDNN inside user models
// (examples/computer_vision/*); semantics are torch.nn.functional.conv2d's.

#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>
#include <type_traits>

#include "det_stats.h"

namespace {

constexpr int kThreads = 256;
constexpr int kBK = 64;  // K tile (elements): one 128-B LDS row per operand row
#ifndef DET_NT_SINGLE_OCC
#define DET_NT_SINGLE_OCC 3
#endif
constexpr int kSingleOcc = DET_NT_SINGLE_OCC;  // workgroups per CU of the K == 64 variant

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) unsigned short us8;

__device__ __forceinline__ float bf2f(unsigned short u) { return __uint_as_float(static_cast<uint32_t>(u) << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));
}
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

// byte offset of 16-B chunk `ch` (0..7) of row `row` in a [rows][64 bf16] tile
__device__ __forceinline__ int swz(int row, int ch) { return row * 128 + ((ch ^ (row & 7)) << 4); }

// Bijective XCD-aware remap: hardware dispatches workgroup ids round-robin over the 8 XCDs; give
// each XCD a contiguous range of logical tiles (cdna_hip_programming.md §5 "XCD swizzle").
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// Input-row gather of a 1x1 stride-2 convolution: output row m = ((n*Ho)+ho)*Wo+wo reads input
// row (n*Hi + 2ho)*Wi + 2wo.
constexpr int kGmDirect = 0, kGmStride2 = 1, kGmStem = 2, kGmConv = 3;  // A/X row gather modes

struct Gather {
  int Ho, Wo, Hi, Wi;
  // kGmConv (wgrad of an R x S conv): channels per input pixel, kernel width, stride, padding
  int cin, ks, cstride, cpad;
  __device__ __forceinline__ int64_t row(int64_t m) const {
    if (static_cast<uint64_t>(m) < (static_cast<uint64_t>(1) << 32)) {
      // 32-bit unsigned divisions (every activation here has < 2^32 rows): the 64-bit ones are a
      // long software sequence per gathered row
      const uint32_t mu = static_cast<uint32_t>(m), hw = static_cast<uint32_t>(Ho) * static_cast<uint32_t>(Wo);
      const uint32_t n = mu / hw, rem = mu - n * hw;
      const uint32_t ho = rem / static_cast<uint32_t>(Wo), wo = rem - ho * static_cast<uint32_t>(Wo);
      return (static_cast<int64_t>(n) * Hi + 2 * ho) * Wi + 2 * wo;
    }
    const int64_t hw = static_cast<int64_t>(Ho) * Wo;
    const int64_t n = m / hw;
    const int rem = static_cast<int>(m - n * hw);
    const int ho = rem / Wo, wo = rem - ho * Wo;
    return (n * Hi + 2 * ho) * Wi + 2 * wo;
  }

  // ResNet stem (7x7, stride 2, pad 3) over an NHWC input with channels padded to 4 (one pixel =
  // 8 B).  K layout of the im2col row: k = r*32 + s*4 + c for r, s in 0..7 (tap 7 and channel 3
  // carry zero weights), so one 16-B chunk q = k/8 is the pixel pair (r = q>>2, s = 2(q&3) + 0/1):
  // adjacent pixels of one input row, contiguous in memory.
  __device__ __forceinline__ const unsigned short* stem(int64_t m, int& ih0, int& iw0,
                                                         const unsigned short* base) const {
    const int64_t hw = static_cast<int64_t>(Ho) * Wo;
    const int64_t n = m / hw;
    const int rem = static_cast<int>(m - n * hw);
    const int ho = rem / Wo, wo = rem - ho * Wo;
    ih0 = 2 * ho - 3;
    iw0 = 2 * wo - 3;
    return base + n * static_cast<int64_t>(Hi) * Wi * 4;
  }
  __device__ __forceinline__ us8 stem_chunk(const unsigned short* img, bool valid, int ih0, int iw0, int q) const {
    const int r = q >> 2, s = (q & 3) * 2;
    const int ih = ih0 + r, iw = iw0 + s;
    const bool rowok = valid && r < 7 && ih >= 0 && ih < Hi;
    typedef __attribute__((ext_vector_type(4))) unsigned short us4;
    us4 lo = us4{0, 0, 0, 0}, hi = us4{0, 0, 0, 0};
    const unsigned short* p = img + (static_cast<int64_t>(ih) * Wi + iw) * 4;
    if (rowok && iw >= 0 && iw < Wi) lo = *reinterpret_cast<const us4*>(p);
    if (rowok && s + 1 < 7 && iw + 1 >= 0 && iw + 1 < Wi) hi = *reinterpret_cast<const us4*>(p + 4);
    return us8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
};

// relu(x * scale + shift) of 8 consecutive channels, re-rounded to bf16
__device__ __forceinline__ us8 affine_relu8(us8 v, const float* __restrict__ scale, const float* __restrict__ shift,
                                            int c0) {
  const float4 s0 = *reinterpret_cast<const float4*>(scale + c0);
  const float4 s1 = *reinterpret_cast<const float4*>(scale + c0 + 4);
  const float4 h0 = *reinterpret_cast<const float4*>(shift + c0);
  const float4 h1 = *reinterpret_cast<const float4*>(shift + c0 + 4);
  const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
  us8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(fmaxf(__fmaf_rn(bf2f(v[j]), sc[j], sh[j]), 0.f));
  return o;
}

// byte offset of 16-B chunk ch of row `row` in a [64][W] bf16 tile (W = 64 or 128): XOR pattern
// that makes the ds_read_b64_tr_b16 fragment reads (4 rows x 2 chunks per 16-lane group, two such
// groups 8 rows apart per 32-lane half) hit distinct banks
template <int W>
__device__ __forceinline__ int tswz(int row, int ch) {
  if (W == 128) return row * 256 + ((ch ^ (((row & 3) << 1) | (((row >> 3) & 1) << 3))) << 4);
  return row * 128 + ((ch ^ ((((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2))) << 4);
}

// MFMA operand (16 columns x 32 k-rows) via two transposed 4x16 reads: lane (g = lane>>4, i = lane&15)
// gets rows k0 + 8g + 0..7 of column c0 + i.
template <int W>
__device__ __forceinline__ bf16x8 tr_frag(const unsigned char* tile, int k0, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = c0 + 4 * p;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const int o0 = tswz<W>(k0 + 8 * g + q, col >> 3) + ((col & 4) << 1);
  const int o1 = tswz<W>(k0 + 8 * g + 4 + q, col >> 3) + ((col & 4) << 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + o0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + o1));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// BN-backward epilogue of an input-gradient GEMM whose output feeds a training BatchNorm's backward
// (C = dL/dy of y = act(bn(x) [+ res])):  d = mask * (C [+ add]) is written instead of C, and the
// BN's backward partial sums over this block's rows, psum = sum d and psumx = sum d (x - mean), go
// to [ceil(M/BM), N] -- the BN backward then needs only its finalize and an unmasked apply
// (det_norm.hip det_bn_bwd_from_partials), and with an identity shortcut d IS the residual's
// gradient, so that pass writes no second tensor.  mode 1: mask = (x*scale + shift > 0);
// mode 2: mask bits of the forward (1 bit per element, with the residual in the sum).
struct BnBwdEpi {
  const unsigned short* x;     // BN input [M, N]
  const float* mean;           // [N]
  const float* scale;          // mode 1
  const float* shift;
  const uint8_t* mbits;        // mode 2: [M*N/8]
  const unsigned short* add;   // nullable: identity-shortcut gradient summed before the mask
  float* psum;
  float* psumx;
  int mode;
  // add_hi > 0: add is given on the stride-2 grid [M/(Hi*Wi)*Ho*Wo, N] of a 1x1 stride-2 projection
  // shortcut (its input gradient is zero off the even (h, w) positions) -- never materialised at
  // the full resolution
  int add_ho, add_wo, add_hi, add_wi;
};

struct NtArgs {
  const unsigned short* A;  // [rows, K]
  const unsigned short* B;  // [N, K]
  unsigned short* C;        // [M, N]
  int64_t M;
  int N, K;
  const float* scale;  // PRO: A <- relu(A*scale[k] + shift[k])
  const float* shift;
  float* pmean;  // STATS: [ceil(M/BM), N] block mean / M2 of the bf16-rounded C
  float* pm2;
  Gather g;  // STRIDE2
  BnBwdEpi bn;  // BNB
  // ABN (input gradient of the conv that produced a training BatchNorm's input): the A operand is
  // the BN backward's apply, dY = coef[0][k] * A + coef[1][k] * A2 + coef[2][k] (A = the BN's
  // masked output gradient, A2 = the BN input), computed while staging; the blocks of the first
  // N tile also write it to Aout (the weight gradient's operand) -- the separate apply pass
  // (read A, A2, write dY) and this GEMM's read of dY become one pass.
  const unsigned short* A2;
  const float* acoef;  // [3][K]
  unsigned short* Aout;
  uint8_t* abits;  // AFWD: ReLU mask bits of Aout (1 per element)
  // AFWD (nullable): A2 is itself a BatchNorm output whose apply was deferred (ResNet's projection
  // shortcut BN): the residual is A2 * a2scale[k] + a2shift[k] (det_norm.hip bn_apply_fwd RES 2)
  const float* a2scale;
  const float* a2shift;
  // nullable: C = op(A) . B^T + bias[n] (bf16 [N]; added to the fp32 accumulators, one rounding)
  const unsigned short* bias;
  // 1: BN statistics before the C stores (DET_STATS_FIRST=1 A/B); 0: after them (default)
  int stats_first;
};

// ------------------------------------------------------------------------------------------------
// C[M,N] = op(A)[M,K] . B[N,K]^T, bf16 in/out, fp32 accumulate.  N % BN == 0, K % 64 == 0.
// ------------------------------------------------------------------------------------------------
// OCC: workgroups per CU the register budget is sized for.  K == 64 (one K tile: layer1's
// 64-channel side, every dgrad into a 64-channel input) is a pure streaming pass with no K loop
// to overlap loads with, so it runs single-buffered (half the LDS) at higher occupancy instead.
// BT: B is given as [K, N] (N contiguous: the conv weight [Cout, Cin] itself for an input gradient),
// staged as it sits ([64 k][BN] image, the wgrad swizzle) and read with ds_read_b64_tr_b16 -- no
// transposed weight copy per call.
// AFWD (forward of the conv that consumes a training BatchNorm(+residual)+ReLU output, ResNet
// bn3 -> the next block's conv1): the A operand is the BN apply itself, relu(A*scale[k] + shift[k]
// + A2) with A = the BN input and A2 = the residual, and the first N tile's blocks write it (Aout)
// and its ReLU mask bits (abits) for the residual add and the backward: the separate apply pass
// and this GEMM's read of its output become one pass.
// PF: register staging sets -- the global loads of K tiles kt+1 .. kt+PF are in flight while tile kt
// is multiplied (PF = 1: one tile ahead).  The short-K, wide-N GEMMs (layer 2-4 expansions, K =
// 128..512) spend most of a block's life waiting for each K tile's loads; deeper prefetch overlaps
// those latencies instead of paying them one after another.
template <int BM, int BN, int WM, int WN, bool PRO, bool STATS, int GM, int OCC, bool BNB = false, bool BT = false,
          bool ABN = false, bool AFWD = false, int PF = 1>
__global__ void __launch_bounds__(kThreads, OCC) gemm_nt_kernel(NtArgs a) {
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int ACH = BM * 8 / kThreads, BCH = BN * 8 / kThreads;
  constexpr int A_BYTES = BM * 128, BUF = (BM + BN) * 128;
  constexpr int LDC = BN + 16;  // epilogue tile row stride (bf16): +32 B keeps the 4 row groups on distinct banks
  static_assert(WM * WN == 4, "4 waves");
  static_assert(FM >= 1 && FN >= 1 && ACH >= 1 && BCH >= 1, "tile");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float red[WM * BN * 3];  // STATS: per (wave row, column) mean, M2, count

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = a.N / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntn, nt = bid - mt * ntn;
  const int64_t m0 = static_cast<int64_t>(mt) * BM;
  const int n0 = nt * BN;
  const int kc = tid & 7, r0 = tid >> 3;
  const int64_t K = a.K;
  const bool first_ntile = nt == 0;  // ABN: these blocks write the staged A operand out

  const unsigned short* aptr[ACH];
  bool aval[ACH];
  int ih0[ACH], iw0[ACH];  // GM_STEM: top-left input pixel of the row's 7x7 window
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int64_t m = m0 + r0 + 32 * i;
    aval[i] = m < a.M;
    int64_t row = aval[i] ? m : 0;
    if (GM == kGmStride2) row = a.g.row(row);
    if (GM == kGmStem) {
      aptr[i] = a.g.stem(row, ih0[i], iw0[i], a.A);
    } else {
      aptr[i] = a.A + row * K + kc * 8;
    }
  }
  const unsigned short* bptr = a.B + static_cast<int64_t>(n0 + r0) * K + kc * 8;
  constexpr int BCPR = BN / 8;  // BT: 16-B chunks per B image row

  constexpr bool A2IN = ABN || AFWD;
  static_assert(PF >= 1 && PF <= 4, "prefetch depth");
  us8 ra_[PF][ACH], rb_[PF][BCH], ra2_[PF][A2IN ? ACH : 1];
  // S: the register set (a compile-time index, std::integral_constant) that holds K tile kt
  auto gload = [&](auto S, int kt) {
    constexpr int s = decltype(S)::value;
    us8* ra = ra_[s];
    us8* rb = rb_[s];
    us8* ra2 = ra2_[s];
    const int64_t k = static_cast<int64_t>(kt) * kBK;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      if (GM == kGmStem) ra[i] = a.g.stem_chunk(aptr[i], aval[i], ih0[i], iw0[i], kt * 8 + kc);
      else if (aval[i]) ra[i] = *reinterpret_cast<const us8*>(aptr[i] + k);
      else ra[i] = us8{0, 0, 0, 0, 0, 0, 0, 0};
      if constexpr (A2IN) {
        if (aval[i]) ra2[i] = *reinterpret_cast<const us8*>(a.A2 + (aptr[i] - a.A) + k);
        else ra2[i] = us8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      if (BT) {
        const int idx = tid + j * kThreads, r = idx / BCPR, c = idx - r * BCPR;
        rb[j] = *reinterpret_cast<const us8*>(a.B + (k + r) * a.N + n0 + c * 8);
      } else {
        rb[j] = *reinterpret_cast<const us8*>(bptr + 32 * j * K + k);
      }
    }
  };
  auto lstore = [&](auto S, int buf, int kt) {
    constexpr int s = decltype(S)::value;
    const us8* ra = ra_[s];
    const us8* rb = rb_[s];
    const us8* ra2 = ra2_[s];
    unsigned char* base = smem + buf * BUF;
    // ABN: this thread's 8 channels of the apply coefficients, loaded once per K tile (before the
    // Aout stores, which the compiler could not move them across)
    float ca[8], cb[8], cc[8], ra_s[8], ra_h[8];
    const bool a2aff = AFWD && a.a2scale != nullptr;
    if constexpr (AFWD) {  // scale, shift of this thread's 8 channels (and of the residual's BN)
      const int k0 = kt * kBK + kc * 8;
#pragma unroll
      for (int j = 0; j < 8; j += 4) {
        const float4 S0 = *reinterpret_cast<const float4*>(a.scale + k0 + j);
        const float4 H0 = *reinterpret_cast<const float4*>(a.shift + k0 + j);
        ca[j] = S0.x; ca[j + 1] = S0.y; ca[j + 2] = S0.z; ca[j + 3] = S0.w;
        cb[j] = H0.x; cb[j + 1] = H0.y; cb[j + 2] = H0.z; cb[j + 3] = H0.w;
        float4 S2 = make_float4(1.f, 1.f, 1.f, 1.f), H2 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a2aff) {
          S2 = *reinterpret_cast<const float4*>(a.a2scale + k0 + j);
          H2 = *reinterpret_cast<const float4*>(a.a2shift + k0 + j);
        }
        ra_s[j] = S2.x; ra_s[j + 1] = S2.y; ra_s[j + 2] = S2.z; ra_s[j + 3] = S2.w;
        ra_h[j] = H2.x; ra_h[j + 1] = H2.y; ra_h[j + 2] = H2.z; ra_h[j + 3] = H2.w;
      }
    }
    if constexpr (ABN) {
      const int k0 = kt * kBK + kc * 8;
#pragma unroll
      for (int j = 0; j < 8; j += 4) {
        const float4 A0 = *reinterpret_cast<const float4*>(a.acoef + k0 + j);
        const float4 B0 = *reinterpret_cast<const float4*>(a.acoef + a.K + k0 + j);
        const float4 C0 = *reinterpret_cast<const float4*>(a.acoef + 2 * a.K + k0 + j);
        ca[j] = A0.x; ca[j + 1] = A0.y; ca[j + 2] = A0.z; ca[j + 3] = A0.w;
        cb[j] = B0.x; cb[j + 1] = B0.y; cb[j + 2] = B0.z; cb[j + 3] = B0.w;
        cc[j] = C0.x; cc[j + 1] = C0.y; cc[j + 2] = C0.z; cc[j + 3] = C0.w;
      }
    }
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      us8 v = ra[i];
      if (PRO) {
        v = affine_relu8(v, a.scale, a.shift, kt * kBK + kc * 8);
        if (!aval[i]) v = us8{0, 0, 0, 0, 0, 0, 0, 0};
      }
      if constexpr (ABN) {
        // exactly det_norm.hip bn_apply_bwd<MASK 0>: fma(A, d, fma(B, x, C)) in fp32, one rounding
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f2bf(__fmaf_rn(ca[j], bf2f(ra[i][j]), __fmaf_rn(cb[j], bf2f(ra2[i][j]), cc[j])));
        if (!aval[i]) v = us8{0, 0, 0, 0, 0, 0, 0, 0};
        else if (first_ntile) *reinterpret_cast<us8*>(a.Aout + (aptr[i] - a.A) + static_cast<int64_t>(kt) * kBK) = v;
      }
      if constexpr (AFWD) {
        // exactly det_norm.hip bn_apply_fwd<RELU, RES>: z = fma(x, scale, shift) + res, relu, mask bits
        // (RES 2: res = bf16(fma(r, rscale, rshift)) of the deferred residual BN)
        unsigned bits = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float r2 = bf2f(ra2[i][j]);
          const float z = __fmaf_rn(bf2f(ra[i][j]), ca[j], cb[j]) + (a2aff ? round_bf(__fmaf_rn(r2, ra_s[j], ra_h[j])) : r2);
          v[j] = f2bf(fmaxf(z, 0.f));
          bits |= (z > 0.f ? 1u : 0u) << j;
        }
        if (!aval[i]) {
          v = us8{0, 0, 0, 0, 0, 0, 0, 0};
        } else if (first_ntile) {
          const int64_t off = (aptr[i] - a.A) + static_cast<int64_t>(kt) * kBK;
          *reinterpret_cast<us8*>(a.Aout + off) = v;
          a.abits[off >> 3] = static_cast<uint8_t>(bits);
        }
      }
      *reinterpret_cast<us8*>(base + swz(r0 + 32 * i, kc)) = v;
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      if (BT) {
        const int idx = tid + j * kThreads, r = idx / BCPR, c = idx - r * BCPR;
        *reinterpret_cast<us8*>(base + A_BYTES + tswz<BN>(r, c)) = rb[j];
      } else {
        *reinterpret_cast<us8*>(base + A_BYTES + swz(r0 + 32 * j, kc)) = rb[j];
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // BNB: the epilogue's operand loads (BN input, shortcut gradient, mask bits) are issued before
  // the K loop, so their HBM latency overlaps the GEMM instead of following it (these dgrads have
  // short K loops and stream 3 activation-sized tensors through the epilogue)
  constexpr int CPR = BN / 8;  // 16-B chunks per output row
  const int64_t rows_left = a.M - m0;
  const int nvalid = rows_left < BM ? static_cast<int>(rows_left) : BM;
  constexpr int NQE = BNB ? BM * CPR / kThreads : 1;
  // hoisted only where the registers allow it (occupancy-2 tiles without the ABN staging: the
  // others spill); elsewhere the loads are issued at the start of the epilogue
  constexpr bool EPRE = BNB && OCC <= 2 && !ABN && PF == 1;
  us8 xs[NQE], as[NQE];
  unsigned bs[NQE];
  auto eload = [&]() {
    static_assert(!BNB || kThreads % CPR == 0, "fixed chunk column per thread");
    const int c0 = n0 + (tid % CPR) * 8;
#pragma unroll
    for (int q = 0; q < NQE; ++q) {
      const int row = (tid + q * kThreads) / CPR;
      const bool ok = row < nvalid;
      const int64_t off = (m0 + (ok ? row : 0)) * a.N + c0;
      xs[q] = ok ? *reinterpret_cast<const us8*>(a.bn.x + off) : us8{0, 0, 0, 0, 0, 0, 0, 0};
      as[q] = us8{0, 0, 0, 0, 0, 0, 0, 0};
      if (ok && a.bn.add) {
        int64_t aoff = off;
        bool on = true;
        if (a.bn.add_hi > 0) {
          // 32-bit unsigned index math (M < 2^32, checked by the host): a 64-bit division is a long
          // software sequence, and every thread does NQE of these before its first store
          const uint32_t r = static_cast<uint32_t>(m0 + row);
          const uint32_t hw = static_cast<uint32_t>(a.bn.add_hi) * static_cast<uint32_t>(a.bn.add_wi);
          const uint32_t img = r / hw, rem = r - img * hw;
          const uint32_t h = rem / static_cast<uint32_t>(a.bn.add_wi), w = rem - h * static_cast<uint32_t>(a.bn.add_wi);
          on = ((h | w) & 1u) == 0;
          aoff = (static_cast<int64_t>(img * static_cast<uint32_t>(a.bn.add_ho) + (h >> 1)) * a.bn.add_wo + (w >> 1)) *
                     a.N + c0;
        }
        if (on) as[q] = *reinterpret_cast<const us8*>(a.bn.add + aoff);
      }
      bs[q] = (ok && a.bn.mode == 2) ? a.bn.mbits[off >> 3] : 0u;
    }
  };
  if constexpr (EPRE) eload();

  const int nk = a.K / kBK;
  using I0 = std::integral_constant<int, 0>;
  gload(I0{}, 0);
  if constexpr (PF > 1) if (1 < nk) gload(std::integral_constant<int, 1 % PF>{}, 1);
  if constexpr (PF > 2) if (2 < nk) gload(std::integral_constant<int, 2 % PF>{}, 2);
  if constexpr (PF > 3) if (3 < nk) gload(std::integral_constant<int, 3 % PF>{}, 3);
  lstore(I0{}, 0, 0);
  if (PF < nk) gload(I0{}, PF);  // set 0 is free again: tile PF
  __syncthreads();
  // one K tile: multiply buffer kt & 1, stage tile kt+1 (register set S) into the other buffer and
  // refill S with tile kt+1+PF
  auto step = [&](auto S, int kt) {
    const unsigned char* base = smem + (kt & 1) * BUF;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + (lane >> 4);
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(base + swz(wm * TM + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if (BT) bfr[j] = tr_frag<BN>(base + A_BYTES, ks * 32, wn * TN + j * 16, lane);
        else bfr[j] = *reinterpret_cast<const bf16x8*>(base + A_BYTES + swz(wn * TN + j * 16 + (lane & 15), ch));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    const int nx = kt + 1;
    if (nx < nk) {
      lstore(S, nx & 1, nx);
      if (nx + PF < nk) gload(S, nx + PF);
    }
    __syncthreads();
  };
  for (int kb = 0; kb < nk; kb += PF) {  // unrolled by PF so every register set index is static
    step(std::integral_constant<int, 1 % PF>{}, kb);
    if constexpr (PF > 1) if (kb + 1 < nk) step(std::integral_constant<int, 2 % PF>{}, kb + 1);
    if constexpr (PF > 2) if (kb + 2 < nk) step(std::integral_constant<int, 3 % PF>{}, kb + 2);
    if constexpr (PF > 3) if (kb + 3 < nk) step(std::integral_constant<int, 4 % PF>{}, kb + 3);
  }

  // ---- epilogue: bf16 tile through LDS (coalesced 16-B row stores) + BN statistics ----
  if constexpr (!BNB) {
    if (a.bias != nullptr) {  // a Linear layer's bias (det_linear_fwd)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const float bj = bf2f(a.bias[n0 + wn * TN + j * 16 + (lane & 15)]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += bj;
      }
    }
  }
  unsigned short* ct = reinterpret_cast<unsigned short*>(smem);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * TM + i * 16 + (lane >> 4) * 4 + r;
        const int col = wn * TN + j * 16 + (lane & 15);
        ct[row * LDC + col] = f2bf(acc[i][j][r]);
      }
  if (STATS && a.stats_first && !BNB)
    det_block_bn_stats<FM, FN, WM, TM, TN, BN>(acc, red, wm, wn, lane, tid, nvalid, a.pmean, a.pm2,
                                                static_cast<int64_t>(mt) * a.N + n0);
  __syncthreads();
  if constexpr (BNB) {
    if (STATS)
      det_block_bn_stats<FM, FN, WM, TM, TN, BN>(acc, red, wm, wn, lane, tid, nvalid, a.pmean, a.pm2,
                                                  static_cast<int64_t>(mt) * a.N + n0);
    // each thread owns one 8-column chunk (kThreads % CPR == 0) over rows tid/CPR + q*kThreads/CPR
    const int cc = tid % CPR;
    const int c0 = n0 + cc * 8;
    float mu[8], sc[8], sh[8], s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mu[j] = a.bn.mean[c0 + j];
      sc[j] = a.bn.mode == 1 ? a.bn.scale[c0 + j] : 0.f;
      sh[j] = a.bn.mode == 1 ? a.bn.shift[c0 + j] : 0.f;
      s1[j] = 0.f;
      s2[j] = 0.f;
    }
    constexpr int NQ = NQE;
    if constexpr (!EPRE) eload();  // all loads before the first store (they may alias it)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int row = (tid + q * kThreads) / CPR;
      if (row >= nvalid) continue;
      const int64_t off = (m0 + row) * a.N + c0;
      const us8 cv = *reinterpret_cast<const us8*>(ct + row * LDC + cc * 8);
      const us8 xv = xs[q];
      const us8 av = as[q];
      const unsigned bits = bs[q];
      us8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xf = bf2f(xv[j]);
        float d = bf2f(cv[j]) + (a.bn.add ? bf2f(av[j]) : 0.f);
        const bool on = a.bn.mode == 2 ? ((bits >> j) & 1u) != 0 : __fmaf_rn(xf, sc[j], sh[j]) > 0.f;
        d = on ? d : 0.f;
        o[j] = f2bf(d);
        const float dr = bf2f(o[j]);  // the sums see exactly what the BN apply reads back
        s1[j] += dr;
        s2[j] += dr * (xf - mu[j]);
      }
      *reinterpret_cast<us8*>(a.C + off) = o;
    }
    float* scratch = reinterpret_cast<float*>(smem + BM * LDC * 2);  // [kThreads][16], past the C tile
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      scratch[tid * 16 + j] = s1[j];
      scratch[tid * 16 + 8 + j] = s2[j];
    }
    __syncthreads();
    if (tid < BN) {
      const int ccol = tid / 8, j = tid % 8;
      float t1 = 0.f, t2 = 0.f;
      for (int g = 0; g < kThreads / CPR; ++g) {
        t1 += scratch[(g * CPR + ccol) * 16 + j];
        t2 += scratch[(g * CPR + ccol) * 16 + 8 + j];
      }
      a.bn.psum[static_cast<int64_t>(mt) * a.N + n0 + tid] = t1;
      a.bn.psumx[static_cast<int64_t>(mt) * a.N + n0 + tid] = t2;
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < BM * CPR / kThreads; ++q) {
    const int idx = tid + q * kThreads;
    const int row = idx / CPR, cc = idx - row * CPR;
    if (row < nvalid)
      *reinterpret_cast<us8*>(a.C + (m0 + row) * a.N + n0 + cc * 8) = *reinterpret_cast<const us8*>(ct + row * LDC + cc * 8);
  }
  // BN statistics after the stores are issued (red is a separate LDS array): they drain meanwhile
  if (STATS && !a.stats_first)
    det_block_bn_stats<FM, FN, WM, TM, TN, BN>(acc, red, wm, wn, lane, tid, nvalid, a.pmean, a.pm2,
                                                static_cast<int64_t>(mt) * a.N + n0);
}

// ------------------------------------------------------------------------------------------------
// wgrad: P[s][N][K] (fp32 slab per M split s) = sum_{m in split s} dY[m][n] * op(X)[g(m)][k]
// ------------------------------------------------------------------------------------------------
struct TnArgs {
  const unsigned short* dY;  // [M, N]
  const unsigned short* X;   // [rows, K]
  float* P;                  // [S, N, K]
  int64_t M;
  int N, K;
  int64_t rows_per_split;  // multiple of 64
  const float* scale;      // PRO: X <- relu(X*scale[k] + shift[k])
  const float* shift;
  Gather g;
};

// KSUB: K sub-tiles of BK columns per workgroup (each a separately swizzled [64][BK] LDS image);
// KSUB = 2 lets one workgroup cover K = 2*BK so every dY row is streamed once (the stem's K = 256).
template <int BN, int BK, bool PRO, int GM, int KSUB = 1>
__global__ void __launch_bounds__(kThreads, 2) gemm_tn_kernel(TnArgs a) {
  constexpr int TN = BN / 2, TK = BK * KSUB / 2, FN = TN / 16, FK = TK / 16;
  constexpr int XSUB = 64 * BK * 2;  // bytes of one X sub-tile
  constexpr int YB = 64 * BN * 2, XB = XSUB * KSUB, BUF = YB + XB;
  constexpr int YCH = 64 * BN / 8 / kThreads, XCH = 64 * BK * KSUB / 8 / kThreads;  // 16-B chunks per thread
  constexpr int YCPR = BN / 8, XCPR = BK * KSUB / 8;                                // chunks per row
  constexpr int SCPR = BK / 8;                                                      // chunks per sub-tile row
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid >> 1, wk = wid & 1;
  const int ntn = a.N / BN, ntk = a.K / (BK * KSUB), ntiles = ntn * ntk;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / ntiles, tile = bid - split * ntiles;
  const int nt = tile / ntk, kt_ = tile - nt * ntk;
  const int n0 = nt * BN, k0 = kt_ * BK * KSUB;
  const int64_t mbeg = static_cast<int64_t>(split) * a.rows_per_split;
  int64_t mend = mbeg + a.rows_per_split;
  if (mend > a.M) mend = a.M;

  us8 ry[YCH], rx[XCH];
  bool xval[XCH];
  // kGmConv: each X chunk row tracks its output pixel (n, ho, wo) and advances it by the 64 rows of
  // an M step with carries (no per-step divisions); the tile's tap (r, s) and channel offset are
  // fixed (one tile never straddles taps: cin % (BK * KSUB) == 0)
  int cn[XCH], cho[XCH], cwo[XCH];
  int ctap_r = 0, ctap_s = 0, cc0 = 0, adv_h = 0, adv_w = 0;
  if (GM == kGmConv) {
    const int tap = k0 / a.g.cin;
    cc0 = k0 - tap * a.g.cin;
    ctap_r = tap / a.g.ks;
    ctap_s = tap - ctap_r * a.g.ks;
    adv_h = 64 / a.g.Wo;
    adv_w = 64 - adv_h * a.g.Wo;
    const int hw = a.g.Ho * a.g.Wo;
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int idx = tid + i * kThreads, r = idx / XCPR;
      const int m = static_cast<int>(mbeg) + r;
      cn[i] = m / hw;
      const int rem = m - cn[i] * hw;
      cho[i] = rem / a.g.Wo;
      cwo[i] = rem - cho[i] * a.g.Wo;
    }
  }
  auto gload = [&](int64_t mb) {
#pragma unroll
    for (int i = 0; i < YCH; ++i) {
      const int idx = tid + i * kThreads, r = idx / YCPR, c = idx - r * YCPR;
      const int64_t m = mb + r;
      if (m < mend) ry[i] = *reinterpret_cast<const us8*>(a.dY + m * a.N + n0 + c * 8);
      else ry[i] = us8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int idx = tid + i * kThreads, r = idx / XCPR, c = idx - r * XCPR;
      const int64_t m = mb + r;
      xval[i] = m < mend;
      if (GM == kGmStem) {
        int ih, iw;
        const unsigned short* img = a.g.stem(xval[i] ? m : 0, ih, iw, a.X);
        rx[i] = a.g.stem_chunk(img, xval[i], ih, iw, (k0 >> 3) + c);
        continue;
      }
      if (GM == kGmConv) {
        const int hi = cho[i] * a.g.cstride - a.g.cpad + ctap_r, wi = cwo[i] * a.g.cstride - a.g.cpad + ctap_s;
        const bool ok = xval[i] && hi >= 0 && hi < a.g.Hi && wi >= 0 && wi < a.g.Wi;
        if (ok)
          rx[i] = *reinterpret_cast<const us8*>(
              a.X + ((static_cast<int64_t>(cn[i]) * a.g.Hi + hi) * a.g.Wi + wi) * a.g.cin + cc0 + c * 8);
        else
          rx[i] = us8{0, 0, 0, 0, 0, 0, 0, 0};
        // advance this row's pixel by one M step (64 rows)
        cwo[i] += adv_w;
        int carry = cwo[i] >= a.g.Wo;
        cwo[i] -= carry ? a.g.Wo : 0;
        cho[i] += adv_h + carry;
        while (cho[i] >= a.g.Ho) {
          cho[i] -= a.g.Ho;
          ++cn[i];
        }
        continue;
      }
      const int64_t row = GM == kGmStride2 ? a.g.row(xval[i] ? m : 0) : (xval[i] ? m : 0);
      if (xval[i]) rx[i] = *reinterpret_cast<const us8*>(a.X + row * a.K + k0 + c * 8);
      else rx[i] = us8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  auto lstore = [&](int buf) {
    unsigned char* base = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < YCH; ++i) {
      const int idx = tid + i * kThreads, r = idx / YCPR, c = idx - r * YCPR;
      *reinterpret_cast<us8*>(base + tswz<BN>(r, c)) = ry[i];
    }
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int idx = tid + i * kThreads, r = idx / XCPR, c = idx - r * XCPR;
      us8 v = rx[i];
      if (PRO) {
        v = affine_relu8(v, a.scale, a.shift, k0 + c * 8);
        if (!xval[i]) v = us8{0, 0, 0, 0, 0, 0, 0, 0};
      }
      *reinterpret_cast<us8*>(base + YB + (c / SCPR) * XSUB + tswz<BK>(r, c % SCPR)) = v;
    }
  };

  f32x4 acc[FN][FK];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = mend > mbeg ? static_cast<int>((mend - mbeg + 63) / 64) : 0;
  if (nsteps > 0) {
    gload(mbeg);
    lstore(0);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    if (s + 1 < nsteps) gload(mbeg + static_cast<int64_t>(s + 1) * 64);
    const unsigned char* base = smem + cur * BUF;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 yf[FN], xf[FK];
#pragma unroll
      for (int i = 0; i < FN; ++i) yf[i] = tr_frag<BN>(base, ks * 32, wn * TN + i * 16, lane);
#pragma unroll
      for (int j = 0; j < FK; ++j) {
        const int kc = wk * TK + j * 16;
        xf[j] = tr_frag<BK>(base + YB + (kc / BK) * XSUB, ks * 32, kc % BK, lane);
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FK; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(yf[i], xf[j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nsteps) lstore(cur ^ 1);
    __syncthreads();
  }
  float* out = a.P + static_cast<int64_t>(split) * a.N * a.K;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * TN + i * 16 + (lane >> 4) * 4 + r;
        const int k = k0 + wk * TK + j * 16 + (lane & 15);
        out[static_cast<int64_t>(n) * a.K + k] = acc[i][j][r];
      }
}

// out[i] = scale * sum_s P[s][i]  (fp32 slabs -> bf16 or fp32), deterministic: a block owns E float4
// columns and L = 256 / E split lanes (lane l sums slabs l, l+L, ...), lane 0 of each column adds the
// L lane sums in order.  L > 1 for small outputs with many slabs (a 64 x 64 weight from 512 slabs
// ran on 4 workgroups).
template <typename TO>
__global__ void __launch_bounds__(kThreads) slab_reduce_kernel(const float* __restrict__ P, int S, int64_t n, float scale,
                                                                TO* __restrict__ out, int E) {
  __shared__ float4 part[kThreads];
  const int L = kThreads / E;
  const int e = threadIdx.x % E, l = threadIdx.x / E;
  const int64_t n4 = n >> 2;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * E + e;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    for (int s = l; s < S; s += L) {
      const float4 v = reinterpret_cast<const float4*>(P + s * n)[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  if (l != 0 || i >= n4) return;
  for (int j = 1; j < L; ++j) {
    const float4 v = part[j * E + e];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if constexpr (sizeof(TO) == 4) {
    reinterpret_cast<float4*>(out)[i] = make_float4(acc.x * scale, acc.y * scale, acc.z * scale, acc.w * scale);
  } else {
    ushort4 o;
    o.x = f2bf(acc.x * scale); o.y = f2bf(acc.y * scale); o.z = f2bf(acc.z * scale); o.w = f2bf(acc.w * scale);
    reinterpret_cast<ushort4*>(out)[i] = o;
  }
}

// launch the slab reduce with enough workgroups: split lanes per column while the output is small
void launch_slab_reduce(hipStream_t st, const float* ws, int splits, int64_t slab, float scale, void* out,
                        int out_dtype) {
  const int64_t n4 = slab / 4;
  int lanes = 1;
  while (lanes < kThreads && lanes < splits && n4 / (kThreads / lanes) < 2048) lanes *= 2;
  const int E = kThreads / lanes;
  const int grid = static_cast<int>((n4 + E - 1) / E);
  if (out_dtype == 1)
    hipLaunchKernelGGL(slab_reduce_kernel<unsigned short>, dim3(grid), dim3(kThreads), 0, st, ws, splits, slab, scale,
                       static_cast<unsigned short*>(out), E);
  else
    hipLaunchKernelGGL(slab_reduce_kernel<float>, dim3(grid), dim3(kThreads), 0, st, ws, splits, slab, scale,
                       static_cast<float*>(out), E);
}

template <int BM, int BN, int NBUF>
constexpr int nt_smem() {
  return (NBUF * (BM + BN) * 128) > (BM * (BN + 16) * 2) ? NBUF * (BM + BN) * 128 : BM * (BN + 16) * 2;
}

// PF (prefetch depth) applies to the plain forward / input-gradient variants; the fused ones
// (AFWD, ABN, BNB) already use their registers for the extra operands and stay at PF = 1.
template <int BM, int BN, int WM, int WN, int OCC, int PF = 1>
int launch_nt(hipStream_t st, const NtArgs& a_in, bool pro, bool stats, bool stride2, bool bnb = false, bool bt = false) {
  NtArgs a = a_in;
  static const int stats_first = [] {
    const char* e = std::getenv("DET_STATS_FIRST");
    return e != nullptr && e[0] == '1' ? 1 : 0;
  }();
  a.stats_first = stats_first;
  const int64_t mtiles = (a.M + BM - 1) / BM;
  const int64_t nwg = mtiles * (a.N / BN);
  if (nwg >= (static_cast<int64_t>(1) << 31)) return -4;
  // double-buffered at occupancy 2, and for the 128 x 64 occupancy-3 tiles of the short-K wide-N
  // forwards (g_nt_wide: 48 KB x 3 fits the 160 KB LDS); the 128 x 128 occupancy-3 K == 64 variant
  // has a single K tile and one buffer
  constexpr int smem = nt_smem<BM, BN, (OCC == 2 || (OCC == 3 && BN == 64)) ? 2 : 1>();
  if (a.abits != nullptr) {  // AFWD: forward with the BN apply (+ residual, ReLU) in the A staging
    if (!a.A2 || !a.Aout || !a.scale || !a.shift || pro || bt || bnb || stride2) return -2;
    if constexpr (OCC > 2) {
      return -6;  // the occupancy-3 single-K-tile variant has no register room for it (K = 64 only)
    } else {
      if (stats)
        hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, false, true, kGmDirect, OCC, false, false, false, true>),
                           dim3(static_cast<unsigned>(nwg)), dim3(kThreads), smem, st, a);
      else
        hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, false, false, kGmDirect, OCC, false, false, false, true>),
                           dim3(static_cast<unsigned>(nwg)), dim3(kThreads), smem, st, a);
      return static_cast<int>(hipGetLastError());
    }
  }
  const bool abn = a.A2 != nullptr;
  if (abn && (!bt || pro || stats || stride2)) return -2;  // the A-apply prologue: input gradients only
  if (bnb) {  // input-gradient GEMM with the BN-backward epilogue (no prologue / stats / gather)
    constexpr int smem_b = smem > BM * (BN + 16) * 2 + kThreads * 16 * 4 ? smem : BM * (BN + 16) * 2 + kThreads * 16 * 4;
    if (abn)
      hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, false, false, kGmDirect, OCC, true, true, true, false, PF>),
                         dim3(static_cast<unsigned>(nwg)), dim3(kThreads), smem_b, st, a);
    else if (bt)
      hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, false, false, kGmDirect, OCC, true, true, false, false, PF>),
                         dim3(static_cast<unsigned>(nwg)), dim3(kThreads), smem_b, st, a);
    else
      hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, false, false, kGmDirect, OCC, true, false, false, false, PF>),
                         dim3(static_cast<unsigned>(nwg)), dim3(kThreads), smem_b, st, a);
    return static_cast<int>(hipGetLastError());
  }
  if (bt) {  // plain input-gradient GEMM against the untransposed weight
    if (abn)
      hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, false, false, kGmDirect, OCC, false, true, true>),
                         dim3(static_cast<unsigned>(nwg)), dim3(kThreads), smem, st, a);
    else
      hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, false, false, kGmDirect, OCC, false, true, false, false, PF>),
                         dim3(static_cast<unsigned>(nwg)), dim3(kThreads), smem, st, a);
    return static_cast<int>(hipGetLastError());
  }
#define DET_NT(P, S, G)                                                                                           \
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, P, S, G, OCC, false, false, false, false, PF>),               \
                     dim3(static_cast<unsigned>(nwg)), dim3(kThreads), smem, st, a)
  if (stride2) {
    if (pro) { if (stats) DET_NT(true, true, kGmStride2); else DET_NT(true, false, kGmStride2); }
    else { if (stats) DET_NT(false, true, kGmStride2); else DET_NT(false, false, kGmStride2); }
  } else {
    if (pro) { if (stats) DET_NT(true, true, kGmDirect); else DET_NT(true, false, kGmDirect); }
    else { if (stats) DET_NT(false, true, kGmDirect); else DET_NT(false, false, kGmDirect); }
  }
#undef DET_NT
  return static_cast<int>(hipGetLastError());
}

template <int BN, int BK>
int launch_tn(hipStream_t st, const TnArgs& a, int splits, bool pro, bool stride2, bool conv = false) {
  const int nwg = (a.N / BN) * (a.K / BK) * splits;
  constexpr int smem = 2 * 64 * (BN + BK) * 2;
#define DET_TN(P, G) \
  hipLaunchKernelGGL((gemm_tn_kernel<BN, BK, P, G>), dim3(nwg), dim3(kThreads), smem, st, a)
  if (conv) DET_TN(false, kGmConv);
  else if (stride2) { if (pro) DET_TN(true, kGmStride2); else DET_TN(false, kGmStride2); }
  else { if (pro) DET_TN(true, kGmDirect); else DET_TN(false, kGmDirect); }
#undef DET_TN
  return static_cast<int>(hipGetLastError());
}

// Prefetch depth of the OCC-2 plain GEMMs: DET_NT_PF (1..3), capped at the K tile count.  Default 3:
// GEMM-only 2-10 % faster than depth 1 on most ResNet 1x1 shapes (profiles/r4_conv1x1_pf_sweep.jsonl);
// neutral on the whole step, where the fused variants carry most calls (r4_nt_pf_ab.jsonl).
int g_nt_pf = -1;  // det_conv_nt_set_pf
// Short-K wide-N plain forwards (the bottleneck expansions, K = 128..512) on 128 x 64 tiles at three
// workgroups per CU instead of 128 x 128 at two: those GEMMs wait on each block's load latency (a
// 2-8 K-tile loop), and a third resident block hides more of it.  -1: DET_NT_WIDE decides (default off).
int g_nt_wide = -1;
bool nt_wide(const NtArgs& a) {
  if (g_nt_wide < 0) {
    const char* e = std::getenv("DET_NT_WIDE");
    g_nt_wide = e != nullptr && e[0] == '1' ? 1 : 0;
  }
  return g_nt_wide == 1 && a.K >= 128 && a.K <= 512 && a.N >= 4 * a.K && a.abits == nullptr && a.A2 == nullptr;
}
int nt_pf(int K) {
  static const int env_pf = [] {
    const char* e = std::getenv("DET_NT_PF");
    const int v = e ? std::atoi(e) : 3;
    return v < 1 ? 1 : (v > 3 ? 3 : v);
  }();
  const int pf = g_nt_pf > 0 ? g_nt_pf : env_pf;
  const int nk = K / kBK;
  return nk < pf ? nk : pf;
}

template <int BM, int BN>
int launch_nt_pf(hipStream_t st, const NtArgs& a, bool pro, bool stats, bool stride2, bool bt) {
  const bool fused = a.abits != nullptr || a.A2 != nullptr;
  int pf = fused ? 1 : nt_pf(a.K);
  if (bt && pf > 2) pf = 2;  // the transposed-B variant spills at 3
  switch (pf) {
    case 3: return launch_nt<BM, BN, 2, 2, 2, 3>(st, a, pro, stats, stride2, false, bt);
    case 2: return launch_nt<BM, BN, 2, 2, 2, 2>(st, a, pro, stats, stride2, false, bt);
    default: return launch_nt<BM, BN, 2, 2, 2, 1>(st, a, pro, stats, stride2, false, bt);
  }
}

}  // namespace

extern "C" {

// Prefetch depth of the plain GEMMs (1..3; 0 = back to DET_NT_PF / the default).  Returns the previous
// override.  For benchmarks and tests; not thread-safe against concurrent launches.
int det_conv_nt_set_wide(int on) {
  const int prev = g_nt_wide;
  g_nt_wide = on < 0 ? -1 : (on ? 1 : 0);
  return prev;
}

int det_conv_nt_set_pf(int pf) {
  const int old = g_nt_pf;
  g_nt_pf = pf <= 0 ? -1 : (pf > 3 ? 3 : pf);
  return old;
}

// Rows per statistics block of det_conv_nt for an N-column output (the BN finalize needs it).
int det_conv_nt_rows_per_block(int N) { return 128; }

// C[M,N] = op(A)[M,K] . B[N,K]^T.  bf16.  N % 64 == 0, K % 64 == 0, pointers 16-B aligned.
// scale/shift (nullable): prologue relu(A*scale+shift) per K channel.  pmean/pm2 (nullable):
// BN statistics partials [ceil(M/rpb), N].  Ho..Wi > 0 selects the 1x1 stride-2 row gather.
// res / aout / abits (all or none; with scale, shift): AFWD -- op(A) = relu(A*scale + shift + res),
// written to aout with its mask bits to abits by the first N tile (the consuming conv applies the
// producing BatchNorm; see the AFWD note at gemm_nt_kernel).  res_scale / res_shift (nullable): the
// residual is res * res_scale + res_shift (a deferred projection-shortcut BN apply).
int det_conv_nt(void* stream, const void* A, const void* B, void* C, int64_t M, int N, int K,
                const float* scale, const float* shift, float* pmean, float* pm2, int Ho, int Wo, int Hi, int Wi,
                const void* res, void* aout, void* abits, const float* res_scale, const float* res_shift) {
  if ((res_scale == nullptr) != (res_shift == nullptr) || (res_scale && !res)) return -2;
  if (M <= 0 || N % 64 != 0 || K % 64 != 0 || N <= 0 || K <= 0) return -1;
  if ((scale == nullptr) != (shift == nullptr) || (pmean == nullptr) != (pm2 == nullptr)) return -2;
  const bool stride2 = Ho > 0;
  if (stride2 && M != static_cast<int64_t>(M / (static_cast<int64_t>(Ho) * Wo)) * Ho * Wo) return -3;
  if ((res == nullptr) != (aout == nullptr) || (res == nullptr) != (abits == nullptr)) return -2;
  if (res && (!scale || stride2)) return -2;
  NtArgs a{static_cast<const unsigned short*>(A), static_cast<const unsigned short*>(B), static_cast<unsigned short*>(C),
           M, N, K, scale, shift, pmean, pm2, Gather{Ho, Wo, Hi, Wi}, BnBwdEpi{},
           static_cast<const unsigned short*>(res), nullptr, static_cast<unsigned short*>(aout),
           static_cast<uint8_t*>(abits), res_scale, res_shift};
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool pro = scale != nullptr && res == nullptr, stats = pmean != nullptr;
  if (K == kBK) {
    if (N % 128 == 0) return launch_nt<128, 128, 2, 2, kSingleOcc>(st, a, pro, stats, stride2);
    return launch_nt<128, 64, 2, 2, kSingleOcc>(st, a, pro, stats, stride2);
  }
  if (nt_wide(a)) return launch_nt<128, 64, 2, 2, 3, 2>(st, a, pro, stats, stride2);
  if (N % 128 == 0) return launch_nt_pf<128, 128>(st, a, pro, stats, stride2, false);
  return launch_nt_pf<128, 64>(st, a, pro, stats, stride2, false);
}

// Linear layer forward: Y[M, N] = X[M, K] . W[N, K]^T (+ bias[N]), bf16, N % 64 == 0, K % 64 == 0
// (a transformer's dense layers on the same MFMA tiles as the 1x1 convs).  Small grids (fewer than
// two 128 x 128 tiles per CU: BERT's M = 4608 token rows against N = 768) take 128 x 64 tiles.
int det_linear_fwd(void* stream, const void* X, const void* W, const void* bias, void* Y, int64_t M, int N, int K) {
  if (M <= 0 || N % 64 != 0 || K % 64 != 0 || N <= 0 || K <= 0) return -1;
  NtArgs a{static_cast<const unsigned short*>(X), static_cast<const unsigned short*>(W), static_cast<unsigned short*>(Y),
           M, N, K, nullptr, nullptr, nullptr, nullptr, Gather{}, BnBwdEpi{}, nullptr, nullptr, nullptr, nullptr,
           nullptr, nullptr, static_cast<const unsigned short*>(bias)};
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t tiles128 = ((M + 127) / 128) * (N / 128);
  if (K == kBK) {
    if (N % 128 == 0 && tiles128 >= 512) return launch_nt<128, 128, 2, 2, kSingleOcc>(st, a, false, false, false);
    return launch_nt<128, 64, 2, 2, kSingleOcc>(st, a, false, false, false);
  }
  if (N % 128 == 0 && tiles128 >= 512) return launch_nt_pf<128, 128>(st, a, false, false, false, false);
  return launch_nt_pf<128, 64>(st, a, false, false, false, false);
}

// dX[M, N] = dY[M, K] . W[K, N]: the input gradient of a 1x1 conv against its weight W = [Cout, Cin]
// as stored (no transposed copy).  bf16, N % 64 == 0, K % 64 == 0.
// abn_x (nullable): with abn_coef [3][K] and abn_out, dY is the BN backward's apply of A = dY (the
// BN's masked gradient) and abn_x (the BN input), computed in the A staging and written to abn_out.
int det_conv_dgrad(void* stream, const void* dY, const void* W, void* dX, int64_t M, int N, int K, const void* abn_x,
                   const float* abn_coef, void* abn_out) {
  if (M <= 0 || N % 64 != 0 || K % 64 != 0 || N <= 0 || K <= 0) return -1;
  if (abn_x && (!abn_coef || !abn_out)) return -2;
  NtArgs a{static_cast<const unsigned short*>(dY), static_cast<const unsigned short*>(W), static_cast<unsigned short*>(dX),
           M, N, K, nullptr, nullptr, nullptr, nullptr, Gather{}, BnBwdEpi{},
           static_cast<const unsigned short*>(abn_x), abn_coef, static_cast<unsigned short*>(abn_out)};
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (K == kBK) {
    if (N % 128 == 0) return launch_nt<128, 128, 2, 2, kSingleOcc>(st, a, false, false, false, false, true);
    return launch_nt<128, 64, 2, 2, kSingleOcc>(st, a, false, false, false, false, true);
  }
  if (N % 128 == 0) return launch_nt_pf<128, 128>(st, a, false, false, false, true);
  return launch_nt_pf<128, 64>(st, a, false, false, false, true);
}

// dX[M, N] = dY[M, K] . W^T[N, K]^T with the BN-backward epilogue (BnBwdEpi above): writes
// d = mask * (dX [+ add]) and the BN's backward partials psum / psumx [ceil(M/128), N].
// mode 1: x, mean, scale, shift; mode 2: x, mean, mbits (add nullable).
// b_kn: B is the untransposed weight [K, N] (the gemm reads it with transposed LDS reads).
int det_conv_nt_bnbwd(void* stream, const void* A, const void* B, void* C, int64_t M, int N, int K, const void* x,
                      const float* mean, const float* scale, const float* shift, const void* mbits, const void* add,
                      float* psum, float* psumx, int mode, int b_kn, const void* abn_x, const float* abn_coef,
                      void* abn_out, int add_ho, int add_wo, int add_hi, int add_wi) {
  if (M <= 0 || N % 64 != 0 || K % 64 != 0 || N <= 0 || K <= 0) return -1;
  if (add_hi > 0 && (add_wi <= 0 || add_ho != (add_hi + 1) / 2 || add_wo != (add_wi + 1) / 2 ||
                     M % (static_cast<int64_t>(add_hi) * add_wi) != 0 || M >= (static_cast<int64_t>(1) << 32)))
    return -3;
  if (!x || !mean || !psum || !psumx || (mode == 1 && (!scale || !shift)) || (mode == 2 && !mbits) || mode < 1 || mode > 2)
    return -2;
  NtArgs a{static_cast<const unsigned short*>(A), static_cast<const unsigned short*>(B), static_cast<unsigned short*>(C),
           M, N, K, nullptr, nullptr, nullptr, nullptr, Gather{}, BnBwdEpi{static_cast<const unsigned short*>(x), mean, scale,
           shift, static_cast<const uint8_t*>(mbits), static_cast<const unsigned short*>(add), psum, psumx, mode,
           add_ho, add_wo, add_hi > 0 ? add_hi : 0, add_wi},
           static_cast<const unsigned short*>(abn_x), abn_coef, static_cast<unsigned short*>(abn_out)};
  if (abn_x && (!abn_coef || !abn_out)) return -2;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool bt = b_kn != 0;
  // K == 64 (one K tile): the occupancy-3 single-buffer variant, or (DET_BNB_SINGLE_OCC=0) the
  // occupancy-2 one, whose BN-backward epilogue loads are issued before the K loop (EPRE)
  static const bool single = [] {
    const char* e = std::getenv("DET_BNB_SINGLE_OCC");
    return !(e && e[0] == '0');
  }();
  if (K == kBK && (single || abn_x)) {
    if (N % 128 == 0) return launch_nt<128, 128, 2, 2, kSingleOcc>(st, a, false, false, false, true, bt);
    return launch_nt<128, 64, 2, 2, kSingleOcc>(st, a, false, false, false, true, bt);
  }
  // BN-backward GEMMs with a K loop of >= 4 tiles (layer 3/4 input gradients): DET_BNB_PF register
  // sets of prefetch (the epilogue operand loads then wait for the loop's end instead of holding
  // their registers through it)
  static const int bnb_pf = [] {
    const char* e = std::getenv("DET_BNB_PF");
    const int v = e ? std::atoi(e) : 1;
    return v < 1 ? 1 : (v > 2 ? 2 : v);
  }();
  if (bnb_pf == 2 && K >= 4 * kBK && !abn_x) {
    if (N % 128 == 0) return launch_nt<128, 128, 2, 2, 2, 2>(st, a, false, false, false, true, bt);
    return launch_nt<128, 64, 2, 2, 2, 2>(st, a, false, false, false, true, bt);
  }
  if (N % 128 == 0) return launch_nt<128, 128, 2, 2, 2>(st, a, false, false, false, true, bt);
  return launch_nt<128, 64, 2, 2, 2>(st, a, false, false, false, true, bt);
}

// fp32 workspace elements det_conv_tn needs (slabs) for an [N, K] output from M rows.
int64_t det_conv_tn_ws_elems(int64_t M, int N, int K) {
  const int bn = N % 128 == 0 ? 128 : 64, bk = K % 128 == 0 ? 128 : 64;
  const int64_t tiles = static_cast<int64_t>(N / bn) * (K / bk);
  int64_t splits = (512 + tiles - 1) / tiles;    // ~2 workgroups per CU
  const int64_t max_rows = (M + 1023) / 1024;    // >= 1024 rows per split
  // fp32 slab traffic (write + reduce read) at most ~1/4 of the operand bytes the GEMM streams
  const int64_t max_bytes = (M * (N + K) * 2) / (4 * 4 * static_cast<int64_t>(N) * K * 2);
  if (splits > max_rows) splits = max_rows;
  if (splits > max_bytes) splits = max_bytes;
  if (splits < 1) splits = 1;
  return splits * N * K;
}

// dW[N,K] (out_dtype 0 fp32 / 1 bf16) = scale * dY[M,N]^T . op(X)[M,K], via fp32 split-M slabs
// in ws (>= det_conv_tn_ws_elems) reduced by a second launch.
int det_conv_tn(void* stream, const void* dY, const void* X, void* out, int out_dtype, int64_t M, int N, int K,
                const float* scale_x, const float* shift_x, float* ws, float out_scale, int Ho, int Wo, int Hi,
                int Wi) {
  if (M <= 0 || N % 64 != 0 || K % 64 != 0) return -1;
  if ((scale_x == nullptr) != (shift_x == nullptr)) return -2;
  const int bn = N % 128 == 0 ? 128 : 64, bk = K % 128 == 0 ? 128 : 64;
  const int64_t slab = static_cast<int64_t>(N) * K;
  const int splits = static_cast<int>(det_conv_tn_ws_elems(M, N, K) / slab);
  int64_t rps = (M + splits - 1) / splits;
  rps = (rps + 63) / 64 * 64;
  TnArgs a{static_cast<const unsigned short*>(dY), static_cast<const unsigned short*>(X), ws, M, N, K, rps,
           scale_x, shift_x, Gather{Ho, Wo, Hi, Wi}};
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool pro = scale_x != nullptr, stride2 = Ho > 0;
  int rc;
  if (bn == 128 && bk == 128) rc = launch_tn<128, 128>(st, a, splits, pro, stride2);
  else if (bn == 128) rc = launch_tn<128, 64>(st, a, splits, pro, stride2);
  else if (bk == 128) rc = launch_tn<64, 128>(st, a, splits, pro, stride2);
  else rc = launch_tn<64, 64>(st, a, splits, pro, stride2);
  if (rc != 0) return rc;
  launch_slab_reduce(st, ws, splits, slab, out_scale, out, out_dtype);
  return static_cast<int>(hipGetLastError());
}

// Weight gradient of an R x S convolution (stride, pad) over NHWC bf16:
//   dW[N, R*S*Cin] (KRSC; out_dtype 0 fp32 / 1 bf16) = out_scale * dY[M, N]^T . im2col(X)[M, R*S*Cin]
// as split-M fp32 slabs in ws (>= det_conv_tn_ws_elems(M, N, R*S*Cin)) reduced by a second launch.
// Cin % 64 == 0, N % 64 == 0.
int det_conv_wgrad(void* stream, const void* dY, const void* X, void* out, int out_dtype, int64_t M, int N, int Cin,
                   int Hi, int Wi, int Ho, int Wo, int R, int S, int stride, int pad, float* ws, float out_scale) {
  if (M <= 0 || N % 64 != 0 || Cin % 64 != 0 || R <= 0 || S <= 0) return -1;
  if (M % (static_cast<int64_t>(Ho) * Wo) != 0 || M >= (static_cast<int64_t>(1) << 31)) return -3;
  if (Ho != (Hi + 2 * pad - R) / stride + 1 || Wo != (Wi + 2 * pad - S) / stride + 1) return -3;
  const int K = R * S * Cin;
  const int bn = N % 128 == 0 ? 128 : 64, bk = Cin % 128 == 0 ? 128 : 64;
  const int64_t slab = static_cast<int64_t>(N) * K;
  const int splits = static_cast<int>(det_conv_tn_ws_elems(M, N, K) / slab);
  int64_t rps = (M + splits - 1) / splits;
  rps = (rps + 63) / 64 * 64;
  Gather g{Ho, Wo, Hi, Wi, Cin, S, stride, pad};
  TnArgs a{static_cast<const unsigned short*>(dY), static_cast<const unsigned short*>(X), ws, M, N, K, rps, nullptr,
           nullptr, g};
  hipStream_t st = static_cast<hipStream_t>(stream);
  int rc;
  if (bn == 128 && bk == 128) rc = launch_tn<128, 128>(st, a, splits, false, false, true);
  else if (bn == 128) rc = launch_tn<128, 64>(st, a, splits, false, false, true);
  else if (bk == 128) rc = launch_tn<64, 128>(st, a, splits, false, false, true);
  else rc = launch_tn<64, 64>(st, a, splits, false, false, true);
  if (rc != 0) return rc;
  launch_slab_reduce(st, ws, splits, slab, out_scale, out, out_dtype);
  return static_cast<int>(hipGetLastError());
}

// ResNet stem convolution (7x7, stride 2, pad 3, 64 filters) as an implicit GEMM on the MFMA tiles
// above: Y[M, 64] = im2col(X)[M, 256] . W[64, 256]^T, X NHWC bf16 with channels padded to 4, W in
// the k = r*32 + s*4 + c layout with zero taps/channel (ops/conv.py pack_stem_weight).  pmean/pm2
// (nullable): BN statistics partials of Y, consumed by the stem BatchNorm (no stats pass).
int det_stem_conv_fwd(void* stream, const void* X, const void* W, void* Y, int64_t M, int Hi, int Wi, int Ho, int Wo,
                      float* pmean, float* pm2) {
  if (M <= 0 || Ho <= 0 || Wo <= 0 || M % (static_cast<int64_t>(Ho) * Wo) != 0) return -1;
  if (Ho != (Hi + 6 - 7) / 2 + 1 || Wo != (Wi + 6 - 7) / 2 + 1) return -3;
  if ((pmean == nullptr) != (pm2 == nullptr)) return -2;
  NtArgs a{static_cast<const unsigned short*>(X), static_cast<const unsigned short*>(W), static_cast<unsigned short*>(Y),
           M, 64, 256, nullptr, nullptr, pmean, pm2, Gather{Ho, Wo, Hi, Wi}};
  const int64_t nwg = (M + 127) / 128;
  if (nwg >= (static_cast<int64_t>(1) << 31)) return -4;
  constexpr int smem = nt_smem<128, 64, 2>();  // double-buffered: 4 K tiles
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>(nwg));
  if (pmean) hipLaunchKernelGGL((gemm_nt_kernel<128, 64, 2, 2, false, true, kGmStem, 2>), grid, dim3(kThreads), smem, st, a);
  else hipLaunchKernelGGL((gemm_nt_kernel<128, 64, 2, 2, false, false, kGmStem, 2>), grid, dim3(kThreads), smem, st, a);
  return static_cast<int>(hipGetLastError());
}

// fp32 workspace elements det_stem_conv_wgrad needs: 512 split-M slabs of [64, 256] (2 workgroups
// per CU over 256 CUs), fewer for small M (>= 1024 rows per split).
int64_t det_stem_conv_wgrad_ws_elems(int64_t M) {
  int64_t splits = (M + 1023) / 1024;
  if (splits > 512) splits = 512;
  if (splits < 1) splits = 1;
  return splits * 64 * 256;
}

// Stem weight gradient dW[64, 256] (out_dtype 0 fp32 / 1 bf16) = out_scale * dY[M, 64]^T . im2col(X),
// split-M fp32 slabs in ws (>= det_stem_conv_wgrad_ws_elems(M)) reduced by a second launch.
int det_stem_conv_wgrad(void* stream, const void* dY, const void* X, void* out, int out_dtype, int64_t M, int Hi,
                        int Wi, int Ho, int Wo, float* ws, float out_scale) {
  if (M <= 0 || Ho <= 0 || Wo <= 0 || M % (static_cast<int64_t>(Ho) * Wo) != 0) return -1;
  if (Ho != (Hi + 6 - 7) / 2 + 1 || Wo != (Wi + 6 - 7) / 2 + 1) return -3;
  constexpr int N = 64, K = 256;
  const int64_t slab = static_cast<int64_t>(N) * K;
  const int splits = static_cast<int>(det_stem_conv_wgrad_ws_elems(M) / slab);
  int64_t rps = (M + splits - 1) / splits;
  rps = (rps + 63) / 64 * 64;
  TnArgs a{static_cast<const unsigned short*>(dY), static_cast<const unsigned short*>(X), ws, M, N, K, rps,
           nullptr, nullptr, Gather{Ho, Wo, Hi, Wi}};
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int nwg = splits;  // one 64 x 256 output tile: every dY row is read once
  constexpr int smem = 2 * 64 * (64 + 2 * 128) * 2;
  hipLaunchKernelGGL((gemm_tn_kernel<64, 128, false, kGmStem, 2>), dim3(nwg), dim3(kThreads), smem, st, a);
  launch_slab_reduce(st, ws, splits, slab, out_scale, out, out_dtype);
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
