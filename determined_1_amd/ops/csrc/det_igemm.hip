// det_igemm.hip — pipelined implicit-GEMM convolution for NHWC bf16 activations on CDNA4 MFMA.
//
//   Y[M, N] = sum_{tap (r,s), c} X[n, ho*st - pad + r, wo*st - pad + s, c] . W[N][r][s][c]
//   (M = Nb*Ho*Wo output pixels, N = output channels, K = R*S*Cin, W in KRSC = torch channels_last
//   weight order, so the B operand is the weight tensor as it sits in memory)
//
// One kernel covers every ResNet conv whose input channel count is a multiple of 64: 1x1 stride 1/2,
// 3x3 stride 1/2 pad 1, and the stride-1 input gradients (dgrad of a 1x1 is this GEMM against W^T;
// dgrad of a 3x3/pad-1 is a 3x3/pad-1 conv of dY against the spatially flipped, transposed weight).
//
// Why a new kernel: the register-staged det_conv GEMM and the library convs both run ResNet-50's
// convolutions at ~19 % of the bf16 MFMA peak (profiles/r2_resnet50_bs512_fin2_steady.csv): with
// one K tile of prefetch in registers, HBM/L2 latency (~1-2 us under load) is not covered by the
// ~0.2 us of MFMA work per K step.  Here (cdna_hip_programming.md §5):
//   * operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4): no staging VGPRs, no
//     ds_write pass; the per-lane SOURCE address does the im2col gather (a 16-B chunk per lane,
//     zero-padding and the M tail read a zero page), so the LDS image stays lane-linear and the
//     XOR swizzle (chunk ^ row&7, conflict-free ds_read_b128 fragments) is applied on the source;
//   * a 3-stage LDS ring with a COUNTED vmcnt: two K tiles are in flight while the MFMAs consume
//     the third, and the barrier is a raw s_barrier (a __syncthreads() would drain the DMA queue);
//   * 256 x BN block tile, 8 waves (2 per SIMD), 64x64 (or 32x64) wave tiles of
//     v_mfma_f32_16x16x32_bf16, one workgroup per CU (3 x 48 KiB ring);
//   * epilogue: bf16 tile through LDS -> coalesced 16-B row stores, optional BatchNorm statistics
//     of the bf16-rounded output per (256-row block, channel) for the consuming BN (det_norm.hip
//     det_bn_fwd_from_partials);
//   * XCD-aware bijective block remap (blocks sharing an A row-panel on one XCD's L2).
//
// Measured (profiles/r2_igemm_microbench.jsonl, ResNet-50 bs512 forward shapes on MI355X): ~590 TF/s
// on every 3x3 (118 GFLOP each), 130-720 TF/s on the 1x1s.  That beats the register-staged det_conv
// GEMM on the K >= 256 1x1 shapes by 5-20 % but not MIOpen's 3x3 forward (700-880 TF/s), so the
// ResNet model does not route through it yet; the next step is the 2-phase-per-K-step interleave
// (ds_read || glds || MFMA) that the one-barrier-per-K-step loop here lacks.
//
// Reference parity: convolutions belong to the user's model in the reference (cuDNN through torch,
// examples/computer_vision/*); semantics are torch.nn.functional.conv2d's.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <type_traits>

#include "det_stats.h"

namespace {

constexpr int kBK = 64;       // K tile: one 128-B LDS row per operand row
constexpr int kStages = 3;    // LDS ring depth

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) unsigned short us8;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ float bf2f(unsigned short u) { return __uint_as_float(static_cast<uint32_t>(u) << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));
}
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

__device__ __forceinline__ int swz(int row, int ch) { return row * 128 + ((ch ^ (row & 7)) << 4); }

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

struct IgArgs {
  const unsigned short* X;     // NHWC [Nb, Hi, Wi, Cin] (DENSE: [M, K] rows)
  const unsigned short* W;     // [N, K], K = R*S*Cin (KRSC)
  unsigned short* Y;           // [M, N]
  const unsigned short* zero;  // >= 128 zero bytes, 16-B aligned
  float* pmean;                // STATS: [ceil(M/BM), N]
  float* pm2;
  int64_t M;
  int N, K, Cin;
  int Hi, Wi, Ho, Wo, stride, pad, S;
  int R;
  int64_t x_bytes;  // X extent for the buffer resource (v2 fetch; < 2^31)
  // BNB (input gradient feeding a training BatchNorm+ReLU backward, mask recomputed from the BN
  // input): Y <- d = (bn_x * bn_scale + bn_shift > 0) ? dX : 0, and the BN's backward partials
  // psum = sum d, psumx = sum d (bn_x - bn_mean) per (BM-row block, column)
  const unsigned short* bn_x;
  const float* bn_mean;
  const float* bn_scale;
  const float* bn_shift;
  float* psum;
  float* psumx;
  // Input gradient of a stride-2 3x3/pad-1 conv as four parity-class convs (igemm3 only; see
  // det_igemm_dgrad_s2): kb_stride = the B row stride (0: K), tapmap = 4-bit B tap per class tap
  // (0: identity), oscat = 1 + 2*ph + pw scatters output row (q = n*Ho + i, j) to the full-resolution
  // row (2q + ph) * 2Wo + 2j + pw, mt_base = first statistics block row of this class.
  int kb_stride;
  unsigned tapmap;
  int oscat;
  int mt_base;
  // conv3p prologue: the input operand is relu(X * pro_scale[c] + pro_shift[c]) (padding stays 0)
  const float* pro_scale;
  const float* pro_shift;
  // 1: the BN-statistics epilogue runs before the C stores (the round-3 order, DET_STATS_FIRST=1 A/B);
  // 0: after them, so the stores drain while the statistics are reduced
  int stats_first;
};

// DET_STATS_FIRST (read once): the statistics-epilogue order of every GEMM with STATS
inline int stats_first_flag() {
  static const int v = [] {
    const char* e = std::getenv("DET_STATS_FIRST");
    return e != nullptr && e[0] == '1' ? 1 : 0;
  }();
  return v;
}

// the row of Y (and of the BN input in the BNB epilogue) that GEMM row m writes
__device__ __forceinline__ int64_t out_row(const IgArgs& a, int64_t m) {
  if (a.oscat == 0) return m;
  const int cls = a.oscat - 1, ph = cls >> 1, pw = cls & 1;
  const int64_t q = m / a.Wo;
  const int j = static_cast<int>(m - q * a.Wo);
  return (2 * q + ph) * (2 * static_cast<int64_t>(a.Wo)) + 2 * j + pw;
}

// BN-backward epilogue of a BM x BN output tile held as bf16 in LDS (ct, row stride LDC): each
// thread owns one 8-column chunk over rows tid/CPR + q*NT/CPR, writes the masked gradient and
// accumulates the two sums of exactly what it wrote; the per-thread sums then overlay the C tile
// ([NT][16] floats) and the NT/CPR threads of a column are added in a fixed order.
template <int BM, int BN, int NT>
__device__ __forceinline__ void bnb_epilogue(const IgArgs& a, unsigned char* smem, const unsigned short* ct, int LDC,
                                             int64_t m0, int n0, int mt, int nvalid, int tid) {
  constexpr int CPR = BN / 8;
  static_assert(NT % CPR == 0, "fixed chunk column per thread");
  const int cc = tid % CPR;
  const int c0 = n0 + cc * 8;
  float mu[8], sc[8], sh[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = a.bn_mean[c0 + j];
    sc[j] = a.bn_scale[c0 + j];
    sh[j] = a.bn_shift[c0 + j];
    s1[j] = 0.f;
    s2[j] = 0.f;
  }
  // every BN-input load of this thread is issued before the first store (the stores could alias
  // the loads as far as the compiler knows, which would serialise each row on the HBM latency)
  constexpr int NQ = BM * CPR / NT;
  us8 xs[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int row = (tid + q * NT) / CPR;
    xs[q] = row < nvalid ? *reinterpret_cast<const us8*>(a.bn_x + out_row(a, m0 + row) * a.N + c0) : us8{0, 0, 0, 0, 0, 0, 0, 0};
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int row = (tid + q * NT) / CPR;
    if (row >= nvalid) continue;
    const int64_t off = out_row(a, m0 + row) * a.N + c0;
    const us8 cv = *reinterpret_cast<const us8*>(ct + row * LDC + cc * 8);
    const us8 xv = xs[q];
    us8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xf = bf2f(xv[j]);
      const float d = __fmaf_rn(xf, sc[j], sh[j]) > 0.f ? bf2f(cv[j]) : 0.f;
      o[j] = f2bf(d);
      const float dr = bf2f(o[j]);  // the sums see exactly what the BN apply reads back
      s1[j] += dr;
      s2[j] += dr * (xf - mu[j]);
    }
    *reinterpret_cast<us8*>(a.Y + off) = o;
  }
  float* scratch = reinterpret_cast<float*>(smem);  // overlays the consumed C tile
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
    for (int g = 0; g < NT / CPR; ++g) {
      t1 += scratch[(g * CPR + ccol) * 16 + j];
      t2 += scratch[(g * CPR + ccol) * 16 + 8 + j];
    }
    a.psum[static_cast<int64_t>(a.mt_base + mt) * a.N + n0 + tid] = t1;
    a.psumx[static_cast<int64_t>(a.mt_base + mt) * a.N + n0 + tid] = t2;
  }
}

__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void*)(const_cast<void*>(g)), (lds_void*)(lds_wave_base), 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void block_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// DENSE: A rows are X rows (1x1 stride-1 conv / plain GEMM).  Otherwise the conv gather.
// WM x WN waves of 64 lanes; each wave owns a (BM/WM) x (BN/WN) accumulator tile.
template <int BM, int BN, int WM, int WN, bool DENSE, bool STATS>
__global__ void __launch_bounds__(WM * WN * 64, 1) igemm_kernel(IgArgs a) {
  constexpr int NW = WM * WN, kThreads = NW * 64;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int AI = BM / (8 * NW), BI = BN / (8 * NW);  // glds instructions per lane per K tile
  static_assert(AI * 8 * NW == BM && BI * 8 * NW == BN, "tile rows split evenly over the waves");
  constexpr int NI = AI + BI;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int LDC = BN + 16;
  constexpr int RED_OFF = kStages * STAGE;  // stats scratch after the ring (one LDS array: no 2nd __shared__)
  static_assert(BM * LDC * 2 <= kStages * STAGE, "C tile fits in the ring");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* red = reinterpret_cast<float*>(smem + RED_OFF);  // [WM][BN]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = a.N / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntn, nt = bid - mt * ntn;
  const int64_t m0 = static_cast<int64_t>(mt) * BM;
  const int n0 = nt * BN;
  const int64_t K = a.K;

  // lane -> (row within an 8-row glds group, swizzled source chunk): LDS slot (row, lane&7) holds
  // source chunk (lane&7) ^ (row&7) with row&7 == lane>>3
  const int lrow = lane >> 3;
  const int gch = (lane & 7) ^ lrow;

  // per-lane A row descriptors for its AI rows
  int64_t arow[AI];  // DENSE: element offset of the row start; else pixel base (n*Hi*Wi) or -1
  int ahi[AI], awi[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = (i * NW + wid) * 8 + lrow;
    const int64_t m = m0 + row;
    if (DENSE) {
      arow[i] = m < a.M ? m * K : -1;
      ahi[i] = awi[i] = 0;
    } else if (m < a.M) {
      const int64_t hw = static_cast<int64_t>(a.Ho) * a.Wo;
      const int64_t n = m / hw;
      const int rem = static_cast<int>(m - n * hw);
      const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
      arow[i] = n * a.Hi;
      ahi[i] = ho * a.stride - a.pad;
      awi[i] = wo * a.stride - a.pad;
    } else {
      arow[i] = -1;
      ahi[i] = awi[i] = 0;
    }
  }
  const unsigned short* bbase = a.W + static_cast<int64_t>(n0) * K + gch * 8;
  const unsigned short* zsrc = a.zero;

  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % kStages) * STAGE;
    const int k0 = kt * kBK;
    if (DENSE) {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const unsigned short* src = arow[i] >= 0 ? a.X + arow[i] + k0 + gch * 8 : zsrc;
        glds16(src, st + ((i * NW + wid) * 8) * 128);
      }
    } else {
      const int tap = k0 / a.Cin, c0 = k0 - tap * a.Cin;
      const int r = tap / a.S, s = tap - r * a.S;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const int hi = ahi[i] + r, wi = awi[i] + s;
        const bool ok = arow[i] >= 0 && hi >= 0 && hi < a.Hi && wi >= 0 && wi < a.Wi;
        const unsigned short* src =
            ok ? a.X + ((arow[i] + hi) * a.Wi + wi) * static_cast<int64_t>(a.Cin) + c0 + gch * 8 : zsrc;
        glds16(src, st + ((i * NW + wid) * 8) * 128);
      }
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int row = (j * NW + wid) * 8 + lrow;
      glds16(bbase + static_cast<int64_t>(row) * K + k0, st + A_BYTES + ((j * NW + wid) * 8) * 128);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.K / kBK;
  issue(0);
  if (nk > 1) issue(1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) wait_vmcnt<NI>();  // tile kt landed (this wave's DMAs); kt+1 may stay in flight
    else wait_vmcnt<0>();
    block_barrier();  // every wave's tile-kt DMAs landed; every wave is done reading tile kt-1
    if (kt + 2 < nk) issue(kt + 2);  // into tile kt-1's buffer
    const unsigned char* base = smem + (kt % kStages) * STAGE;
    // both 32-deep k halves' fragments are read up front (two register sets): the second half's
    // ds_reads are in flight under the first half's MFMAs
    bf16x8 af[2][FM], bfr[2][FN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[ks][i] = *reinterpret_cast<const bf16x8*>(base + swz(wm * TM + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[ks][j] = *reinterpret_cast<const bf16x8*>(base + A_BYTES + swz(wn * TN + j * 16 + (lane & 15), ch));
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
  }
  __syncthreads();  // all fragment reads done before the ring is reused for the C tile

  // ---- epilogue: bf16 tile through LDS (coalesced 16-B row stores) + BN statistics ----
  unsigned short* ct = reinterpret_cast<unsigned short*>(smem);
  const int64_t rows_left = a.M - m0;
  const int nvalid = rows_left < BM ? static_cast<int>(rows_left) : BM;
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
  if (STATS && a.stats_first)
    det_block_bn_stats<FM, FN, WM, TM, TN, BN>(acc, red, wm, wn, lane, tid, nvalid, a.pmean, a.pm2,
                                                static_cast<int64_t>(mt) * a.N + n0);
  __syncthreads();
  constexpr int CPR = BN / 8;
#pragma unroll
  for (int q = 0; q < BM * CPR / kThreads; ++q) {
    const int idx = tid + q * kThreads;
    const int row = idx / CPR, cc = idx - row * CPR;
    if (row < nvalid)
      *reinterpret_cast<us8*>(a.Y + (m0 + row) * a.N + n0 + cc * 8) = *reinterpret_cast<const us8*>(ct + row * LDC + cc * 8);
  }
  // BN statistics after the stores are issued (red is its own LDS region): they drain meanwhile
  if (STATS && !a.stats_first)
    det_block_bn_stats<FM, FN, WM, TM, TN, BN>(acc, red, wm, wn, lane, tid, nvalid, a.pmean, a.pm2,
                                                static_cast<int64_t>(mt) * a.N + n0);
}

// ------------------------------------------------------------------------------------------------
// v2: the same LDS-DMA ring, with the fragment reads software-pipelined against the MFMAs.
//
// v1 issues all of a K tile's 16 fragment reads and then all 32 MFMAs, and every wave of the block
// meets at one barrier per K tile, so the whole CU alternates between an LDS-read phase (matrix pipe
// idle) and an MFMA phase (LDS idle).  v2 keeps two fragment register sets, one per 32-deep k half:
//
//   read F1 = half 1 of tile kt      || MFMAs on F0 (half 0 of tile kt, read last iteration)
//   wait tile kt+1 (counted vmcnt), barrier, issue tile kt+NS-1 into the buffer tile kt-1 vacated
//   read F0 = half 0 of tile kt+1    || MFMAs on F1
//
// so every ds_read burst has an independent MFMA cluster beside it (s_setprio(1) around the
// clusters, cdna_hip_programming.md T5).  WAR on the ring: tile kt-1's fragments were all consumed
// by MFMAs issued before this iteration's barrier, so every wave is past its reads of that buffer.
// RAW: each wave's vmcnt retires its own DMAs of tile kt+1 and the barrier publishes all waves'.
// ------------------------------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, int NS, bool DENSE, bool STATS, int OCC, bool BNB = false>
__global__ void __launch_bounds__(WM * WN * 64, OCC) igemm2_kernel(IgArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)  // buffer-resource builtins exist only in the device pass
  constexpr int NW = WM * WN, kThreads = NW * 64;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int AI = BM / (8 * NW), BI = BN / (8 * NW);
  static_assert(AI * 8 * NW == BM && BI * 8 * NW == BN, "tile rows split evenly over the waves");
  static_assert(NS >= 3, "the prefetch distance needs >= 3 ring stages");
  constexpr int NI = AI + BI;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int LDC = BN + 16;
  static_assert(BM * LDC * 2 + 12 * WM * BN <= NS * STAGE, "C tile + stats scratch fit in the ring");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* red = reinterpret_cast<float*>(smem + BM * LDC * 2);  // [WM][BN], after the C tile

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = a.N / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntn, nt = bid - mt * ntn;
  const int64_t m0 = static_cast<int64_t>(mt) * BM;
  const int n0 = nt * BN;
  const int64_t K = a.K;
  const int lrow = lane >> 3;
  const int gch = (lane & 7) ^ lrow;

  // Operand fetch through buffer_load ... lds (raw buffer resources, 32-bit offsets): per A row the
  // byte offset of its top-left input pixel (may be negative: padding) and a bitmask of the R*S
  // taps that land inside the image; per K tile the tap offset is a wave-uniform scalar, so each
  // A fetch costs an add, a bit test and a select, and an invalid tap or a row past M fetches at
  // an out-of-range offset, which the buffer unit returns as zeros (no zero page, no branches).
  // B offsets are fixed per lane; the K advance rides in the scalar soffset.
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(a.X), 0, static_cast<int>(a.x_bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(a.W), 0, static_cast<int>(static_cast<int64_t>(a.N) * K * 2), 0x00020000);
  constexpr unsigned kOOB = 0xFFFFFFF0u;
  int aoff[AI];
  unsigned amask[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = (i * NW + wid) * 8 + lrow;
    const int64_t m = m0 + row;
    aoff[i] = 0;
    amask[i] = 0;
    if (m < a.M) {
      const int64_t hw = static_cast<int64_t>(a.Ho) * a.Wo;
      const int64_t n = m / hw;
      const int rem = static_cast<int>(m - n * hw);
      const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
      const int hi0 = ho * a.stride - a.pad, wi0 = wo * a.stride - a.pad;
      aoff[i] = static_cast<int>(((n * a.Hi + hi0) * a.Wi + wi0) * a.Cin * 2 + gch * 16);
      for (int r = 0; r < a.R; ++r)
        for (int s2 = 0; s2 < a.S; ++s2) {
          const int hi = hi0 + r, wi = wi0 + s2;
          if (hi >= 0 && hi < a.Hi && wi >= 0 && wi < a.Wi) amask[i] |= 1u << (r * a.S + s2);
        }
    }
  }
  unsigned boff[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j)
    boff[j] = static_cast<unsigned>(((static_cast<int64_t>(n0) + (j * NW + wid) * 8 + lrow) * K + gch * 8) * 2);

  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % NS) * STAGE;
    const int k0 = kt * kBK;
    const int tap = k0 / a.Cin, c0 = k0 - tap * a.Cin;
    const int r = tap / a.S, s2 = tap - r * a.S;
    const int toff = ((r * a.Wi + s2) * a.Cin + c0) * 2;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const unsigned v = ((amask[i] >> tap) & 1u) ? static_cast<unsigned>(aoff[i] + toff) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(st + ((i * NW + wid) * 8) * 128), 16, v, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < BI; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void*)(st + A_BYTES + ((j * NW + wid) * 8) * 128), 16, boff[j],
                                               k0 * 2, 0, 0);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 a0[FM], b0[FN], a1[FM], b1[FN];
  auto read_half = [&](const unsigned char* base, int ks, bf16x8* af, bf16x8* bfr) {
    const int ch = ks * 4 + (lane >> 4);
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(base + swz(wm * TM + i * 16 + (lane & 15), ch));
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(base + A_BYTES + swz(wn * TN + j * 16 + (lane & 15), ch));
  };
  auto mfma_half = [&](const bf16x8* af, const bf16x8* bfr) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = a.K / kBK;
  // prologue: NS-1 tiles in flight, wait for tile 0
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(t);
  if (nk >= NS - 1) wait_vmcnt<NI * (NS - 2)>();
  else wait_vmcnt<0>();
  block_barrier();
  read_half(smem, 0, a0, b0);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // loop entry with nothing pending on lgkm (see the loop tail)
  // every iteration but the last, with no data-dependent join between a read burst and the MFMA
  // cluster that consumes the burst before it (a join makes the waitcnt pass fall back to lgkmcnt(0))
  for (int kt = 0; kt + 1 < nk; ++kt) {
    read_half(smem + (kt % NS) * STAGE, 1, a1, b1);
    mfma_half(a0, b0);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // F1 landed under the F0 cluster: nothing pending past here
    // tiles issued so far: 0 .. min(nk-1, kt+NS-2); tile kt+1 must land, the younger may fly
    if (kt + NS - 2 < nk) wait_vmcnt<NI * (NS - 3)>();
    else wait_vmcnt<0>();
    block_barrier();
    if (kt + NS - 1 < nk) issue(kt + NS - 1);
    read_half(smem + ((kt + 1) % NS) * STAGE, 0, a0, b0);
    mfma_half(a1, b1);
    // retire F0's reads (they ran under the F1 cluster) with a real S_WAITCNT the waitcnt pass sees:
    // otherwise it merges the back edge conservatively and puts lgkmcnt(0) AFTER the next F1 reads,
    // i.e. in front of the F0 MFMAs, serialising every read burst with its cluster
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt/expcnt untouched
  }
  read_half(smem + ((nk - 1) % NS) * STAGE, 1, a1, b1);
  mfma_half(a0, b0);
  mfma_half(a1, b1);
  __syncthreads();  // every wave's last fragment reads are done before the ring holds the C tile

  unsigned short* ct = reinterpret_cast<unsigned short*>(smem);
  const int64_t rows_left = a.M - m0;
  const int nvalid = rows_left < BM ? static_cast<int>(rows_left) : BM;
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
    bnb_epilogue<BM, BN, kThreads>(a, smem, ct, LDC, m0, n0, mt, nvalid, tid);
    return;
  }
  constexpr int CPR = BN / 8;
#pragma unroll
  for (int q = 0; q < (BM * CPR + kThreads - 1) / kThreads; ++q) {
    const int idx = tid + q * kThreads;
    const int row = idx / CPR, cc = idx - row * CPR;
    if (idx < BM * CPR && row < nvalid)
      *reinterpret_cast<us8*>(a.Y + (m0 + row) * a.N + n0 + cc * 8) = *reinterpret_cast<const us8*>(ct + row * LDC + cc * 8);
  }
  // BN statistics after the stores are issued (red is its own LDS region): they drain meanwhile
  if (STATS && !a.stats_first)
    det_block_bn_stats<FM, FN, WM, TM, TN, BN>(acc, red, wm, wn, lane, tid, nvalid, a.pmean, a.pm2,
                                                static_cast<int64_t>(mt) * a.N + n0);
#endif
}

// ------------------------------------------------------------------------------------------------
// v3: 32-deep K tiles and 256 x 256 block tiles (8 waves, 128 x 64 wave tiles).
//
// v2's 256 x 128 tile stages (256 + 128) rows per 2 * 256 * 128 * K FLOP; its 6 LDS-DMA pieces per
// wave per 32 MFMAs cost ~60-185 issue cycles each among the MFMAs (MI355X_MICROARCH.md, "LDS-DMA
// piece issue cost"), which is what held it at ~35 % of the MFMA rate.  A 256 x 256 tile stages
// 1.5x fewer bytes per FLOP: 4 pieces per wave per 32 MFMAs.  At BK = 64 a 256 x 256 stage is
// 64 KiB, two stages are all the ring LDS allows, which leaves no prefetch distance in this loop
// structure; at BK = 32 a stage is 32 KiB and a 4-stage ring keeps two tiles in flight.
//
// LDS rows are 64 B: a ds_read_b128 fragment read (16 rows, one 16-B chunk each, lane groups
// {0-3,12-15,20-27} ...) is conflict-free with the chunk XOR f(row) = (-(row >> 2)) & 3 (each group
// then covers 16 distinct (row & 3, chunk') bank slots); as everywhere the LDS image is lane-linear
// and the XOR is applied to the per-lane source address.
//
// Software pipeline per K tile: the wave tile is cut into its upper and lower A halves;
//   read A_hi(kt)                  || MFMAs A_lo(kt) x B(kt)
//   wait tile kt+1, barrier, issue tile kt+NS-1
//   read A_lo(kt+1)                || MFMAs A_hi(kt) x B(kt), then read B(kt+1) into the B registers
//                                     as the j-outer cluster releases them
// (acc 128 + 3 x 16 fragment VGPRs: a second B set would push the 256 x 256 tile past 256 VGPRs).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int swz64(int row, int ch) { return row * 64 + ((ch ^ ((-(row >> 2)) & 3)) << 4); }

template <int BM, int BN, int WM, int WN, int NS, bool STATS, bool BNB = false, int OCC = 1>
__global__ void __launch_bounds__(WM * WN * 64, OCC) igemm3_kernel(IgArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int BK = 32;
  constexpr int NW = WM * WN, kThreads = NW * 64;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16, FH = FM / 2;
  static_assert(FM % 2 == 0, "two A halves");
  // 16 rows of 64 B per LDS-DMA piece.  When B has fewer pieces than there are waves (BN = 64 at 8
  // waves) only waves wid < BP fetch B, one piece each, and count their own extra piece in vmcnt.
  constexpr int AI = BM / (16 * NW), BP = BN / 16, BI = BP >= NW ? BP / NW : 1;
  static_assert(AI * 16 * NW == BM && (BP >= NW ? BI * NW == BP : NW % BP == 0), "tile rows split over the waves");
  static_assert(NS >= 3, "prefetch distance");
  constexpr bool BPART = BP < NW;
  constexpr int NI = AI + BI, NIA = AI;  // pieces per tile of a B-fetching / a non-fetching wave
  constexpr int A_BYTES = BM * 64, STAGE = (BM + BN) * 64;
  constexpr int LDC = BN + 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* red = reinterpret_cast<float*>(smem + BM * LDC * 2);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = a.N / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntn, nt = bid - mt * ntn;
  const int64_t m0 = static_cast<int64_t>(mt) * BM;
  const int n0 = nt * BN;
  const int64_t K = a.K;
  const int lrow = lane >> 2;                       // row within a 16-row piece
  const int gch = (lane & 3) ^ ((-(lrow >> 2)) & 3);  // source chunk of this lane's LDS slot

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(a.X), 0, static_cast<int>(a.x_bytes), 0x00020000);
  const int64_t KB = a.kb_stride > 0 ? a.kb_stride : K;  // B row stride (elements)
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(a.W), 0, static_cast<int>(static_cast<int64_t>(a.N) * KB * 2), 0x00020000);
  constexpr unsigned kOOB = 0xFFFFFFF0u;
  int aoff[AI];
  unsigned amask[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = (i * NW + wid) * 16 + lrow;
    const int64_t m = m0 + row;
    aoff[i] = 0;
    amask[i] = 0;
    if (m < a.M) {
      const int64_t hw = static_cast<int64_t>(a.Ho) * a.Wo;
      const int64_t n = m / hw;
      const int rem = static_cast<int>(m - n * hw);
      const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
      const int hi0 = ho * a.stride - a.pad, wi0 = wo * a.stride - a.pad;
      aoff[i] = static_cast<int>(((n * a.Hi + hi0) * a.Wi + wi0) * a.Cin * 2 + gch * 16);
      for (int r = 0; r < a.R; ++r)
        for (int s2 = 0; s2 < a.S; ++s2) {
          const int hi = hi0 + r, wi = wi0 + s2;
          if (hi >= 0 && hi < a.Hi && wi >= 0 && wi < a.Wi) amask[i] |= 1u << (r * a.S + s2);
        }
    }
  }
  unsigned boff[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j)
    boff[j] = static_cast<unsigned>(((static_cast<int64_t>(n0) + ((j * NW + wid) % BP) * 16 + lrow) * KB + gch * 8) * 2);

  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % NS) * STAGE;
    const int k0 = kt * BK;
    const int tap = k0 / a.Cin, c0 = k0 - tap * a.Cin;
    const int r = tap / a.S, s2 = tap - r * a.S;
    const int toff = ((r * a.Wi + s2) * a.Cin + c0) * 2;
    const int kb = a.tapmap ? static_cast<int>((a.tapmap >> (4 * tap)) & 15u) * a.Cin + c0 : k0;  // B column
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const unsigned v = ((amask[i] >> tap) & 1u) ? static_cast<unsigned>(aoff[i] + toff) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(st + ((i * NW + wid) * 16) * 64), 16, v, 0, 0, 0);
    }
    if (!BPART || wid < BP) {
#pragma unroll
      for (int j = 0; j < BI; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void*)(st + A_BYTES + ((j * NW + wid) * 16) * 64), 16, boff[j],
                                                 kb * 2, 0, 0);
    }
  };
  const bool bwave = !BPART || __builtin_amdgcn_readfirstlane(wid) < BP;
  // counted waits on this wave's own LDS-DMA pieces: `tiles` younger tiles may stay in flight
  auto wait_tiles = [&](auto tiles) {
    constexpr int T = decltype(tiles)::value;
    if (bwave) wait_vmcnt<NI * T>();
    else wait_vmcnt<NIA * T>();
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ch = lane >> 4;
  auto read_a = [&](const unsigned char* base, int h, bf16x8* af) {
#pragma unroll
    for (int i = 0; i < FH; ++i) af[i] = *reinterpret_cast<const bf16x8*>(base + swz64(wm * TM + (h * FH + i) * 16 + (lane & 15), ch));
  };
  auto read_b = [&](const unsigned char* base, bf16x8* bfr) {
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(base + A_BYTES + swz64(wn * TN + j * 16 + (lane & 15), ch));
  };
  // h = 0: i-outer; h = 1: j-outer, so each b[j] dies after its FH MFMAs and the next tile's B
  // reads (issued after the cluster in source order) can be scheduled into the cluster's tail
  auto mfma = [&](int h, const bf16x8* af, const bf16x8* bfr) {
    __builtin_amdgcn_s_setprio(1);
    if (h == 0) {
#pragma unroll
      for (int i = 0; i < FH; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FH; ++i)
          acc[FH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[FH + i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  };

  bf16x8 alo[FH], ahi[FH], bf[FN];
  const int nk = a.K / BK;
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(t);
  if (nk >= NS - 1) wait_tiles(std::integral_constant<int, NS - 2>{});
  else wait_vmcnt<0>();
  block_barrier();
  read_a(smem, 0, alo);
  read_b(smem, bf);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  for (int kt = 0; kt + 1 < nk; ++kt) {
    read_a(smem + (kt % NS) * STAGE, 1, ahi);
    mfma(0, alo, bf);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (kt + NS - 2 < nk) wait_tiles(std::integral_constant<int, NS - 3>{});
    else wait_vmcnt<0>();
    block_barrier();
    if (kt + NS - 1 < nk) issue(kt + NS - 1);
    const unsigned char* nb = smem + ((kt + 1) % NS) * STAGE;
    read_a(nb, 0, alo);
    mfma(1, ahi, bf);
    read_b(nb, bf);
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
  read_a(smem + ((nk - 1) % NS) * STAGE, 1, ahi);
  mfma(0, alo, bf);
  mfma(1, ahi, bf);
  __syncthreads();

  unsigned short* ct = reinterpret_cast<unsigned short*>(smem);
  const int64_t rows_left = a.M - m0;
  const int nvalid = rows_left < BM ? static_cast<int>(rows_left) : BM;
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
    bnb_epilogue<BM, BN, kThreads>(a, smem, ct, LDC, m0, n0, mt, nvalid, tid);
    return;
  }
  constexpr int CPR = BN / 8;
#pragma unroll
  for (int q = 0; q < (BM * CPR + kThreads - 1) / kThreads; ++q) {
    const int idx = tid + q * kThreads;
    const int row = idx / CPR, cc = idx - row * CPR;
    if (idx < BM * CPR && row < nvalid)
      *reinterpret_cast<us8*>(a.Y + out_row(a, m0 + row) * a.N + n0 + cc * 8) = *reinterpret_cast<const us8*>(ct + row * LDC + cc * 8);
  }
  // BN statistics after the stores are issued (red is its own LDS region): they drain meanwhile
  if (STATS && !a.stats_first)
    det_block_bn_stats<FM, FN, WM, TM, TN, BN>(acc, red, wm, wn, lane, tid, nvalid, a.pmean, a.pm2,
                                                static_cast<int64_t>(mt) * a.N + n0);
#endif
}

// ------------------------------------------------------------------------------------------------
// v8: the eight-phase ping-pong schedule of det_gemm8.hip (see its header) on igemm3's implicit-GEMM
// gather.  256 x 256 block tile, 8 waves of 128 x 64 (the igemm3 cfg-8 wave decomposition, so the
// igemm3 epilogues apply unchanged), K tiles of 64 = one tap x 64 channels (Cin % 64 == 0), LDS as
// two K tiles x four 16 KiB half-tiles (A rows 0-127 / 128-255, B rows 0-127 / 128-255) of two
// 64-B-row sub-images each.  Per K tile: P1 reads A rows 0-63 + B cols 0-31 and issues A(t+1),
// P2 reads A rows 64-127 + B cols 32-63, P3 only computes, P4 issues B(t+2) into this tile's buffer
// and retires tile t+1 (vmcnt 4).  The wave group of the lower 128 rows runs one barrier late.
// ------------------------------------------------------------------------------------------------
template <int BM, int BN, bool STATS, bool BNB>
__global__ void __launch_bounds__(512, 1) igemm8_kernel(IgArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  // 8 waves of 128 x 64: BM x BN = 256 x 256 (2 x 4 waves) or 512 x 128 (4 x 2)
  constexpr int WM = BM / 128, WN = BN / 64, NW = 8, kThreads = 512;
  static_assert(WM * WN == NW, "eight waves");
  constexpr int NA = BM / 128, NB = BN / 128;  // A / B half-tiles per K tile
  constexpr int TM = 128, TN = 64, FM = 8, FN = 4;
  constexpr int HALF = 128 * 64 * 2, BUF = (NA + NB) * HALF;
  constexpr int LDC = BN + 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* red = reinterpret_cast<float*>(smem + BM * LDC * 2);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = a.N / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntn, nt = bid - mt * ntn;
  const int64_t m0 = static_cast<int64_t>(mt) * BM;
  const int n0 = nt * BN;
  const int lrow = lane >> 2;
  const int gch = (lane & 3) ^ ((-(lrow >> 2)) & 3);

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(a.X), 0, static_cast<int>(a.x_bytes), 0x00020000);
  const int64_t KB = a.kb_stride > 0 ? a.kb_stride : a.K;
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(a.W), 0, static_cast<int>(static_cast<int64_t>(a.N) * KB * 2), 0x00020000);
  constexpr unsigned kOOB = 0xFFFFFFF0u;
  // this lane's DMA rows: half h, row h*128 + wid*16 + lrow (4 lanes per 64-B row, chunk gch)
  int aoff[NA];
  unsigned amask[NA], boff[NB];
#pragma unroll
  for (int h = 0; h < NA; ++h) {
    const int64_t m = m0 + h * 128 + wid * 16 + lrow;
    aoff[h] = 0;
    amask[h] = 0;
    if (m < a.M) {
      const int64_t hw = static_cast<int64_t>(a.Ho) * a.Wo;
      const int64_t n = m / hw;
      const int rem = static_cast<int>(m - n * hw);
      const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
      const int hi0 = ho * a.stride - a.pad, wi0 = wo * a.stride - a.pad;
      aoff[h] = static_cast<int>(((n * a.Hi + hi0) * a.Wi + wi0) * a.Cin * 2 + gch * 16);
      for (int r = 0; r < a.R; ++r)
        for (int s2 = 0; s2 < a.S; ++s2) {
          const int hi = hi0 + r, wi = wi0 + s2;
          if (hi >= 0 && hi < a.Hi && wi >= 0 && wi < a.Wi) amask[h] |= 1u << (r * a.S + s2);
        }
    }
  }
#pragma unroll
  for (int h = 0; h < NB; ++h)
    boff[h] = static_cast<unsigned>(((static_cast<int64_t>(n0) + h * 128 + wid * 16 + lrow) * KB + gch * 8) * 2);
  auto stage = [&](int ht, int kt) {
    unsigned char* dst = smem + (kt & 1) * BUF + ht * HALF + wid * 1024;
    const int k0 = kt * 64;
    const int tap = k0 / a.Cin, c0 = k0 - tap * a.Cin;
    if (ht < NA) {
      const int r = tap / a.S, s2 = tap - r * a.S;
      const int toff = ((r * a.Wi + s2) * a.Cin + c0) * 2;
      const bool ok = (amask[ht] >> tap) & 1u;
      const unsigned v = ok ? static_cast<unsigned>(aoff[ht] + toff) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)dst, 16, v, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(dst + 8192), 16, ok ? v + 64u : kOOB, 0, 0, 0);
    } else {
      const int kb = a.tapmap ? static_cast<int>((a.tapmap >> (4 * tap)) & 15u) * a.Cin + c0 : k0;
      const unsigned v = boff[ht - NA] + static_cast<unsigned>(kb) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_void*)dst, 16, v, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_void*)(dst + 8192), 16, v + 64u, 0, 0, 0);
    }
  };
  // a raw barrier that also keeps every instruction in its phase
  auto phase_barrier = []() {
    __builtin_amdgcn_sched_barrier(0);
    block_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[FM][2], bfm[FN][2];
  const int fr = lane & 15, fch = lane >> 4;
  auto read_a = [&](int kt, int i0) {
    const unsigned char* base = smem + (kt & 1) * BUF + wm * HALF;
#pragma unroll
    for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) af[i][kh] = *reinterpret_cast<const bf16x8*>(base + kh * 8192 + swz64(i * 16 + fr, fch));
  };
  auto read_b = [&](int kt, int j0) {
    const unsigned char* base = smem + (kt & 1) * BUF + (NA + (wn >> 1)) * HALF;
#pragma unroll
    for (int j = j0; j < j0 + 2; ++j)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
        bfm[j][kh] = *reinterpret_cast<const bf16x8*>(base + kh * 8192 + swz64((wn & 1) * 64 + j * 16 + fr, fch));
  };
  auto mfma = [&](int i0, int j0) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
        for (int j = j0; j < j0 + 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kh], bfm[j][kh], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = a.K / 64;
  // the late wave group: waves 4-7 (each SIMD holds waves s and s + 4)
  const bool late = wid >= 4;
#pragma unroll
  for (int h = 0; h < NA + NB; ++h) stage(h, 0);
  if (nk > 1) {
#pragma unroll
    for (int h = 0; h < NB; ++h) stage(NA + h, 1);
    wait_vmcnt<2 * NB>();
  } else {
    wait_vmcnt<0>();
  }
  phase_barrier();
  if (late) phase_barrier();
  for (int t = 0; t < nk; ++t) {
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    // P1: A rows 0-63 + B cols 0-31 of tile t; A(t+1) (first two half-tiles)
    read_a(t, 0);
    read_b(t, 0);
    if (n1) { stage(0, t + 1); stage(1, t + 1); }
    phase_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mfma(0, 0);
    phase_barrier();
    // P2: A rows 64-127 + B cols 32-63 (the tile is now in registers); A(t+1) half-tiles 2-3
    read_a(t, 4);
    read_b(t, 2);
    if (NA > 2 && n1) { stage(2, t + 1); stage(3, t + 1); }
    phase_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mfma(0, 2);
    phase_barrier();
    phase_barrier();
    mfma(4, 2);
    phase_barrier();
    // P4: B(t+2) into this tile's buffer (its last reads were in P2), then retire tile t+1
    if (n2) {
#pragma unroll
      for (int h = 0; h < NB; ++h) stage(NA + h, t + 2);
      wait_vmcnt<2 * NB>();
    } else {
      wait_vmcnt<0>();
    }
    phase_barrier();
    mfma(4, 0);
    phase_barrier();
  }
  if (!late) phase_barrier();
  __syncthreads();

  unsigned short* ct = reinterpret_cast<unsigned short*>(smem);
  const int64_t rows_left = a.M - m0;
  const int nvalid = rows_left < BM ? static_cast<int>(rows_left) : BM;
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
    bnb_epilogue<BM, BN, kThreads>(a, smem, ct, LDC, m0, n0, mt, nvalid, tid);
    return;
  }
  constexpr int CPR = BN / 8;
#pragma unroll
  for (int q = 0; q < (BM * CPR + kThreads - 1) / kThreads; ++q) {
    const int idx = tid + q * kThreads;
    const int row = idx / CPR, cc = idx - row * CPR;
    if (idx < BM * CPR && row < nvalid)
      *reinterpret_cast<us8*>(a.Y + out_row(a, m0 + row) * a.N + n0 + cc * 8) = *reinterpret_cast<const us8*>(ct + row * LDC + cc * 8);
  }
  if (STATS && !a.stats_first)
    det_block_bn_stats<FM, FN, WM, TM, TN, BN>(acc, red, wm, wn, lane, tid, nvalid, a.pmean, a.pm2,
                                                static_cast<int64_t>(mt) * a.N + n0);
  (void)NW;
#endif
}

template <int BM, int BN>
int launch8(hipStream_t st, const IgArgs& a_in, bool stats, bool bnb) {
  IgArgs a = a_in;
  a.stats_first = stats_first_flag();
  if (a.N % BN != 0 || a.Cin % 64 != 0 || a.K % 64 != 0) return -6;
  const int64_t nwg = ((a.M + BM - 1) / BM) * (a.N / BN);
  if (nwg >= (static_cast<int64_t>(1) << 31)) return -4;
  constexpr int ring = 2 * (BM + BN) * 64 * 2, ctile = BM * (BN + 16) * 2 + 12 * (BM / 128) * BN;
  constexpr int smem = ring > ctile ? ring : ctile;
  static_assert(smem <= 163840, "LDS");
  if (bnb)
    hipLaunchKernelGGL((igemm8_kernel<BM, BN, false, true>), dim3(static_cast<unsigned>(nwg)), dim3(512), smem, st, a);
  else if (stats)
    hipLaunchKernelGGL((igemm8_kernel<BM, BN, true, false>), dim3(static_cast<unsigned>(nwg)), dim3(512), smem, st, a);
  else
    hipLaunchKernelGGL((igemm8_kernel<BM, BN, false, false>), dim3(static_cast<unsigned>(nwg)), dim3(512), smem, st, a);
  return static_cast<int>(hipGetLastError());
}

// OCC: workgroups per CU the LDS footprint and register budget are sized for.  At OCC 2 one
// workgroup's epilogue (C tile through LDS, 16-B stores, BN statistics) overlaps the other's K loop;
// with one workgroup per CU the short-K GEMMs (1x1 expansions, K = 64..512) serialise load ->
// compute -> store per tile.
template <int BM, int BN, int WM, int WN, int NS, int OCC = 1>
int launch3(hipStream_t st, const IgArgs& a_in, bool stats, bool bnb = false) {
  IgArgs a = a_in;
  a.stats_first = stats_first_flag();
  constexpr int kThreads = WM * WN * 64;
  if (a.N % BN != 0 || a.Cin % 32 != 0) return -6;
  const int64_t nwg = ((a.M + BM - 1) / BM) * (a.N / BN);
  if (nwg >= (static_cast<int64_t>(1) << 31)) return -4;
  constexpr int ring = NS * (BM + BN) * 64, ctile = BM * (BN + 16) * 2 + 12 * WM * BN;
  constexpr int smem = ring > ctile ? ring : ctile;
  static_assert(smem * OCC <= 163840, "LDS");
  static_assert(BM * (BN + 16) * 2 >= kThreads * 16 * 4, "BN-backward scratch fits in the C tile");
  if (bnb)
    hipLaunchKernelGGL((igemm3_kernel<BM, BN, WM, WN, NS, false, true, OCC>), dim3(static_cast<unsigned>(nwg)), dim3(kThreads),
                       smem, st, a);
  else if (stats)
    hipLaunchKernelGGL((igemm3_kernel<BM, BN, WM, WN, NS, true, false, OCC>), dim3(static_cast<unsigned>(nwg)), dim3(kThreads),
                       smem, st, a);
  else
    hipLaunchKernelGGL((igemm3_kernel<BM, BN, WM, WN, NS, false, false, OCC>), dim3(static_cast<unsigned>(nwg)), dim3(kThreads),
                       smem, st, a);
  return static_cast<int>(hipGetLastError());
}

template <int BM, int BN, int WM, int WN, int NS, int OCC>
int launch2(hipStream_t st, const IgArgs& a_in, bool dense, bool stats, bool bnb = false) {
  IgArgs a = a_in;
  a.stats_first = stats_first_flag();
  constexpr int kThreads = WM * WN * 64;
  if (a.N % BN != 0 || a.Cin % 64 != 0) return -6;
  const int64_t nwg = ((a.M + BM - 1) / BM) * (a.N / BN);
  if (nwg >= (static_cast<int64_t>(1) << 31)) return -4;
  constexpr int smem = NS * (BM + BN) * 128;
#define DET_IG2(D, S)                                                                                          \
  hipLaunchKernelGGL((igemm2_kernel<BM, BN, WM, WN, NS, D, S, OCC>), dim3(static_cast<unsigned>(nwg)), dim3(kThreads), \
                     smem, st, a)
  (void)dense;  // the tap-mask fetch covers 1x1 / strided / padded alike
  static_assert(BM * (BN + 16) * 2 >= kThreads * 16 * 4, "BN-backward scratch fits in the C tile");
  if (bnb)
    hipLaunchKernelGGL((igemm2_kernel<BM, BN, WM, WN, NS, false, false, OCC, true>), dim3(static_cast<unsigned>(nwg)),
                       dim3(kThreads), smem, st, a);
  else if (stats) DET_IG2(false, true); else DET_IG2(false, false);
#undef DET_IG2
  return static_cast<int>(hipGetLastError());
}

template <int BM, int BN, int WM, int WN>
int launch(hipStream_t st, const IgArgs& a_in, bool dense, bool stats) {
  IgArgs a = a_in;
  a.stats_first = stats_first_flag();
  constexpr int kThreads = WM * WN * 64;
  const int64_t nwg = ((a.M + BM - 1) / BM) * (a.N / BN);
  if (nwg >= (static_cast<int64_t>(1) << 31)) return -4;
  constexpr int smem = kStages * (BM + BN) * 128 + 12 * WM * BN;
#define DET_IG(D, S) \
  hipLaunchKernelGGL((igemm_kernel<BM, BN, WM, WN, D, S>), dim3(static_cast<unsigned>(nwg)), dim3(kThreads), smem, st, a)
  if (dense) { if (stats) DET_IG(true, true); else DET_IG(true, false); }
  else { if (stats) DET_IG(false, true); else DET_IG(false, false); }
#undef DET_IG
  return static_cast<int>(hipGetLastError());
}

// Tile configurations (det_igemm_conv_cfg): 0 = automatic; 1 = v1 (256 x BN, 8 waves); 2..7 = v2:
//   2: 256x128, 8 waves (4x2, 64x64 wave tiles), 3-stage ring (144 KiB), 1 block/CU
//   3: 256x64,  4 waves (4x1, 64x64), 3 stages (120 KiB)
//   4: 128x128, 4 waves (2x2, 64x64), 4 stages (128 KiB)
//   5: 256x64,  8 waves (8x1, 32x64), 3 stages (120 KiB)
//   6: 128x64,  4 waves (2x2, 64x32), 3 stages (72 KiB), 2 blocks/CU
//   7: 128x128, 4 waves (2x2, 64x64), 3 stages (96 KiB)
static int run_cfg(int cfg, hipStream_t st, const IgArgs& a, bool dense, bool stats, bool bnb = false) {
  switch (cfg) {
    case 1:
      if (a.Cin % 64 || bnb) return -6;
      if (a.N % 128 == 0) return launch<256, 128, 4, 2>(st, a, dense, stats);
      return launch<256, 64, 8, 1>(st, a, dense, stats);
    case 2: return launch2<256, 128, 4, 2, 3, 1>(st, a, dense, stats, bnb);
    case 3: return launch2<256, 64, 4, 1, 3, 1>(st, a, dense, stats, bnb);
    case 4: return launch2<128, 128, 2, 2, 4, 1>(st, a, dense, stats, bnb);
    case 5: return launch2<256, 64, 8, 1, 3, 1>(st, a, dense, stats, bnb);
    case 6: return launch2<128, 64, 2, 2, 3, 2>(st, a, dense, stats, bnb);
    case 7: return launch2<128, 128, 2, 2, 3, 1>(st, a, dense, stats, bnb);
    case 8: return launch3<256, 256, 2, 4, 4>(st, a, stats, bnb);   // 128x64 wave tiles, BK 32, 4 stages
    case 9: return launch3<256, 128, 4, 2, 4>(st, a, stats, bnb);   // 64x64 wave tiles, BK 32
    case 10: return launch3<256, 256, 2, 4, 3>(st, a, stats, bnb);  // 3 stages
    case 11: return launch3<256, 64, 4, 1, 4>(st, a, stats, bnb);   // 4 waves, 64x64 wave tiles (N = 64)
    case 12: return launch3<512, 128, 4, 2, 3>(st, a, stats, bnb);  // 128x64 wave tiles at N = 128
    case 13: return launch3<512, 128, 4, 2, 4>(st, a, stats, bnb);
    case 14: return launch3<512, 64, 8, 1, 4>(st, a, stats, bnb);   // 64x64 wave tiles at N = 64, 8 waves
    case 15: return launch3<512, 64, 4, 1, 4>(st, a, stats, bnb);   // 128x64 wave tiles at N = 64, 4 waves
    // two workgroups per CU (one's epilogue under the other's K loop)
    case 16: return launch3<256, 128, 4, 2, 3, 2>(st, a, stats, bnb);  // 64x64 wave tiles, 3 stages
    case 17: return launch3<256, 64, 4, 1, 4, 2>(st, a, stats, bnb);   // cfg 11 at 2 per CU
    case 18: return launch3<256, 64, 4, 1, 3, 2>(st, a, stats, bnb);
    case 19: return launch3<128, 128, 2, 2, 4, 2>(st, a, stats, bnb);  // 64x64 wave tiles, 4 waves
    case 20: return launch3<128, 256, 2, 4, 3, 2>(st, a, stats, bnb);  // 64x64 wave tiles, 8 waves
    case 21: return launch8<256, 256>(st, a, stats, bnb);  // eight-phase ping-pong, 256x256, BK 64
    case 22: return launch8<512, 128>(st, a, stats, bnb);  // eight-phase, 512x128 (4 x 2 waves of 128x64)
    default: return -7;
  }
}

// block-tile N (output channels) of a tile configuration
static int cfg_bn(int c) {
  switch (c) {
    case 3: case 5: case 6: case 11: case 14: case 15: case 17: case 18: return 64;
    case 8: case 10: case 20: case 21: return 256;
    default: return 128;
  }
}

static int auto_cfg(const IgArgs& a) {
  static const int forced = [] {
    const char* e = std::getenv("DET_IGEMM_CFG");
    return e ? std::atoi(e) : 0;
  }();
  // a forced configuration (sweeps) applies where its tile fits; other shapes keep the heuristic
  if (forced > 0 && a.N % cfg_bn(forced) == 0 && ((forced < 8 || forced >= 21) ? a.Cin % 64 == 0 : a.Cin % 32 == 0))
    return forced;
  // measured per ResNet-50 shape (profiles/r3_igemm_cfgs.jsonl): 256 x 256 / BK 32 wherever N
  // allows, 256 x 128 / BK 64 at N = 128, 256 x 64 / BK 32 (4 waves) at N = 64
  // R x S convolutions with 256-multiple N on the eight-phase schedule (cfg 21): 7-9 % faster than
  // cfg 8 on ResNet-50's 256/512-channel 3x3 forward and stride-1 input-gradient passes; the
  // stride-2 parity-class input gradients (tapmap) and 1x1 gathers (short K) stay on cfg 8
  // (profiles/r6_igemm8_conv3x3.jsonl).  DET_IGEMM8=0 turns it off (A/B).
  static const bool use8 = [] {
    const char* e = std::getenv("DET_IGEMM8");
    return !(e && e[0] == '0');
  }();
  // 1x1 convolutions (opt-in DET_IGEMM8_1X1=1): in isolation the stride-2 gathers, K = 64 and
  // K >= 2048 expansions gain 2-9 % on cfg 21 (profiles/r6_igemm8_conv1x1.jsonl), but in the step
  // the bench reads 0.15 % lower with them than with the 3x3 convs alone (r6s35, three rounds)
  static const bool use8_1x1 = [] {
    const char* e = std::getenv("DET_IGEMM8_1X1");
    return e && e[0] == '1';
  }();
  const bool one = a.R * a.S == 1;
  const bool one8 = one && use8_1x1 && (a.stride == 2 || a.K == 64 || a.K >= 2048);
  if (use8 && a.N % 256 == 0 && a.Cin % 64 == 0 && a.tapmap == 0 && (!one || one8)) return 21;
  // 128-channel convolutions: the 512 x 128 eight-phase tile, 2-4 % faster forward (r6s30, r6s33)
  if (use8 && a.N % 128 == 0 && a.N % 256 != 0 && a.Cin % 64 == 0 && a.tapmap == 0 && (!one || (use8_1x1 && a.K >= 512)))
    return 22;
  if (a.N % 256 == 0 && a.Cin % 32 == 0) return 8;
  if (a.N % 128 == 0 && a.Cin % 64 == 0) return 2;
  return a.Cin % 32 == 0 ? 11 : 1;
}

// ------------------------------------------------------------------------------------------------
// v5 (conv3p): 3x3 / stride-1 / pad-1 convolution with the input staged ONCE per tile as a halo
// patch, for the thin-N layers (ResNet layer1/2: N = 64/128, K = 9 x 64/128).
//
// igemm3 gathers the im2col A operand tap by tap: every output pixel's row is staged 9 times per
// channel slice, and with N = 64 the 16 KiB of A per K tile carry only 256 x 64 x 32 MACs -- the
// LDS-DMA issue cost per KiB (MI355X_MICROARCH.md "LDS-DMA piece issue cost") then exceeds the MFMA
// time (layer1 3x3 forward at ~400 TF/s, profiles/r3_conv3x3_passes.jsonl).  Here a 256-pixel output
// tile stages, per 32-channel slice, the padded input rows it touches (<= 640 pixels x 64 B) and the
// slice's 9-tap weights [9][64][32] once; the 9 taps then read their A fragments from the patch at
// a row offset of r * (W + 2) + s (per-lane patch rows, the 64-B-row swizzle of igemm3).  Staging
// is register-path (global_load -> ds_write), which lets the preceding BatchNorm + ReLU be applied
// on the way in (PRO: the normalised activation is never written to HBM; padding stays zero).
//   * 256 x 64 block tile, 8 waves of 32 x 64 (v_mfma_f32_16x16x32_bf16), one block per CU (the
//     staged slice is held in registers while the MFMAs run: 4 waves of 64 x 64 spill);
//   * persistent blocks over a contiguous chunk of (M tile, N tile) pairs, N fastest: the next
//     slice (or the next tile's first) is loaded into registers while the current one computes;
//   * epilogues of igemm3: bf16 tile via LDS, BN statistics (STATS) or the BN-backward partials
//     of the producing BatchNorm (BNB, for the stride-1 input gradient over the flipped weight).
// ------------------------------------------------------------------------------------------------
constexpr int kP3BM = 256, kP3BN = 64, kP3BK = 32, kP3PMAX = 640;  // PMAX: a 56-wide tile across an image boundary needs 580
constexpr int kP3PATCH = kP3PMAX * 64, kP3BT = 9 * kP3BN * 64;
constexpr int kP3SMEM = kP3PATCH + kP3BT;  // 69632 B

struct P3Tile {
  int64_t m0;
  int n0, g0;  // first padded input row ((H + 2) per image) the tile reads
  int rows;    // padded rows in the patch
};

__device__ __forceinline__ P3Tile p3_tile(const IgArgs& a, int t, int ntn) {
  P3Tile T;
  const int mt = t / ntn;
  T.n0 = (t - mt * ntn) * kP3BN;
  T.m0 = static_cast<int64_t>(mt) * kP3BM;
  const int64_t hw = static_cast<int64_t>(a.Hi) * a.Wi;
  int64_t mlast = T.m0 + kP3BM - 1;
  if (mlast >= a.M) mlast = a.M - 1;
  const int64_t na = T.m0 / hw, nb = mlast / hw;
  const int ha = static_cast<int>((T.m0 - na * hw) / a.Wi), hb = static_cast<int>((mlast - nb * hw) / a.Wi);
  T.g0 = static_cast<int>(na * (a.Hi + 2) + ha);
  T.rows = static_cast<int>(nb * (a.Hi + 2) + hb + 2) - T.g0 + 1;
  return T;
}

template <bool PRO, bool STATS, bool BNB>
__global__ void __launch_bounds__(512, 2) conv3p_kernel(IgArgs a, int ntiles, int ntn) {
  constexpr int BM = kP3BM, BN = kP3BN, NT = 512, WM = 8, TM = 32, TN = 64, FM = 2, FN = 4;
  constexpr int PCH = kP3PMAX * 4 / NT;  // patch 16-B chunks per thread (max)
  constexpr int BCHUNKS = 9 * BN * 4, BCH = (BCHUNKS + NT - 1) / NT;  // weight chunks (per thread)
  static_assert(kP3PMAX * 4 % NT == 0, "patch chunks split evenly");
  constexpr int LDC = BN + 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* patch = smem;
  unsigned char* bt = smem + kP3PATCH;
  float* red = reinterpret_cast<float*>(smem + BM * LDC * 2);

  const int tid = threadIdx.x, lane = tid & 63, wm = tid >> 6;
  const int Wp = a.Wi + 2;
  const int ns = a.Cin / kP3BK;  // channel slices per tile
  // this block's contiguous chunk of tiles (N tile fastest)
  const int G = gridDim.x;
  const int tbeg = static_cast<int>((static_cast<int64_t>(ntiles) * blockIdx.x) / G);
  const int tend = static_cast<int>((static_cast<int64_t>(ntiles) * (blockIdx.x + 1)) / G);
  const int items = (tend - tbeg) * ns;
  if (items <= 0) return;

  us8 rp[PCH], rw[BCH];
  const int cch = tid & 3;  // the 16-B channel chunk every patch chunk of this thread carries
  auto gload = [&](int it) {
    const int t = tbeg + it / ns, sl = it - (it / ns) * ns;
    const P3Tile T = p3_tile(a, t, ntn);
    const int c0 = sl * kP3BK;
    const int np = T.rows * Wp;
#pragma unroll
    for (int q = 0; q < PCH; ++q) {
      const int idx = tid + q * NT, p = idx >> 2;
      us8 v = us8{0, 0, 0, 0, 0, 0, 0, 0};
      if (p < np) {
        const int gr = T.g0 + p / Wp, wp = p - (p / Wp) * Wp;
        const int n = gr / (a.Hi + 2), h = gr - n * (a.Hi + 2) - 1, w = wp - 1;
        if (h >= 0 && h < a.Hi && w >= 0 && w < a.Wi)
          v = *reinterpret_cast<const us8*>(a.X + ((static_cast<int64_t>(n) * a.Hi + h) * a.Wi + w) * a.Cin + c0 + cch * 8);
      }
      rp[q] = v;
    }
#pragma unroll
    for (int q = 0; q < BCH; ++q) {
      const int idx = tid + q * NT, row = idx >> 2, ch = idx & 3;  // row = tap * BN + n
      const int tap = row / BN, n = row - tap * BN;
      if (BCHUNKS % NT == 0 || idx < BCHUNKS)
        rw[q] = *reinterpret_cast<const us8*>(a.W + (static_cast<int64_t>(T.n0 + n) * 9 + tap) * a.Cin + c0 + ch * 8);
    }
  };
  auto lstore = [&](int it) {
    const int t = tbeg + it / ns, sl = it - (it / ns) * ns;
    const P3Tile T = p3_tile(a, t, ntn);
    const int np = T.rows * Wp;
    float psc[8], psh[8];  // (loaded here, not with the slice: no registers held across the MFMAs)
    if constexpr (PRO) {
      const int c = sl * kP3BK + cch * 8;
#pragma unroll
      for (int j = 0; j < 8; j += 4) {
        const float4 s4 = *reinterpret_cast<const float4*>(a.pro_scale + c + j);
        const float4 h4 = *reinterpret_cast<const float4*>(a.pro_shift + c + j);
        psc[j] = s4.x; psc[j + 1] = s4.y; psc[j + 2] = s4.z; psc[j + 3] = s4.w;
        psh[j] = h4.x; psh[j + 1] = h4.y; psh[j + 2] = h4.z; psh[j + 3] = h4.w;
      }
    }
#pragma unroll
    for (int q = 0; q < PCH; ++q) {
      const int idx = tid + q * NT, p = idx >> 2;
      if (p >= np) continue;
      us8 v = rp[q];
      if constexpr (PRO) {
        const int gr = T.g0 + p / Wp, wp = p - (p / Wp) * Wp;
        const int h = gr - (gr / (a.Hi + 2)) * (a.Hi + 2) - 1, w = wp - 1;
        if (h >= 0 && h < a.Hi && w >= 0 && w < a.Wi) {  // the BN output of real pixels; padding stays 0
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = f2bf(fmaxf(__fmaf_rn(bf2f(v[j]), psc[j], psh[j]), 0.f));
        }
      }
      *reinterpret_cast<us8*>(patch + swz64(p, cch)) = v;
    }
#pragma unroll
    for (int q = 0; q < BCH; ++q) {
      const int idx = tid + q * NT, row = idx >> 2, ch = idx & 3;
      if (BCHUNKS % NT == 0 || idx < BCHUNKS) *reinterpret_cast<us8*>(bt + swz64(row, ch)) = rw[q];
    }
  };

  f32x4 acc[FM][FN];
  int abase[FM];  // patch row of this lane's A rows at tap (0, 0)
  const int ch = lane >> 4;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int it = 0; it < items; ++it) {
    const int t = tbeg + it / ns, sl = it - (it / ns) * ns;
    if (sl == 0) {
      const P3Tile T = p3_tile(a, t, ntn);
      const int64_t hw = static_cast<int64_t>(a.Hi) * a.Wi;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        int64_t m = T.m0 + wm * TM + i * 16 + (lane & 15);
        if (m >= a.M) m = a.M - 1;  // tail rows read a real pixel; their outputs are not stored
        const int64_t n = m / hw;
        const int rem = static_cast<int>(m - n * hw);
        const int ho = rem / a.Wi, wo = rem - ho * a.Wi;
        abase[i] = static_cast<int>(n * (a.Hi + 2) + ho - T.g0) * Wp + wo;
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (it + 1 < items) gload(it + 1);  // in flight under the 9 x 16 MFMAs below
    // taps software-pipelined over two fragment sets: the reads of tap+1 are in flight under the
    // 16 MFMAs of tap (sched_barrier keeps the compiler from hoisting further reads: registers)
    bf16x8 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
    auto rd = [&](int tap, bf16x8* fa, bf16x8* fb) {
      const int toff = (tap / 3) * Wp + (tap % 3);
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(patch + swz64(abase[i] + toff, ch));
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(bt + swz64(tap * BN + j * 16 + (lane & 15), ch));
    };
    auto mm = [&](const bf16x8* fa, const bf16x8* fb) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    rd(0, fa0, fb0);
#pragma unroll
    for (int tap = 0; tap < 9; tap += 2) {
      if (tap + 1 < 9) rd(tap + 1, fa1, fb1);
      mm(fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      if (tap + 1 < 9) {
        if (tap + 2 < 9) rd(tap + 2, fa0, fb0);
        mm(fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __syncthreads();  // every wave is done with this slice's patch and weights
    if (sl == ns - 1) {
      const P3Tile T = p3_tile(a, t, ntn);
      const int64_t m0 = T.m0;
      const int n0 = T.n0, mt = static_cast<int>(m0 / BM);
      unsigned short* ct = reinterpret_cast<unsigned short*>(smem);
      const int64_t rows_left = a.M - m0;
      const int nvalid = rows_left < BM ? static_cast<int>(rows_left) : BM;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ct[(wm * TM + i * 16 + (lane >> 4) * 4 + r) * LDC + j * 16 + (lane & 15)] = f2bf(acc[i][j][r]);
      if (STATS)
        det_block_bn_stats<FM, FN, WM, TM, TN, BN>(acc, red, wm, 0, lane, tid, nvalid, a.pmean, a.pm2,
                                                    static_cast<int64_t>(mt) * a.N + n0);
      __syncthreads();
      if constexpr (BNB) {
        bnb_epilogue<BM, BN, NT>(a, smem, ct, LDC, m0, n0, mt, nvalid, tid);
      } else {
        constexpr int CPR = BN / 8;
#pragma unroll
        for (int q = 0; q < BM * CPR / NT; ++q) {
          const int idx = tid + q * NT, row = idx / CPR, cc = idx - row * CPR;
          if (row < nvalid)
            *reinterpret_cast<us8*>(a.Y + (m0 + row) * a.N + n0 + cc * 8) = *reinterpret_cast<const us8*>(ct + row * LDC + cc * 8);
        }
      }
      __syncthreads();  // the C tile (LDS) is consumed before the next slice lands there
    }
    if (it + 1 < items) {
      lstore(it + 1);
      __syncthreads();
    }
  }
}

// Largest patch (pixels) any 256-pixel tile of an Nb x H x W image batch needs (host side).
static int64_t p3_max_patch(int64_t M, int H, int W) {
  const int64_t hw = static_cast<int64_t>(H) * W;
  int64_t best = 0;
  for (int64_t m0 = 0; m0 < M; m0 += kP3BM) {
    int64_t ml = m0 + kP3BM - 1;
    if (ml >= M) ml = M - 1;
    const int64_t na = m0 / hw, nb = ml / hw;
    const int64_t ga = na * (H + 2) + (m0 - na * hw) / W, gb = nb * (H + 2) + (ml - nb * hw) / W + 2;
    const int64_t p = (gb - ga + 1) * (W + 2);
    if (p > best) best = p;
    if (best > kP3PMAX) break;
  }
  return best;
}

// Input-gradient weight of an R x S conv in one pass: out[c][r][s][k] = W[k][R-1-r][S-1-s][c]
// (W in KRSC = channels_last memory, fp32 or bf16 in, bf16 out), 64 x 64 LDS-tiled transpose per tap.
template <typename TI>
__global__ void __launch_bounds__(256) dgrad_weight_kernel(const TI* __restrict__ W, unsigned short* __restrict__ out,
                                                           int K, int C, int R, int S) {
  __shared__ float tile[64][65];
  const int c0 = blockIdx.x * 64, k0 = blockIdx.y * 64, tap = blockIdx.z;
  const int r = tap / S, s2 = tap - r * S;
  const int src_tap = (R - 1 - r) * S + (S - 1 - s2);
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int k = k0 + i, c = c0 + tx;
    float v = 0.f;
    if (k < K && c < C) {
      const TI x = W[(static_cast<int64_t>(k) * R * S + src_tap) * C + c];
      if constexpr (sizeof(TI) == 2) v = bf2f(x); else v = x;
    }
    tile[i][tx] = v;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, k = k0 + tx;
    if (c < C && k < K) out[(static_cast<int64_t>(c) * R * S + tap) * K + k] = f2bf(tile[tx][i]);
  }
}

// The same transpose for up to kDwMulti weights in ONE launch (ops/conv.py flips every R x S weight a
// backward pass needs at its first input gradient): one launch per weight was 16 latency-bound
// launches of 9-576 workgroups per ResNet-50 step (0.19 ms, profiles/r5_resnet50_steady.csv).
constexpr int kDwMulti = 32;
struct DwMultiArgs {
  int n;
  int start[kDwMulti + 1];  // first workgroup of each weight (prefix sums)
  const void* w[kDwMulti];
  unsigned short* out[kDwMulti];
  int K[kDwMulti], C[kDwMulti], R[kDwMulti], S[kDwMulti], bf16[kDwMulti];
};

__global__ void __launch_bounds__(256) dgrad_weight_multi_kernel(DwMultiArgs a) {
  __shared__ float tile[64][65];
  int t = 0;
  while (t + 1 < a.n && static_cast<int>(blockIdx.x) >= a.start[t + 1]) ++t;
  const int K = a.K[t], C = a.C[t], R = a.R[t], S = a.S[t];
  const int gx = (C + 63) / 64, gy = (K + 63) / 64;
  const int local = static_cast<int>(blockIdx.x) - a.start[t];
  const int tap = local / (gx * gy), rem = local - tap * gx * gy;
  const int k0 = (rem / gx) * 64, c0 = (rem % gx) * 64;
  const int r = tap / S, s2 = tap - r * S;
  const int src_tap = (R - 1 - r) * S + (S - 1 - s2);
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const bool bf = a.bf16[t] != 0;
  for (int i = ty; i < 64; i += 4) {
    const int k = k0 + i, c = c0 + tx;
    float v = 0.f;
    if (k < K && c < C) {
      const int64_t off = (static_cast<int64_t>(k) * R * S + src_tap) * C + c;
      v = bf ? bf2f(static_cast<const unsigned short*>(a.w[t])[off]) : static_cast<const float*>(a.w[t])[off];
    }
    tile[i][tx] = v;
  }
  __syncthreads();
  unsigned short* out = a.out[t];
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, k = k0 + tx;
    if (c < C && k < K) out[(static_cast<int64_t>(c) * R * S + tap) * K + k] = f2bf(tile[tx][i]);
  }
}

// ------------------------------------------------------------------------------------------------
// Weight gradient on the LDS-DMA ring: P[split][N][RSC] (fp32 slab per pixel split) =
//   sum_{m in split} dY[m][n] . im2col(X)[m][rsc]            (rsc = (r*S + s)*Cin + c, KRSC order)
//
// Both operands arrive pixel-major ([m][channel], channels contiguous), i.e. K-major for this GEMM,
// so they are staged as they sit in HBM and read K-contiguous with ds_read_b64_tr_b16 (T10).  Each
// operand image is a stack of [32 pixels][64 channels] sub-tiles (128-B rows, 4 KiB), filled by
// buffer_load ... lds (16-B pieces, lane-linear: one instruction = 8 rows of one sub-tile) with the
// transposed-read swizzle applied on the SOURCE chunk; any multiple of 64 works for both tile
// sides, so the 9-tap column dimension (576 = 9 x 64 at Cin 64) needs no padding.
//   * dY pieces: fixed column per lane, the row advances 32 pixels per K step (one VALU add);
//   * X pieces: per lane a fixed (tap r,s, channel c) and an output pixel (n, ho, wo) advanced 32
//     pixels per step with carries (no divisions in the loop); padding taps and the split tail
//     fetch at an out-of-range offset, which the buffer unit returns as zeros;
//   * NS-stage ring with a counted vmcnt and raw s_barrier (as igemm3);
//   * blocks of one pixel split are consecutive in the XCD remap, so the N tiles that re-read the
//     same dY/X rows share an XCD's L2.
// ------------------------------------------------------------------------------------------------
struct WgArgs {
  const unsigned short* dY;  // [M, N]
  const unsigned short* X;   // NHWC [Nb, Hi, Wi, Cin]
  float* P;                  // [splits, N, RSC]
  int64_t M;
  int N, RSC, Cin;
  int Hi, Wi, Ho, Wo, stride, pad, S;
  int rows_per_split;  // multiple of 32
  int dy_bytes, x_bytes;
};

__device__ __forceinline__ int wswz(int row, int ch) {
  return row * 128 + ((ch ^ ((((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2))) << 4);
}

// MFMA operand (16 columns x 32 pixels) of a [32][64] sub-tile via two transposed 4x16 reads: lane
// (g = lane>>4, i = lane&15) gets pixels 8g + 0..7 of column c0 + i.
__device__ __forceinline__ bf16x8 wtr_frag(const unsigned char* sub, int c0, int lane) {
  typedef __attribute__((ext_vector_type(4))) short s16x4;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = c0 + 4 * p;
  const int o0 = wswz(8 * g + q, col >> 3) + ((col & 4) << 1);
  const int o1 = wswz(8 * g + 4 + q, col >> 3) + ((col & 4) << 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sub + o0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sub + o1));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int BM, int BN, int WM, int WN, int NS, int KB, int OCC>
__global__ void __launch_bounds__(WM * WN * 64, OCC) wgrad3_kernel(WgArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  // a stage = KB groups of 32 pixels (KB > 1: fewer barriers / waits per MFMA for small tiles)
  constexpr int BK = 32, SK = BK * KB;
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int PA = BM / 16, PB = BN / 16, PT = PA + PB;  // 1-KiB pieces per 32-pixel group
  static_assert(BM % 64 == 0 && BN % 64 == 0 && TM % 16 == 0 && TN % 16 == 0, "tile shape");
  static_assert(PT % NW == 0, "pieces split evenly over the waves");
  static_assert(NS >= 3, "prefetch distance");
  constexpr int PW = PT / NW;  // pieces per wave per group
  constexpr int A_BYTES = BM * 64, GROUP = (BM + BN) * 64, STAGE = GROUP * KB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: piece kinds branch per wave
  const int wm = wid / WN, wn = wid % WN;
  const int ntm = a.N / BM, ntn = a.RSC / BN, ntiles = ntm * ntn;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / ntiles, tile = bid - split * ntiles;
  const int mt = tile / ntn, nt = tile - mt * ntn;
  const int n0 = mt * BM, k0 = nt * BN;
  const int64_t mbeg = static_cast<int64_t>(split) * a.rows_per_split;
  int64_t mend = mbeg + a.rows_per_split;
  if (mend > a.M) mend = a.M;
  const int nk = mend > mbeg ? static_cast<int>((mend - mbeg + SK - 1) / SK) : 0;

  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(a.dY), 0, a.dy_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(a.X), 0, a.x_bytes, 0x00020000);
  constexpr unsigned kOOB = 0xFFFFFFF0u;

  // per piece: LDS slot (row, slot chunk) of this lane and the source it stands for
  const int prow = lane >> 3;  // row within the piece's 8
  int row_[PW];                // pixel row within a 32-pixel group
  bool isa[PW];
  int yoff[PW];                // A: byte offset of (mbeg + row, column)
  int xc[PW], xr_[PW], xs[PW]; // B: channel, tap row/col
  int xn[PW], xho[PW], xwo[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int p = i * NW + wid;
    const bool pa = p < PA;
    const int q = pa ? p : p - PA;  // piece within the operand
    const int sub = q >> 2, row = (q & 3) * 8 + prow;
    const int ch = (lane & 7) ^ ((((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2));
    row_[i] = row;
    isa[i] = pa;
    yoff[i] = 0;
    xc[i] = xr_[i] = xs[i] = xn[i] = xho[i] = xwo[i] = 0;
    if (pa) {
      yoff[i] = static_cast<int>(((mbeg + row) * a.N + n0 + sub * 64 + ch * 8) * 2);
    } else {
      const int k = k0 + sub * 64 + ch * 8;
      const int tap = k / a.Cin;
      xc[i] = k - tap * a.Cin;
      xr_[i] = tap / a.S;
      xs[i] = tap - xr_[i] * a.S;
      const int64_t m = mbeg + row;
      const int hw = a.Ho * a.Wo;
      xn[i] = static_cast<int>(m / hw);
      const int rem = static_cast<int>(m - static_cast<int64_t>(xn[i]) * hw);
      xho[i] = rem / a.Wo;
      xwo[i] = rem - xho[i] * a.Wo;
    }
  }
  const int adv_h = BK / a.Wo, adv_w = BK - adv_h * a.Wo;
  const int ystep = BK * a.N * 2;

  // issue stage kt's pieces (kt advances monotonically: the X pixel state is stepped here, 32
  // pixels per group)
  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % NS) * STAGE;
#pragma unroll
    for (int g = 0; g < KB; ++g) {
      const int grp = kt * KB + g;
      const int64_t mrow0 = mbeg + static_cast<int64_t>(grp) * BK;
#pragma unroll
      for (int i = 0; i < PW; ++i) {
        const int p = i * NW + wid;
        const bool valid = mrow0 + row_[i] < mend;
        unsigned v;
        if (isa[i]) {
          v = valid ? static_cast<unsigned>(yoff[i] + grp * ystep) : kOOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_void*)(st + g * GROUP + p * 1024), 16, v, 0, 0, 0);
        } else {
          const int hi = xho[i] * a.stride - a.pad + xr_[i], wi = xwo[i] * a.stride - a.pad + xs[i];
          const bool ok = valid && hi >= 0 && hi < a.Hi && wi >= 0 && wi < a.Wi;
          v = ok ? static_cast<unsigned>((((xn[i] * a.Hi + hi) * a.Wi + wi) * a.Cin + xc[i]) * 2) : kOOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(st + g * GROUP + p * 1024), 16, v, 0, 0, 0);
          // advance this row's output pixel by one group
          xwo[i] += adv_w;
          const int carry = xwo[i] >= a.Wo;
          xwo[i] -= carry ? a.Wo : 0;
          xho[i] += adv_h + carry;
          while (xho[i] >= a.Ho) {
            xho[i] -= a.Ho;
            ++xn[i];
          }
        }
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(t);
  for (int kt = 0; kt < nk; ++kt) {
    // stages issued: 0 .. min(nk-1, kt+NS-2); stage kt must land, the younger may stay in flight
    if (kt + NS - 2 < nk) wait_vmcnt<KB * PW * (NS - 2)>();
    else wait_vmcnt<0>();
    block_barrier();  // every wave's stage-kt pieces landed; every wave is done reading stage kt-1
    if (kt + NS - 1 < nk) issue(kt + NS - 1);  // into stage kt-1's buffer
#pragma unroll
    for (int g = 0; g < KB; ++g) {
      const unsigned char* base = smem + (kt % NS) * STAGE + g * GROUP;
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int c = wm * TM + i * 16;
        af[i] = wtr_frag(base + (c >> 6) * 4096, c & 63, lane);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = wn * TN + j * 16;
        bfr[j] = wtr_frag(base + A_BYTES + (c >> 6) * 4096, c & 63, lane);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }

  float* out = a.P + static_cast<int64_t>(split) * a.N * a.RSC;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wm * TM + i * 16 + (lane >> 4) * 4 + r;
        const int k = k0 + wn * TN + j * 16 + (lane & 15);
        out[static_cast<int64_t>(n) * a.RSC + k] = acc[i][j][r];
      }
#endif
}

// ------------------------------------------------------------------------------------------------
// wgrad8: the ring weight gradient (wgrad3, above) on the eight-phase ping-pong schedule of
// det_gemm8.hip: a 256 (Cout) x 256 (R*S*Cin) tile, 8 waves of 128 x 64 in two staggered groups, K
// tiles of 64 pixels held as four 16 KiB half-tiles (dY channels 0-127 / 128-255, im2col columns
// 0-127 / 128-255), each half-tile two 32-pixel groups of two [32][64] sub-tiles in wgrad3's
// transposed-read image.  P1 reads the wave's dY rows 0-63 and im2col columns 0-31 and issues
// dY(t+1), P2 reads the rest, P3 computes, P4 issues im2col(t+2) and retires tile t+1.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(512, 1) wgrad8_kernel(WgArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int BM = 256, BN = 256, WN = 4, TM = 128, TN = 64, FM = 8, FN = 4;
  constexpr int HALF = 16384, BUF = 4 * HALF;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntm = a.N / BM, ntn = a.RSC / BN, ntiles = ntm * ntn;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / ntiles, tile = bid - split * ntiles;
  const int mt = tile / ntn, nt = tile - mt * ntn;
  const int n0 = mt * BM, k0 = nt * BN;
  const int64_t mbeg = static_cast<int64_t>(split) * a.rows_per_split;
  int64_t mend = mbeg + a.rows_per_split;
  if (mend > a.M) mend = a.M;
  const int nk = mend > mbeg ? static_cast<int>((mend - mbeg + 63) / 64) : 0;

  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(a.dY), 0, a.dy_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(a.X), 0, a.x_bytes, 0x00020000);
  constexpr unsigned kOOB = 0xFFFFFFF0u;

  // this wave's pieces of every half-tile: sub-tile `sub`, pixel row `row` (of a 32-pixel group), two
  // groups (pieces wid and wid + 8); the lane's 16-B chunk pre-swizzled for the transposed reads
  const int q = wid;
  const int sub = q >> 2, row = (q & 3) * 8 + (lane >> 3);
  const int ch = (lane & 7) ^ ((((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2));
  int yoff[2];
  int xc[2], xrr[2], xss[2], xn[2], xho[2], xwo[2];  // im2col half h: column state, pixel (group 0)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    yoff[h] = static_cast<int>(((mbeg + row) * a.N + n0 + h * 128 + sub * 64 + ch * 8) * 2);
    const int k = k0 + h * 128 + sub * 64 + ch * 8;
    const int tap = k / a.Cin;
    xc[h] = k - tap * a.Cin;
    xrr[h] = tap / a.S;
    xss[h] = tap - xrr[h] * a.S;
    const int64_t m = mbeg + row;
    const int hw = a.Ho * a.Wo;
    xn[h] = static_cast<int>(m / hw);
    const int rem = static_cast<int>(m - static_cast<int64_t>(xn[h]) * hw);
    xho[h] = rem / a.Wo;
    xwo[h] = rem - xho[h] * a.Wo;
  }
  const int adv_h = 32 / a.Wo, adv_w = 32 - adv_h * a.Wo;
  auto adv32 = [&](int& n, int& ho, int& wo) {
    wo += adv_w;
    const int carry = wo >= a.Wo;
    wo -= carry ? a.Wo : 0;
    ho += adv_h + carry;
    while (ho >= a.Ho) {
      ho -= a.Ho;
      ++n;
    }
  };
  auto xsrc = [&](int h, int n, int ho, int wo, bool valid) -> unsigned {
    const int hi = ho * a.stride - a.pad + xrr[h], wi = wo * a.stride - a.pad + xss[h];
    const bool ok = valid && hi >= 0 && hi < a.Hi && wi >= 0 && wi < a.Wi;
    return ok ? static_cast<unsigned>((((n * a.Hi + hi) * a.Wi + wi) * a.Cin + xc[h]) * 2) : kOOB;
  };
  // half-tile ht (0/1 dY channel halves, 2/3 im2col column halves) of K tile kt; the im2col halves
  // must be issued in increasing kt (their pixel state advances 64 per call)
  auto stage = [&](int ht, int kt) {
    unsigned char* dst = smem + (kt & 1) * BUF + ht * HALF + q * 1024;
    const int64_t px0 = mbeg + static_cast<int64_t>(kt) * 64 + row;
    if (ht < 2) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const bool valid = px0 + g * 32 < mend;
        const unsigned v = valid ? static_cast<unsigned>(yoff[ht] + (kt * 64 + g * 32) * a.N * 2) : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_void*)(dst + g * 8192), 16, v, 0, 0, 0);
      }
    } else {
      const int h = ht - 2;
      const unsigned v0 = xsrc(h, xn[h], xho[h], xwo[h], px0 < mend);
      int n1 = xn[h], ho1 = xho[h], wo1 = xwo[h];
      adv32(n1, ho1, wo1);
      const unsigned v1 = xsrc(h, n1, ho1, wo1, px0 + 32 < mend);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)dst, 16, v0, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(dst + 8192), 16, v1, 0, 0, 0);
      adv32(n1, ho1, wo1);
      xn[h] = n1;
      xho[h] = ho1;
      xwo[h] = wo1;
    }
  };
  auto phase_barrier = []() {
    __builtin_amdgcn_sched_barrier(0);
    block_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[FM][2], bfm[FN][2];
  auto read_a = [&](int kt, int i0) {
    const unsigned char* base = smem + (kt & 1) * BUF + wm * HALF;
#pragma unroll
    for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
      for (int g = 0; g < 2; ++g) af[i][g] = wtr_frag(base + g * 8192 + (i >> 2) * 4096, (i * 16) & 63, lane);
  };
  auto read_b = [&](int kt, int j0) {
    const unsigned char* base = smem + (kt & 1) * BUF + (2 + (wn >> 1)) * HALF + (wn & 1) * 4096;
#pragma unroll
    for (int j = j0; j < j0 + 2; ++j)
#pragma unroll
      for (int g = 0; g < 2; ++g) bfm[j][g] = wtr_frag(base + g * 8192, j * 16, lane);
  };
  auto mfma = [&](int i0, int j0) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
        for (int j = j0; j < j0 + 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][g], bfm[j][g], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const bool late = wid >= 4;
  if (nk > 0) {
    stage(0, 0); stage(1, 0); stage(2, 0); stage(3, 0);
    if (nk > 1) { stage(2, 1); stage(3, 1); wait_vmcnt<4>(); } else wait_vmcnt<0>();
  }
  phase_barrier();
  if (late) phase_barrier();
  for (int t = 0; t < nk; ++t) {
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    read_a(t, 0);
    read_b(t, 0);
    if (n1) { stage(0, t + 1); stage(1, t + 1); }
    phase_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mfma(0, 0);
    phase_barrier();
    read_a(t, 4);
    read_b(t, 2);
    phase_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mfma(0, 2);
    phase_barrier();
    phase_barrier();
    mfma(4, 2);
    phase_barrier();
    if (n2) { stage(2, t + 2); stage(3, t + 2); wait_vmcnt<4>(); } else wait_vmcnt<0>();
    phase_barrier();
    mfma(4, 0);
    phase_barrier();
  }
  if (!late) phase_barrier();

  float* out = a.P + static_cast<int64_t>(split) * a.N * a.RSC;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wm * TM + i * 16 + (lane >> 4) * 4 + r;
        const int k = k0 + wn * TN + j * 16 + (lane & 15);
        out[static_cast<int64_t>(n) * a.RSC + k] = acc[i][j][r];
      }
#endif
}

// ------------------------------------------------------------------------------------------------
// conv3p_wgrad: weight gradient of a 3x3 / stride-1 / pad-1 convolution on the halo patch.
//   P[split][n][tap * Cin + c] = sum_{m in split} dY[m][n] . Xpad[patch(m) + off(tap)][c]
// A 512-thread block owns one 64 (Cout) x 9 x 64 (Cin) tile of the weight gradient and a range of
// output pixels, staged 256 at a time: dY [256][64] and the input patch those pixels read
// (<= 640 padded pixels x 64 channels) once for all 9 taps -- the per-tap im2col gather of the
// ring wgrad (wgrad3) stages each input row 9 times, which is what left it behind MIOpen at 64/128
// channels (profiles/r3_wgrad_ring_sweep.jsonl: 0.44 vs 0.33 ms).  Both MFMA operands are read
// K(pixel)-major with ds_read_b64_tr_b16: dY from 32-pixel sub-tiles (wtr_frag), the input from the
// patch at per-lane rows (the pixel's patch row + the tap offset, from a per-stage row table).
// Wave w holds Cout rows 32 (w & 1) .. +32 and Cin columns 16 (w >> 1) .. +16 of all 9 taps: 18
// accumulator tiles per 32-pixel step from 2 dY fragments and 9 input fragments, each input
// fragment feeding 2 MFMAs (LDS reads ~0.6 of the MFMA time; 16 x 32 wave columns would need 19
// fragments per 18 MFMAs and be LDS-bound).
// ------------------------------------------------------------------------------------------------
struct WpArgs {
  const unsigned short* dY;  // [M, N]
  const unsigned short* X;   // NHWC [Nb, H, W, Cin]
  float* P;                  // [splits, N, 9 * Cin]
  int64_t M;
  int N, Cin, H, W;
  int rows_per_split;        // multiple of 256
  int ntiles;                // (N / 64) * (Cin / 64)
};
constexpr int kWpDY = 256 * 128, kWpPATCH = kP3PMAX * 128;
constexpr int kWpSMEM = kWpDY + kWpPATCH + 256 * 4;  // dY [256][64] + patch [512][64] + row table

__global__ void __launch_bounds__(512, 1) conv3p_wgrad_kernel(WpArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((ext_vector_type(4))) short s16x4;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  constexpr int NT = 512, DYCH = 256 * 8 / NT, XCH = kP3PMAX * 8 / NT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* dys = smem;
  unsigned char* xps = smem + kWpDY;
  int* prow = reinterpret_cast<int*>(smem + kWpDY + kWpPATCH);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nh = w & 1, cb = w >> 1;  // Cout 32-row half, Cin 16-column block
  const int tile = blockIdx.x % a.ntiles, split = blockIdx.x / a.ntiles;
  const int ntc = a.Cin / 64;
  const int n0 = (tile / ntc) * 64, c0 = (tile % ntc) * 64;
  const int64_t pbeg = static_cast<int64_t>(split) * a.rows_per_split;
  int64_t pend = pbeg + a.rows_per_split;
  if (pend > a.M) pend = a.M;
  const int nst = pend > pbeg ? static_cast<int>((pend - pbeg + 255) / 256) : 0;
  const int Wp = a.W + 2;
  const int64_t hw = static_cast<int64_t>(a.H) * a.W;
  const int RSC = 9 * a.Cin;

  us8 ry[DYCH], rx[XCH];
  int g0s = 0, rows_s = 0;  // patch geometry of the staged chunk
  auto geom = [&](int64_t m0, int& g0, int& rows) {
    int64_t ml = m0 + 255;
    if (ml >= a.M) ml = a.M - 1;
    const int64_t na = m0 / hw, nbb = ml / hw;
    g0 = static_cast<int>(na * (a.H + 2) + (m0 - na * hw) / a.W);
    rows = static_cast<int>(nbb * (a.H + 2) + (ml - nbb * hw) / a.W + 2) - g0 + 1;
  };
  auto gload = [&](int st) {
    const int64_t m0 = pbeg + static_cast<int64_t>(st) * 256;
    int g0, rows;
    geom(m0, g0, rows);
#pragma unroll
    for (int q = 0; q < DYCH; ++q) {
      const int idx = tid + q * NT, r = idx >> 3, cc = idx & 7;
      const int64_t m = m0 + r;
      ry[q] = m < pend ? *reinterpret_cast<const us8*>(a.dY + m * a.N + n0 + cc * 8) : us8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    const int np = rows * Wp;
#pragma unroll
    for (int q = 0; q < XCH; ++q) {
      const int idx = tid + q * NT, pp = idx >> 3, cc = idx & 7;
      us8 v = us8{0, 0, 0, 0, 0, 0, 0, 0};
      if (pp < np) {
        const int gr = g0 + pp / Wp, wp = pp - (pp / Wp) * Wp;
        const int n = gr / (a.H + 2), h = gr - n * (a.H + 2) - 1, x = wp - 1;
        if (h >= 0 && h < a.H && x >= 0 && x < a.W)
          v = *reinterpret_cast<const us8*>(a.X + ((static_cast<int64_t>(n) * a.H + h) * a.W + x) * a.Cin + c0 + cc * 8);
      }
      rx[q] = v;
    }
  };
  auto lstore = [&](int st) {
    const int64_t m0 = pbeg + static_cast<int64_t>(st) * 256;
    geom(m0, g0s, rows_s);
#pragma unroll
    for (int q = 0; q < DYCH; ++q) {
      const int idx = tid + q * NT, r = idx >> 3, cc = idx & 7;
      *reinterpret_cast<us8*>(dys + (r >> 5) * 4096 + wswz(r & 31, cc)) = ry[q];
    }
    const int np = rows_s * Wp;
#pragma unroll
    for (int q = 0; q < XCH; ++q) {
      const int idx = tid + q * NT, pp = idx >> 3, cc = idx & 7;
      if (pp < np) *reinterpret_cast<us8*>(xps + wswz(pp, cc)) = rx[q];
    }
    if (tid < 256) {  // patch row of output pixel m0 + tid at tap (0, 0); rows past M read row 0 (dY = 0)
      int64_t m = m0 + tid;
      int r = 0;
      if (m < pend) {
        const int64_t n = m / hw;
        const int rem = static_cast<int>(m - n * hw);
        const int ho = rem / a.W, wo = rem - ho * a.W;
        r = static_cast<int>(n * (a.H + 2) + ho - g0s) * Wp + wo;
      }
      prow[tid] = r;
    }
  };

  f32x4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  if (nst > 0) {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    if (st + 1 < nst) gload(st + 1);
#pragma unroll 1
    for (int ks = 0; ks < 8; ++ks) {
      bf16x8 af[2];  // dY^T: 2 x (16 Cout x 32 pixels)
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = wtr_frag(dys + ks * 4096, nh * 32 + i * 16, lane);
      // this lane's two K rows (pixels) of the B reads: 8g + q4 and 8g + 4 + q4
      const int r0 = prow[ks * 32 + 8 * g + q4], r1 = prow[ks * 32 + 8 * g + 4 + q4];
      const int col = cb * 16 + 4 * p4;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int toff = (tap / 3) * Wp + (tap % 3);
        const int o0 = wswz(r0 + toff, col >> 3) + ((col & 4) << 1);
        const int o1 = wswz(r1 + toff, col >> 3) + ((col & 4) << 1);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xps + o0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xps + o1));
        const bf16x8 bfr = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][tap] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][tap], 0, 0, 0);
      }
    }
    __syncthreads();
    if (st + 1 < nst) {
      lstore(st + 1);
      __syncthreads();
    }
  }
  float* out = a.P + static_cast<int64_t>(split) * a.N * RSC;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + nh * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int c = c0 + cb * 16 + (lane & 15);
        out[static_cast<int64_t>(n) * RSC + t * a.Cin + c] = acc[i][t][r];
      }
#endif
}

// ------------------------------------------------------------------------------------------------
// stemp_wgrad: weight gradient of the ResNet stem (7x7 / stride 2 / pad 3 over 4-channel NHWC
// images) in the packed layout of det_conv's stem GEMM: P[split][n][k], k = r*32 + s*4 + c over an
// 8x8x4 box (tap 7 and channel 3 carry zero weights; their gradient is computed and dropped).
// Per 256-output-pixel chunk the block stages dY [256][64] and the input rows the chunk reads
// (<= 14 padded rows x (W + 6) pixels x 8 B) once; the B fragment of column block (r, s0..s0+3) is
// 4 transposed reads per lane pair straight from the patch: lane (q, p) addresses the input pixel
// (2 ho - 3 + r, 2 wo - 3 + s0 + p) of K row q -- its 4 channels are the 8 contiguous bytes the
// transposed read takes.  Replaces MIOpen's NHWC C=4 wrw kernel (0.46 ms/step at batch 512).
// Wave w: Cout rows 32 (w & 1) .. +32, packed columns 64 (w >> 1) .. +64 (two r values).
// ------------------------------------------------------------------------------------------------
struct SpArgs {
  const unsigned short* dY;  // [M, 64]
  const unsigned short* X;   // [Nb, Hi, Wi, 4]
  float* P;                  // [splits, 64, 256]
  int64_t M;
  int Hi, Wi, Ho, Wo;
  int rows_per_split;        // multiple of 256
  // ABN (nullable): dY is the stem BatchNorm's backward apply, computed while staging:
  // dY = coef[0][c] * dY_in + coef[1][c] * bn_x + coef[2][c] (dY_in = the BN's masked output gradient,
  // bn_x = its input [M, 64]); the materialised input gradient of the BN is never written
  const unsigned short* bn_x;
  const float* coef;  // [3][64]
};
constexpr int kSpPMAX = 14 * 240;  // padded input pixels per chunk (Wi <= 234)
constexpr int kSpSMEM = 256 * 128 + kSpPMAX * 8 + 256 * 4;

template <bool ABN>
__global__ void __launch_bounds__(512, 1) stemp_wgrad_kernel(SpArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((ext_vector_type(4))) short s16x4;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef __attribute__((ext_vector_type(4))) unsigned short us4;
  constexpr int NT = 512, DYCH = 256 * 8 / NT, XCH = (kSpPMAX * 8 / 16 + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* dys = smem;
  unsigned char* xps = smem + 256 * 128;
  int* prow = reinterpret_cast<int*>(smem + 256 * 128 + kSpPMAX * 8);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nh = w & 1, cq = w >> 1;
  const int64_t pbeg = static_cast<int64_t>(blockIdx.x) * a.rows_per_split;
  int64_t pend = pbeg + a.rows_per_split;
  if (pend > a.M) pend = a.M;
  const int nst = pend > pbeg ? static_cast<int>((pend - pbeg + 255) / 256) : 0;
  const int Hp = a.Hi + 6, Wp = a.Wi + 6;  // 3 pixels of zero padding on every side
  const int64_t hw = static_cast<int64_t>(a.Ho) * a.Wo;

  us8 ry[DYCH], rx[XCH], rz[ABN ? DYCH : 1];
  float ca[8], cb[8], cc8[8];  // ABN: this thread's 8 channels (tid & 7) of the apply coefficients
  if constexpr (ABN) {
    const int c0 = (tid & 7) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ca[j] = a.coef[c0 + j];
      cb[j] = a.coef[64 + c0 + j];
      cc8[j] = a.coef[128 + c0 + j];
    }
  }
  auto geom = [&](int64_t m0, int& g0, int& rows) {
    int64_t ml = m0 + 255;
    if (ml >= a.M) ml = a.M - 1;
    const int64_t na = m0 / hw, nb = ml / hw;
    g0 = static_cast<int>(na * Hp + 2 * ((m0 - na * hw) / a.Wo));
    rows = static_cast<int>(nb * Hp + 2 * ((ml - nb * hw) / a.Wo) + 7) - g0 + 1;
  };
  auto gload = [&](int st) {
    const int64_t m0 = pbeg + static_cast<int64_t>(st) * 256;
    int g0, rows;
    geom(m0, g0, rows);
#pragma unroll
    for (int q = 0; q < DYCH; ++q) {
      const int idx = tid + q * NT, r = idx >> 3, cc = idx & 7;
      const int64_t m = m0 + r;
      ry[q] = m < pend ? *reinterpret_cast<const us8*>(a.dY + m * 64 + cc * 8) : us8{0, 0, 0, 0, 0, 0, 0, 0};
      if constexpr (ABN)
        rz[q] = m < pend ? *reinterpret_cast<const us8*>(a.bn_x + m * 64 + cc * 8) : us8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    // the patch in 16-B pieces = 2 padded pixels of 4 channels
    const int npc = (rows * Wp + 1) / 2;
#pragma unroll
    for (int q = 0; q < XCH; ++q) {
      const int idx = tid + q * NT;
      us8 v = us8{0, 0, 0, 0, 0, 0, 0, 0};
      if (idx < npc) {
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int pp = 2 * idx + h2;
          const int gr = g0 + pp / Wp, wp = pp - (pp / Wp) * Wp;
          const int n = gr / Hp, h = gr - n * Hp - 3, x = wp - 3;
          if (pp < rows * Wp && h >= 0 && h < a.Hi && x >= 0 && x < a.Wi) {
            const us4 px = *reinterpret_cast<const us4*>(a.X + ((static_cast<int64_t>(n) * a.Hi + h) * a.Wi + x) * 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[h2 * 4 + j] = px[j];
          }
        }
      }
      rx[q] = v;
    }
  };
  auto lstore = [&](int st) {
    const int64_t m0 = pbeg + static_cast<int64_t>(st) * 256;
    int g0, rows;
    geom(m0, g0, rows);
#pragma unroll
    for (int q = 0; q < DYCH; ++q) {
      const int idx = tid + q * NT, r = idx >> 3, cc = idx & 7;
      us8 v = ry[q];
      if constexpr (ABN) {
        // exactly det_norm.hip bn_apply_bwd<MASK 0>: fma(A, d, fma(B, x, C)) in fp32, one rounding;
        // rows past the end stay zero
        if (m0 + r < pend) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[j] = f2bf(__fmaf_rn(ca[j], bf2f(ry[q][j]), __fmaf_rn(cb[j], bf2f(rz[q][j]), cc8[j])));
        }
      }
      *reinterpret_cast<us8*>(dys + (r >> 5) * 4096 + wswz(r & 31, cc)) = v;
    }
    const int npc = (rows * Wp + 1) / 2;
#pragma unroll
    for (int q = 0; q < XCH; ++q) {
      const int idx = tid + q * NT;
      if (idx < npc) *reinterpret_cast<us8*>(xps + idx * 16) = rx[q];
    }
    if (tid < 256) {  // padded-patch pixel of (row 2 ho, col 2 wo) for output pixel m0 + tid
      const int64_t m = m0 + tid;
      int r = 0;
      if (m < pend) {
        const int64_t n = m / hw;
        const int rem = static_cast<int>(m - n * hw);
        const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
        r = static_cast<int>(n * Hp + 2 * ho - g0) * Wp + 2 * wo;
      }
      prow[tid] = r;
    }
  };

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  if (nst > 0) {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    if (st + 1 < nst) gload(st + 1);
#pragma unroll 1
    for (int ks = 0; ks < 8; ++ks) {
      bf16x8 af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = wtr_frag(dys + ks * 4096, nh * 32 + i * 16, lane);
      const int r0 = prow[ks * 32 + 8 * g + q4], r1 = prow[ks * 32 + 8 * g + 4 + q4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cb = cq * 4 + j;            // 16-column block: r = cb / 2, s0 = 4 (cb % 2)
        const int off = (cb >> 1) * Wp + (cb & 1) * 4 + p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xps + (r0 + off) * 8));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xps + (r1 + off) * 8));
        const bf16x8 bfr = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
    if (st + 1 < nst) {
      lstore(st + 1);
      __syncthreads();
    }
  }
  float* out = a.P + static_cast<int64_t>(blockIdx.x) * 64 * 256;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = nh * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int k = (cq * 4 + j) * 16 + (lane & 15);
        out[n * 256 + k] = acc[i][j][r];
      }
#endif
}

// out[i] = scale * sum_s P[s][i]  (fp32 slabs -> bf16 or fp32), deterministic: a block owns E float4
// columns and L = 256 / E split lanes (lane l sums splits l, l+L, ...), then lane 0 of each column
// adds the L lane sums in order.  L > 1 when the output is small and the split count large (the
// layer-1 shapes: 4096 outputs x ~1000 splits would otherwise run on a handful of workgroups).
template <typename TO>
__global__ void __launch_bounds__(256) wg_reduce_kernel(const float* __restrict__ P, int S, int64_t n, float scale,
                                                        TO* __restrict__ out, int E) {
  __shared__ float4 part[256];
  const int L = 256 / E;
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

// wgrad tile configurations: {BM (output channels), BN (R*S*Cin columns), waves, occupancy, KB}
struct WgCfg {
  int bm, bn, nw, occ, kb;
};
constexpr WgCfg kWgCfgs[] = {
    {0, 0, 0, 0, 0},
    {64, 192, 4, 2, 1},    // 1: 1 x 4 waves of 64 x 48 (Cout 64 at 3 x 3: 576 = 3 x 192)
    {128, 384, 8, 1, 1},   // 2: 2 x 4 waves of 64 x 96 (Cout 128 at 3 x 3: 1152 = 3 x 384)
    {256, 256, 8, 1, 1},   // 3: 2 x 4 waves of 128 x 64
    {128, 128, 4, 2, 1},   // 4: 2 x 2 waves of 64 x 64
    {64, 256, 4, 2, 1},    // 5: 1 x 4 waves of 64 x 64
    {256, 128, 8, 1, 1},   // 6: 4 x 2 waves of 64 x 64
    {128, 256, 8, 1, 1},   // 7: 2 x 4 waves of 64 x 64
    {64, 128, 4, 1, 2},    // 8: 1 x 4 waves of 64 x 32, 64 pixels per stage
    {64, 64, 4, 2, 2},     // 9: 2 x 2 waves of 32 x 32, 64 pixels per stage
    {256, 64, 4, 2, 1},    // 10: 4 x 1 waves of 64 x 64
    {128, 64, 4, 1, 2},    // 11: 2 x 2 waves of 64 x 32, 64 pixels per stage
    {64, 192, 4, 1, 2},    // 12: cfg 1 at 64 pixels per stage
    {64, 64, 4, 1, 4},     // 13: cfg 9 at 128 pixels per stage
    {256, 256, 8, 1, 2},   // 14: wgrad8 -- cfg 3's tile on the eight-phase schedule, 64 pixels per K tile
                           //     (in isolation -2..-6 % at 256 channels, +1-2 % at 512, r6s36; in the
                           //     side-stream step at 1,024 images/GPU +0.7 %, r6s62: the default where it fits)
};
constexpr int kWgNumCfgs = sizeof(kWgCfgs) / sizeof(kWgCfgs[0]);

int wg_auto_cfg(int N, int RSC) {
  static const int forced = [] {
    const char* e = std::getenv("DET_WGRAD_CFG");
    return e ? std::atoi(e) : 0;
  }();
  auto fits = [&](int c) { return N % kWgCfgs[c].bm == 0 && RSC % kWgCfgs[c].bn == 0; };
  if (forced > 0 && forced < kWgNumCfgs && fits(forced)) return forced;
  static const bool use8 = [] {  // DET_WGRAD8=0: cfg 3 (the 4-stage ring) where cfg 14 fits
    const char* e = std::getenv("DET_WGRAD8");
    return !(e != nullptr && std::atoi(e) == 0);
  }();
  if (use8 && fits(14)) return 14;
  for (int c : {3, 2, 7, 6, 10, 1, 5, 4, 11, 8, 9})
    if (fits(c)) return c;
  return 0;
}

int wg_splits(int64_t M, int N, int RSC, int cfg) {
  const WgCfg& c = kWgCfgs[cfg];
  const int64_t tiles = static_cast<int64_t>(N / c.bm) * (RSC / c.bn);
  static const int target = [] {
    const char* e = std::getenv("DET_WGRAD_WGS");
    return e ? std::atoi(e) : 512;
  }();
  // ~two waves of workgroups over the 256 CUs (one wave: -20 % at Cout 128, profiles/r3_wgrad_ring_sweep.jsonl)
  int64_t splits = (target * c.occ + tiles - 1) / tiles;
  const int64_t max_rows = (M + 511) / 512;                  // >= 512 pixels (16 K steps) per split
  // fp32 slab traffic (write + reduce read) at most the operand bytes ...
  const int64_t max_bytes = (M * (static_cast<int64_t>(N) + RSC) * 2) / (8 * static_cast<int64_t>(N) * RSC);
  if (splits > max_bytes) splits = max_bytes;
  // ... but never fewer workgroups than one per CU slot (small-M deep layers)
  const int64_t one_wave = (256 * c.occ + tiles - 1) / tiles;
  if (splits < one_wave) splits = one_wave;
  if (splits > max_rows) splits = max_rows;
  if (splits < 1) splits = 1;
  return static_cast<int>(splits);
}

template <int BM, int BN, int WM, int WN, int OCC, int KB>
void launch_wg(hipStream_t st, const WgArgs& a, int nwg) {
  constexpr int NS = 4;
  constexpr int smem = NS * KB * (BM + BN) * 64;
  static_assert(smem * OCC <= 163840, "LDS");
  hipLaunchKernelGGL((wgrad3_kernel<BM, BN, WM, WN, NS, KB, OCC>), dim3(nwg), dim3(WM * WN * 64), smem, st, a);
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// stemp_fwd: the ResNet stem forward Y[M, 64] = im2col(X) . W^T (7x7 / stride 2 / pad 3 over
// 4-channel NHWC images, W packed k = r*32 + s*4 + c) on stemp_wgrad's input patch.  The implicit
// GEMM of det_conv (GM_STEM) gathers every A fragment from global memory -- each input pixel is
// fetched ~12 times (49 taps / stride 4) through L2 and the MFMAs wait on it (0.58 ms/step at batch
// 512, 27 % of the bandwidth bound).  Here a block stages the <= 14 padded input rows of a 256-pixel
// chunk once into LDS; an A fragment (row m, k-group g of k-step r) is then the 16 contiguous bytes
// of padded pixels (2 ho + r, 2 wo + 2g .. 2g + 1) -- two 8-B LDS reads, no transposes.  The weights
// (32 KB) stay resident in LDS for the whole run: persistent blocks walk a contiguous range of chunks
// (the next chunk's halo rows are this chunk's, so their re-read hits L2), prefetching the next
// patch into registers under the MFMAs.  The k order (8 steps of 32) is the GEMM kernel's, so the
// outputs are bit-identical to det_stem_conv_fwd.  Epilogue: BN statistics partials per 256 rows
// (det_stats.h) and a C tile restaged in LDS for coalesced 16-B row stores.
// Wave w: rows 32 w .. +32, all 64 filters (2 x 4 MFMA 16x16x32 tiles).
// ------------------------------------------------------------------------------------------------
struct SfArgs {
  const unsigned short* X;  // [Nb, Hi, Wi, 4]
  const unsigned short* W;  // [64, 256] packed
  unsigned short* Y;        // [M, 64]
  float* pmean;             // [ceil(M / 256), 64] (nullable, with pm2)
  float* pm2;
  int64_t M;
  int Hi, Wi, Ho, Wo;
  int chunks_per_block;
};
constexpr int kSfLDC = 72;                     // C tile row pitch (elements): 16-B stores conflict-free
constexpr int kSfU = 256 * kSfLDC * 2;         // patch + prow while computing, the C tile after
static_assert(kSpPMAX * 8 + 256 * 4 <= kSfU, "patch region");
constexpr int kSfSMEM = 64 * 256 * 2 + kSfU + 3 * 8 * 64 * 4;  // weights | patch / C tile | stats

template <bool STATS>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) stemp_fwd_kernel(SfArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((ext_vector_type(4))) unsigned short us4;
  typedef __attribute__((ext_vector_type(4))) short s16x4;
  constexpr int NT = 512, XCH = (kSpPMAX * 8 / 16 + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* wl = smem;
  unsigned char* xps = smem + 64 * 256 * 2;
  int* prow = reinterpret_cast<int*>(xps + kSpPMAX * 8);
  unsigned short* ct = reinterpret_cast<unsigned short*>(xps);
  float* red = reinterpret_cast<float*>(smem + 64 * 256 * 2 + kSfU);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int64_t nch = (a.M + 255) / 256;
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * a.chunks_per_block;
  int64_t c1 = c0 + a.chunks_per_block;
  if (c1 > nch) c1 = nch;
  if (c0 >= c1) return;  // uniform over the block, before any barrier
  const int Hp = a.Hi + 6, Wp = a.Wi + 6;
  const int64_t hw = static_cast<int64_t>(a.Ho) * a.Wo;

  // the weights, [k-step][filter][4 x 16 B] swizzled: 2048 16-B pieces
#pragma unroll
  for (int q = 0; q < 64 * 32 / NT; ++q) {
    const int idx = tid + q * NT, n = idx >> 5, ch = idx & 31;
    *reinterpret_cast<us8*>(wl + (ch >> 2) * 4096 + swz64(n, ch & 3)) =
        *reinterpret_cast<const us8*>(a.W + n * 256 + ch * 8);
  }
  us8 rx[XCH];
  auto geom = [&](int64_t m0, int& g0, int& rows) {
    int64_t ml = m0 + 255;
    if (ml >= a.M) ml = a.M - 1;
    const int64_t na = m0 / hw, nb = ml / hw;
    g0 = static_cast<int>(na * Hp + 2 * ((m0 - na * hw) / a.Wo));
    rows = static_cast<int>(nb * Hp + 2 * ((ml - nb * hw) / a.Wo) + 7) - g0 + 1;
  };
  auto gload = [&](int64_t m0) {
    int g0, rows;
    geom(m0, g0, rows);
    const int npc = (rows * Wp + 1) / 2;  // 16-B pieces = 2 padded pixels of 4 channels
#pragma unroll
    for (int q = 0; q < XCH; ++q) {
      const int idx = tid + q * NT;
      us8 v = us8{0, 0, 0, 0, 0, 0, 0, 0};
      if (idx < npc) {
        // one division pair per piece: the second pixel is the first's right neighbour
        const int pp0 = 2 * idx, q0 = pp0 / Wp;
        int gr = g0 + q0, wp = pp0 - q0 * Wp, n = gr / Hp, h = gr - n * Hp - 3;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          if (h2 == 1 && ++wp == Wp) {
            wp = 0;
            if (++h == a.Hi + 3) {
              h = -3;
              ++n;
            }
          }
          const int x = wp - 3;
          if (pp0 + h2 < rows * Wp && h >= 0 && h < a.Hi && x >= 0 && x < a.Wi) {
            const us4 px = *reinterpret_cast<const us4*>(a.X + ((static_cast<int64_t>(n) * a.Hi + h) * a.Wi + x) * 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[h2 * 4 + j] = px[j];
          }
        }
      }
      rx[q] = v;
    }
  };
  auto lstore = [&](int64_t m0) {
    int g0, rows;
    geom(m0, g0, rows);
    const int npc = (rows * Wp + 1) / 2;
#pragma unroll
    for (int q = 0; q < XCH; ++q) {
      const int idx = tid + q * NT;
      if (idx < npc) *reinterpret_cast<us8*>(xps + idx * 16) = rx[q];
    }
    if (tid < 256) {  // padded-patch pixel (row 2 ho, col 2 wo) of output pixel m0 + tid
      const int64_t m = m0 + tid;
      int r = 0;
      if (m < a.M) {
        const int64_t n = m / hw;
        const int rem = static_cast<int>(m - n * hw);
        const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
        r = static_cast<int>(n * Hp + 2 * ho - g0) * Wp + 2 * wo;
      }
      prow[tid] = r;
    }
  };

  gload(c0 * 256);
  lstore(c0 * 256);
  __syncthreads();
  for (int64_t c = c0; c < c1; ++c) {
    const int64_t m0 = c * 256;
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int pr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) pr[i] = prow[w * 32 + i * 16 + (lane & 15)] + 2 * g;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      bf16x8 fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        // 8-B aligned only (odd Wp): two 8-B reads
        const unsigned char* p = xps + (pr[i] + ks * Wp) * 8;
        const s16x4 lo = *reinterpret_cast<const s16x4*>(p), hi = *reinterpret_cast<const s16x4*>(p + 8);
        fa[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(wl + ks * 4096 + swz64(j * 16 + (lane & 15), g));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);  // one k-step's fragments in flight (registers)
    }
    __syncthreads();  // every wave is done with the patch: the C tile overlays it
    const int64_t rows_left = a.M - m0;
    const int nvalid = rows_left < 256 ? static_cast<int>(rows_left) : 256;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ct[(w * 32 + i * 16 + g * 4 + r) * kSfLDC + j * 16 + (lane & 15)] = f2bf(acc[i][j][r]);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 256 * 8 / NT; ++q) {
      const int idx = tid + q * NT, row = idx >> 3, cc = idx & 7;
      if (row < nvalid)
        *reinterpret_cast<us8*>(a.Y + (m0 + row) * 64 + cc * 8) = *reinterpret_cast<const us8*>(ct + row * kSfLDC + cc * 8);
    }
    if constexpr (STATS)  // after the stores are issued (red is its own LDS region)
      det_block_bn_stats<2, 4, 8, 32, 64, 64>(acc, red, w, 0, lane, tid, nvalid, a.pmean, a.pm2, c * 64);
    if (c + 1 < c1) {
      // the next chunk's patch: fetched here, not under the MFMAs or the epilogue (both spill at
      // 4 waves / SIMD); the other block on the CU computes meanwhile
      gload(m0 + 256);
      __syncthreads();  // the C tile is consumed before the next patch lands there
      lstore(m0 + 256);
      __syncthreads();
    }
  }
#endif
}

extern "C" {

// fp32 workspace elements det_igemm_wgrad needs for an [N, R*S*Cin] output from M pixels.
int64_t det_igemm_wgrad_ws_elems(int64_t M, int N, int RSC, int cfg) {
  const int c = cfg > 0 && cfg < kWgNumCfgs ? cfg : wg_auto_cfg(N, RSC);
  if (c == 0 || N % kWgCfgs[c].bm != 0 || RSC % kWgCfgs[c].bn != 0) return 0;  // no tile fits
  return static_cast<int64_t>(wg_splits(M, N, RSC, c)) * N * RSC;
}

// Weight gradient of an R x S convolution (stride, pad) over NHWC bf16 on the LDS-DMA ring:
//   dW[N, R*S*Cin] (KRSC; out_dtype 0 fp32 / 1 bf16) = out_scale * dY[M, N]^T . im2col(X)[M, R*S*Cin]
// as split-pixel fp32 slabs in ws (>= det_igemm_wgrad_ws_elems) reduced by a second launch.
// N % 64 == 0, R*S*Cin divisible by the tile, Cin % 8 == 0, operands < 2 GiB, 16-B aligned.
int det_igemm_wgrad(void* stream, const void* dY, const void* X, void* out, int out_dtype, int64_t M, int N, int Cin,
                    int Hi, int Wi, int Ho, int Wo, int R, int S, int stride, int pad, float* ws, float out_scale,
                    int cfg) {
  if (M <= 0 || N <= 0 || Cin <= 0 || Cin % 8 != 0 || R <= 0 || S <= 0 || stride <= 0 || pad < 0) return -1;
  const int64_t hw = static_cast<int64_t>(Ho) * Wo;
  if (hw <= 0 || M % hw != 0) return -3;
  if (Ho != (Hi + 2 * pad - R) / stride + 1 || Wo != (Wi + 2 * pad - S) / stride + 1) return -3;
  if (((reinterpret_cast<uintptr_t>(dY) | reinterpret_cast<uintptr_t>(X)) & 15) != 0) return -5;
  const int RSC = R * S * Cin;
  const int c = cfg > 0 && cfg < kWgNumCfgs ? cfg : wg_auto_cfg(N, RSC);
  if (c == 0 || N % kWgCfgs[c].bm != 0 || RSC % kWgCfgs[c].bn != 0) return -6;
  const int64_t dy_bytes = M * N * 2, x_bytes = (M / hw) * Hi * static_cast<int64_t>(Wi) * Cin * 2;
  if (dy_bytes >= (static_cast<int64_t>(1) << 31) || x_bytes >= (static_cast<int64_t>(1) << 31)) return -8;
  const int splits = wg_splits(M, N, RSC, c);
  int64_t rps = (M + splits - 1) / splits;
  const int sk = 32 * kWgCfgs[c].kb;
  rps = (rps + sk - 1) / sk * sk;
  const int real_splits = static_cast<int>((M + rps - 1) / rps);
  WgArgs a{static_cast<const unsigned short*>(dY), static_cast<const unsigned short*>(X), ws, M, N, RSC, Cin, Hi, Wi,
           Ho, Wo, stride, pad, S, static_cast<int>(rps), static_cast<int>(dy_bytes), static_cast<int>(x_bytes)};
  const int nwg = (N / kWgCfgs[c].bm) * (RSC / kWgCfgs[c].bn) * real_splits;
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (c) {
    case 1: launch_wg<64, 192, 1, 4, 2, 1>(st, a, nwg); break;
    case 2: launch_wg<128, 384, 2, 4, 1, 1>(st, a, nwg); break;
    case 3: launch_wg<256, 256, 2, 4, 1, 1>(st, a, nwg); break;
    case 4: launch_wg<128, 128, 2, 2, 2, 1>(st, a, nwg); break;
    case 5: launch_wg<64, 256, 1, 4, 2, 1>(st, a, nwg); break;
    case 6: launch_wg<256, 128, 4, 2, 1, 1>(st, a, nwg); break;
    case 7: launch_wg<128, 256, 2, 4, 1, 1>(st, a, nwg); break;
    case 8: launch_wg<64, 128, 1, 4, 1, 2>(st, a, nwg); break;
    case 9: launch_wg<64, 64, 2, 2, 2, 2>(st, a, nwg); break;
    case 10: launch_wg<256, 64, 4, 1, 2, 1>(st, a, nwg); break;
    case 11: launch_wg<128, 64, 2, 2, 1, 2>(st, a, nwg); break;
    case 12: launch_wg<64, 192, 1, 4, 1, 2>(st, a, nwg); break;
    case 13: launch_wg<64, 64, 2, 2, 1, 4>(st, a, nwg); break;
    case 14: {
      constexpr int smem = 2 * 4 * 16384;
      hipLaunchKernelGGL(wgrad8_kernel, dim3(nwg), dim3(512), smem, st, a);
      break;
    }
    default: return -7;
  }
  const int rc = static_cast<int>(hipGetLastError());
  if (rc != 0) return rc;
  const int64_t slab = static_cast<int64_t>(N) * RSC, n4 = slab / 4;
  int lanes = 1;  // split lanes per output column: enough workgroups for small outputs
  while (lanes < 256 && lanes < real_splits && n4 / (256 / lanes) < 2048) lanes *= 2;
  const int E = 256 / lanes;
  const int grid = static_cast<int>((n4 + E - 1) / E);
  if (out_dtype == 1)
    hipLaunchKernelGGL(wg_reduce_kernel<unsigned short>, dim3(grid), dim3(256), 0, st, ws, real_splits, slab, out_scale,
                       static_cast<unsigned short*>(out), E);
  else
    hipLaunchKernelGGL(wg_reduce_kernel<float>, dim3(grid), dim3(256), 0, st, ws, real_splits, slab, out_scale,
                       static_cast<float*>(out), E);
  return static_cast<int>(hipGetLastError());
}

// conv3p_wgrad splits: enough (tile, pixel-range) blocks for the 256 CUs, >= 8 stages of 256 pixels each.
static int wp_splits(int64_t M, int ntiles) {
  int64_t s = (256 + ntiles - 1) / ntiles;
  const int64_t max_s = (M + 2047) / 2048;
  if (s > max_s) s = max_s;
  return static_cast<int>(s < 1 ? 1 : s);
}
int64_t det_conv3p_wgrad_ws_elems(int64_t M, int N, int Cin) {
  if (N % 64 || Cin % 64) return 0;
  return static_cast<int64_t>(wp_splits(M, (N / 64) * (Cin / 64))) * N * 9 * Cin;
}

// Weight gradient of a 3x3 / stride-1 / pad-1 convolution (NHWC bf16 dY [M, N] and X) on the halo
// patch (conv3p_wgrad above): out [N, 9 * Cin] (KRSC; out_dtype 0 fp32 / 1 bf16) = out_scale *
// dY^T . im2col(X), as split-pixel fp32 slabs in ws (>= det_conv3p_wgrad_ws_elems) reduced by a
// second launch.  N % 64 == 0, Cin % 64 == 0; -6 when a 256-pixel chunk's patch exceeds 640 pixels.
int det_conv3p_wgrad(void* stream, const void* dY, const void* X, void* out, int out_dtype, int Nb, int H, int W, int Cin,
                     int N, float* ws, float out_scale) {
  if (Nb <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cin % 64 != 0 || N <= 0 || N % 64 != 0) return -1;
  if (((reinterpret_cast<uintptr_t>(dY) | reinterpret_cast<uintptr_t>(X)) & 15) != 0) return -5;
  const int64_t M = static_cast<int64_t>(Nb) * H * W;
  if (p3_max_patch(M, H, W) > kP3PMAX) return -6;
  const int ntiles = (N / 64) * (Cin / 64);
  const int splits = wp_splits(M, ntiles);
  int64_t rps = (M + splits - 1) / splits;
  rps = (rps + 255) / 256 * 256;
  const int real = static_cast<int>((M + rps - 1) / rps);
  WpArgs a{static_cast<const unsigned short*>(dY), static_cast<const unsigned short*>(X), ws, M, N, Cin, H, W,
           static_cast<int>(rps), ntiles};
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(conv3p_wgrad_kernel, dim3(static_cast<unsigned>(ntiles * real)), dim3(512), kWpSMEM, st, a);
  int rc = static_cast<int>(hipGetLastError());
  if (rc != 0) return rc;
  const int64_t slab = static_cast<int64_t>(N) * 9 * Cin, n4 = slab / 4;
  int lanes = 1;
  while (lanes < 256 && lanes < real && n4 / (256 / lanes) < 2048) lanes *= 2;
  const int E = 256 / lanes;
  const int grid = static_cast<int>((n4 + E - 1) / E);
  if (out_dtype == 1)
    hipLaunchKernelGGL(wg_reduce_kernel<unsigned short>, dim3(grid), dim3(256), 0, st, ws, real, slab, out_scale,
                       static_cast<unsigned short*>(out), E);
  else
    hipLaunchKernelGGL(wg_reduce_kernel<float>, dim3(grid), dim3(256), 0, st, ws, real, slab, out_scale,
                       static_cast<float*>(out), E);
  return static_cast<int>(hipGetLastError());
}

static bool sp_patch_fits(int64_t M, int Hi, int Wi, int Ho, int Wo);

static int sp_splits(int64_t M) {
  int64_t s = 256;
  const int64_t max_s = (M + 4095) / 4096;  // >= 16 chunks of 256 pixels per block
  if (s > max_s) s = max_s;
  return static_cast<int>(s < 1 ? 1 : s);
}
int64_t det_stemp_wgrad_ws_elems(int64_t M) { return static_cast<int64_t>(sp_splits(M)) * 64 * 256; }

// ResNet stem weight gradient (7x7 / stride 2 / pad 3, 64 filters, NHWC input padded to 4 channels)
// on the patch kernel above: out [64, 256] (packed k = r*32 + s*4 + c; fp32 or bf16) = out_scale *
// sum over pixels, via split fp32 slabs in ws (>= det_stemp_wgrad_ws_elems(M)).  -6 for widths the
// patch cannot hold (Wi > 234).
// bn_x / coef (nullable, both or neither): dY is the stem BatchNorm's backward apply of the given
// masked gradient (SpArgs ABN).
int det_stemp_wgrad(void* stream, const void* dY, const void* X, void* out, int out_dtype, int64_t M, int Hi, int Wi,
                    int Ho, int Wo, float* ws, float out_scale, const void* bn_x, const float* coef) {
  if (M <= 0 || Hi <= 0 || Wi <= 0 || Ho != (Hi - 1) / 2 + 1 || Wo != (Wi - 1) / 2 + 1) return -1;
  if (M % (static_cast<int64_t>(Ho) * Wo) != 0) return -1;
  if (!sp_patch_fits(M, Hi, Wi, Ho, Wo)) return -6;
  if ((bn_x == nullptr) != (coef == nullptr)) return -2;
  if (((reinterpret_cast<uintptr_t>(dY) | reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(bn_x)) & 15) != 0)
    return -5;
  const int splits = sp_splits(M);
  int64_t rps = (M + splits - 1) / splits;
  rps = (rps + 255) / 256 * 256;
  const int real = static_cast<int>((M + rps - 1) / rps);
  SpArgs a{static_cast<const unsigned short*>(dY), static_cast<const unsigned short*>(X), ws, M, Hi, Wi, Ho, Wo,
           static_cast<int>(rps), static_cast<const unsigned short*>(bn_x), coef};
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (bn_x)
    hipLaunchKernelGGL(stemp_wgrad_kernel<true>, dim3(static_cast<unsigned>(real)), dim3(512), kSpSMEM, st, a);
  else
    hipLaunchKernelGGL(stemp_wgrad_kernel<false>, dim3(static_cast<unsigned>(real)), dim3(512), kSpSMEM, st, a);
  int rc = static_cast<int>(hipGetLastError());
  if (rc != 0) return rc;
  const int64_t slab = 64 * 256, n4 = slab / 4;
  int lanes = 1;
  while (lanes < 256 && lanes < real && n4 / (256 / lanes) < 2048) lanes *= 2;
  const int E = 256 / lanes;
  const int grid = static_cast<int>((n4 + E - 1) / E);
  if (out_dtype == 1)
    hipLaunchKernelGGL(wg_reduce_kernel<unsigned short>, dim3(grid), dim3(256), 0, st, ws, real, slab, out_scale,
                       static_cast<unsigned short*>(out), E);
  else
    hipLaunchKernelGGL(wg_reduce_kernel<float>, dim3(grid), dim3(256), 0, st, ws, real, slab, out_scale,
                       static_cast<float*>(out), E);
  return static_cast<int>(hipGetLastError());
}

// Host side: do the input rows of every 256-pixel chunk fit the stem patch (kSpPMAX pixels)?  A
// chunk that straddles two images spans both images' rows plus the padding between them; cached
// per shape (one pass over the chunks, the first call of a shape only).
static bool sp_patch_fits(int64_t M, int Hi, int Wi, int Ho, int Wo) {
  thread_local int64_t key_m = -1;
  thread_local int key_h = -1, key_w = -1;
  thread_local bool key_ok = false;
  if (M == key_m && Hi == key_h && Wi == key_w) return key_ok;
  const int64_t Hp = Hi + 6, Wp = Wi + 6, hw = static_cast<int64_t>(Ho) * Wo;
  bool ok = Wp <= 240;
  for (int64_t m0 = 0; ok && m0 < M; m0 += 256) {
    int64_t ml = m0 + 255;
    if (ml >= M) ml = M - 1;
    const int64_t na = m0 / hw, nb = ml / hw;
    const int64_t rows = nb * Hp + 2 * ((ml - nb * hw) / Wo) + 8 - (na * Hp + 2 * ((m0 - na * hw) / Wo));
    ok = rows * Wp <= kSpPMAX;
  }
  key_m = M;
  key_h = Hi;
  key_w = Wi;
  key_ok = ok;
  return ok;
}

int det_stemp_fwd_rows_per_block() { return 256; }

// ResNet stem convolution on the patch kernel above (same contract as det_conv's det_stem_conv_fwd,
// except that the statistics partials pmean / pm2 are per det_stemp_fwd_rows_per_block() rows).
// -6: a chunk's input rows do not fit the patch (very wide images) -- use det_stem_conv_fwd.
int det_stemp_fwd(void* stream, const void* X, const void* W, void* Y, int64_t M, int Hi, int Wi, int Ho, int Wo,
                  float* pmean, float* pm2) {
  if (M <= 0 || Hi <= 0 || Wi <= 0 || Ho != (Hi - 1) / 2 + 1 || Wo != (Wi - 1) / 2 + 1) return -1;
  if (M % (static_cast<int64_t>(Ho) * Wo) != 0) return -1;
  if ((pmean == nullptr) != (pm2 == nullptr)) return -2;
  if (((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(Y)) & 15) != 0)
    return -5;
  if (!sp_patch_fits(M, Hi, Wi, Ho, Wo)) return -6;
  const int64_t nch = (M + 255) / 256;
  // two blocks per CU over 256 CUs; at least 4 chunks a block so the weight staging amortises
  int64_t blocks = 512;
  if (blocks > (nch + 3) / 4) blocks = (nch + 3) / 4;
  const int64_t cpb = (nch + blocks - 1) / blocks;
  if (cpb >= (static_cast<int64_t>(1) << 30)) return -4;
  blocks = (nch + cpb - 1) / cpb;
  SfArgs a{static_cast<const unsigned short*>(X), static_cast<const unsigned short*>(W), static_cast<unsigned short*>(Y),
           pmean, pm2, M, Hi, Wi, Ho, Wo, static_cast<int>(cpb)};
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (pmean)
    hipLaunchKernelGGL(stemp_fwd_kernel<true>, dim3(static_cast<unsigned>(blocks)), dim3(512), kSfSMEM, st, a);
  else
    hipLaunchKernelGGL(stemp_fwd_kernel<false>, dim3(static_cast<unsigned>(blocks)), dim3(512), kSfSMEM, st, a);
  return static_cast<int>(hipGetLastError());
}

// out[C][R*S*K] bf16 = the flipped, transposed KRSC weight the stride-1 input gradient convolves with.
// det_conv_dgrad_weight for n weights in one launch per kDwMulti: w[i] (KRSC, fp32 or bf16 per
// dims[i*5+4] = 1 for bf16) -> out[i] (bf16 [C, R*S*K]); dims[i*5 .. +3] = K, C, R, S.
int det_conv_dgrad_weight_multi(void* stream, int n, const int64_t* w, const int64_t* out, const int* dims) {
  if (n <= 0) return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  for (int b = 0; b < n; b += kDwMulti) {
    DwMultiArgs a{};
    a.n = n - b < kDwMulti ? n - b : kDwMulti;
    int64_t total = 0;
    for (int i = 0; i < a.n; ++i) {
      const int* d = dims + 5 * (b + i);
      if (d[0] <= 0 || d[1] <= 0 || d[2] <= 0 || d[3] <= 0) return -1;
      a.K[i] = d[0]; a.C[i] = d[1]; a.R[i] = d[2]; a.S[i] = d[3]; a.bf16[i] = d[4];
      a.w[i] = reinterpret_cast<const void*>(w[b + i]);
      a.out[i] = reinterpret_cast<unsigned short*>(out[b + i]);
      a.start[i] = static_cast<int>(total);
      total += static_cast<int64_t>((d[1] + 63) / 64) * ((d[0] + 63) / 64) * d[2] * d[3];
      if (total >= (static_cast<int64_t>(1) << 31)) return -3;
    }
    a.start[a.n] = static_cast<int>(total);
    hipLaunchKernelGGL(dgrad_weight_multi_kernel, dim3(static_cast<unsigned>(total)), dim3(256), 0, st, a);
    const int rc = static_cast<int>(hipGetLastError());
    if (rc != 0) return rc;
  }
  return 0;
}

int det_conv_dgrad_weight(void* stream, const void* W, int in_dtype, void* out, int K, int C, int R, int S) {
  if (K <= 0 || C <= 0 || R <= 0 || S <= 0) return -1;
  const dim3 grid((C + 63) / 64, (K + 63) / 64, R * S);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (in_dtype == 1)
    hipLaunchKernelGGL(dgrad_weight_kernel<unsigned short>, grid, dim3(256), 0, st,
                       static_cast<const unsigned short*>(W), static_cast<unsigned short*>(out), K, C, R, S);
  else
    hipLaunchKernelGGL(dgrad_weight_kernel<float>, grid, dim3(256), 0, st, static_cast<const float*>(W),
                       static_cast<unsigned short*>(out), K, C, R, S);
  return static_cast<int>(hipGetLastError());
}

// Rows per statistics block of det_igemm for configuration cfg (0 = the automatic choice for N).
int det_igemm_rows_per_block_cfg(int N, int cfg) {
  IgArgs a{};
  a.N = N;
  const int c = cfg > 0 ? cfg : auto_cfg(a);
  return (c == 4 || c == 6 || c == 7 || c == 19 || c == 20) ? 128 : (((c >= 12 && c <= 15) || c == 22) ? 512 : 256);
}
int det_igemm_rows_per_block() { return 256; }

// Y[M, N] = conv(X, W) as described at the top.  bf16 NHWC.  Requirements (checked): Cin % 64 == 0,
// N % 64 == 0, K == R*S*Cin, pointers 16-B aligned, zero -> >= 128 zero bytes.  R == S == 1,
// stride 1, pad 0 with Hi*Wi == Ho*Wo takes the dense path.  pmean/pm2 (nullable, [ceil(M/rpb), N],
// rpb = det_igemm_rows_per_block_cfg(N, cfg)): BatchNorm statistics partials of the bf16-rounded Y.
int det_igemm_conv_cfg(void* stream, const void* X, const void* W, void* Y, const void* zero, int64_t M, int N, int Cin,
                       int Hi, int Wi, int Ho, int Wo, int R, int S, int stride, int pad, float* pmean, float* pm2,
                       int cfg) {
  if (M <= 0 || N <= 0 || N % 64 != 0 || Cin <= 0 || Cin % 32 != 0 || R <= 0 || S <= 0 || stride <= 0 || pad < 0)
    return -1;
  if ((pmean == nullptr) != (pm2 == nullptr) || zero == nullptr) return -2;
  if (((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(Y) |
        reinterpret_cast<uintptr_t>(zero)) & 15) != 0)
    return -5;
  const int64_t hw = static_cast<int64_t>(Ho) * Wo;
  if (hw <= 0 || M % hw != 0) return -3;
  if (Ho != (Hi + 2 * pad - R) / stride + 1 || Wo != (Wi + 2 * pad - S) / stride + 1) return -3;
  const int K = R * S * Cin;
  const int64_t x_bytes = (M / hw) * Hi * static_cast<int64_t>(Wi) * Cin * 2;
  if (cfg != 1 && (x_bytes >= (static_cast<int64_t>(1) << 31) || static_cast<int64_t>(N) * K * 2 >= (static_cast<int64_t>(1) << 31)))
    return -8;  // 32-bit buffer offsets
  if (R * S > 32) return -1;
  IgArgs a{static_cast<const unsigned short*>(X), static_cast<const unsigned short*>(W), static_cast<unsigned short*>(Y),
           static_cast<const unsigned short*>(zero), pmean, pm2, M, N, K, Cin, Hi, Wi, Ho, Wo, stride, pad, S, R, x_bytes};
  const bool dense = R == 1 && S == 1 && stride == 1 && pad == 0 && Hi == Ho && Wi == Wo;
  hipStream_t st = static_cast<hipStream_t>(stream);
  return run_cfg(cfg > 0 ? cfg : auto_cfg(a), st, a, dense, pmean != nullptr);
}

// det_igemm_conv_cfg for an input gradient whose output feeds a training BatchNorm(+ReLU) backward:
// Y <- the ReLU-masked gradient d (mask = bn_x*bn_scale + bn_shift > 0) and psum / psumx
// [ceil(M/rpb), N] (rpb = det_igemm_rows_per_block_cfg(N, cfg)) = sum d, sum d (bn_x - bn_mean)
// per row block: the BN backward is then finalize + unmasked apply (det_bn_bwd_from_partials).
int det_igemm_conv_bnbwd(void* stream, const void* X, const void* W, void* Y, const void* zero, int64_t M, int N, int Cin,
                         int Hi, int Wi, int Ho, int Wo, int R, int S, int stride, int pad, const void* bn_x,
                         const float* bn_mean, const float* bn_scale, const float* bn_shift, float* psum, float* psumx,
                         int cfg) {
  if (M <= 0 || N <= 0 || N % 64 != 0 || Cin <= 0 || Cin % 32 != 0 || R <= 0 || S <= 0 || stride <= 0 || pad < 0)
    return -1;
  if (!bn_x || !bn_mean || !bn_scale || !bn_shift || !psum || !psumx || zero == nullptr) return -2;
  if (((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(Y) |
        reinterpret_cast<uintptr_t>(zero) | reinterpret_cast<uintptr_t>(bn_x)) & 15) != 0)
    return -5;
  const int64_t hw = static_cast<int64_t>(Ho) * Wo;
  if (hw <= 0 || M % hw != 0) return -3;
  if (Ho != (Hi + 2 * pad - R) / stride + 1 || Wo != (Wi + 2 * pad - S) / stride + 1) return -3;
  const int K = R * S * Cin;
  const int64_t x_bytes = (M / hw) * Hi * static_cast<int64_t>(Wi) * Cin * 2;
  if (x_bytes >= (static_cast<int64_t>(1) << 31) || static_cast<int64_t>(N) * K * 2 >= (static_cast<int64_t>(1) << 31))
    return -8;
  if (R * S > 32) return -1;
  IgArgs a{static_cast<const unsigned short*>(X), static_cast<const unsigned short*>(W), static_cast<unsigned short*>(Y),
           static_cast<const unsigned short*>(zero), nullptr, nullptr, M, N, K, Cin, Hi, Wi, Ho, Wo, stride, pad, S, R, x_bytes,
           static_cast<const unsigned short*>(bn_x), bn_mean, bn_scale, bn_shift, psum, psumx};
  hipStream_t st = static_cast<hipStream_t>(stream);
  return run_cfg(cfg > 0 ? cfg : auto_cfg(a), st, a, false, false, true);
}

// igemm3 tile configuration of the stride-2 input gradient for Cin output channels (the launch3
// family: the class gather needs the 32-deep K tiles); rows per statistics block follow from it.
static int s2_cfg(int cin, int cfg) {
  if (cfg > 0) return cfg;
  return cin % 256 == 0 ? 8 : (cin % 128 == 0 ? 9 : 11);
}
int det_igemm_dgrad_s2_rows_per_block(int Cin, int cfg) {
  return det_igemm_rows_per_block_cfg(Cin, s2_cfg(Cin, cfg));
}

// Input gradient of a 3x3 / stride-2 / pad-1 convolution (Hi = 2 Ho, Wi = 2 Wo) without MIOpen:
//   dX[n, h, w, c] = sum_{r,s,k} dY[n, (h+1-r)/2, (w+1-s)/2, k] W[k][c][r][s]   ((h+1-r), (w+1-s) even)
// Output pixels of one parity class (h % 2, w % 2) = (ph, pw) see only the taps r == ph + 1 (mod 2):
// ph = 0 -> r = 1; ph = 1 -> r in {2, 0} at dY rows i, i + 1 (h = 2i + ph), likewise for w.  So each
// class is a stride-1, pad-0 implicit GEMM over dY with a (1+ph) x (1+pw) kernel whose B taps are
// gathered from the flipped dgrad weight Wd [Cin][9 * Cout] (det_conv_dgrad_weight: tap r' = 2 - r)
// through `tapmap`, and whose output rows scatter to the class's pixels (`oscat`): 2.25 taps per
// pixel on average, no zero-inserted MACs (a dilated stride-1 conv would do 9).  Four launches.
// bn_x..psumx (all or none): the BNB epilogue of the BatchNorm(+ReLU) whose output this is (mask
// mode 1), partials [4 * ceil(Nb*Ho*Wo / rpb), Cin], rpb = det_igemm_dgrad_s2_rows_per_block.
int det_igemm_dgrad_s2(void* stream, const void* dY, const void* Wd, void* dX, const void* zero, int Nb, int Ho, int Wo,
                       int Cout, int Cin, const void* bn_x, const float* bn_mean, const float* bn_scale,
                       const float* bn_shift, float* psum, float* psumx, int cfg) {
  if (Nb <= 0 || Ho <= 0 || Wo <= 0 || Cout <= 0 || Cout % 32 != 0 || Cin <= 0 || Cin % 64 != 0) return -1;
  const bool bnb = bn_x != nullptr;
  if (bnb && (!bn_mean || !bn_scale || !bn_shift || !psum || !psumx)) return -2;
  if (((reinterpret_cast<uintptr_t>(dY) | reinterpret_cast<uintptr_t>(Wd) | reinterpret_cast<uintptr_t>(dX) |
        reinterpret_cast<uintptr_t>(zero) | reinterpret_cast<uintptr_t>(bn_x)) & 15) != 0)
    return -5;
  const int64_t M = static_cast<int64_t>(Nb) * Ho * Wo;
  const int64_t dy_bytes = M * Cout * 2;
  if (dy_bytes >= (static_cast<int64_t>(1) << 31) || static_cast<int64_t>(Cin) * 9 * Cout * 2 >= (static_cast<int64_t>(1) << 31))
    return -8;
  const int c = s2_cfg(Cin, cfg);
  if (c < 8) return -7;
  const int rpb = det_igemm_dgrad_s2_rows_per_block(Cin, cfg);
  const int nblk = static_cast<int>((M + rpb - 1) / rpb);
  hipStream_t st = static_cast<hipStream_t>(stream);
  for (int cls = 0; cls < 4; ++cls) {
    const int ph = cls >> 1, pw = cls & 1;
    const int R = 1 + ph, S = 1 + pw;
    unsigned tapmap = 0;
    for (int rr = 0; rr < R; ++rr)
      for (int ss = 0; ss < S; ++ss) {
        const int rp = ph ? 2 * rr : 1, sp = pw ? 2 * ss : 1;  // flipped-weight tap of class tap (rr, ss)
        tapmap |= static_cast<unsigned>(rp * 3 + sp) << (4 * (rr * S + ss));
      }
    IgArgs a{static_cast<const unsigned short*>(dY), static_cast<const unsigned short*>(Wd), static_cast<unsigned short*>(dX),
             static_cast<const unsigned short*>(zero), nullptr, nullptr, M, Cin, R * S * Cout, Cout, Ho, Wo, Ho, Wo, 1, 0,
             S, R, dy_bytes, static_cast<const unsigned short*>(bn_x), bn_mean, bn_scale, bn_shift, psum, psumx,
             9 * Cout, tapmap, 1 + cls, cls * nblk};
    const int rc = run_cfg(c, st, a, false, false, bnb);
    if (rc != 0) return rc;
  }
  return 0;
}

// 3x3 / stride-1 / pad-1 convolution on the halo-patch kernel (conv3p, see above): Y[M, N] (M = Nb*H*W)
// = conv(op(X), W) with W in KRSC [N][9][Cin], op = relu(x * pro_scale + pro_shift) when given (the
// preceding BatchNorm + ReLU; zero padding is not transformed).  pmean/pm2 (nullable, [ceil(M/256),
// N]): BN statistics partials of Y.  bn_x..psumx (all or none): the BN-backward epilogue of a BN
// whose output X this conv's input gradient is (mask mode 1), partials [ceil(M/256), N].  Cin % 32,
// N % 64, 16-B aligned; -6 when a tile's patch would exceed 640 pixels (very wide images).
int det_conv3p(void* stream, const void* X, const void* W, void* Y, int Nb, int H, int Wd, int Cin, int N,
               const float* pro_scale, const float* pro_shift, float* pmean, float* pm2, const void* bn_x,
               const float* bn_mean, const float* bn_scale, const float* bn_shift, float* psum, float* psumx,
               int grid) {
  if (Nb <= 0 || H <= 0 || Wd <= 0 || Cin <= 0 || Cin % 32 != 0 || N <= 0 || N % kP3BN != 0) return -1;
  if ((pro_scale == nullptr) != (pro_shift == nullptr) || (pmean == nullptr) != (pm2 == nullptr)) return -2;
  const bool bnb = bn_x != nullptr;
  if (bnb && (!bn_mean || !bn_scale || !bn_shift || !psum || !psumx || pmean || pro_scale)) return -2;
  if (((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(Y) |
        reinterpret_cast<uintptr_t>(bn_x)) & 15) != 0)
    return -5;
  const int64_t M = static_cast<int64_t>(Nb) * H * Wd;
  if (p3_max_patch(M, H, Wd) > kP3PMAX) return -6;
  IgArgs a{};
  a.X = static_cast<const unsigned short*>(X);
  a.W = static_cast<const unsigned short*>(W);
  a.Y = static_cast<unsigned short*>(Y);
  a.pmean = pmean;
  a.pm2 = pm2;
  a.M = M;
  a.N = N;
  a.K = 9 * Cin;
  a.Cin = Cin;
  a.Hi = a.Ho = H;
  a.Wi = a.Wo = Wd;
  a.stride = 1;
  a.pad = 1;
  a.R = a.S = 3;
  a.bn_x = static_cast<const unsigned short*>(bn_x);
  a.bn_mean = bn_mean;
  a.bn_scale = bn_scale;
  a.bn_shift = bn_shift;
  a.psum = psum;
  a.psumx = psumx;
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
  const int ntn = N / kP3BN;
  const int64_t ntiles64 = ((M + kP3BM - 1) / kP3BM) * ntn;
  if (ntiles64 >= (static_cast<int64_t>(1) << 31)) return -4;
  const int ntiles = static_cast<int>(ntiles64);
  static const int env_grid = [] {
    const char* e = std::getenv("DET_CONV3P_GRID");
    return e ? std::atoi(e) : 0;
  }();
  int g = grid > 0 ? grid : (env_grid > 0 ? env_grid : 256);  // one persistent block per CU
  if (g > ntiles) g = ntiles;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 gd(static_cast<unsigned>(g)), bd(512);
  if (bnb) hipLaunchKernelGGL((conv3p_kernel<false, false, true>), gd, bd, kP3SMEM, st, a, ntiles, ntn);
  else if (pro_scale && pmean) hipLaunchKernelGGL((conv3p_kernel<true, true, false>), gd, bd, kP3SMEM, st, a, ntiles, ntn);
  else if (pro_scale) hipLaunchKernelGGL((conv3p_kernel<true, false, false>), gd, bd, kP3SMEM, st, a, ntiles, ntn);
  else if (pmean) hipLaunchKernelGGL((conv3p_kernel<false, true, false>), gd, bd, kP3SMEM, st, a, ntiles, ntn);
  else hipLaunchKernelGGL((conv3p_kernel<false, false, false>), gd, bd, kP3SMEM, st, a, ntiles, ntn);
  return static_cast<int>(hipGetLastError());
}

int det_igemm_conv(void* stream, const void* X, const void* W, void* Y, const void* zero, int64_t M, int N, int Cin,
                   int Hi, int Wi, int Ho, int Wo, int R, int S, int stride, int pad, float* pmean, float* pm2) {
  return det_igemm_conv_cfg(stream, X, W, Y, zero, M, N, Cin, Hi, Wi, Ho, Wo, R, S, stride, pad, pmean, pm2, 1);
}

}  // extern "C"
