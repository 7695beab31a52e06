// det_gemm8: a 256 x 256 bf16 GEMM tile on an eight-phase ping-pong schedule, C = A . B^T (+ bias).
//
// A [M, K] and B [N, K] are K-contiguous bf16 rows (torch Linear: x @ W^T, and its dgrad/wgrad
// forms once the operands are laid out K-contiguous); C [M, N] bf16, fp32 accumulation.
//
// Structure (MI355X_MICROARCH.md / cdna_hip_programming.md §5 "256² 8-phase"; written for this
// framework, not copied):
//   * 512 threads = 8 waves as 2 (rows) x 4 (cols); each wave owns a 128 x 64 accumulator tile
//     (8 x 4 fragments of v_mfma_f32_16x16x32_bf16, 128 accumulator VGPRs).
//   * K tiles of 64.  LDS holds two K tiles (even / odd), each as four 16 KiB half-tiles: A rows
//     0-127, A rows 128-255, B rows 0-127, B rows 128-255.  A half-tile is two 64-B-row sub-images
//     (k 0-31, k 32-63) filled by LDS-DMA (buffer_load ... lds, 16 B per lane, lane-linear
//     destination) with the chunk XOR swizzle applied to the SOURCE address, so the 16 x 16 x 32
//     fragment reads (ds_read_b128) are conflict-free.
//   * Four phases per K tile, one C quadrant (64 x 32 of the wave tile, 16 MFMAs) per phase:
//       P1 read A rows 0-63 + B cols 0-31 | MFMA quadrant (0,0)
//       P2 read A rows 64-127 + B cols 32-63 | MFMA (0,1)
//       P3 (no reads)  | MFMA (1,1)        P4 (no reads) | MFMA (1,0)
//     every fragment of the tile is in registers after P2, so the buffer can be restaged from P4 on.
//   * Each phase: reads, LDS-DMA issue, [counted vmcnt in P4 only], barrier, lgkmcnt(0), MFMA
//     cluster at raised priority, barrier.  The wave group of the lower 128 rows starts one barrier
//     late, so on every SIMD one wave runs its MFMA cluster while the other issues reads and DMAs.
//   * Staging (MODE 1, "paired"): P1(t) issues A(t+1), P4(t) issues B(t+2); the P4 wait leaves
//     B(t+2) in flight (vmcnt 4), so A(t+1) has three phases to land.  MODE 0 ("balanced") issues one
//     half-tile per phase: P1 B1(t+1), P2 A0(t+1), P3 A1(t+1), P4 B0(t+2), wait vmcnt 2.
//   RAW: a half-tile is read only in a phase after the P4 wait that retired it, one barrier more for
//   the late group.  WAR: a buffer is restaged two phases after its last read (P2 -> P4).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) unsigned short us8;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kBM = 256, kBN = 256, kNW = 8, kNT = 512;
constexpr int kHalf = 128 * 64 * 2;   // one half-tile: 128 rows x 64 k, bf16
constexpr int kBuf = 4 * kHalf;       // A0 A1 B0 B1
constexpr int kLDC = kBN + 16;
constexpr int kSmem = (2 * kBuf > kBM * kLDC * 2) ? 2 * kBuf : kBM * kLDC * 2;
constexpr unsigned kOOB = 0x80000000u;  // >= every buffer's num_records: the load returns zeros

__device__ __forceinline__ float bf2f(unsigned short u) { return __uint_as_float(static_cast<uint32_t>(u) << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) { return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f)); }

// bijective XCD-aware block order: consecutive tiles land on the same XCD (shared L2)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// 64-B LDS rows: chunk ch of row r sits at chunk ch ^ f(r), f(r) = (-(r >> 2)) & 3
__device__ __forceinline__ int swz64(int row, int ch) { return row * 64 + ((ch ^ ((-(row >> 2)) & 3)) << 4); }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// a raw s_barrier (no fence: LDS-DMA stays in flight across it) that also pins the instruction
// order: nothing, MFMAs included, is scheduled across a phase boundary
__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

struct G8Args {
  const unsigned short* A;  // [M, lda]
  const unsigned short* B;  // [N, ldb]
  unsigned short* C;        // [M, ldc]
  const void* bias;         // [N] fp32 (bias_dt 1) or bf16 (2), or null
  int64_t M;
  int N, K, lda, ldb, ldc, bias_dt;
  unsigned a_bytes, b_bytes;  // buffer ranges
  unsigned short* C2;         // epi 1 / 2: gelu(C) [M, ldc] (C keeps the pre-activation for the backward)
  int epi;                    // 0 none, 1 erf GELU (BERT), 2 tanh GELU (gelu_new)
};

// the GELU of ops/csrc/det_transformer.hip gelu_f, applied to the bf16-rounded pre-activation (so
// the fused output equals the separate det_tf_gelu_fwd pass bit for bit)
__device__ __forceinline__ float gelu_epi(float z, int epi) {
  if (epi == 1) return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
  const float u = 0.7978845608028654f * (z + 0.044715f * z * z * z);
  return 0.5f * z * (1.f + tanhf(u));
}

template <int MODE>
__global__ void __launch_bounds__(kNT, 1) gemm8_kernel(G8Args g) {
#if defined(__HIP_DEVICE_COMPILE__)
  // MODE bits (schedule experiments, scripts/bench_gemm8.py): 1 paired staging (else balanced),
  // 2 issue the phase's DMAs before its fragment reads, 4 no explicit lgkmcnt(0) before the MFMA
  // cluster (the compiler's per-operand waits only), 8 no group stagger (both groups in lockstep)
  constexpr bool kPaired = MODE & 1, kStageFirst = MODE & 2, kNoLgkm = MODE & 4, kNoStagger = MODE & 8;
  constexpr bool kNoPrio = MODE & 16;  // 16: MFMA clusters at normal priority
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;  // 2 x 4 waves; SIMD s holds waves s (wr 0) and s + 4 (wr 1)
  const int ntn = (g.N + kBN - 1) / kBN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntn, nt = bid - mt * ntn;
  const int64_t m0 = static_cast<int64_t>(mt) * kBM;
  const int n0 = nt * kBN;

  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(g.A), 0, g.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(g.B), 0, g.b_bytes, 0x00020000);

  // this lane's DMA source rows: wave `wid` fills rows wid*16 .. +15 of every half-tile, 4 lanes per
  // 64-B row, source chunk pre-swizzled so the lane-linear LDS image matches swz64
  const int lrow = lane >> 2;
  const int gch = (lane & 3) ^ ((-(lrow >> 2)) & 3);
  unsigned voff[4];
  bool vok[4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t am = m0 + h * 128 + wid * 16 + lrow;
    vok[h] = am < g.M;
    voff[h] = vok[h] ? static_cast<unsigned>(am * g.lda * 2 + gch * 16) : 0u;
    const int bn = n0 + h * 128 + wid * 16 + lrow;
    vok[2 + h] = bn < g.N;
    voff[2 + h] = vok[2 + h] ? static_cast<unsigned>(static_cast<int64_t>(bn) * g.ldb * 2 + gch * 16) : 0u;
  }
  // half-tile ht (0 A rows 0-127, 1 A rows 128-255, 2 B rows 0-127, 3 B rows 128-255) of K tile kt
  auto stage = [&](int ht, int kt) {
    unsigned char* dst = smem + (kt & 1) * kBuf + ht * kHalf + wid * 1024;
    const unsigned kb = static_cast<unsigned>(kt) * 128u;
    const unsigned v0 = vok[ht] ? voff[ht] + kb : kOOB;
    const unsigned v1 = vok[ht] ? voff[ht] + kb + 64u : kOOB;
    if (ht < 2) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ar, (lds_void*)dst, 16, v0, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ar, (lds_void*)(dst + 8192), 16, v1, 0, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(br, (lds_void*)dst, 16, v0, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(br, (lds_void*)(dst + 8192), 16, v1, 0, 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[8][2], bfm[4][2];
  const int fr = lane & 15, fch = lane >> 4;
  // fragments of K tile kt: A rows i*16.. of the wave's half (wr), B cols (wc & 1) * 64 + j * 16 of half wc >> 1
  auto read_a = [&](int kt, int i0) {
    const unsigned char* base = smem + (kt & 1) * kBuf + wr * kHalf;
#pragma unroll
    for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
        af[i][kh] = *reinterpret_cast<const bf16x8*>(base + kh * 8192 + swz64(i * 16 + fr, fch));
  };
  auto read_b = [&](int kt, int j0) {
    const unsigned char* base = smem + (kt & 1) * kBuf + (2 + (wc >> 1)) * kHalf;
#pragma unroll
    for (int j = j0; j < j0 + 2; ++j)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
        bfm[j][kh] = *reinterpret_cast<const bf16x8*>(base + kh * 8192 + swz64((wc & 1) * 64 + j * 16 + fr, fch));
  };
  auto mfma = [&](int i0, int j0) {
    if (!kNoPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
        for (int j = j0; j < j0 + 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kh], bfm[j][kh], acc[i][j], 0, 0, 0);
    if (!kNoPrio) __builtin_amdgcn_s_setprio(0);
  };
  auto lgkm0 = [&]() {
    if (!kNoLgkm) __builtin_amdgcn_s_waitcnt(0xC07F);
  };

  const int nk = g.K / 64;
  // prologue: tile 0 complete plus what the steady state expects in flight at tile 0's entry
  if (kPaired) {
    stage(0, 0); stage(1, 0); stage(2, 0); stage(3, 0);
    if (nk > 1) { stage(2, 1); stage(3, 1); wait_vmcnt<4>(); } else wait_vmcnt<0>();
  } else {
    stage(0, 0); stage(1, 0); stage(2, 0); stage(3, 0);
    if (nk > 1) { stage(2, 1); wait_vmcnt<2>(); } else wait_vmcnt<0>();
  }
  barrier();
  if (!kNoStagger && wr == 1) barrier();  // the late group: one barrier behind from here on

  for (int t = 0; t < nk; ++t) {
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    // P1
    if (kStageFirst && kPaired && n1) { stage(0, t + 1); stage(1, t + 1); }
    read_a(t, 0);
    read_b(t, 0);
    if (kPaired) { if (!kStageFirst && n1) { stage(0, t + 1); stage(1, t + 1); } }
    else { if (n1) stage(3, t + 1); }
    barrier();
    lgkm0();
    mfma(0, 0);
    barrier();
    // P2
    read_a(t, 4);
    read_b(t, 2);
    if (!kPaired && n1) stage(0, t + 1);
    barrier();
    lgkm0();
    mfma(0, 2);
    barrier();
    // P3
    if (!kPaired && n1) stage(1, t + 1);
    barrier();
    mfma(4, 2);
    barrier();
    // P4: restage this tile's buffer with B(t+2); then retire tile t+1 (everything older than the
    // B(t+2) pieces just issued)
    if (kPaired) {
      if (n2) { stage(2, t + 2); stage(3, t + 2); wait_vmcnt<4>(); } else wait_vmcnt<0>();
    } else {
      if (n2) { stage(2, t + 2); wait_vmcnt<2>(); } else wait_vmcnt<0>();
    }
    barrier();
    mfma(4, 0);
    barrier();
  }
  if (!kNoStagger && wr == 0) barrier();  // the early group catches up: every wave has passed the same barriers
  __syncthreads();

  // epilogue: C tile through LDS (bias added in fp32), 16-B row stores
  unsigned short* ct = reinterpret_cast<unsigned short*>(smem);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wc * 64 + j * 16 + fr;
      float bv = 0.f;
      if (g.bias_dt != 0 && n0 + col < g.N)
        bv = g.bias_dt == 1 ? static_cast<const float*>(g.bias)[n0 + col]
                            : bf2f(static_cast<const unsigned short*>(g.bias)[n0 + col]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 128 + i * 16 + fch * 4 + r;
        ct[row * kLDC + col] = f2bf(acc[i][j][r] + bv);
      }
    }
  __syncthreads();
  const int64_t rows_left = g.M - m0;
  const int nvalid = rows_left < kBM ? static_cast<int>(rows_left) : kBM;
  const int cols_left = g.N - n0;
  constexpr int CPR = kBN / 8;
#pragma unroll
  for (int q = 0; q < kBM * CPR / kNT; ++q) {
    const int idx = tid + q * kNT;
    const int row = idx / CPR, cc = idx - row * CPR;
    if (row < nvalid && cc * 8 < cols_left) {
      const us8 z = *reinterpret_cast<const us8*>(ct + row * kLDC + cc * 8);
      *reinterpret_cast<us8*>(g.C + (m0 + row) * g.ldc + n0 + cc * 8) = z;
      if (g.epi != 0) {
        us8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf(gelu_epi(bf2f(z[e]), g.epi));
        *reinterpret_cast<us8*>(g.C2 + (m0 + row) * g.ldc + n0 + cc * 8) = o;
      }
    }
  }
#endif
}

template <int MODE>
int launch(hipStream_t st, const G8Args& a) {
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm8_kernel<MODE>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kSmem);
    if (e != hipSuccess) return static_cast<int>(e);
    attr = true;
  }
  const int64_t nwg = ((a.M + kBM - 1) / kBM) * ((a.N + kBN - 1) / kBN);
  hipLaunchKernelGGL((gemm8_kernel<MODE>), dim3(static_cast<unsigned>(nwg)), dim3(kNT), kSmem, st, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace

extern "C" {

// C[M, N] = A[M, K] . B[N, K]^T (+ bias[N]); bf16 operands and output, fp32 accumulation.
// Requirements (checked): K % 64 == 0, N % 8 == 0, lda/ldb/ldc % 8 == 0, 16-B aligned pointers,
// operand byte ranges < 2^31.  mode 0 / 1: staging schedule (see the header).
// epi 1 / 2: C2 [M, ldc] = gelu(C) (erf / tanh form), C keeps the pre-activation.
int det_gemm8(void* stream, const void* A, const void* B, void* C, const void* bias, int bias_dt, int64_t M, int N,
              int K, int lda, int ldb, int ldc, int mode, void* C2, int epi) {
  if (epi != 0 && (C2 == nullptr || (reinterpret_cast<uintptr_t>(C2) & 15) || epi > 2)) return -5;
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 != 0 || N % 8 != 0 || lda % 8 || ldb % 8 || ldc % 8) return -1;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B) | reinterpret_cast<uintptr_t>(C)) & 15) return -2;
  const int64_t ab = ((M - 1) * lda + K) * 2, bb = (static_cast<int64_t>(N - 1) * ldb + K) * 2;
  if (ab >= (int64_t(1) << 31) || bb >= (int64_t(1) << 31)) return -3;
  if (((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN) >= (int64_t(1) << 31)) return -4;
  G8Args a{static_cast<const unsigned short*>(A), static_cast<const unsigned short*>(B), static_cast<unsigned short*>(C), bias,
           M, N, K, lda, ldb, ldc, bias ? bias_dt : 0, static_cast<unsigned>(ab), static_cast<unsigned>(bb),
           static_cast<unsigned short*>(C2), epi};
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (mode) {
    case 0: return launch<0>(st, a);
    case 3: return launch<3>(st, a);
    case 5: return launch<5>(st, a);
    case 7: return launch<7>(st, a);
    case 9: return launch<9>(st, a);
    case 21: return launch<21>(st, a);
    case 23: return launch<23>(st, a);
    default: return launch<1>(st, a);
  }
}

}  // extern "C"
