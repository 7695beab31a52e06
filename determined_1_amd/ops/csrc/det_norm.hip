// det_norm.hip — fused training BatchNorm (+ residual add) (+ ReLU) for channels_last activations.
//
// Why this exists: in the ResNet-50 north-star step (profiles/r1_resnet50_bs256_o1_kernel_stats.csv)
// MIOpen's NHWC batch-norm kernels plus the separate residual-add / ReLU / ReLU-backward
// elementwise launches are ~20 ms of a 44 ms step (>45%).  Every one of them is HBM-bound, so the
// only way to speed them up is to touch fewer bytes: fold the add and the activation into the
// normalisation pass and recompute the ReLU mask from the saved input instead of materialising it.
//
// Layout: x is a [M, C] row-major matrix (M = N*H*W, channels contiguous = torch channels_last),
// C % 8 == 0, 16-byte aligned.  A lane owns 8 consecutive channels (one 16 B bf16 vector) and
// walks rows; a 256-thread block covers `tpr` channel groups x `R` rows per iteration.
//
// Forward (training), 3 launches, x read twice (the 2nd read often hits the 256 MiB MALL):
//   1. stats_partial : per (row-block, channel) mean / M2 from shifted sums (no cancellation)
//   2. stats_finalize: Chan merge of the partials -> mean, rstd, scale=g*rstd, shift=b-mean*scale,
//                      running-stat update and num_batches_tracked += 1 (no extra torch launch)
//   3. apply_fwd     : y = act(x*scale + shift [+ res])
// Backward, 3 launches:
//   1. bwd_partial   : sum(dz), sum(dz*(x-mean)) with dz = dy * relu'(.)
//                      relu' comes from x itself (z = x*scale+shift > 0, bit-identical to fwd) when
//                      there is no residual, else from the saved output y > 0
//   2. bwd_finalize  : dgamma, dbeta and the affine dx coefficients  dx = A*dz + B*x + C
//   3. apply_bwd     : dx (and d_residual = dz when the block had a residual input)
//
// Reductions are two-level (LDS, then a finalize launch) with no float atomics: results are
// bitwise reproducible run to run.  No host syncs: capturable in a hipGraph.
//
// Reference parity: the reference delegates BN to torch/cuDNN inside user models
// (examples/computer_vision/*); SURVEY §2.4 K7.  Semantics follow torch.nn.BatchNorm2d
// (biased variance for normalisation, unbiased for running_var, momentum=None -> cumulative).

#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>


namespace {

constexpr int kThreads = 256;
constexpr int kFinThreads = 1024;  // finalize: 64 channels x 16 waves
constexpr int kFinCh = 64;
constexpr int kFinLanes = kFinThreads / kFinCh;

typedef unsigned short us8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(unsigned short u) { return __uint_as_float(static_cast<uint32_t>(u) << 16); }
// RNE; adjacent conversions pair into gfx950's v_cvt_pk_bf16_f32 (1 op per 2 elements instead of
// ~6 per element: the apply kernels are close enough to the HBM roof that VALU work shows)
__device__ __forceinline__ unsigned short f2bf(float f) {
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));
}

// 8-element vector IO: bf16 = one 16 B load, fp32 = two 16 B loads.
template <typename T> struct IO8;
template <> struct IO8<unsigned short> {
  static __device__ __forceinline__ void load(const unsigned short* p, float (&v)[8]) {
    us8 r = *reinterpret_cast<const us8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f(r[j]);
  }
  // streaming read of data this pass alone consumes: the nt hint (det_stream.hip measured 6.4 vs
  // 5.4 TB/s for 16-B/lane reads of 2 GiB, profiles/r5_hbm_stream.txt)
  static __device__ __forceinline__ void load_nt(const unsigned short* p, float (&v)[8]) {
    us8 r = __builtin_nontemporal_load(reinterpret_cast<const us8*>(p));
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
template <> struct IO8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    float4 a = reinterpret_cast<const float4*>(p)[0];
    float4 b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void load_nt(const float* p, float (&v)[8]) { load(p, v); }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

__device__ __forceinline__ void load8f(const float* p, float (&v)[8]) { IO8<float>::load(p, v); }
template <bool NT, typename T>
__device__ __forceinline__ void sload8(const T* p, float (&v)[8]) {
  if constexpr (NT) IO8<T>::load_nt(p, v);
  else IO8<T>::load(p, v);
}

// DET_BN_NT=1: the BatchNorm apply passes read their activation streams with the nontemporal hint
inline bool bn_nt() {  // nontemporal activation reads in the apply passes: on (+0.6 %, round-5 A/B); DET_BN_NT=0 off
  static const bool v = [] {
    const char* e = std::getenv("DET_BN_NT");
    return e == nullptr || e[0] != '0';
  }();
  return v;
}

#ifndef DET_BN_CF
#define DET_BN_CF 1  // channel-fixed apply mapping (0: the grid-stride vector mapping, for A/B builds)
#endif

struct Geom {
  int64_t M;   // rows
  int C;       // channels
  int tpr;     // threads per row (channel groups per block)
  int R;       // rows per block iteration
  int64_t rpb; // rows per row-block
  int nrb;     // number of row-blocks
};

// ---------------------------------------------------------------------------------------------
// Forward stats: per-thread shifted sums -> (mean, M2) -> block merge in LDS -> partials.
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(kThreads)
bn_stats_partial(const T* __restrict__ x, Geom g, float* __restrict__ pmean, float* __restrict__ pm2) {
  __shared__ float lmean[kThreads * 8];
  __shared__ float lm2[kThreads * 8];
  __shared__ int lcnt[kThreads];
  const int tx = threadIdx.x % g.tpr, ty = threadIdx.x / g.tpr;
  const int cgrp = blockIdx.y * g.tpr + tx;
  const bool active = ty < g.R && cgrp * 8 < g.C;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * g.rpb;
  const int64_t r1 = min(g.M, r0 + g.rpb);
  float k[8], s[8], ss[8];
  int n = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) { k[j] = 0.f; s[j] = 0.f; ss[j] = 0.f; }
  if (active && r0 + ty < r1) {
    const int64_t C = g.C;
    const T* base = x + cgrp * 8;
    IO8<T>::load(base + (r0 + ty) * C, k);  // shift = first sample of this lane
    int64_t r = r0 + ty;
    const int64_t R = g.R;
    for (; r + 3 * R < r1; r += 4 * R) {
      float a[8], b[8], c[8], d[8];
      IO8<T>::load(base + r * C, a);
      IO8<T>::load(base + (r + R) * C, b);
      IO8<T>::load(base + (r + 2 * R) * C, c);
      IO8<T>::load(base + (r + 3 * R) * C, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float da = a[j] - k[j], db = b[j] - k[j], dc = c[j] - k[j], dd = d[j] - k[j];
        s[j] += (da + db) + (dc + dd);
        ss[j] += (da * da + db * db) + (dc * dc + dd * dd);
      }
      n += 4;
    }
    for (; r < r1; r += R) {
      float a[8];
      IO8<T>::load(base + r * C, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float da = a[j] - k[j];
        s[j] += da;
        ss[j] += da * da;
      }
      n += 1;
    }
  }
  const float inv_n = n > 0 ? 1.f / static_cast<float>(n) : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float m = s[j] * inv_n;
    lmean[threadIdx.x * 8 + j] = n > 0 ? k[j] + m : 0.f;
    lm2[threadIdx.x * 8 + j] = n > 0 ? fmaxf(ss[j] - s[j] * m, 0.f) : 0.f;
  }
  lcnt[threadIdx.x] = n;
  __syncthreads();
  if (ty == 0 && cgrp * 8 < g.C) {
    // closed-form merge of the R row-lanes of this channel group
    float tot = 0.f, mu[8], m2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { mu[j] = 0.f; m2[j] = 0.f; }
    for (int q = 0; q < g.R; ++q) {
      const int t = q * g.tpr + tx;
      const float nq = static_cast<float>(lcnt[t]);
      tot += nq;
#pragma unroll
      for (int j = 0; j < 8; ++j) mu[j] += nq * lmean[t * 8 + j];
    }
    const float inv_tot = tot > 0.f ? 1.f / tot : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) mu[j] *= inv_tot;
    for (int q = 0; q < g.R; ++q) {
      const int t = q * g.tpr + tx;
      const float nq = static_cast<float>(lcnt[t]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = lmean[t * 8 + j] - mu[j];
        m2[j] += lm2[t * 8 + j] + nq * d * d;
      }
    }
    const int64_t o = static_cast<int64_t>(blockIdx.x) * g.C + cgrp * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      pmean[o + j] = mu[j];
      pm2[o + j] = m2[j];
    }
  }
}

__global__ void bump_counter(int64_t* c) { *c += 1; }

struct FinArgs {
  const float* gamma;  // may be null (affine=False)
  const float* beta;
  float* running_mean;  // may be null (track_running_stats=False)
  float* running_var;
  int64_t* num_batches_tracked;  // may be null
  float momentum;                // < 0: cumulative moving average (torch momentum=None)
  float eps;
  float* save_mean;
  float* save_rstd;
  float* scale;
  float* shift;
  // nullable: a counter the finalize increments once (block 0, thread 0) -- num_batches_tracked when no
  // apply kernel follows to bump it; only with momentum >= 0, where no block reads the counter
  int64_t* bump;
};

// One block = 64 channels x 16 row-lanes (one wave per row-lane: 256 B coalesced partial rows).
// Single pass in fp64: S1 = sum n_b*mean_b, S2 = sum(M2_b + n_b*mean_b^2); var = S2/M - mean^2.
// fp64 keeps the cancellation harmless, and the 4-way unroll keeps 4 independent partial loads
// in flight per lane (the loop is L2-latency bound, not bandwidth bound).
__global__ void __launch_bounds__(kFinThreads)
bn_stats_finalize(const float* __restrict__ pmean, const float* __restrict__ pm2, Geom g, FinArgs a) {
  if (a.bump && blockIdx.x == 0 && threadIdx.x == 0) *a.bump += 1;
  __shared__ double red1[kFinLanes][kFinCh];
  __shared__ double red2[kFinLanes][kFinCh];
  const int cl = threadIdx.x % kFinCh, lane = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + cl;
  const bool ok = c < g.C;
  double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  if (ok) {
    const int last = g.nrb - 1;
    const double n_full = static_cast<double>(g.rpb);
    const double n_last = static_cast<double>(g.M - static_cast<int64_t>(last) * g.rpb);
    int b = lane;
    for (; b + 3 * kFinLanes < g.nrb; b += 4 * kFinLanes) {
      float mv[4], qv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = static_cast<int64_t>(b + u * kFinLanes) * g.C + c;
        mv[u] = pmean[o];
        qv[u] = pm2[o];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double nb = (b + u * kFinLanes) == last ? n_last : n_full;
        const double m = mv[u];
        s1[u] += nb * m;
        s2[u] += static_cast<double>(qv[u]) + nb * m * m;
      }
    }
    for (; b < g.nrb; b += kFinLanes) {
      const int64_t o = static_cast<int64_t>(b) * g.C + c;
      const double nb = b == last ? n_last : n_full;
      const double m = pmean[o];
      s1[0] += nb * m;
      s2[0] += static_cast<double>(pm2[o]) + nb * m * m;
    }
  }
  red1[lane][cl] = (s1[0] + s1[1]) + (s1[2] + s1[3]);
  red2[lane][cl] = (s2[0] + s2[1]) + (s2[2] + s2[3]);
  __syncthreads();
  if (lane == 0 && ok) {
    double t1 = 0, t2 = 0;
#pragma unroll
    for (int q = 0; q < kFinLanes; ++q) {
      t1 += red1[q][cl];
      t2 += red2[q][cl];
    }
    const double M = static_cast<double>(g.M);
    const double meand = t1 / M;
    double m2 = t2 - M * meand * meand;
    if (m2 < 0) m2 = 0;
    const float mean = static_cast<float>(meand);
    const float var = static_cast<float>(m2 / M);
    const float rstd = rsqrtf(var + a.eps);
    const float gm = a.gamma ? a.gamma[c] : 1.f;
    const float bt = a.beta ? a.beta[c] : 0.f;
    const float sc = gm * rstd;
    a.save_mean[c] = mean;
    a.save_rstd[c] = rstd;
    a.scale[c] = sc;
    a.shift[c] = bt - mean * sc;
    if (a.running_mean) {
      float f = a.momentum;
      if (f < 0.f) f = a.num_batches_tracked ? 1.f / static_cast<float>(*a.num_batches_tracked + 1) : 0.f;
      const float unbiased = g.M > 1 ? static_cast<float>(m2 / (M - 1.0)) : var;
      a.running_mean[c] = (1.f - f) * a.running_mean[c] + f * mean;
      a.running_var[c] = (1.f - f) * a.running_var[c] + f * unbiased;
    }
  }
}

// Two-stage finalize for long partial lists (the GEMM-epilogue partials of det_conv.hip come in
// 128-row blocks: 12,544 rows of partials for a layer1 activation, which one 64-channel block
// walked serially in ~30 us).  Stage 1 spreads the row-blocks over S slices x C/64 channel blocks
// and writes fp64 (S1, S2) per (slice, channel); stage 2 merges the S slices in a fixed order
// (deterministic, no atomics) and applies the same epilogue as bn_stats_finalize.
constexpr int kMaxSlices = 64;

__global__ void __launch_bounds__(kFinThreads)
bn_stats_reduce(const float* __restrict__ pmean, const float* __restrict__ pm2, Geom g, int per_slice,
                double* __restrict__ part) {
  __shared__ double red1[kFinLanes][kFinCh];
  __shared__ double red2[kFinLanes][kFinCh];
  const int cl = threadIdx.x % kFinCh, lane = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + cl;
  const bool ok = c < g.C;
  const int b0 = blockIdx.y * per_slice;
  const int b1 = min(g.nrb, b0 + per_slice);
  double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  if (ok) {
    const int last = g.nrb - 1;
    const double n_full = static_cast<double>(g.rpb);
    const double n_last = static_cast<double>(g.M - static_cast<int64_t>(last) * g.rpb);
    int b = b0 + lane;
    for (; b + 3 * kFinLanes < b1; b += 4 * kFinLanes) {
      float mv[4], qv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = static_cast<int64_t>(b + u * kFinLanes) * g.C + c;
        mv[u] = pmean[o];
        qv[u] = pm2[o];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double nb = (b + u * kFinLanes) == last ? n_last : n_full;
        const double m = mv[u];
        s1[u] += nb * m;
        s2[u] += static_cast<double>(qv[u]) + nb * m * m;
      }
    }
    for (; b < b1; b += kFinLanes) {
      const int64_t o = static_cast<int64_t>(b) * g.C + c;
      const double nb = b == last ? n_last : n_full;
      const double m = pmean[o];
      s1[0] += nb * m;
      s2[0] += static_cast<double>(pm2[o]) + nb * m * m;
    }
  }
  red1[lane][cl] = (s1[0] + s1[1]) + (s1[2] + s1[3]);
  red2[lane][cl] = (s2[0] + s2[1]) + (s2[2] + s2[3]);
  __syncthreads();
  if (lane == 0 && ok) {
    double t1 = 0, t2 = 0;
#pragma unroll
    for (int q = 0; q < kFinLanes; ++q) {
      t1 += red1[q][cl];
      t2 += red2[q][cl];
    }
    const int64_t o = (static_cast<int64_t>(blockIdx.y) * g.C + c) * 2;
    part[o] = t1;
    part[o + 1] = t2;
  }
}

// Combine of the S slices (fp64 pairs) per channel, 16 lanes per channel in a fixed order
// (deterministic): a lane walks S / 16 slices instead of one thread walking all S (the serial
// 256-thread combine took ~10 us per call).  A one-launch variant that merged in the last-arriving
// reduce block was slower (41 vs 16 us per BN: every block's agent-scope fence writes back L2,
// profiles/r3_resnet50_lastblock_finalize_negative_steady.csv).
__global__ void __launch_bounds__(kFinThreads)
bn_stats_combine_par(const double* __restrict__ part, int S, Geom g, FinArgs a) {
  if (a.bump && blockIdx.x == 0 && threadIdx.x == 0) *a.bump += 1;
  __shared__ double red1[kFinLanes][kFinCh];
  __shared__ double red2[kFinLanes][kFinCh];
  const int cl = threadIdx.x % kFinCh, lane = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + cl;
  const bool ok = c < g.C;
  double t1 = 0, t2 = 0;
  if (ok) {
    for (int q = lane; q < S; q += kFinLanes) {
      const int64_t o = (static_cast<int64_t>(q) * g.C + c) * 2;
      t1 += part[o];
      t2 += part[o + 1];
    }
  }
  red1[lane][cl] = t1;
  red2[lane][cl] = t2;
  __syncthreads();
  if (lane != 0 || !ok) return;
  t1 = 0;
  t2 = 0;
#pragma unroll
  for (int q = 0; q < kFinLanes; ++q) {
    t1 += red1[q][cl];
    t2 += red2[q][cl];
  }
  const double M = static_cast<double>(g.M);
  const double meand = t1 / M;
  double m2 = t2 - M * meand * meand;
  if (m2 < 0) m2 = 0;
  const float mean = static_cast<float>(meand);
  const float var = static_cast<float>(m2 / M);
  const float rstd = rsqrtf(var + a.eps);
  const float gm = a.gamma ? a.gamma[c] : 1.f;
  const float bt = a.beta ? a.beta[c] : 0.f;
  const float sc = gm * rstd;
  a.save_mean[c] = mean;
  a.save_rstd[c] = rstd;
  a.scale[c] = sc;
  a.shift[c] = bt - mean * sc;
  if (a.running_mean) {
    float f = a.momentum;
    if (f < 0.f) f = a.num_batches_tracked ? 1.f / static_cast<float>(*a.num_batches_tracked + 1) : 0.f;
    const float unbiased = g.M > 1 ? static_cast<float>(m2 / (M - 1.0)) : var;
    a.running_mean[c] = (1.f - f) * a.running_mean[c] + f * mean;
    a.running_var[c] = (1.f - f) * a.running_var[c] + f * unbiased;
  }
}

// One-launch sliced finalize: bn_stats_reduce, then the block that arrives last for its channel
// block merges the S slices (bn_stats_combine_par's work) -- one launch per BN instead of two.  The
// round-3 version of this published the slices with an agent-scope release fence per block, which
// writes back the XCD's whole L2 (41 vs 16 us per BN, profiles/r3_resnet50_lastblock_finalize_
// negative_steady.csv).  Here the slice sums go out as write-through (sc1) stores, the storing wave
// drains them (vmcnt(0)) before its lane 0 adds to the channel block's arrival counter, and the last
// arriver reads every slice back with sc1 loads behind a workgroup barrier -- the hand-off form the
// guide measures without fences (MI355X_MICROARCH.md "Valid forms", first table row).  The counter
// goes back to 0 for the next BatchNorm on the stream.  No spinning: blocks that are not last exit.
constexpr int kMaxChanBlocks = 64;  // C <= 4096
__device__ unsigned g_bn_stats_arrivals[kMaxChanBlocks];
__device__ unsigned g_bn_bwd_arrivals[kMaxChanBlocks];

__device__ __forceinline__ void stats_finish(double t1, double t2, int c, const Geom& g, const FinArgs& a) {
  const double M = static_cast<double>(g.M);
  const double meand = t1 / M;
  double m2 = t2 - M * meand * meand;
  if (m2 < 0) m2 = 0;
  const float mean = static_cast<float>(meand);
  const float var = static_cast<float>(m2 / M);
  const float rstd = rsqrtf(var + a.eps);
  const float gm = a.gamma ? a.gamma[c] : 1.f;
  const float bt = a.beta ? a.beta[c] : 0.f;
  const float sc = gm * rstd;
  a.save_mean[c] = mean;
  a.save_rstd[c] = rstd;
  a.scale[c] = sc;
  a.shift[c] = bt - mean * sc;
  if (a.running_mean) {
    float f = a.momentum;
    if (f < 0.f) f = a.num_batches_tracked ? 1.f / static_cast<float>(*a.num_batches_tracked + 1) : 0.f;
    const float unbiased = g.M > 1 ? static_cast<float>(m2 / (M - 1.0)) : var;
    a.running_mean[c] = (1.f - f) * a.running_mean[c] + f * mean;
    a.running_var[c] = (1.f - f) * a.running_var[c] + f * unbiased;
  }
}

// true in every thread of the block that arrives last (wave 0 published this block's slice)
__device__ __forceinline__ bool last_arrival(unsigned* counter, unsigned total, int* flag) {
  if (threadIdx.x < 64) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // wave 0's write-through slice stores landed
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = old == total - 1 ? 1 : 0;
    }
  }
  __syncthreads();
  return *flag != 0;
}

__global__ void __launch_bounds__(kFinThreads)
bn_stats_reduce_last(const float* __restrict__ pmean, const float* __restrict__ pm2, Geom g, int per_slice,
                     double* __restrict__ part, FinArgs a) {
  __shared__ double red1[kFinLanes][kFinCh];
  __shared__ double red2[kFinLanes][kFinCh];
  __shared__ int is_last;
  const int cl = threadIdx.x % kFinCh, lane = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + cl;
  const bool ok = c < g.C;
  const int b0 = blockIdx.y * per_slice;
  const int b1 = min(g.nrb, b0 + per_slice);
  double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  if (ok) {
    const int last = g.nrb - 1;
    const double n_full = static_cast<double>(g.rpb);
    const double n_last = static_cast<double>(g.M - static_cast<int64_t>(last) * g.rpb);
    int b = b0 + lane;
    for (; b + 3 * kFinLanes < b1; b += 4 * kFinLanes) {
      float mv[4], qv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = static_cast<int64_t>(b + u * kFinLanes) * g.C + c;
        mv[u] = pmean[o];
        qv[u] = pm2[o];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double nb = (b + u * kFinLanes) == last ? n_last : n_full;
        const double m = mv[u];
        s1[u] += nb * m;
        s2[u] += static_cast<double>(qv[u]) + nb * m * m;
      }
    }
    for (; b < b1; b += kFinLanes) {
      const int64_t o = static_cast<int64_t>(b) * g.C + c;
      const double nb = b == last ? n_last : n_full;
      const double m = pmean[o];
      s1[0] += nb * m;
      s2[0] += static_cast<double>(pm2[o]) + nb * m * m;
    }
  }
  red1[lane][cl] = (s1[0] + s1[1]) + (s1[2] + s1[3]);
  red2[lane][cl] = (s2[0] + s2[1]) + (s2[2] + s2[3]);
  __syncthreads();
  if (lane == 0 && ok) {  // wave 0
    double t1 = 0, t2 = 0;
#pragma unroll
    for (int q = 0; q < kFinLanes; ++q) {
      t1 += red1[q][cl];
      t2 += red2[q][cl];
    }
    const int64_t o = (static_cast<int64_t>(blockIdx.y) * g.C + c) * 2;
    __hip_atomic_store(part + o, t1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part + o + 1, t2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!last_arrival(&g_bn_stats_arrivals[blockIdx.x], gridDim.y, &is_last)) return;
  // the last block of this channel block: merge the S slices in a fixed order (deterministic)
  if (a.bump && blockIdx.x == 0 && threadIdx.x == 0) *a.bump += 1;
  double t1 = 0, t2 = 0;
  if (ok) {
    for (int q = lane; q < static_cast<int>(gridDim.y); q += kFinLanes) {
      const int64_t o = (static_cast<int64_t>(q) * g.C + c) * 2;
      t1 += __hip_atomic_load(part + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t2 += __hip_atomic_load(part + o + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();  // red1/red2 reuse
  red1[lane][cl] = t1;
  red2[lane][cl] = t2;
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&g_bn_stats_arrivals[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane != 0 || !ok) return;
  t1 = 0;
  t2 = 0;
#pragma unroll
  for (int q = 0; q < kFinLanes; ++q) {
    t1 += red1[q][cl];
    t2 += red2[q][cl];
  }
  stats_finish(t1, t2, c, g, a);
}

__global__ void __launch_bounds__(256)
bn_stats_combine(const double* __restrict__ part, int S, Geom g, FinArgs a) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= g.C) return;
  double t1 = 0, t2 = 0;
  for (int s = 0; s < S; ++s) {
    const int64_t o = (static_cast<int64_t>(s) * g.C + c) * 2;
    t1 += part[o];
    t2 += part[o + 1];
  }
  const double M = static_cast<double>(g.M);
  const double meand = t1 / M;
  double m2 = t2 - M * meand * meand;
  if (m2 < 0) m2 = 0;
  const float mean = static_cast<float>(meand);
  const float var = static_cast<float>(m2 / M);
  const float rstd = rsqrtf(var + a.eps);
  const float gm = a.gamma ? a.gamma[c] : 1.f;
  const float bt = a.beta ? a.beta[c] : 0.f;
  const float sc = gm * rstd;
  a.save_mean[c] = mean;
  a.save_rstd[c] = rstd;
  a.scale[c] = sc;
  a.shift[c] = bt - mean * sc;
  if (a.running_mean) {
    float f = a.momentum;
    if (f < 0.f) f = a.num_batches_tracked ? 1.f / static_cast<float>(*a.num_batches_tracked + 1) : 0.f;
    const float unbiased = g.M > 1 ? static_cast<float>(m2 / (M - 1.0)) : var;
    a.running_mean[c] = (1.f - f) * a.running_mean[c] + f * mean;
    a.running_var[c] = (1.f - f) * a.running_var[c] + f * unbiased;
  }
}

// DET_BN_LASTBLOCK=0: the two-launch sliced finalizes (reduce, then combine) instead of the one-launch
// last-arriving-block form (A/B switch, read once)
inline bool bn_last_block() {
  static const bool v = [] {
    const char* e = std::getenv("DET_BN_LASTBLOCK");
    return !(e != nullptr && e[0] == '0');
  }();
  return v;
}

// fp32 elements of scratch the two-stage finalize needs for C channels (fp64 pairs per slice)
inline int64_t fin_scratch_elems(int C) { return static_cast<int64_t>(kMaxSlices) * C * 4; }

// Statistics finalize over g.nrb partial rows: one launch when the list is short, two otherwise.
void launch_stats_finalize(hipStream_t st, const float* pmean, const float* pm2, const Geom& g, const FinArgs& fa,
                           float* scratch) {
  const int cb = (g.C + kFinCh - 1) / kFinCh;
  int S = 1024 / cb;
  if (S > kMaxSlices) S = kMaxSlices;
  const int by_rows = g.nrb / (4 * kFinLanes);  // >= 4 partial rows per lane
  if (S > by_rows) S = by_rows;
  if (scratch == nullptr || S < 4) {
    hipLaunchKernelGGL(bn_stats_finalize, dim3(cb), dim3(kFinThreads), 0, st, pmean, pm2, g, fa);
    return;
  }
  const int per = (g.nrb + S - 1) / S;
  S = (g.nrb + per - 1) / per;
  double* part = reinterpret_cast<double*>(scratch);
  if (bn_last_block() && cb <= kMaxChanBlocks) {
    hipLaunchKernelGGL(bn_stats_reduce_last, dim3(cb, S), dim3(kFinThreads), 0, st, pmean, pm2, g, per, part, fa);
    return;
  }
  hipLaunchKernelGGL(bn_stats_reduce, dim3(cb, S), dim3(kFinThreads), 0, st, pmean, pm2, g, per, part);
  hipLaunchKernelGGL(bn_stats_combine_par, dim3(cb), dim3(kFinThreads), 0, st, part, S, g, fa);
}

// ---------------------------------------------------------------------------------------------
// Elementwise apply: y = act(x*scale + shift [+ res]); grid-stride over 8-element vectors, 4 in
// flight per thread.  RES 2: the residual is itself a BatchNorm output whose apply was deferred
// (ResNet's projection-shortcut BN): res = bf16(r * rscale + rshift), computed here from its input r
// -- that BN's own apply pass (read r, write res) and this pass's read of res become one read of r.
// ---------------------------------------------------------------------------------------------
template <typename T, bool RELU, int RES, bool NTL = false>
__global__ void __launch_bounds__(kThreads)
bn_apply_fwd(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y,
             const float* __restrict__ scale, const float* __restrict__ shift, int64_t nvec, int C,
             int64_t* __restrict__ bump, uint8_t* __restrict__ mbits, const float* __restrict__ rscale = nullptr,
             const float* __restrict__ rshift = nullptr) {
  // num_batches_tracked += 1 rides on this launch (stream-ordered after the finalize that read it)
  if (bump && blockIdx.x == 0 && threadIdx.x == 0) *bump += 1;
#if DET_BN_CF
  // channel-fixed mapping when C/8 divides the block: each thread keeps one 8-channel group for the
  // whole pass (scale/shift loaded once, no per-vector channel modulo), a block covers 256/(C/8)
  // whole rows per iteration (consecutive threads = consecutive 16-B chunks of a row)
  const int cv = C >> 3;
  if (cv <= kThreads && (kThreads % cv) == 0) {
    const int lc = static_cast<int>(threadIdx.x) % cv, rpb = kThreads / cv, c0 = lc << 3;
    float sc[8], sh[8], rsc[8], rsh[8];
    load8f(scale + c0, sc);
    load8f(shift + c0, sh);
    if (RES == 2) {
      load8f(rscale + c0, rsc);
      load8f(rshift + c0, rsh);
    }
    const int64_t nrow = nvec / cv, RS = static_cast<int64_t>(gridDim.x) * rpb;
    for (int64_t r0 = static_cast<int64_t>(blockIdx.x) * rpb + threadIdx.x / cv; r0 < nrow; r0 += 4 * RS) {
      float xv[4][8], rv[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t r = r0 + u * RS;
        if (r < nrow) {
          sload8<NTL>(x + (r * cv + lc) * 8, xv[u]);
          if (RES) sload8<NTL>(res + (r * cv + lc) * 8, rv[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t r = r0 + u * RS;
        if (r < nrow) {
          const int64_t v = r * cv + lc;
          float o[8];
          unsigned bits = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float z = __fmaf_rn(xv[u][j], sc[j], sh[j]);
            if (RES == 1) z += rv[u][j];
            if (RES == 2) z += __uint_as_float(static_cast<uint32_t>(f2bf(__fmaf_rn(rv[u][j], rsc[j], rsh[j]))) << 16);
            o[j] = RELU ? fmaxf(z, 0.f) : z;
            bits |= (z > 0.f ? 1u : 0u) << j;
          }
          IO8<T>::store(y + v * 8, o);
          if (RELU && RES && mbits) mbits[v] = static_cast<uint8_t>(bits);
        }
      }
    }
    return;
  }
#endif
  const int64_t S = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t v0 = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; v0 < nvec; v0 += 4 * S) {
    float xv[4][8], rv[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t v = v0 + u * S;
      if (v < nvec) {
        sload8<NTL>(x + v * 8, xv[u]);
        if (RES) sload8<NTL>(res + v * 8, rv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t v = v0 + u * S;
      if (v < nvec) {
        // vector index -> first channel; 32-bit modulo (nvec < 2^32 checked on the host)
        const int c0 = static_cast<int>(static_cast<uint32_t>(v) % static_cast<uint32_t>(C >> 3)) << 3;
        float sc[8], sh[8], o[8], rsc[8], rsh[8];
        load8f(scale + c0, sc);
        load8f(shift + c0, sh);
        if (RES == 2) {
          load8f(rscale + c0, rsc);
          load8f(rshift + c0, rsh);
        }
        unsigned bits = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float z = __fmaf_rn(xv[u][j], sc[j], sh[j]);
          if (RES == 1) z += rv[u][j];
          // rounded to bf16 like the materialised shortcut-BN output: bit-identical to that path
          if (RES == 2) z += __uint_as_float(static_cast<uint32_t>(f2bf(__fmaf_rn(rv[u][j], rsc[j], rsh[j]))) << 16);
          o[j] = RELU ? fmaxf(z, 0.f) : z;
          bits |= (z > 0.f ? 1u : 0u) << j;
        }
        IO8<T>::store(y + v * 8, o);
        // ReLU mask, 1 bit per element (1/16 of a bf16 stream): the residual-block backward
        // reads it instead of re-reading the 16-bit output twice
        if (RELU && RES && mbits) mbits[v] = static_cast<uint8_t>(bits);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Backward partial sums.  MASK: 0 = identity, 1 = relu mask recomputed from x, 2 = from y > 0.
// ---------------------------------------------------------------------------------------------
template <typename T, int MASK>
__global__ void __launch_bounds__(kThreads)
bn_bwd_partial(const T* __restrict__ dy, const T* __restrict__ dy2, const T* __restrict__ x,
               const uint8_t* __restrict__ mbits, Geom g,
               const float* __restrict__ mean, const float* __restrict__ scale,
               const float* __restrict__ shift, float* __restrict__ psum, float* __restrict__ psumx) {
  __shared__ float l1[kThreads * 8];
  __shared__ float l2[kThreads * 8];
  const int tx = threadIdx.x % g.tpr, ty = threadIdx.x / g.tpr;
  const int cgrp = blockIdx.y * g.tpr + tx;
  const bool chan_ok = cgrp * 8 < g.C;
  const bool active = ty < g.R && chan_ok;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * g.rpb;
  const int64_t r1 = min(g.M, r0 + g.rpb);
  float s[8], sx[8], mu[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s[j] = 0.f; sx[j] = 0.f; mu[j] = 0.f; sc[j] = 0.f; sh[j] = 0.f; }
  if (active) {
    const int c0 = cgrp * 8;
    load8f(mean + c0, mu);
    if (MASK == 1) { load8f(scale + c0, sc); load8f(shift + c0, sh); }
    const int64_t C = g.C, R = g.R;
    const int64_t off = c0;
    int64_t r = r0 + ty;
    for (; r + R < r1; r += 2 * R) {
      float d0[8], x0[8], d1[8], x1[8];
      unsigned b0 = 0xFFu, b1 = 0xFFu;
      IO8<T>::load(dy + r * C + off, d0);
      IO8<T>::load(x + r * C + off, x0);
      IO8<T>::load(dy + (r + R) * C + off, d1);
      IO8<T>::load(x + (r + R) * C + off, x1);
      if (dy2) {
        float e0[8], e1[8];
        IO8<T>::load(dy2 + r * C + off, e0);
        IO8<T>::load(dy2 + (r + R) * C + off, e1);
#pragma unroll
        for (int j = 0; j < 8; ++j) { d0[j] += e0[j]; d1[j] += e1[j]; }
      }
      if (MASK == 2) { b0 = mbits[(r * C + off) >> 3]; b1 = mbits[((r + R) * C + off) >> 3]; }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = d0[j], b = d1[j];
        if (MASK == 1) {
          a = __fmaf_rn(x0[j], sc[j], sh[j]) > 0.f ? a : 0.f;
          b = __fmaf_rn(x1[j], sc[j], sh[j]) > 0.f ? b : 0.f;
        } else if (MASK == 2) {
          a = (b0 >> j) & 1u ? a : 0.f;
          b = (b1 >> j) & 1u ? b : 0.f;
        }
        s[j] += a + b;
        sx[j] += a * (x0[j] - mu[j]) + b * (x1[j] - mu[j]);
      }
    }
    for (; r < r1; r += R) {
      float d0[8], x0[8];
      unsigned b0 = 0xFFu;
      IO8<T>::load(dy + r * C + off, d0);
      IO8<T>::load(x + r * C + off, x0);
      if (dy2) {
        float e0[8];
        IO8<T>::load(dy2 + r * C + off, e0);
#pragma unroll
        for (int j = 0; j < 8; ++j) d0[j] += e0[j];
      }
      if (MASK == 2) b0 = mbits[(r * C + off) >> 3];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = d0[j];
        if (MASK == 1) a = __fmaf_rn(x0[j], sc[j], sh[j]) > 0.f ? a : 0.f;
        else if (MASK == 2) a = (b0 >> j) & 1u ? a : 0.f;
        s[j] += a;
        sx[j] += a * (x0[j] - mu[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    l1[threadIdx.x * 8 + j] = s[j];
    l2[threadIdx.x * 8 + j] = sx[j];
  }
  __syncthreads();
  if (ty == 0 && chan_ok) {
    float a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = 0.f; b[j] = 0.f; }
    for (int q = 0; q < g.R; ++q) {
      const int t = q * g.tpr + tx;
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] += l1[t * 8 + j]; b[j] += l2[t * 8 + j]; }
    }
    const int64_t o = static_cast<int64_t>(blockIdx.x) * g.C + cgrp * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) { psum[o + j] = a[j]; psumx[o + j] = b[j]; }
  }
}

struct BwdFin {
  const float* gamma;  // may be null
  const float* rstd;
  const float* mean;
  float* dgamma;  // may be null
  float* dbeta;   // may be null
  float* coef;    // [3][C]: A, B, C
};

__global__ void __launch_bounds__(kFinThreads)
bn_bwd_finalize(const float* __restrict__ psum, const float* __restrict__ psumx, Geom g, BwdFin a) {
  __shared__ float r1[kFinLanes][kFinCh];
  __shared__ float r2[kFinLanes][kFinCh];
  const int cl = threadIdx.x % kFinCh, lane = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + cl;
  const bool ok = c < g.C;
  float s = 0.f, sx = 0.f;
  if (ok) {
    float sa[4] = {0.f, 0.f, 0.f, 0.f}, sb[4] = {0.f, 0.f, 0.f, 0.f};
    int b = lane;
    for (; b + 3 * kFinLanes < g.nrb; b += 4 * kFinLanes) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = static_cast<int64_t>(b + u * kFinLanes) * g.C + c;
        sa[u] += psum[o];
        sb[u] += psumx[o];
      }
    }
    for (; b < g.nrb; b += kFinLanes) {
      const int64_t o = static_cast<int64_t>(b) * g.C + c;
      sa[0] += psum[o];
      sb[0] += psumx[o];
    }
    s = (sa[0] + sa[1]) + (sa[2] + sa[3]);
    sx = (sb[0] + sb[1]) + (sb[2] + sb[3]);
  }
  r1[lane][cl] = s;
  r2[lane][cl] = sx;
  __syncthreads();
  if (lane == 0 && ok) {
    float ts = 0.f, tsx = 0.f;
#pragma unroll
    for (int q = 0; q < kFinLanes; ++q) { ts += r1[q][cl]; tsx += r2[q][cl]; }
    const float rstd = a.rstd[c], mu = a.mean[c];
    const float gm = a.gamma ? a.gamma[c] : 1.f;
    const float dbeta = ts;
    const float dgamma = tsx * rstd;
    if (a.dgamma) a.dgamma[c] = dgamma;
    if (a.dbeta) a.dbeta[c] = dbeta;
    const float invM = 1.f / static_cast<float>(g.M);
    const float A = gm * rstd;
    const float B = -gm * rstd * rstd * dgamma * invM;
    const float C0 = -A * dbeta * invM - B * mu;
    a.coef[c] = A;
    a.coef[g.C + c] = B;
    a.coef[2 * g.C + c] = C0;
  }
}

// Sliced backward finalize: blocks (channel block, slice) sum their slice of the [nrb, C] partials
// into part[S][C][2]; a combine launch merges the slices (16 lanes per channel, fixed order) and
// writes dgamma, dbeta and the apply coefficients (the single-block finalize walked 12,544 partial
// rows serially for a layer-1 activation: ~22 us).
__global__ void __launch_bounds__(kFinThreads)
bn_bwd_reduce(const float* __restrict__ psum, const float* __restrict__ psumx, Geom g, int per_slice,
              float* __restrict__ part) {
  __shared__ float r1[kFinLanes][kFinCh];
  __shared__ float r2[kFinLanes][kFinCh];
  const int cl = threadIdx.x % kFinCh, lane = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + cl;
  const bool ok = c < g.C;
  const int b0 = blockIdx.y * per_slice;
  const int b1 = min(g.nrb, b0 + per_slice);
  float sa[4] = {0.f, 0.f, 0.f, 0.f}, sb[4] = {0.f, 0.f, 0.f, 0.f};
  if (ok) {
    int b = b0 + lane;
    for (; b + 3 * kFinLanes < b1; b += 4 * kFinLanes) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = static_cast<int64_t>(b + u * kFinLanes) * g.C + c;
        sa[u] += psum[o];
        sb[u] += psumx[o];
      }
    }
    for (; b < b1; b += kFinLanes) {
      const int64_t o = static_cast<int64_t>(b) * g.C + c;
      sa[0] += psum[o];
      sb[0] += psumx[o];
    }
  }
  r1[lane][cl] = (sa[0] + sa[1]) + (sa[2] + sa[3]);
  r2[lane][cl] = (sb[0] + sb[1]) + (sb[2] + sb[3]);
  __syncthreads();
  if (lane == 0 && ok) {
    float ts = 0.f, tsx = 0.f;
#pragma unroll
    for (int q = 0; q < kFinLanes; ++q) { ts += r1[q][cl]; tsx += r2[q][cl]; }
    const int64_t o = (static_cast<int64_t>(blockIdx.y) * g.C + c) * 2;
    part[o] = ts;
    part[o + 1] = tsx;
  }
}

__global__ void __launch_bounds__(kFinThreads)
bn_bwd_combine(const float* __restrict__ part, int S, Geom g, BwdFin a) {
  __shared__ float r1[kFinLanes][kFinCh];
  __shared__ float r2[kFinLanes][kFinCh];
  const int cl = threadIdx.x % kFinCh, lane = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + cl;
  const bool ok = c < g.C;
  float ts = 0.f, tsx = 0.f;
  if (ok) {
    for (int q = lane; q < S; q += kFinLanes) {
      const int64_t o = (static_cast<int64_t>(q) * g.C + c) * 2;
      ts += part[o];
      tsx += part[o + 1];
    }
  }
  r1[lane][cl] = ts;
  r2[lane][cl] = tsx;
  __syncthreads();
  if (lane != 0 || !ok) return;
  ts = 0.f;
  tsx = 0.f;
#pragma unroll
  for (int q = 0; q < kFinLanes; ++q) { ts += r1[q][cl]; tsx += r2[q][cl]; }
  const float rstd = a.rstd[c], mu = a.mean[c];
  const float gm = a.gamma ? a.gamma[c] : 1.f;
  const float dbeta = ts;
  const float dgamma = tsx * rstd;
  if (a.dgamma) a.dgamma[c] = dgamma;
  if (a.dbeta) a.dbeta[c] = dbeta;
  const float invM = 1.f / static_cast<float>(g.M);
  const float A = gm * rstd;
  const float B = -gm * rstd * rstd * dgamma * invM;
  const float C0 = -A * dbeta * invM - B * mu;
  a.coef[c] = A;
  a.coef[g.C + c] = B;
  a.coef[2 * g.C + c] = C0;
}

__device__ __forceinline__ void bwd_finish(float ts, float tsx, int c, const Geom& g, const BwdFin& a) {
  const float rstd = a.rstd[c], mu = a.mean[c];
  const float gm = a.gamma ? a.gamma[c] : 1.f;
  const float dbeta = ts;
  const float dgamma = tsx * rstd;
  if (a.dgamma) a.dgamma[c] = dgamma;
  if (a.dbeta) a.dbeta[c] = dbeta;
  const float invM = 1.f / static_cast<float>(g.M);
  const float A = gm * rstd;
  const float B = -gm * rstd * rstd * dgamma * invM;
  const float C0 = -A * dbeta * invM - B * mu;
  a.coef[c] = A;
  a.coef[g.C + c] = B;
  a.coef[2 * g.C + c] = C0;
}

// bn_bwd_reduce + bn_bwd_combine in one launch (the hand-off of bn_stats_reduce_last)
__global__ void __launch_bounds__(kFinThreads)
bn_bwd_reduce_last(const float* __restrict__ psum, const float* __restrict__ psumx, Geom g, int per_slice,
                   float* __restrict__ part, BwdFin a) {
  __shared__ float r1[kFinLanes][kFinCh];
  __shared__ float r2[kFinLanes][kFinCh];
  __shared__ int is_last;
  const int cl = threadIdx.x % kFinCh, lane = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + cl;
  const bool ok = c < g.C;
  const int b0 = blockIdx.y * per_slice;
  const int b1 = min(g.nrb, b0 + per_slice);
  float sa[4] = {0.f, 0.f, 0.f, 0.f}, sb[4] = {0.f, 0.f, 0.f, 0.f};
  if (ok) {
    int b = b0 + lane;
    for (; b + 3 * kFinLanes < b1; b += 4 * kFinLanes) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = static_cast<int64_t>(b + u * kFinLanes) * g.C + c;
        sa[u] += psum[o];
        sb[u] += psumx[o];
      }
    }
    for (; b < b1; b += kFinLanes) {
      const int64_t o = static_cast<int64_t>(b) * g.C + c;
      sa[0] += psum[o];
      sb[0] += psumx[o];
    }
  }
  r1[lane][cl] = (sa[0] + sa[1]) + (sa[2] + sa[3]);
  r2[lane][cl] = (sb[0] + sb[1]) + (sb[2] + sb[3]);
  __syncthreads();
  if (lane == 0 && ok) {  // wave 0
    float ts = 0.f, tsx = 0.f;
#pragma unroll
    for (int q = 0; q < kFinLanes; ++q) { ts += r1[q][cl]; tsx += r2[q][cl]; }
    const int64_t o = (static_cast<int64_t>(blockIdx.y) * g.C + c) * 2;
    __hip_atomic_store(part + o, ts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part + o + 1, tsx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!last_arrival(&g_bn_bwd_arrivals[blockIdx.x], gridDim.y, &is_last)) return;
  float ts = 0.f, tsx = 0.f;
  if (ok) {
    for (int q = lane; q < static_cast<int>(gridDim.y); q += kFinLanes) {
      const int64_t o = (static_cast<int64_t>(q) * g.C + c) * 2;
      ts += __hip_atomic_load(part + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tsx += __hip_atomic_load(part + o + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  r1[lane][cl] = ts;
  r2[lane][cl] = tsx;
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&g_bn_bwd_arrivals[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane != 0 || !ok) return;
  ts = 0.f;
  tsx = 0.f;
#pragma unroll
  for (int q = 0; q < kFinLanes; ++q) { ts += r1[q][cl]; tsx += r2[q][cl]; }
  bwd_finish(ts, tsx, c, g, a);
}

// Backward finalize: sliced reduce + parallel combine when the partial list is long and scratch
// (>= 2 * kMaxSlices * C floats) is given, else the single-launch walk.
void launch_bwd_finalize(hipStream_t st, const float* psum, const float* psumx, const Geom& g, const BwdFin& bf,
                         float* scratch) {
  const int cb = (g.C + kFinCh - 1) / kFinCh;
  int S = 1024 / cb;
  if (S > kMaxSlices) S = kMaxSlices;
  const int by_rows = g.nrb / (4 * kFinLanes);
  if (S > by_rows) S = by_rows;
  if (!scratch || S < 4) {
    hipLaunchKernelGGL(bn_bwd_finalize, dim3(cb), dim3(kFinThreads), 0, st, psum, psumx, g, bf);
    return;
  }
  const int per = (g.nrb + S - 1) / S;
  S = (g.nrb + per - 1) / per;
  if (bn_last_block() && cb <= kMaxChanBlocks) {
    hipLaunchKernelGGL(bn_bwd_reduce_last, dim3(cb, S), dim3(kFinThreads), 0, st, psum, psumx, g, per, scratch, bf);
    return;
  }
  hipLaunchKernelGGL(bn_bwd_reduce, dim3(cb, S), dim3(kFinThreads), 0, st, psum, psumx, g, per, scratch);
  hipLaunchKernelGGL(bn_bwd_combine, dim3(cb), dim3(kFinThreads), 0, st, scratch, S, g, bf);
}

template <typename T, int MASK, bool DRES, bool NTL = false>
__global__ void __launch_bounds__(kThreads)
bn_apply_bwd(const T* __restrict__ dy, const T* __restrict__ dy2, const T* __restrict__ x,
             const uint8_t* __restrict__ mbits,
             const float* __restrict__ coef, const float* __restrict__ scale,
             const float* __restrict__ shift, T* __restrict__ dx, T* __restrict__ dres,
             int64_t nvec, int C) {
#if DET_BN_CF
  const int cv = C >> 3;
  if (cv <= kThreads && (kThreads % cv) == 0) {  // channel-fixed mapping (see bn_apply_fwd)
    const int lc = static_cast<int>(threadIdx.x) % cv, rpb = kThreads / cv, c0 = lc << 3;
    float A[8], B[8], Cc[8], sc[8], sh[8];
    load8f(coef + c0, A);
    load8f(coef + C + c0, B);
    load8f(coef + 2 * C + c0, Cc);
    if (MASK == 1) {
      load8f(scale + c0, sc);
      load8f(shift + c0, sh);
    }
    const int64_t nrow = nvec / cv, RS = static_cast<int64_t>(gridDim.x) * rpb;
    for (int64_t r0 = static_cast<int64_t>(blockIdx.x) * rpb + threadIdx.x / cv; r0 < nrow; r0 += 2 * RS) {
      float dv[2][8], xv[2][8];
      unsigned mb[2] = {0xFFu, 0xFFu};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t r = r0 + u * RS;
        if (r < nrow) {
          const int64_t v = r * cv + lc;
          sload8<NTL>(dy + v * 8, dv[u]);
          sload8<NTL>(x + v * 8, xv[u]);
          if (dy2) {
            float e[8];
            sload8<NTL>(dy2 + v * 8, e);
#pragma unroll
            for (int j = 0; j < 8; ++j) dv[u][j] += e[j];
          }
          if (MASK == 2) mb[u] = mbits[v];
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t r = r0 + u * RS;
        if (r < nrow) {
          const int64_t v = r * cv + lc;
          float o[8], dz[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float d = dv[u][j];
            if (MASK == 1) d = __fmaf_rn(xv[u][j], sc[j], sh[j]) > 0.f ? d : 0.f;
            else if (MASK == 2) d = (mb[u] >> j) & 1u ? d : 0.f;
            dz[j] = d;
            o[j] = __fmaf_rn(A[j], d, __fmaf_rn(B[j], xv[u][j], Cc[j]));
          }
          IO8<T>::store(dx + v * 8, o);
          if (DRES) IO8<T>::store(dres + v * 8, dz);
        }
      }
    }
    return;
  }
#endif
  const int64_t S = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t v0 = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; v0 < nvec; v0 += 2 * S) {
    float dv[2][8], xv[2][8];
    unsigned mb[2] = {0xFFu, 0xFFu};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t v = v0 + u * S;
      if (v < nvec) {
        sload8<NTL>(dy + v * 8, dv[u]);
        sload8<NTL>(x + v * 8, xv[u]);
        if (dy2) {
          float e[8];
          sload8<NTL>(dy2 + v * 8, e);
#pragma unroll
          for (int j = 0; j < 8; ++j) dv[u][j] += e[j];
        }
        if (MASK == 2) mb[u] = mbits[v];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t v = v0 + u * S;
      if (v < nvec) {
        // vector index -> first channel; 32-bit modulo (nvec < 2^32 checked on the host)
        const int c0 = static_cast<int>(static_cast<uint32_t>(v) % static_cast<uint32_t>(C >> 3)) << 3;
        float A[8], B[8], Cc[8], o[8], dz[8];
        load8f(coef + c0, A);
        load8f(coef + C + c0, B);
        load8f(coef + 2 * C + c0, Cc);
        float sc[8], sh[8];
        if (MASK == 1) { load8f(scale + c0, sc); load8f(shift + c0, sh); }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float d = dv[u][j];
          if (MASK == 1) d = __fmaf_rn(xv[u][j], sc[j], sh[j]) > 0.f ? d : 0.f;
          else if (MASK == 2) d = (mb[u] >> j) & 1u ? d : 0.f;
          dz[j] = d;
          o[j] = __fmaf_rn(A[j], d, __fmaf_rn(B[j], xv[u][j], Cc[j]));
        }
        IO8<T>::store(dx + v * 8, o);
        if (DRES) IO8<T>::store(dres + v * 8, dz);
      }
    }
  }
}

Geom make_geom(int64_t M, int C) {
  Geom g;
  g.M = M;
  g.C = C;
  const int cg = C / 8;
  g.tpr = cg < kThreads ? cg : kThreads;
  g.R = kThreads / g.tpr;
  const int cblocks = (cg + g.tpr - 1) / g.tpr;
  const int64_t target = cblocks >= 1024 ? 1 : 1024 / cblocks;
  const int64_t min_rows_per_thread = 48;
  int64_t by_work = (M + g.R * min_rows_per_thread - 1) / (g.R * min_rows_per_thread);
  int64_t nrb = target < by_work ? target : by_work;
  if (nrb < 1) nrb = 1;
  int64_t rpb = (M + nrb - 1) / nrb;
  rpb = (rpb + g.R - 1) / g.R * g.R;
  g.rpb = rpb;
  g.nrb = static_cast<int>((M + rpb - 1) / rpb);
  return g;
}

int apply_grid(int64_t nvec, int per_thread) {
  int64_t blocks = (nvec + static_cast<int64_t>(kThreads) * per_thread - 1) / (static_cast<int64_t>(kThreads) * per_thread);
  if (blocks < 1) blocks = 1;
  if (blocks > 256 * 16) blocks = 256 * 16;
  return static_cast<int>(blocks);
}

}  // namespace

extern "C" {

// Number of fp32 workspace elements the fwd/bwd entry points need for an [M, C] activation.
int64_t det_bn_ws_elems(int64_t M, int C) {
  Geom g = make_geom(M, C);
  return 2 * static_cast<int64_t>(g.nrb) * C + 3 * static_cast<int64_t>(C) + fin_scratch_elems(C);
}

// fp32 workspace elements det_bn_fwd_from_partials needs (two-stage finalize scratch).
int64_t det_bn_fin_ws_elems(int C) { return fin_scratch_elems(C); }

// fp32 scratch elements of det_bn_bwd_from_partials' sliced finalize.
int64_t det_bn_bwd_scratch_elems(int C) { return 2 * static_cast<int64_t>(kMaxSlices) * C; }

// dtype: 0 = fp32, 1 = bf16.  res may be null.  Outputs save_mean/save_rstd/scale/shift [C].
int det_bn_fwd_train(void* stream, int dtype, const void* x, const void* res, void* y, int64_t M, int C,
                     const float* gamma, const float* beta, float* running_mean, float* running_var,
                     int64_t* num_batches_tracked, float momentum, float eps, int relu,
                     float* save_mean, float* save_rstd, float* scale, float* shift, float* ws,
                     uint8_t* mbits) {
  if (C % 8 != 0 || M <= 0) return -1;
  if (M * (C / 8) >= (static_cast<int64_t>(1) << 32)) return -3;  // 32-bit vector indexing in apply
  hipStream_t st = static_cast<hipStream_t>(stream);
  Geom g = make_geom(M, C);
  float* pmean = ws;
  float* pm2 = ws + static_cast<int64_t>(g.nrb) * C;
  dim3 grid(g.nrb, (C / 8 + g.tpr - 1) / g.tpr);
  if (dtype == 1)
    hipLaunchKernelGGL(bn_stats_partial<unsigned short>, grid, dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), g, pmean, pm2);
  else
    hipLaunchKernelGGL(bn_stats_partial<float>, grid, dim3(kThreads), 0, st, static_cast<const float*>(x), g,
                       pmean, pm2);
  FinArgs fa{gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps,
             save_mean, save_rstd, scale, shift};
  launch_stats_finalize(st, pmean, pm2, g, fa, ws + 2 * static_cast<int64_t>(g.nrb) * C + 3 * static_cast<int64_t>(C));
  int64_t* bump = num_batches_tracked;
  const int64_t nvec = M * C / 8;
  const int grid2 = apply_grid(nvec, 4);
#define DET_BN_FWD(T, RL, RS)                                                                          \
  do {                                                                                                 \
    if (bn_nt())                                                                                       \
      hipLaunchKernelGGL((bn_apply_fwd<T, RL, RS, true>), dim3(grid2), dim3(kThreads), 0, st,          \
                         static_cast<const T*>(x), static_cast<const T*>(res), static_cast<T*>(y), scale, \
                         shift, nvec, C, bump, mbits);                                                 \
    else                                                                                               \
      hipLaunchKernelGGL((bn_apply_fwd<T, RL, RS>), dim3(grid2), dim3(kThreads), 0, st,                \
                         static_cast<const T*>(x), static_cast<const T*>(res), static_cast<T*>(y), scale, \
                         shift, nvec, C, bump, mbits);                                                 \
  } while (0)
  if (dtype == 1) {
    if (relu && res) DET_BN_FWD(unsigned short, true, true);
    else if (relu) DET_BN_FWD(unsigned short, true, false);
    else if (res) DET_BN_FWD(unsigned short, false, true);
    else DET_BN_FWD(unsigned short, false, false);
  } else {
    if (relu && res) DET_BN_FWD(float, true, true);
    else if (relu) DET_BN_FWD(float, true, false);
    else if (res) DET_BN_FWD(float, false, true);
    else DET_BN_FWD(float, false, false);
  }
  return static_cast<int>(hipGetLastError());
}

// Training statistics only (stats_partial + finalize + num_batches_tracked bump), no apply pass:
// the consumer applies relu(x*scale + shift) itself in its GEMM prologue (det_conv.hip), so the
// normalised activation is never written to HBM.  ResNet bottlenecks use it for bn2 -> conv3.
int det_bn_stats_train(void* stream, int dtype, const void* x, int64_t M, int C, const float* gamma,
                       const float* beta, float* running_mean, float* running_var, int64_t* num_batches_tracked,
                       float momentum, float eps, float* save_mean, float* save_rstd, float* scale, float* shift,
                       float* ws) {
  if (C % 8 != 0 || M <= 0) return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  Geom g = make_geom(M, C);
  float* pmean = ws;
  float* pm2 = ws + static_cast<int64_t>(g.nrb) * C;
  dim3 grid(g.nrb, (C / 8 + g.tpr - 1) / g.tpr);
  if (dtype == 1)
    hipLaunchKernelGGL(bn_stats_partial<unsigned short>, grid, dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), g, pmean, pm2);
  else
    hipLaunchKernelGGL(bn_stats_partial<float>, grid, dim3(kThreads), 0, st, static_cast<const float*>(x), g,
                       pmean, pm2);
  FinArgs fa{gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps,
             save_mean, save_rstd, scale, shift};
  if (momentum >= 0.f) fa.bump = num_batches_tracked;  // bumped by the finalize itself
  launch_stats_finalize(st, pmean, pm2, g, fa, ws + 2 * static_cast<int64_t>(g.nrb) * C + 3 * static_cast<int64_t>(C));
  if (num_batches_tracked && !fa.bump) hipLaunchKernelGGL(bump_counter, dim3(1), dim3(1), 0, st, num_batches_tracked);
  return static_cast<int>(hipGetLastError());
}

// Training forward when the producer already computed the statistics partials (det_conv.hip GEMM
// epilogue): Chan-merge the [nrb, C] (mean, M2) partials over row-blocks of `rpb` rows, then apply.
// ws (nullable, >= det_bn_fin_ws_elems(C) floats, 8-B aligned): scratch of the two-stage finalize.
// Skips the stats pass over x entirely.  apply = 0 stops after the finalize (the consumer applies
// scale/shift itself, e.g. in its GEMM prologue); num_batches_tracked is then bumped here.
int det_bn_fwd_from_partials(void* stream, int dtype, const void* x, const void* res, void* y, int64_t M, int C,
                             int rpb, int nrb, const float* pmean, const float* pm2, const float* gamma,
                             const float* beta, float* running_mean, float* running_var,
                             int64_t* num_batches_tracked, float momentum, float eps, int relu, int apply,
                             float* save_mean, float* save_rstd, float* scale, float* shift, uint8_t* mbits,
                             float* ws, const float* res_scale, const float* res_shift) {
  if (C % 8 != 0 || M <= 0 || rpb <= 0 || nrb != static_cast<int>((M + rpb - 1) / rpb)) return -1;
  if ((res_scale == nullptr) != (res_shift == nullptr) || (res_scale && (!res || dtype != 1 || !relu))) return -2;
  if (M * (C / 8) >= (static_cast<int64_t>(1) << 32)) return -3;
  hipStream_t st = static_cast<hipStream_t>(stream);
  Geom g = make_geom(M, C);
  g.rpb = rpb;
  g.nrb = nrb;
  FinArgs fa{gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps,
             save_mean, save_rstd, scale, shift};
  if (!apply && momentum >= 0.f) fa.bump = num_batches_tracked;  // no apply kernel to bump it
  launch_stats_finalize(st, pmean, pm2, g, fa, ws);
  int64_t* bump = num_batches_tracked;
  if (!apply) {
    if (bump && !fa.bump) hipLaunchKernelGGL(bump_counter, dim3(1), dim3(1), 0, st, bump);
    return static_cast<int>(hipGetLastError());
  }
  const int64_t nvec = M * C / 8;
  const int grid2 = apply_grid(nvec, 4);
  if (res_scale) {  // the residual is a deferred BN apply of its input res (RES 2)
    if (bn_nt())
      hipLaunchKernelGGL((bn_apply_fwd<unsigned short, true, 2, true>), dim3(grid2), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(res),
                       static_cast<unsigned short*>(y), scale, shift, nvec, C, bump, mbits, res_scale, res_shift);
    else
      hipLaunchKernelGGL((bn_apply_fwd<unsigned short, true, 2>), dim3(grid2), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(res),
                       static_cast<unsigned short*>(y), scale, shift, nvec, C, bump, mbits, res_scale, res_shift);
    return static_cast<int>(hipGetLastError());
  }
#define DET_BN_FWD(T, RL, RS)                                                                          \
  do {                                                                                                 \
    if (bn_nt())                                                                                       \
      hipLaunchKernelGGL((bn_apply_fwd<T, RL, RS, true>), dim3(grid2), dim3(kThreads), 0, st,          \
                         static_cast<const T*>(x), static_cast<const T*>(res), static_cast<T*>(y), scale, \
                         shift, nvec, C, bump, mbits);                                                 \
    else                                                                                               \
      hipLaunchKernelGGL((bn_apply_fwd<T, RL, RS>), dim3(grid2), dim3(kThreads), 0, st,                \
                         static_cast<const T*>(x), static_cast<const T*>(res), static_cast<T*>(y), scale, \
                         shift, nvec, C, bump, mbits);                                                 \
  } while (0)
  if (dtype == 1) {
    if (relu && res) DET_BN_FWD(unsigned short, true, true);
    else if (relu) DET_BN_FWD(unsigned short, true, false);
    else if (res) DET_BN_FWD(unsigned short, false, true);
    else DET_BN_FWD(unsigned short, false, false);
  } else {
    if (relu && res) DET_BN_FWD(float, true, true);
    else if (relu) DET_BN_FWD(float, true, false);
    else if (res) DET_BN_FWD(float, false, true);
    else DET_BN_FWD(float, false, false);
  }
  return static_cast<int>(hipGetLastError());
}

// Training apply with precomputed scale/shift: y = relu(x*scale + shift + res) and its mask bits
// (the materialisation of a BN apply deferred onto a consuming conv that could not take it).
// res_scale / res_shift (nullable): the residual is a deferred BN apply of res (bn_apply_fwd RES 2).
int det_bn_apply_res_mbits(void* stream, const void* x, const void* res, void* y, int64_t M, int C, const float* scale,
                           const float* shift, uint8_t* mbits, const float* res_scale, const float* res_shift) {
  if (C % 8 != 0 || M <= 0 || !res || !mbits) return -1;
  if ((res_scale == nullptr) != (res_shift == nullptr)) return -2;
  if (M * (C / 8) >= (static_cast<int64_t>(1) << 32)) return -3;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t nvec = M * C / 8;
  if (res_scale)
    if (bn_nt())
      hipLaunchKernelGGL((bn_apply_fwd<unsigned short, true, 2, true>), dim3(apply_grid(nvec, 4)), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(res),
                       static_cast<unsigned short*>(y), scale, shift, nvec, C, static_cast<int64_t*>(nullptr), mbits,
                       res_scale, res_shift);
    else
      hipLaunchKernelGGL((bn_apply_fwd<unsigned short, true, 2>), dim3(apply_grid(nvec, 4)), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(res),
                       static_cast<unsigned short*>(y), scale, shift, nvec, C, static_cast<int64_t*>(nullptr), mbits,
                       res_scale, res_shift);
  else
    if (bn_nt())
      hipLaunchKernelGGL((bn_apply_fwd<unsigned short, true, 1, true>), dim3(apply_grid(nvec, 4)), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(res),
                       static_cast<unsigned short*>(y), scale, shift, nvec, C, static_cast<int64_t*>(nullptr), mbits);
    else
      hipLaunchKernelGGL((bn_apply_fwd<unsigned short, true, 1>), dim3(apply_grid(nvec, 4)), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(res),
                       static_cast<unsigned short*>(y), scale, shift, nvec, C, static_cast<int64_t*>(nullptr), mbits);
  return static_cast<int>(hipGetLastError());
}

// Inference / frozen-stats path: y = act(x*scale + shift [+ res]) with host-prepared scale/shift.
int det_bn_apply(void* stream, int dtype, const void* x, const void* res, void* y, int64_t M, int C,
                 const float* scale, const float* shift, int relu) {
  if (C % 8 != 0 || M <= 0) return -1;
  if (M * (C / 8) >= (static_cast<int64_t>(1) << 32)) return -3;  // 32-bit vector indexing in apply
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t nvec = M * C / 8;
  const int grid2 = apply_grid(nvec, 4);
  int64_t* bump = nullptr;
  uint8_t* mbits = nullptr;
  if (dtype == 1) {
    if (relu && res) DET_BN_FWD(unsigned short, true, true);
    else if (relu) DET_BN_FWD(unsigned short, true, false);
    else if (res) DET_BN_FWD(unsigned short, false, true);
    else DET_BN_FWD(unsigned short, false, false);
  } else {
    if (relu && res) DET_BN_FWD(float, true, true);
    else if (relu) DET_BN_FWD(float, true, false);
    else if (res) DET_BN_FWD(float, false, true);
    else DET_BN_FWD(float, false, false);
  }
#undef DET_BN_FWD
  return static_cast<int>(hipGetLastError());
}

// mask_mode: 0 none, 1 relu (mask recomputed from x), 2 relu (bitmask written by the forward).
// dy2 (nullable): a second upstream gradient of the output, summed with dy inside both passes —
// the identity-shortcut gradient of a residual block, which would otherwise cost an elementwise
// add over the whole activation (read 2, write 1) before this backward.
// dres may be null.
// dgamma/dbeta may be null.  ws >= det_bn_ws_elems(M, C).
// BatchNorm backward whose partial sums (psum = sum d, psumx = sum d * (x - mean) over row-blocks of
// rpb rows, [nrb, C]) were produced by the epilogue of the GEMM that computed d (the dgrad of the
// consuming conv, with the ReLU mask and the identity-shortcut gradient already applied:
// det_conv_nt's BN-backward epilogue).  Runs the finalize and an unmasked apply: dx = A d + B x + C.
int det_bn_bwd_from_partials(void* stream, int dtype, const void* d, const void* x, int64_t M, int C, const float* gamma,
                             const float* save_mean, const float* save_rstd, const float* psum, const float* psumx,
                             int nrb, int64_t rpb, void* dx, float* dgamma, float* dbeta, float* coef, float* scratch) {
  if (C % 8 != 0 || M <= 0 || nrb <= 0) return -1;
  if (M * (C / 8) >= (static_cast<int64_t>(1) << 32)) return -3;
  hipStream_t st = static_cast<hipStream_t>(stream);
  Geom g = make_geom(M, C);
  g.nrb = nrb;
  g.rpb = rpb;
  BwdFin bf{gamma, save_rstd, save_mean, dgamma, dbeta, coef};
  launch_bwd_finalize(st, psum, psumx, g, bf, scratch);
  const int64_t nvec = M * C / 8;
  const int grid2 = apply_grid(nvec, 2);
  if (dtype == 1)
    if (bn_nt())
      hipLaunchKernelGGL((bn_apply_bwd<unsigned short, 0, false, true>), dim3(grid2), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(d), static_cast<const unsigned short*>(nullptr),
                       static_cast<const unsigned short*>(x), static_cast<const uint8_t*>(nullptr), coef,
                       static_cast<const float*>(nullptr), static_cast<const float*>(nullptr),
                       static_cast<unsigned short*>(dx), static_cast<unsigned short*>(nullptr), nvec, C);
    else
      hipLaunchKernelGGL((bn_apply_bwd<unsigned short, 0, false>), dim3(grid2), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(d), static_cast<const unsigned short*>(nullptr),
                       static_cast<const unsigned short*>(x), static_cast<const uint8_t*>(nullptr), coef,
                       static_cast<const float*>(nullptr), static_cast<const float*>(nullptr),
                       static_cast<unsigned short*>(dx), static_cast<unsigned short*>(nullptr), nvec, C);
  else
    if (bn_nt())
      hipLaunchKernelGGL((bn_apply_bwd<float, 0, false, true>), dim3(grid2), dim3(kThreads), 0, st, static_cast<const float*>(d),
                       static_cast<const float*>(nullptr), static_cast<const float*>(x),
                       static_cast<const uint8_t*>(nullptr), coef, static_cast<const float*>(nullptr),
                       static_cast<const float*>(nullptr), static_cast<float*>(dx), static_cast<float*>(nullptr), nvec, C);
    else
      hipLaunchKernelGGL((bn_apply_bwd<float, 0, false>), dim3(grid2), dim3(kThreads), 0, st, static_cast<const float*>(d),
                       static_cast<const float*>(nullptr), static_cast<const float*>(x),
                       static_cast<const uint8_t*>(nullptr), coef, static_cast<const float*>(nullptr),
                       static_cast<const float*>(nullptr), static_cast<float*>(dx), static_cast<float*>(nullptr), nvec, C);
  return static_cast<int>(hipGetLastError());
}

// det_bn_bwd_from_partials split in two for a consumer that applies the BN backward itself (the
// input-gradient GEMM of the conv that produced x stages dx = A d + B x + C as its A operand,
// det_conv.hip ABN): the finalize only (dgamma, dbeta, coef [3][C]) ...
int det_bn_bwd_finalize_partials(void* stream, int64_t M, int C, const float* gamma, const float* save_mean,
                                 const float* save_rstd, const float* psum, const float* psumx, int nrb, int64_t rpb,
                                 float* dgamma, float* dbeta, float* coef, float* scratch) {
  if (C % 8 != 0 || M <= 0 || nrb <= 0) return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  Geom g = make_geom(M, C);
  g.nrb = nrb;
  g.rpb = rpb;
  BwdFin bf{gamma, save_rstd, save_mean, dgamma, dbeta, coef};
  launch_bwd_finalize(st, psum, psumx, g, bf, scratch);
  return static_cast<int>(hipGetLastError());
}

// ... and the unmasked apply alone, dx = A d + B x + C (the fallback when that consumer cannot).
int det_bn_bwd_apply_coef(void* stream, int dtype, const void* d, const void* x, int64_t M, int C, const float* coef,
                          void* dx) {
  if (C % 8 != 0 || M <= 0) return -1;
  if (M * (C / 8) >= (static_cast<int64_t>(1) << 32)) return -3;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t nvec = M * C / 8;
  const int grid2 = apply_grid(nvec, 2);
  if (dtype == 1)
    if (bn_nt())
      hipLaunchKernelGGL((bn_apply_bwd<unsigned short, 0, false, true>), dim3(grid2), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(d), static_cast<const unsigned short*>(nullptr),
                       static_cast<const unsigned short*>(x), static_cast<const uint8_t*>(nullptr), coef,
                       static_cast<const float*>(nullptr), static_cast<const float*>(nullptr),
                       static_cast<unsigned short*>(dx), static_cast<unsigned short*>(nullptr), nvec, C);
    else
      hipLaunchKernelGGL((bn_apply_bwd<unsigned short, 0, false>), dim3(grid2), dim3(kThreads), 0, st,
                       static_cast<const unsigned short*>(d), static_cast<const unsigned short*>(nullptr),
                       static_cast<const unsigned short*>(x), static_cast<const uint8_t*>(nullptr), coef,
                       static_cast<const float*>(nullptr), static_cast<const float*>(nullptr),
                       static_cast<unsigned short*>(dx), static_cast<unsigned short*>(nullptr), nvec, C);
  else
    if (bn_nt())
      hipLaunchKernelGGL((bn_apply_bwd<float, 0, false, true>), dim3(grid2), dim3(kThreads), 0, st, static_cast<const float*>(d),
                       static_cast<const float*>(nullptr), static_cast<const float*>(x),
                       static_cast<const uint8_t*>(nullptr), coef, static_cast<const float*>(nullptr),
                       static_cast<const float*>(nullptr), static_cast<float*>(dx), static_cast<float*>(nullptr), nvec, C);
    else
      hipLaunchKernelGGL((bn_apply_bwd<float, 0, false>), dim3(grid2), dim3(kThreads), 0, st, static_cast<const float*>(d),
                       static_cast<const float*>(nullptr), static_cast<const float*>(x),
                       static_cast<const uint8_t*>(nullptr), coef, static_cast<const float*>(nullptr),
                       static_cast<const float*>(nullptr), static_cast<float*>(dx), static_cast<float*>(nullptr), nvec, C);
  return static_cast<int>(hipGetLastError());
}

// Offset (floats) of the [3][C] apply coefficients inside det_bn_bwd's workspace.
int64_t det_bn_bwd_coef_offset(int64_t M, int C) { return 2 * static_cast<int64_t>(make_geom(M, C).nrb) * C; }

int det_bn_bwd(void* stream, int dtype, const void* dy, const void* dy2, const void* x, const void* mbits, int64_t M, int C,
               int mask_mode, const float* gamma, const float* save_mean, const float* save_rstd,
               const float* scale, const float* shift, void* dx, void* dres, float* dgamma, float* dbeta,
               float* ws, int apply) {
  if (C % 8 != 0 || M <= 0) return -1;
  if (M * (C / 8) >= (static_cast<int64_t>(1) << 32)) return -3;  // 32-bit vector indexing in apply
  if (mask_mode == 2 && !mbits) return -2;
  hipStream_t st = static_cast<hipStream_t>(stream);
  Geom g = make_geom(M, C);
  float* psum = ws;
  float* psumx = ws + static_cast<int64_t>(g.nrb) * C;
  float* coef = psumx + static_cast<int64_t>(g.nrb) * C;
  dim3 grid(g.nrb, (C / 8 + g.tpr - 1) / g.tpr);
#define DET_BN_P(T, MK)                                                                                \
  hipLaunchKernelGGL((bn_bwd_partial<T, MK>), grid, dim3(kThreads), 0, st, static_cast<const T*>(dy),   \
                     static_cast<const T*>(dy2), static_cast<const T*>(x), static_cast<const uint8_t*>(mbits), g, save_mean, scale, shift, psum, psumx)
  if (dtype == 1) {
    if (mask_mode == 0) DET_BN_P(unsigned short, 0);
    else if (mask_mode == 1) DET_BN_P(unsigned short, 1);
    else DET_BN_P(unsigned short, 2);
  } else {
    if (mask_mode == 0) DET_BN_P(float, 0);
    else if (mask_mode == 1) DET_BN_P(float, 1);
    else DET_BN_P(float, 2);
  }
#undef DET_BN_P
  BwdFin bf{gamma, save_rstd, save_mean, dgamma, dbeta, coef};
  launch_bwd_finalize(st, psum, psumx, g, bf, coef + 3 * static_cast<int64_t>(C));
  // apply = 0: stop at the coefficients (ws + det_bn_bwd_coef_offset): a consuming GEMM stages the
  // apply dx = coef[0] dy + coef[1] x + coef[2] itself (mask mode 0, no dy2 / dres)
  if (!apply) return (mask_mode == 0 && !dy2 && !dres) ? static_cast<int>(hipGetLastError()) : -2;
  const int64_t nvec = M * C / 8;
  const int grid2 = apply_grid(nvec, 2);
#define DET_BN_B(T, MK, DR)                                                                            \
  do {                                                                                                 \
    if (bn_nt())                                                                                       \
      hipLaunchKernelGGL((bn_apply_bwd<T, MK, DR, true>), dim3(grid2), dim3(kThreads), 0, st,          \
                         static_cast<const T*>(dy), static_cast<const T*>(dy2), static_cast<const T*>(x), \
                         static_cast<const uint8_t*>(mbits), coef, scale, shift, static_cast<T*>(dx),  \
                         static_cast<T*>(dres), nvec, C);                                              \
    else                                                                                               \
      hipLaunchKernelGGL((bn_apply_bwd<T, MK, DR>), dim3(grid2), dim3(kThreads), 0, st,                \
                         static_cast<const T*>(dy), static_cast<const T*>(dy2), static_cast<const T*>(x), \
                         static_cast<const uint8_t*>(mbits), coef, scale, shift, static_cast<T*>(dx),  \
                         static_cast<T*>(dres), nvec, C);                                              \
  } while (0)
#define DET_BN_B_MASK(T, DR)                 \
  if (mask_mode == 0) DET_BN_B(T, 0, DR);    \
  else if (mask_mode == 1) DET_BN_B(T, 1, DR); \
  else DET_BN_B(T, 2, DR);
  if (dtype == 1) {
    if (dres) { DET_BN_B_MASK(unsigned short, true) } else { DET_BN_B_MASK(unsigned short, false) }
  } else {
    if (dres) { DET_BN_B_MASK(float, true) } else { DET_BN_B_MASK(float, false) }
  }
#undef DET_BN_B_MASK
#undef DET_BN_B
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
