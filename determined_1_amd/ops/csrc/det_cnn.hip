// det_cnn.hip — the CIFAR-10 CNN of the ASHA benchmark (BASELINE configs #2/#4) on one generic
// gather-GEMM kernel: every conv / linear pass of forward and backward, with bias, ReLU, 2x2 max-pool,
// dropout and the pooling / dropout backward folded into operand loaders and epilogues.
//
// Network (reference examples/computer_vision/cifar10_pytorch/model_def.py:47-65), NHWC:
//   x [N,32,32,3] -> conv1 3->32 -> relu -> a1 [N,30,30,32]
//   -> conv2 32->32 -> relu -> maxpool2 -> dropout2d -> a2 [N,14,14,32] (+ argmax idx2)
//   -> conv3 32->64 pad 1 -> relu -> a3 [N,14,14,64]
//   -> conv4 64->64 -> relu -> maxpool2 -> dropout2d -> a4 [N,6,6,64] (+ idx4)
//   -> flatten (torch's NCHW order: k = c*36 + h*6 + w) -> fc1 2304->512 -> relu -> dropout -> a5
//   -> fc2 512->10 -> logits (fp32)
//
// Why gather-GEMMs: at batch 16-64 every pass is a few microseconds of work on a few hundred
// workgroups, so the step is launch- and latency-bound (round 4: ~130 library kernels per batch,
// profiles/r4_cifar_trial_steady.txt).  What matters is the number of passes and that no activation
// is written just to be re-read by an elementwise kernel: here the forward is 8 launches (masks +
// 6 GEMMs + split-K finishes, pooling/dropout in the conv epilogues), the backward ~10 (each layer's
// weight- and input-gradient GEMMs share one launch, one launch reduces every split-K weight
// gradient into the grad arena), and the unpooling / ReLU / dropout backward never materialise: the
// gradient operand loader routes the pooled gradient to the argmax position as it stages the tile.
//
// GEMM: C[M,N] = sum_k A[m,k] B[k,n] on MFMA (64x64 block tile, BK 64, bf16 or exact-fp32 MFMA,
// fp32 accumulate), one kernel instantiation per (A source, B source, epilogue) kind.  Every pass is
// latency-bound (a tile's global loads take longer than its MFMAs), so the levers are loads in
// flight per iteration (BK 64, 16-B gathers), split-K for launches with few tiles, and small
// per-kind code (see gemm_tile).
//
// Dropout masks: one launch per forward draws every mask from Philox4x32-10 keyed by (seed, offset) +
// the device offset counter (ops/transformer.py rng_base), so hipGraph replays draw fresh masks and
// backward reads the masks the forward used.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace {

constexpr int BM = 64, BN = 64, NT = 256;

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

// element access for T = float (dtype 0) or bf16 (dtype 1)
__device__ __forceinline__ float ld(const void* p, int dt, int64_t i) {
  return dt == 0 ? static_cast<const float*>(p)[i] : bf2f(static_cast<const uint16_t*>(p)[i]);
}
__device__ __forceinline__ void st(void* p, int dt, int64_t i, float v) {
  if (dt == 0) static_cast<float*>(p)[i] = v;
  else static_cast<uint16_t*>(p)[i] = f2bf(v);
}

// ---- operand loaders ---------------------------------------------------------------------------
// Operand roles: ACT = an activation gathered as im2col (conv) or flattened (fc); GRAD = a gradient
// w.r.t. a layer output; WGT = a weight through its strides; ONES is the bias column of a wgrad.
enum Src : int {
  S_ACT_CONV = 0,     // act[n][h][w][c], (pix, kk=(r*S+s)*C+c): h = ho*1 + r - pad (zero outside)
  S_ACT_FLAT = 1,     // act[n][h][w][c] read in torch's NCHW flatten order: kk = c*HW + h*W + w
  S_ACT_ROWS = 2,     // act[n][j] (fc input rows)
  S_GRAD_ROWS = 3,    // g[n][j]
  S_GRAD_CONV_T = 4,  // dgrad gather: g over output pixels, kk = (r*S+s)*Cg + o, input pixel (h, w):
                      //   output (h + pad - r, w + pad - s)
  S_WGT_CONV = 5,     // W[o][c][r][s] via strides: B[kk=(r*S+s)*C+c][n=o]        (forward)
  S_WGT_CONV_T = 6,   // W[o][c][r][s]: B[kk=(r*S+s)*Cout+o][n=c]                 (dgrad)
  S_WGT_FC = 7,       // W[o][j]: B[k=j][n=o]                                        (fc forward)
  S_WGT_FC_T = 8,     // W[o][j]: B[k=o][n=j]                                        (fc dgrad)
};

struct Operand {
  const void* p;     // tensor
  int dt;            // 0 f32, 1 bf16, 2 f32 regardless of the GEMM's dtype (logits-side fp32)
  int src;           // Src
  // geometry of the tensor the index maps read (activation / gradient grid)
  int H, W, C;       // grid of p (for GRAD_CONV_T: the output-gradient grid Ho, Wo, Cout)
  int R, S, pad;     // conv kernel
  int OH, OW;        // the GEMM's pixel grid (conv forward/wgrad: output grid; dgrad: input grid)
  int pool;          // 1: the pixel grid is a 2x2-window-ordered pre-pool grid (m = win*4 + q)
  // unpool (GRAD operands of a pooled layer): p holds the pooled gradient [n][OH/2][OW/2][C];
  // idx the argmax (0..3) per pooled element; the value is routed to the argmax position only
  const uint8_t* idx;
  int64_t so, sc, sr, ss;  // weight strides (o, c, r, s) in elements / (o, j) for fc
  int transpose;     // the operand is read as A[m][k] = T[k][m] (wgrad's gradient operand)
};

// All index math is 32-bit unsigned (every tensor here has < 2^31 elements; 64-bit divisions are a
// long software sequence per element): the decomposition of the thread's fixed row is done once per
// 8-element group, and 8 consecutive reduction indices that share one kernel tap (C % 8 == 0) are
// one 16-B (bf16) / 32-B (fp32) vector load.

// 8 consecutive elements at p[e .. e+7] (contiguous), converted to fp32
__device__ __forceinline__ void ld8(const void* p, int dt, uint32_t e, float (&v)[8]) {
  if (dt == 1) {
    typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
    const u16x8 r = *reinterpret_cast<const u16x8*>(static_cast<const uint16_t*>(p) + e);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f(r[j]);
  } else {
    const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + e);
    const float4 b = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + e + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}
__device__ __forceinline__ float ld32(const void* p, int dt, uint32_t e) {
  return dt == 0 ? static_cast<const float*>(p)[e] : bf2f(static_cast<const uint16_t*>(p)[e]);
}
__device__ __forceinline__ int odt(const Operand& o) { return o.dt == 2 ? 0 : o.dt; }

// pixel index -> (n, h, w) over an OH x OW grid (window-ordered 2x2 groups if pool)
__device__ __forceinline__ void pix_nhw(const Operand& o, uint32_t pix, uint32_t& n, int& h, int& w) {
  if (o.pool) {
    const uint32_t q = pix & 3u, win = pix >> 2;
    const uint32_t PW = static_cast<uint32_t>(o.OW) >> 1, PH = static_cast<uint32_t>(o.OH) >> 1;
    const uint32_t t = win / PW, pw = win - t * PW;
    n = t / PH;
    const uint32_t ph = t - n * PH;
    h = static_cast<int>(2 * ph + (q >> 1));
    w = static_cast<int>(2 * pw + (q & 1u));
  } else {
    const uint32_t t = pix / static_cast<uint32_t>(o.OW);
    w = static_cast<int>(pix - t * static_cast<uint32_t>(o.OW));
    n = t / static_cast<uint32_t>(o.OH);
    h = static_cast<int>(t - n * static_cast<uint32_t>(o.OH));
  }
}

// the unpooled gradient at pre-pool position (n, h, w, c): the pooled gradient routed to the argmax
__device__ __forceinline__ float unpool_at(const Operand& o, uint32_t n, int h, int w, uint32_t c) {
  const uint32_t PH = static_cast<uint32_t>(o.H) >> 1, PW = static_cast<uint32_t>(o.W) >> 1;
  const uint32_t pe = ((n * PH + static_cast<uint32_t>(h >> 1)) * PW + static_cast<uint32_t>(w >> 1)) *
                      static_cast<uint32_t>(o.C) + c;
  return o.idx[pe] == static_cast<uint8_t>((h & 1) << 1 | (w & 1)) ? ld32(o.p, o.dt, pe) : 0.f;
}

// A[row][kk0 .. kk0+7] (or B[kk0 .. kk0+7][row]) for a fixed GEMM row; nk <= 8 of them are in range
template <int SRC>
__device__ __forceinline__ void opval8(const Operand& o, uint32_t row, uint32_t kk0, int nk, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
  const int dt = odt(o);
  switch (SRC) {
    case S_ACT_CONV: {
      uint32_t n;
      int oh, ow;
      pix_nhw(o, row, n, oh, ow);
      const uint32_t C = static_cast<uint32_t>(o.C);
      if ((C & 7u) == 0 && nk == 8) {  // one tap, 8 consecutive channels: one vector load
        const uint32_t rs = kk0 / C, c0 = kk0 - rs * C;
        const int r = static_cast<int>(rs / static_cast<uint32_t>(o.S)), s = static_cast<int>(rs) - r * o.S;
        const int h = oh + r - o.pad, w = ow + s - o.pad;
        if (h >= 0 && h < o.H && w >= 0 && w < o.W)
          ld8(o.p, dt, ((n * static_cast<uint32_t>(o.H) + h) * static_cast<uint32_t>(o.W) + w) * C + c0, v);
        return;
      }
      for (int j = 0; j < nk; ++j) {
        const uint32_t kk = kk0 + j, rs = kk / C, c = kk - rs * C;
        const int r = static_cast<int>(rs / static_cast<uint32_t>(o.S)), s = static_cast<int>(rs) - r * o.S;
        const int h = oh + r - o.pad, w = ow + s - o.pad;
        if (h >= 0 && h < o.H && w >= 0 && w < o.W)
          v[j] = ld32(o.p, dt, ((n * static_cast<uint32_t>(o.H) + h) * static_cast<uint32_t>(o.W) + w) * C + c);
      }
      return;
    }
    case S_ACT_FLAT: {  // torch's NCHW flatten order over an NHWC tensor
      const uint32_t hw = static_cast<uint32_t>(o.H * o.W), C = static_cast<uint32_t>(o.C);
      for (int j = 0; j < nk; ++j) {
        const uint32_t kk = kk0 + j, c = kk / hw;
        v[j] = ld32(o.p, dt, (row * hw + (kk - c * hw)) * C + c);
      }
      return;
    }
    case S_ACT_ROWS:
    case S_GRAD_ROWS: {
      const uint32_t e = row * static_cast<uint32_t>(o.C) + kk0;
      if (nk == 8 && (o.C & 7) == 0) {
        ld8(o.p, dt, e, v);
        return;
      }
      for (int j = 0; j < nk; ++j) v[j] = ld32(o.p, dt, e + j);
      return;
    }
    case S_GRAD_CONV_T: {  // input pixel `row` of the dgrad grid; kk = (r*S+s)*C + og
      uint32_t n;
      int ih, iw;
      pix_nhw(o, row, n, ih, iw);
      const uint32_t C = static_cast<uint32_t>(o.C);
      const bool vec = (C & 7u) == 0 && nk == 8;
      for (int j = 0; j < (vec ? 1 : nk); ++j) {
        const uint32_t kk = kk0 + j, rs = kk / C, og = kk - rs * C;
        const int r = static_cast<int>(rs / static_cast<uint32_t>(o.S)), s = static_cast<int>(rs) - r * o.S;
        const int h = ih + o.pad - r, w = iw + o.pad - s;  // output-gradient position
        if (h < 0 || h >= o.H || w < 0 || w >= o.W) continue;
        if (o.idx != nullptr) {
          if (vec) {
            for (int q = 0; q < 8; ++q) v[q] = unpool_at(o, n, h, w, og + q);
          } else {
            v[j] = unpool_at(o, n, h, w, og);
          }
        } else {
          const uint32_t e = ((n * static_cast<uint32_t>(o.H) + h) * static_cast<uint32_t>(o.W) + w) * C + og;
          if (vec) ld8(o.p, dt, e, v);
          else v[j] = ld32(o.p, dt, e);
        }
      }
      return;
    }
    case S_WGT_CONV: {  // B[kk = (r*S+s)*C + c][n = o] = W[o][c][r][s]
      const uint32_t C = static_cast<uint32_t>(o.C);
      if ((C & 7u) == 0 && nk == 8 && o.sc == 1) {
        const uint32_t rs = kk0 / C, c0 = kk0 - rs * C;
        const uint32_t r = rs / static_cast<uint32_t>(o.S), s = rs - r * static_cast<uint32_t>(o.S);
        ld8(o.p, dt, static_cast<uint32_t>(row * o.so + c0 + r * o.sr + s * o.ss), v);
        return;
      }
      for (int j = 0; j < nk; ++j) {
        const uint32_t kk = kk0 + j, rs = kk / C, c = kk - rs * C;
        const uint32_t r = rs / static_cast<uint32_t>(o.S), s = rs - r * static_cast<uint32_t>(o.S);
        v[j] = ld32(o.p, dt, static_cast<uint32_t>(row * o.so + c * o.sc + r * o.sr + s * o.ss));
      }
      return;
    }
    case S_WGT_CONV_T: {  // B[kk = (r*S+s)*Cout + og][n = c] = W[og][c][r][s]
      const uint32_t C = static_cast<uint32_t>(o.C);
      for (int j = 0; j < nk; ++j) {
        const uint32_t kk = kk0 + j, rs = kk / C, og = kk - rs * C;
        const uint32_t r = rs / static_cast<uint32_t>(o.S), s = rs - r * static_cast<uint32_t>(o.S);
        v[j] = ld32(o.p, dt, static_cast<uint32_t>(og * o.so + row * o.sc + r * o.sr + s * o.ss));
      }
      return;
    }
    case S_WGT_FC: {  // B[k = j][n = o] = W[o][j]
      const uint32_t e = static_cast<uint32_t>(row * o.so + kk0 * o.sc);
      if (nk == 8 && o.sc == 1 && (o.so & 7) == 0) {
        ld8(o.p, dt, e, v);
        return;
      }
      for (int j = 0; j < nk; ++j) v[j] = ld32(o.p, dt, static_cast<uint32_t>(e + j * o.sc));
      return;
    }
    case S_WGT_FC_T:  // B[k = o][n = j] = W[o][j]
      for (int j = 0; j < nk; ++j) v[j] = ld32(o.p, dt, static_cast<uint32_t>((kk0 + j) * o.so + row * o.sc));
      return;
  }
}

// weight-gradient operands, 8 consecutive reduction indices (pixels / images) k0 .. k0+7:
//   A[m = out channel][k] = g[k][m] (with the unpool routing of a pooled layer)
template <int SRC>
__device__ __forceinline__ void gradval8(const Operand& o, uint32_t m, uint32_t k0, int nk, float (&v)[8]) {
  const int dt = odt(o);
  const uint32_t C = static_cast<uint32_t>(o.C);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
  if (SRC == S_GRAD_ROWS || o.idx == nullptr) {
    for (int j = 0; j < nk; ++j) v[j] = ld32(o.p, dt, (k0 + j) * C + m);
    return;
  }
  uint32_t n;
  int h, w;
  Operand g = o;
  g.pool = 0;
  g.H = o.OH;  // unpool_at reads the pooled grid of the OH x OW pre-pool grid
  g.W = o.OW;
  pix_nhw(g, k0, n, h, w);
  for (int j = 0; j < nk; ++j) {
    v[j] = unpool_at(g, n, h, w, m);
    if (++w == o.OW) {  // next pixel, row-major
      w = 0;
      if (++h == o.OH) {
        h = 0;
        ++n;
      }
    }
  }
}
//   B[k][n = weight column] = the activation of pixel / image k at column n (conv: kk = n)
template <int SRC>
__device__ __forceinline__ void actcol8(const Operand& o, uint32_t k0, uint32_t col, int nk, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
  const int dt = odt(o);
  if (SRC == S_ACT_ROWS) {
    for (int j = 0; j < nk; ++j) v[j] = ld32(o.p, dt, (k0 + j) * static_cast<uint32_t>(o.C) + col);
    return;
  }
  if (SRC == S_ACT_FLAT) {
    const uint32_t hw = static_cast<uint32_t>(o.H * o.W), C = static_cast<uint32_t>(o.C);
    const uint32_t c = col / hw, rem = col - c * hw;
    for (int j = 0; j < nk; ++j) v[j] = ld32(o.p, dt, ((k0 + j) * hw + rem) * C + c);
    return;
  }
  // S_ACT_CONV: the tap / channel of column `col` is fixed, the pixel advances
  const uint32_t C = static_cast<uint32_t>(o.C);
  const uint32_t rs = col / C, c = col - rs * C;
  const int r = static_cast<int>(rs / static_cast<uint32_t>(o.S)), s = static_cast<int>(rs) - r * o.S;
  uint32_t n;
  int oh, ow;
  Operand g = o;
  g.pool = 0;
  pix_nhw(g, k0, n, oh, ow);
  for (int j = 0; j < nk; ++j) {
    const int h = oh + r - o.pad, w = ow + s - o.pad;
    if (h >= 0 && h < o.H && w >= 0 && w < o.W)
      v[j] = ld32(o.p, dt, ((n * static_cast<uint32_t>(o.H) + h) * static_cast<uint32_t>(o.W) + w) * C + c);
    if (++ow == o.OW) {
      ow = 0;
      if (++oh == o.OH) {
        oh = 0;
        ++n;
      }
    }
  }
}

// ---- epilogues ---------------------------------------------------------------------------------
enum Epi : int {
  E_BIAS_RELU = 0,       // out[m][n] = relu(acc + bias[n])                                 (T)
  E_BIAS_RELU_POOL = 1,  // 2x2 windows of 4 consecutive m: out[m/4][n] = max * drop(img, n), idx
  E_BIAS_RELU_DROP = 2,  // fc1: out[m][n] = relu(acc + bias) * drop(m, n)
  E_BIAS = 3,            // fc2 logits: out[m][n] = acc + bias[n]                            (fp32)
  E_MASK_POS = 4,        // dgrad into a ReLU output a: out = acc * (a[m][n] > 0)            (T)
  E_DROP_POS = 5,        // dgrad into a dropout(relu) output a (pooled / fc): out = acc * drop * (a > 0);
                         //   with idx: written unpooled (the 2x2 window of the pre-pool grid, see unpool_store)
  E_DROP_POS_FLAT = 6,   // fc1 dgrad: as 5, written at the NHWC position of flat index n (c*HW + hw); idx: unpooled
  E_GRAD_FC = 7,         // weight gradient W[m][n] (+)= acc via (gso, gsc); n == N-1 with gbias: bias
  E_GRAD_CONV = 8,       // weight gradient W[o=m][c][r][s] (+)= acc, n = (r*S+s)*C + c; bias column
};

struct Job {
  Operand a, b;
  int64_t M, N, K;
  int tiles_m, tiles_n, splits;  // blocks = tiles_m * tiles_n * splits
  int64_t k_per_split;           // multiple of BK
  int epi;
  void* out;
  int out_dt;
  const void* bias;              // [N] (epilogues 0-3), dtype bias_dt
  int bias_dt;
  const float* drop;             // dropout factors [rows of the image / batch][drop_cols] or null (1)
  int drop_cols;
  const void* act;               // E_MASK_POS / E_DROP_POS*: the activation a
  uint8_t* idx;                  // E_BIAS_RELU_POOL: argmax out
  int HW, C;                     // E_DROP_POS(_FLAT): pooled grid size, channels
  int PW, PH;                    // E_BIAS_RELU_POOL: pooled grid (image = window / (PH*PW))
  int64_t gso, gsc, gsr, gss;    // E_GRAD_*: weight-gradient strides
  int gC, gS;                    // E_GRAD_CONV: kk = (r*gS+s)*gC + c
  void* gbias;                   // bias gradient (its column is N-1) or null
  int accumulate;                // E_GRAD_*: add into the existing gradient
  float* slab;                   // split-K partials [splits][M][N] (splits > 1)
};

struct Launch {
  Job job[2];
  int nblocks0;
};

__device__ __forceinline__ float drop_factor(const Job& j, int64_t row, int64_t col) {
  return j.drop == nullptr ? 1.f : j.drop[row * j.drop_cols + col];
}

// the gradient of one pooled element routed to its 2x2 window of the (2PH, 2PW) pre-pool grid: g at
// the argmax q, zero at the other three (so the unpooled gradient needs no memset)
__device__ __forceinline__ void unpool_store(const Job& J, uint32_t img, uint32_t ph, uint32_t pw, uint32_t c,
                                             uint32_t C, float g, uint8_t q) {
  const uint32_t W2 = 2u * static_cast<uint32_t>(J.PW), H2 = 2u * static_cast<uint32_t>(J.PH);
  const uint32_t base = ((img * H2 + 2u * ph) * W2 + 2u * pw) * C + c;
#pragma unroll
  for (uint32_t d = 0; d < 4; ++d)
    st(J.out, J.out_dt, base + ((d >> 1) * W2 + (d & 1u)) * C, d == q ? g : 0.f);
}

// bias + ReLU + 2x2 max-pool + channel dropout of one pooled output (win, n) from its 4 window rows,
// with the argmax (first maximum of the row-major window, as torch's max_pool2d) to idx
__device__ __forceinline__ void pool_store(const Job& J, uint32_t win, int64_t n, float v0, float v1, float v2, float v3) {
  const uint32_t img = win / static_cast<uint32_t>(J.PH * J.PW);
  const float bb = ld(J.bias, J.bias_dt, n);
  const float v[4] = {v0, v1, v2, v3};
  float best = fmaxf(v[0] + bb, 0.f);
  int arg = 0;
#pragma unroll
  for (int q = 1; q < 4; ++q) {
    const float x = fmaxf(v[q] + bb, 0.f);
    if (x > best) {
      best = x;
      arg = q;
    }
  }
  best = J.out_dt == 1 ? bf2f(f2bf(best)) : best;
  st(J.out, J.out_dt, static_cast<int64_t>(win) * J.N + n, best * drop_factor(J, img, n));
  J.idx[static_cast<int64_t>(win) * J.N + n] = static_cast<uint8_t>(arg);
}

// every epilogue but the pooling one, for one output element (GEMM or split-K finish)
template <int EPI>
__device__ __forceinline__ void epi_store_t(const Job& J, int64_t m, int64_t n, float v) {
  switch (EPI) {
    case E_BIAS_RELU:
      st(J.out, J.out_dt, m * J.N + n, fmaxf(v + ld(J.bias, J.bias_dt, n), 0.f));
      break;
    case E_BIAS_RELU_DROP: {
      float r = fmaxf(v + ld(J.bias, J.bias_dt, n), 0.f);
      r = J.out_dt == 1 ? bf2f(f2bf(r)) : r;  // the reference rounds the Linear output first
      st(J.out, J.out_dt, m * J.N + n, r * drop_factor(J, m, n));
      break;
    }
    case E_BIAS:
      static_cast<float*>(J.out)[m * J.N + n] = v + ld(J.bias, J.bias_dt, n);
      break;
    case E_MASK_POS:
      st(J.out, J.out_dt, m * J.N + n, ld(J.act, J.out_dt, m * J.N + n) > 0.f ? v : 0.f);
      break;
    case E_DROP_POS: {
      const float a = ld(J.act, J.out_dt, m * J.N + n);
      const float g = a > 0.f ? v * drop_factor(J, m / J.HW, n) : 0.f;
      if (J.idx == nullptr) {
        st(J.out, J.out_dt, m * J.N + n, g);
      } else {  // unpooled: m is a pooled pixel (img, ph, pw) of the HW = PH * PW grid
        const uint32_t mu = static_cast<uint32_t>(m), hw = static_cast<uint32_t>(J.HW);
        const uint32_t img = mu / hw, rem = mu - img * hw;
        const uint32_t ph = rem / static_cast<uint32_t>(J.PW), pw = rem - ph * static_cast<uint32_t>(J.PW);
        unpool_store(J, img, ph, pw, static_cast<uint32_t>(n), static_cast<uint32_t>(J.N), g, J.idx[m * J.N + n]);
      }
      break;
    }
    case E_DROP_POS_FLAT: {
      const int c = static_cast<int>(n / J.HW);
      const int hw = static_cast<int>(n - static_cast<int64_t>(c) * J.HW);
      const int64_t e = (m * J.HW + hw) * J.C + c;
      const float a = ld(J.act, J.out_dt, e);
      const float g = a > 0.f ? v * drop_factor(J, m, c) : 0.f;
      if (J.idx == nullptr) {
        st(J.out, J.out_dt, e, g);
      } else {
        const uint32_t ph = static_cast<uint32_t>(hw) / static_cast<uint32_t>(J.PW);
        const uint32_t pw = static_cast<uint32_t>(hw) - ph * static_cast<uint32_t>(J.PW);
        unpool_store(J, static_cast<uint32_t>(m), ph, pw, static_cast<uint32_t>(c), static_cast<uint32_t>(J.C), g, J.idx[e]);
      }
      break;
    }
    case E_GRAD_FC:
    case E_GRAD_CONV: {
      if (J.gbias != nullptr && n == J.N - 1) {
        const float prev = J.accumulate ? ld(J.gbias, J.out_dt, m) : 0.f;
        st(J.gbias, J.out_dt, m, prev + v);
        break;
      }
      int64_t e;
      if (EPI == E_GRAD_FC) {
        e = m * J.gso + n * J.gsc;
      } else {
        const int c = static_cast<int>(n % J.gC), rs = static_cast<int>(n / J.gC);
        const int r = rs / J.gS, sx = rs - r * J.gS;
        e = m * J.gso + c * J.gsc + r * J.gsr + sx * J.gss;
      }
      const float prev = J.accumulate ? ld(J.out, J.out_dt, e) : 0.f;
      st(J.out, J.out_dt, e, prev + v);
      break;
    }
  }
}
__device__ __forceinline__ void epi_store(const Job& J, int64_t m, int64_t n, float v) {
  switch (J.epi) {
    case E_BIAS_RELU: epi_store_t<E_BIAS_RELU>(J, m, n, v); break;
    case E_BIAS_RELU_DROP: epi_store_t<E_BIAS_RELU_DROP>(J, m, n, v); break;
    case E_BIAS: epi_store_t<E_BIAS>(J, m, n, v); break;
    case E_MASK_POS: epi_store_t<E_MASK_POS>(J, m, n, v); break;
    case E_DROP_POS: epi_store_t<E_DROP_POS>(J, m, n, v); break;
    case E_DROP_POS_FLAT: epi_store_t<E_DROP_POS_FLAT>(J, m, n, v); break;
    case E_GRAD_FC: epi_store_t<E_GRAD_FC>(J, m, n, v); break;
    case E_GRAD_CONV: epi_store_t<E_GRAD_CONV>(J, m, n, v); break;
  }
}

// ---- the GEMM core on MFMA ---------------------------------------------------------------------
// 64 x 64 block tile, BK = 64, 4 waves of 32 x 32 (2 x 2 tiles of 16 x 16).  bf16 storage runs
// v_mfma_f32_16x16x32_bf16 (lane l: A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15]); fp32 storage runs the
// exact-fp32 v_mfma_f32_16x16x4_f32 (A[l&15][l>>4], B[l>>4][l&15]), so O0 keeps fp32 products.
// C/D: col = l&15, row = 4(l>>4) + i.  Staging: each lane gathers two groups of 8 consecutive k of
// one tile row (the operand loaders above: one 16-B load per group where the layout allows),
// double-buffered through LDS (one vector store per group) with the next tile's gathers issued
// before the current tile's MFMAs.
//
// The kernel is specialised per (A source, B source, epilogue) at compile time -- a job's loaders
// and epilogue are all a launch executes, so each instantiation stays a few KB of code: one generic
// kernel with every path inlined was 148 KB, beyond the 64 KB instruction cache, and its small
// launches ran 20-30 us on cold instruction fetches (round-5 trace, profiles/r5_cifar_native_trace.txt).
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <bool BF>
struct Stage;
template <>
struct Stage<true> {
  static constexpr int LDK = 64 + 8;  // row stride 144 B: 16-B fragment reads stay aligned
  typedef uint16_t E;
  __device__ static E cvt(float v) { return f2bf(v); }
  // values that came from bf16 storage convert back exactly: keep the high half (v_perm packs two)
  __device__ static E cvt_exact(float v) { return static_cast<E>(__float_as_uint(v) >> 16); }
  __device__ static void put8_exact(E* dst, const float (&v)[8]) {
    uint4 q;
    q.x = __builtin_amdgcn_perm(__float_as_uint(v[1]), __float_as_uint(v[0]), 0x07060302u);
    q.y = __builtin_amdgcn_perm(__float_as_uint(v[3]), __float_as_uint(v[2]), 0x07060302u);
    q.z = __builtin_amdgcn_perm(__float_as_uint(v[5]), __float_as_uint(v[4]), 0x07060302u);
    q.w = __builtin_amdgcn_perm(__float_as_uint(v[7]), __float_as_uint(v[6]), 0x07060302u);
    *reinterpret_cast<uint4*>(dst) = q;
  }
  __device__ static void put8(E* dst, const float (&v)[8]) {
    uint4 q;
    q.x = static_cast<uint32_t>(f2bf(v[0])) | static_cast<uint32_t>(f2bf(v[1])) << 16;
    q.y = static_cast<uint32_t>(f2bf(v[2])) | static_cast<uint32_t>(f2bf(v[3])) << 16;
    q.z = static_cast<uint32_t>(f2bf(v[4])) | static_cast<uint32_t>(f2bf(v[5])) << 16;
    q.w = static_cast<uint32_t>(f2bf(v[6])) | static_cast<uint32_t>(f2bf(v[7])) << 16;
    *reinterpret_cast<uint4*>(dst) = q;
  }
};
template <>
struct Stage<false> {
  static constexpr int LDK = 64 + 4;
  typedef float E;
  __device__ static E cvt(float v) { return v; }
  __device__ static E cvt_exact(float v) { return v; }
  __device__ static void put8(E* dst, const float (&v)[8]) {
    *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
  __device__ static void put8_exact(E* dst, const float (&v)[8]) { put8(dst, v); }
};

constexpr int GBK = 64;

// a job kind: A source, B source, epilogue (weight-gradient jobs read A transposed)
template <int SA_, int SB_, int EP_>
struct Kind {
  static constexpr int SA = SA_, SB = SB_, EP = EP_;
  static constexpr bool WG = EP_ == E_GRAD_FC || EP_ == E_GRAD_CONV;
};
struct NoKind {};

template <bool BF>
struct Smem {
  typename Stage<BF>::E As[2][BM][Stage<BF>::LDK];
  typename Stage<BF>::E Bs[2][BN][Stage<BF>::LDK];
};

// Convolution operands address an element as (row's pixel) + (the k index's tap and channel): the
// k part comes from a per-block LDS table built once (ktab: A delta, packed (dh, dw) offset, B
// delta), the row part is decomposed once per tile, so the K loop does no integer division.
constexpr int KTAB = 576;  // largest conv reduction of the network (3 x 3 x 64)

template <bool BF, class KD>
__device__ __forceinline__ void gemm_tile(const Job& J, int bid, Smem<BF>& sm, int4* ktab) {
  constexpr int LDK = Stage<BF>::LDK;
  const int z = bid % J.splits;
  bid /= J.splits;
  const int tn = bid % J.tiles_n;
  const int tm = bid / J.tiles_n;
  const int64_t m0 = static_cast<int64_t>(tm) * BM, n0 = static_cast<int64_t>(tn) * BN;
  const int64_t k_lo = static_cast<int64_t>(z) * J.k_per_split;
  const int64_t k_hi = k_lo + J.k_per_split < J.K ? k_lo + J.k_per_split : J.K;

  const int t = threadIdx.x;
  const int lr = t >> 2, lk = (t & 3) * 8;  // staging: tile row lr, k = lk .. lk+7 and lk+32 .. lk+39
  const int lane = t & 63, w = t >> 6;
  const int wm = (w & 1) * 32, wn = (w >> 1) * 32;
  const bool bias_col = KD::WG && J.gbias != nullptr;

  constexpr bool ATAB = !KD::WG && (KD::SA == S_ACT_CONV || KD::SA == S_GRAD_CONV_T);
  constexpr bool BTAB = !KD::WG && (KD::SB == S_WGT_CONV || KD::SB == S_WGT_CONV_T);
  if constexpr (ATAB || BTAB) {
    for (int k = t; k < J.K; k += NT) {
      int4 e = make_int4(0, 0, 0, 0);
      if constexpr (ATAB) {
        const Operand& o = J.a;
        const int rs = k / o.C, c = k - rs * o.C, r = rs / o.S, sx = rs - r * o.S;
        const int dh = KD::SA == S_ACT_CONV ? r - o.pad : o.pad - r;
        const int dw = KD::SA == S_ACT_CONV ? sx - o.pad : o.pad - sx;
        e.x = (dh * o.W + dw) * o.C + c;
        e.y = static_cast<int>(static_cast<uint32_t>(dh) << 16 | (static_cast<uint32_t>(dw) & 0xffffu));
      }
      if constexpr (BTAB) {
        const Operand& o = J.b;
        const int rs = k / o.C, c = k - rs * o.C, r = rs / o.S, sx = rs - r * o.S;
        e.z = static_cast<int>((KD::SB == S_WGT_CONV ? c * o.sc : c * o.so) + r * o.sr + sx * o.ss);
      }
      ktab[k] = e;
    }
    __syncthreads();
  }
  // this thread's A row (a pixel of the conv's GEMM grid), decomposed once
  int a_base = 0, a_h = 0, a_w = 0;
  if constexpr (ATAB) {
    const Operand& o = J.a;
    if (m0 + lr < J.M) {
      uint32_t n;
      Operand g = o;
      if (KD::SA == S_GRAD_CONV_T) g.pool = 0;
      pix_nhw(g, static_cast<uint32_t>(m0 + lr), n, a_h, a_w);
      a_base = ((static_cast<int>(n) * o.H + a_h) * o.W + a_w) * o.C;
    }
  }
  auto tab_a = [&](int64_t kg, int nk, float (&v)[8]) {
    const Operand& o = J.a;
    const int dt = odt(o);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    if (nk == 8 && (o.C & 7) == 0) {  // one tap, 8 channels
      const int4 e = ktab[kg];
      const int h = a_h + (e.y >> 16), w = a_w + static_cast<int>(static_cast<short>(e.y & 0xffff));
      if (h >= 0 && h < o.H && w >= 0 && w < o.W) ld8(o.p, dt, static_cast<uint32_t>(a_base + e.x), v);
      return;
    }
    for (int j = 0; j < nk; ++j) {
      const int4 e = ktab[kg + j];
      const int h = a_h + (e.y >> 16), w = a_w + static_cast<int>(static_cast<short>(e.y & 0xffff));
      if (h >= 0 && h < o.H && w >= 0 && w < o.W) v[j] = ld32(o.p, dt, static_cast<uint32_t>(a_base + e.x));
    }
  };
  auto tab_b = [&](uint32_t row, int64_t kg, int nk, float (&v)[8]) {
    const Operand& o = J.b;
    const int dt = odt(o);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    const uint32_t rb = static_cast<uint32_t>(row * (KD::SB == S_WGT_CONV ? o.so : o.sc));
    if (KD::SB == S_WGT_CONV && nk == 8 && o.sc == 1 && (o.C & 7) == 0) {
      ld8(o.p, dt, rb + static_cast<uint32_t>(ktab[kg].z), v);
      return;
    }
    for (int j = 0; j < nk; ++j) v[j] = ld32(o.p, dt, rb + static_cast<uint32_t>(ktab[kg + j].z));
  };

  // Operands whose 8 contiguous elements run along the GEMM row (not along k) are staged k-major:
  // thread t takes k = t & 63 of the tile and rows 8 rg .. 8 rg + 7 (rg = t >> 6, then + 4), one 16-B
  // load each, written to LDS transposed -- the weight-gradient operands (A = dY^T: channels
  // contiguous; B = the activation column block: a tap's channels contiguous) and the input-gradient
  // weights (W[o][c][r][s] with c contiguous).  The others are staged row-major (row lr, 8 k).
  constexpr bool AKM = KD::WG;
  constexpr bool BKM = KD::WG || KD::SB == S_WGT_CONV_T || KD::SB == S_WGT_FC_T;
  const int kk = t & 63, rg = t >> 6;
  // k-major B of a conv weight gradient: per row group, the tap offset and channel of its 8 columns
  int bc_dh[2] = {0, 0}, bc_dw[2] = {0, 0}, bc_c0[2] = {0, 0};
  bool bc_vec[2] = {false, false};
  const int nreal = bias_col ? static_cast<int>(J.N) - 1 : static_cast<int>(J.N);  // non-bias columns
  if constexpr (KD::WG && KD::SB == S_ACT_CONV) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int col0 = static_cast<int>(n0) + 8 * (rg + 4 * g);
      const int C = J.b.C;
      const int rs = col0 / C, c0 = col0 - rs * C, r = rs / J.b.S, sx = rs - r * J.b.S;
      bc_dh[g] = r - J.b.pad;
      bc_dw[g] = sx - J.b.pad;
      bc_c0[g] = c0;
      bc_vec[g] = (C & 7) == 0 && col0 + 8 <= nreal;
    }
  }
  auto km_a = [&](int64_t k, int g, float (&v)[8]) {  // A[m][k] = dY[k][m], m = m0 + 8 (rg + 4g) + i
    const Operand& o = J.a;
    const int dt = odt(o);
    const int mr = static_cast<int>(m0) + 8 * (rg + 4 * g);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
    if (k >= k_hi) return;
    const uint32_t base = static_cast<uint32_t>(k) * static_cast<uint32_t>(o.C);
    if ((o.C & 7) == 0 && mr + 8 <= J.M) {
      ld8(o.p, dt, base + static_cast<uint32_t>(mr), v);
    } else {
      for (int i = 0; i < 8; ++i)
        if (mr + i < J.M) v[i] = ld32(o.p, dt, base + static_cast<uint32_t>(mr + i));
    }
  };
  // the pixel of k-major k (weight gradients of a conv: k runs over the OH x OW grid, row-major)
  auto km_b = [&](int64_t k, int g, uint32_t pn, int ph, int pw, float (&v)[8]) {
    const Operand& o = J.b;
    const int dt = odt(o);
    const int col0 = static_cast<int>(n0) + 8 * (rg + 4 * g);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
    if (k >= k_hi) return;
    if constexpr (KD::WG) {
      if constexpr (KD::SB == S_ACT_CONV) {
        if (bc_vec[g]) {
          const int h = ph + bc_dh[g], w = pw + bc_dw[g];
          if (h >= 0 && h < o.H && w >= 0 && w < o.W)
            ld8(o.p, dt, ((pn * static_cast<uint32_t>(o.H) + h) * static_cast<uint32_t>(o.W) + w) * o.C + bc_c0[g], v);
          return;
        }
        for (int i = 0; i < 8; ++i) {
          const int col = col0 + i;
          if (col >= static_cast<int>(J.N)) break;
          if (col == nreal) {  // the bias column
            v[i] = 1.f;
            continue;
          }
          const int rs = col / o.C, c = col - rs * o.C, r = rs / o.S, sx = rs - r * o.S;
          const int h = ph + r - o.pad, w = pw + sx - o.pad;
          if (h >= 0 && h < o.H && w >= 0 && w < o.W)
            v[i] = ld32(o.p, dt, ((pn * static_cast<uint32_t>(o.H) + h) * static_cast<uint32_t>(o.W) + w) * o.C + c);
        }
      } else if constexpr (KD::SB == S_ACT_ROWS) {
        const uint32_t base = static_cast<uint32_t>(k) * static_cast<uint32_t>(o.C);
        if ((o.C & 7) == 0 && col0 + 8 <= nreal) {
          ld8(o.p, dt, base + static_cast<uint32_t>(col0), v);
          return;
        }
        for (int i = 0; i < 8; ++i) {
          const int col = col0 + i;
          if (col < nreal) v[i] = ld32(o.p, dt, base + static_cast<uint32_t>(col));
          else if (col == nreal && col < static_cast<int>(J.N)) v[i] = 1.f;
        }
      } else {  // S_ACT_FLAT: column c*HW + hw of image k
        const int hw = o.H * o.W;
        for (int i = 0; i < 8; ++i) {
          const int col = col0 + i;
          if (col < nreal) {
            const int c = col / hw, rem = col - c * hw;
            v[i] = ld32(o.p, dt, (static_cast<uint32_t>(k) * static_cast<uint32_t>(hw) + rem) * o.C + c);
          } else if (col == nreal && col < static_cast<int>(J.N)) {
            v[i] = 1.f;
          }
        }
      }
    } else if constexpr (KD::SB == S_WGT_CONV_T) {  // B[k = (tap, o)][n = c] = W[o][c][r][s]
      const uint32_t base = static_cast<uint32_t>(ktab[k].z);
      if (o.sc == 1 && col0 + 8 <= static_cast<int>(J.N)) {
        ld8(o.p, dt, base + static_cast<uint32_t>(col0), v);
        return;
      }
      for (int i = 0; i < 8; ++i)
        if (col0 + i < J.N) v[i] = ld32(o.p, dt, base + static_cast<uint32_t>((col0 + i) * o.sc));
    } else {  // S_WGT_FC_T: B[k = o][n = j] = W[o][j]
      const uint32_t base = static_cast<uint32_t>(k * o.so);
      if (o.sc == 1 && col0 + 8 <= static_cast<int>(J.N) && (o.so & 7) == 0) {
        ld8(o.p, dt, base + static_cast<uint32_t>(col0), v);
        return;
      }
      for (int i = 0; i < 8; ++i)
        if (col0 + i < J.N) v[i] = ld32(o.p, dt, base + static_cast<uint32_t>((col0 + i) * o.sc));
    }
  };

  float ra[2][8], rb[2][8];
  auto gather = [&](int64_t k0) {
    const int64_t m = m0 + lr, n = n0 + lr;
    if constexpr (AKM || BKM) {
      const int64_t k = k0 + kk;
      uint32_t pn = 0;
      int ph = 0, pw = 0;
      if constexpr (KD::WG && KD::SB == S_ACT_CONV) {  // this thread's pixel, once per tile
        const uint32_t ku = static_cast<uint32_t>(k), OW = static_cast<uint32_t>(J.b.OW);
        const uint32_t q = ku / OW;
        pw = static_cast<int>(ku - q * OW);
        pn = q / static_cast<uint32_t>(J.b.OH);
        ph = static_cast<int>(q - pn * static_cast<uint32_t>(J.b.OH));
      }
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        if constexpr (AKM) km_a(k, g, ra[g]);
        if constexpr (BKM) km_b(k, g, pn, ph, pw, rb[g]);
      }
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int64_t kg = k0 + lk + 32 * g;
      const int nk = kg >= k_hi ? 0 : (k_hi - kg < 8 ? static_cast<int>(k_hi - kg) : 8);
      if constexpr (!AKM) {
        if (m < J.M && nk > 0) {
          if constexpr (ATAB) tab_a(kg, nk, ra[g]);
          else opval8<KD::SA>(J.a, static_cast<uint32_t>(m), static_cast<uint32_t>(kg), nk, ra[g]);
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) ra[g][i] = 0.f;
        }
      }
      if constexpr (!BKM) {
        if (n < J.N && nk > 0) {
          if constexpr (BTAB) tab_b(static_cast<uint32_t>(n), kg, nk, rb[g]);
          else opval8<KD::SB>(J.b, static_cast<uint32_t>(n), static_cast<uint32_t>(kg), nk, rb[g]);
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) rb[g][i] = 0.f;
        }
      }
    }
  };
  // bf16-stored operands round-trip exactly (truncate); only fp32 ones (the logits gradient) round
  const bool a_exact = J.a.dt == 1, b_exact = J.b.dt == 1;
  auto stash = [&](int b) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if constexpr (AKM) {
        if (a_exact) {
#pragma unroll
          for (int i = 0; i < 8; ++i) sm.As[b][8 * (rg + 4 * g) + i][kk] = Stage<BF>::cvt_exact(ra[g][i]);
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) sm.As[b][8 * (rg + 4 * g) + i][kk] = Stage<BF>::cvt(ra[g][i]);
        }
      } else {
        if (a_exact) Stage<BF>::put8_exact(&sm.As[b][lr][lk + 32 * g], ra[g]);
        else Stage<BF>::put8(&sm.As[b][lr][lk + 32 * g], ra[g]);
      }
      if constexpr (BKM) {
        if (b_exact) {
#pragma unroll
          for (int i = 0; i < 8; ++i) sm.Bs[b][8 * (rg + 4 * g) + i][kk] = Stage<BF>::cvt_exact(rb[g][i]);
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) sm.Bs[b][8 * (rg + 4 * g) + i][kk] = Stage<BF>::cvt(rb[g][i]);
        }
      } else {
        if (b_exact) Stage<BF>::put8_exact(&sm.Bs[b][lr][lk + 32 * g], rb[g]);
        else Stage<BF>::put8(&sm.Bs[b][lr][lk + 32 * g], rb[g]);
      }
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one gather call site (the loaders are most of the code): iteration i gathers tile i, runs the
  // MFMAs of tile i-1 (staged in the other buffer) while the loads are in flight, then stages tile i
  auto compute = [&](int cb) {
    if constexpr (BF) {
#pragma unroll
      for (int ks = 0; ks < GBK; ks += 32) {
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(&sm.As[cb][wm + i * 16 + (lane & 15)][ks + 8 * (lane >> 4)]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(&sm.Bs[cb][wn + j * 16 + (lane & 15)][ks + 8 * (lane >> 4)]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kq = 0; kq < GBK; kq += 4) {
        float af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = sm.As[cb][wm + i * 16 + (lane & 15)][kq + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bfr[j] = sm.Bs[cb][wn + j * 16 + (lane & 15)][kq + (lane >> 4)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  int buf = 0;
  for (int64_t k0 = k_lo; k0 < k_hi; k0 += GBK) {
    gather(k0);
    if (k0 > k_lo) compute(buf ^ 1);
    stash(buf);
    __syncthreads();  // tile i staged; every wave is past tile i-1's reads of the buffer i+1 reuses
    buf ^= 1;
  }
  compute(buf ^ 1);
  (void)LDK;

  // ---- epilogue: lane holds rows 4(lane>>4)+r, r = 0..3, of column lane&15 of each 16x16 tile
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t mrow = m0 + wm + i * 16 + 4 * (lane >> 4);
      const int64_t n = n0 + wn + j * 16 + (lane & 15);
      if (n >= J.N) continue;
      const f32x4 v = acc[i][j];
      if (J.splits > 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (mrow + r < J.M) J.slab[(static_cast<int64_t>(z) * J.M + mrow + r) * J.N + n] = v[r];
        continue;
      }
      if constexpr (KD::EP == E_BIAS_RELU_POOL) {
        // the 4 rows are one 2x2 window (M window-ordered, M % 4 == 0)
        if (mrow >= J.M) continue;
        pool_store(J, static_cast<uint32_t>(mrow >> 2), n, v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (mrow + r < J.M) epi_store_t<KD::EP>(J, mrow + r, n, v[r]);
      }
    }
  }
}

// one launch runs job 0 (kind K0) and, if K1 is a Kind, job 1 side by side
template <bool BF, class K0, class K1>
__global__ void __launch_bounds__(NT) cnn_gemm_kernel(Launch L) {
  __shared__ __attribute__((aligned(16))) Smem<BF> sm;
  __shared__ int4 ktab[KTAB];
  if constexpr (!std::is_same<K1, NoKind>::value) {
    if (static_cast<int>(blockIdx.x) >= L.nblocks0) {
      gemm_tile<BF, K1>(L.job[1], static_cast<int>(blockIdx.x) - L.nblocks0, sm, ktab);
      return;
    }
  }
  gemm_tile<BF, K0>(L.job[0], static_cast<int>(blockIdx.x), sm, ktab);
}

// the job kinds the network launches (ops/cnn.py): forward, then backward (weight grad, input grad)
typedef Kind<S_ACT_CONV, S_WGT_CONV, E_BIAS_RELU> KConv;
typedef Kind<S_ACT_CONV, S_WGT_CONV, E_BIAS_RELU_POOL> KConvPool;
typedef Kind<S_ACT_FLAT, S_WGT_FC, E_BIAS_RELU_DROP> KFc1;
typedef Kind<S_ACT_ROWS, S_WGT_FC, E_BIAS> KFc2;
typedef Kind<S_GRAD_ROWS, S_ACT_ROWS, E_GRAD_FC> KFc2W;
typedef Kind<S_GRAD_ROWS, S_WGT_FC_T, E_DROP_POS> KFc2D;
typedef Kind<S_GRAD_ROWS, S_ACT_FLAT, E_GRAD_FC> KFc1W;
typedef Kind<S_GRAD_ROWS, S_WGT_FC_T, E_DROP_POS_FLAT> KFc1D;
typedef Kind<S_GRAD_CONV_T, S_ACT_CONV, E_GRAD_CONV> KConvW;
typedef Kind<S_GRAD_CONV_T, S_WGT_CONV_T, E_MASK_POS> KConvD;
typedef Kind<S_GRAD_CONV_T, S_WGT_CONV_T, E_DROP_POS> KConvDDrop;

template <class KD>
__host__ bool kind_is(const Job& j) {
  const bool tab = !KD::WG && (KD::SA == S_ACT_CONV || KD::SA == S_GRAD_CONV_T || KD::SB == S_WGT_CONV ||
                               KD::SB == S_WGT_CONV_T);
  return j.a.src == KD::SA && j.b.src == KD::SB && j.epi == KD::EP && (j.a.transpose != 0) == KD::WG &&
         (!tab || j.K <= KTAB);
}

template <bool BF, class K0, class K1>
bool try_launch(const Launch& L, bool has1, int blocks, hipStream_t st) {
  if (!kind_is<K0>(L.job[0])) return false;
  if constexpr (std::is_same<K1, NoKind>::value) {
    if (has1) return false;
  } else {
    if (!has1 || !kind_is<K1>(L.job[1])) return false;
  }
  cnn_gemm_kernel<BF, K0, K1><<<blocks, NT, 0, st>>>(L);
  return true;
}

template <bool BF>
bool launch_kinds(const Launch& L, bool has1, int blocks, hipStream_t st) {
  return try_launch<BF, KConv, NoKind>(L, has1, blocks, st) || try_launch<BF, KConvPool, NoKind>(L, has1, blocks, st) ||
         try_launch<BF, KFc1, NoKind>(L, has1, blocks, st) || try_launch<BF, KFc2, NoKind>(L, has1, blocks, st) ||
         try_launch<BF, KFc2W, KFc2D>(L, has1, blocks, st) || try_launch<BF, KFc1W, KFc1D>(L, has1, blocks, st) ||
         try_launch<BF, KConvW, KConvD>(L, has1, blocks, st) || try_launch<BF, KConvW, KConvDDrop>(L, has1, blocks, st) ||
         try_launch<BF, KConvW, NoKind>(L, has1, blocks, st);
}

// ---- split-K finish: sum the slabs of up to 4 jobs and apply their epilogues --------------------
constexpr int kMaxFin = 4;
struct FinishLaunch {
  Job job[kMaxFin];
  // lanes of job j: [lfirst[j], lfirst[j + 1]), its output elements x tpe[j], padded to whole waves so a
  // wave never straddles two jobs (the group sums shuffle within a wave)
  int64_t lfirst[kMaxFin + 1];
  int tpe[kMaxFin];  // lanes per output element of each job (power of two <= 32): they split its slab sum
  int njobs;
};

// sum of the slabs of (m, n) taken by lane `sub` of a group of T: 4 independent partial sums
__device__ __forceinline__ float slab_part(const Job& J, int64_t m, int64_t n, int sub, int T) {
  const float* sp = J.slab + m * J.N + n;
  const int64_t stride = J.M * J.N;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int zz = sub;
  for (; zz + 3 * T < J.splits; zz += 4 * T) {
    a0 += sp[zz * stride];
    a1 += sp[(zz + T) * stride];
    a2 += sp[(zz + 2 * T) * stride];
    a3 += sp[(zz + 3 * T) * stride];
  }
  for (; zz < J.splits; zz += T) a0 += sp[zz * stride];
  return (a0 + a1) + (a2 + a3);
}

__device__ __forceinline__ float group_sum(float v, int T) {
  for (int o = T >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(NT) cnn_finish_kernel(FinishLaunch L) {
  // T adjacent lanes per output element, each summing every T-th slab, with T sized per job: the
  // weight-gradient slabs run to ~450 splits (one lane per element would be a serial chain of load
  // latencies) while an input gradient finished in the same launch has a handful
  const int64_t total = L.lfirst[L.njobs];
  const int64_t stride = static_cast<int64_t>(gridDim.x) * NT;
  for (int64_t gl = static_cast<int64_t>(blockIdx.x) * NT + threadIdx.x; gl < total; gl += stride) {
    int ji = 0;
    while (ji + 1 < L.njobs && gl >= L.lfirst[ji + 1]) ++ji;
    const Job& J = L.job[ji];
    const int T = L.tpe[ji];
    const int64_t rel = gl - L.lfirst[ji];
    const int sub = static_cast<int>(rel & (T - 1));
    const int64_t e = rel / T;
    if (J.epi == E_BIAS_RELU_POOL) {  // e = (window, n): the window's 4 rows summed, then pooled
      const bool act = e < (J.M / 4) * J.N;
      const int64_t win = act ? e / J.N : 0, n = act ? e - win * J.N : 0;
      const float s0 = group_sum(act ? slab_part(J, 4 * win, n, sub, T) : 0.f, T);
      const float s1 = group_sum(act ? slab_part(J, 4 * win + 1, n, sub, T) : 0.f, T);
      const float s2 = group_sum(act ? slab_part(J, 4 * win + 2, n, sub, T) : 0.f, T);
      const float s3 = group_sum(act ? slab_part(J, 4 * win + 3, n, sub, T) : 0.f, T);
      if (act && sub == 0) pool_store(J, static_cast<uint32_t>(win), n, s0, s1, s2, s3);
    } else {
      const bool act = e < J.M * J.N;
      const int64_t m = act ? e / J.N : 0, n = act ? e - m * J.N : 0;
      const float sum = group_sum(act ? slab_part(J, m, n, sub, T) : 0.f, T);
      if (act && sub == 0) epi_store(J, m, n, sum);
    }
  }
}

// ---- dropout factors ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t philox_u0(uint64_t idx, uint32_t k0, uint32_t k1, uint32_t c2, uint32_t c3) {
  uint32_t c0 = static_cast<uint32_t>(idx), c1 = static_cast<uint32_t>(idx >> 32);
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
  return c0;
}

struct MaskLaunch {
  float* out[3];
  int64_t n[3];
  float p[3];
  uint64_t seed, offset;
  const uint32_t* rng_base;
};

__global__ void __launch_bounds__(NT) cnn_masks_kernel(MaskLaunch L) {
  const uint32_t base = L.rng_base != nullptr ? *L.rng_base : 0u;
  const uint32_t k0 = static_cast<uint32_t>(L.seed), k1 = static_cast<uint32_t>(L.seed >> 32);
  for (int s = 0; s < 3; ++s) {
    if (L.out[s] == nullptr) continue;
    const float p = L.p[s];
    const float keep = 1.f - p;
    const uint32_t thr = p >= 1.f ? 0xffffffffu : static_cast<uint32_t>(static_cast<double>(p) * 4294967296.0);
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * NT + threadIdx.x; i < L.n[s];
         i += static_cast<int64_t>(gridDim.x) * NT) {
      const uint32_t u = philox_u0(static_cast<uint64_t>(i), k0, k1, static_cast<uint32_t>(L.offset) + s * 0x9E3779B9u,
                                   static_cast<uint32_t>(L.offset >> 32) + base);
      L.out[s][i] = (p <= 0.f) ? 1.f : (u >= thr && keep > 0.f ? 1.f / keep : 0.f);
    }
  }
}

// ---- cross entropy -----------------------------------------------------------------------------
// loss = mean_n (logsumexp(z_n) - z_n[y_n]); correct = #(argmax z_n == y_n) (first max, as torch);
// backward dz = g * (softmax(z) - onehot(y)) / N.
// dz1 (nullable): the backward for a seed gradient of exactly 1, written by the same pass (the
// autograd backward then hands it over without a launch when its seed is the shared unit tensor)
__global__ void __launch_bounds__(NT) cnn_xent_fwd_kernel(const float* z, const int64_t* y, int N, int C,
                                                          float* loss_out, float* acc_out, float* dz1) {
  __shared__ float sl[NT], sa[NT];
  float l = 0.f, a = 0.f;
  for (int n = threadIdx.x; n < N; n += NT) {
    const float* r = z + static_cast<int64_t>(n) * C;
    float mx = r[0];
    int arg = 0;
    for (int c = 1; c < C; ++c)
      if (r[c] > mx) {
        mx = r[c];
        arg = c;
      }
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += expf(r[c] - mx);
    const int yy = static_cast<int>(y[n]);
    l += logf(se) + mx - r[yy];
    a += arg == yy ? 1.f : 0.f;
    if (dz1 != nullptr) {  // exactly cnn_xent_bwd_kernel's arithmetic with g = 1
      const float gs = 1.f / N, inv = 1.f / se;
      for (int c = 0; c < C; ++c) dz1[static_cast<int64_t>(n) * C + c] = gs * (expf(r[c] - mx) * inv - (c == yy ? 1.f : 0.f));
    }
  }
  sl[threadIdx.x] = l;
  sa[threadIdx.x] = a;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      sl[threadIdx.x] += sl[threadIdx.x + o];
      sa[threadIdx.x] += sa[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    loss_out[0] = sl[0] / N;
    if (acc_out != nullptr) {  // accuracy, then the error rate in the next float
      acc_out[0] = sa[0] / N;
      acc_out[1] = 1.f - sa[0] / N;
    }
  }
}

__global__ void __launch_bounds__(NT) cnn_xent_bwd_kernel(const float* z, const int64_t* y, const float* g, int N,
                                                          int C, float* dz) {
  const float gs = g[0] / N;
  for (int n = blockIdx.x * NT + threadIdx.x; n < N; n += gridDim.x * NT) {
    const float* r = z + static_cast<int64_t>(n) * C;
    float mx = r[0];
    for (int c = 1; c < C; ++c) mx = fmaxf(mx, r[c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += expf(r[c] - mx);
    const float inv = 1.f / se;
    const int yy = static_cast<int>(y[n]);
    for (int c = 0; c < C; ++c) dz[static_cast<int64_t>(n) * C + c] = gs * (expf(r[c] - mx) * inv - (c == yy ? 1.f : 0.f));
  }
}

}  // namespace

extern "C" {

// mirrored by determined_1_amd/ops/cnn.py (ctypes Structures, field order matters)
struct DetCnnOperand {
  const void* p;
  int32_t dt, src, H, W, C, R, S, pad, OH, OW, pool, transpose;
  const uint8_t* idx;
  int64_t so, sc, sr, ss;
};
struct DetCnnJob {
  DetCnnOperand a, b;
  int64_t M, N, K;
  int32_t splits, epi, out_dt, bias_dt, drop_cols, HW, C, PW, PH, gC, gS, accumulate;
  void* out;
  const void* bias;
  const float* drop;
  const void* act;
  uint8_t* idx;
  int64_t gso, gsc, gsr, gss;
  void* gbias;
  float* slab;
};

static Operand to_operand(const DetCnnOperand& d) {
  Operand o;
  o.p = d.p;
  o.dt = d.dt;
  o.src = d.src;
  o.H = d.H;
  o.W = d.W;
  o.C = d.C;
  o.R = d.R;
  o.S = d.S;
  o.pad = d.pad;
  o.OH = d.OH;
  o.OW = d.OW;
  o.pool = d.pool;
  o.idx = d.idx;
  o.so = d.so;
  o.sc = d.sc;
  o.sr = d.sr;
  o.ss = d.ss;
  o.transpose = d.transpose;
  return o;
}

static int64_t k_per_split(int64_t K, int splits) {
  int64_t kps = (K + splits - 1) / splits;
  return (kps + GBK - 1) / GBK * GBK;
}

// the split count a job with reduction length K and requested splits runs with
int det_cnn_splits(int64_t K, int32_t splits) {
  if (splits < 1) splits = 1;
  const int64_t kps = k_per_split(K, splits);
  return static_cast<int>((K + kps - 1) / kps);
}

static int fill_job(const DetCnnJob& d, Job* j) {
  if (d.M < 1 || d.N < 1 || d.K < 1) return -1;
  j->a = to_operand(d.a);
  j->b = to_operand(d.b);
  j->M = d.M;
  j->N = d.N;
  j->K = d.K;
  j->tiles_m = static_cast<int>((d.M + BM - 1) / BM);
  j->tiles_n = static_cast<int>((d.N + BN - 1) / BN);
  j->splits = det_cnn_splits(d.K, d.splits);
  j->k_per_split = k_per_split(d.K, j->splits > 1 ? j->splits : 1);
  if (j->splits == 1) j->k_per_split = d.K;
  j->epi = d.epi;
  j->out = d.out;
  j->out_dt = d.out_dt;
  j->bias = d.bias;
  j->bias_dt = d.bias_dt;
  j->drop = d.drop;
  j->drop_cols = d.drop_cols;
  j->act = d.act;
  j->idx = d.idx;
  j->HW = d.HW < 1 ? 1 : d.HW;
  j->C = d.C;
  j->PW = d.PW;
  j->PH = d.PH;
  j->gso = d.gso;
  j->gsc = d.gsc;
  j->gsr = d.gsr;
  j->gss = d.gss;
  j->gC = d.gC < 1 ? 1 : d.gC;
  j->gS = d.gS < 1 ? 1 : d.gS;
  j->gbias = d.gbias;
  j->accumulate = d.accumulate;
  j->slab = d.slab;
  if (j->splits > 1 && d.slab == nullptr) return -1;
  if (d.epi == E_BIAS_RELU_POOL && (d.M & 3)) return -1;
  return j->tiles_m * j->tiles_n * j->splits;
}

// one launch running job0 and (optionally) job1 side by side (both of storage dtype `bf16`)
int det_cnn_gemm(void* stream, int32_t bf16, const DetCnnJob* j0, const DetCnnJob* j1) {
  Launch L;
  const int b0 = fill_job(*j0, &L.job[0]);
  if (b0 <= 0) return static_cast<int>(hipErrorInvalidValue);
  int b1 = 0;
  if (j1 != nullptr) {
    b1 = fill_job(*j1, &L.job[1]);
    if (b1 <= 0) return static_cast<int>(hipErrorInvalidValue);
  } else {
    L.job[1] = L.job[0];
  }
  L.nblocks0 = b0;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const bool ok = bf16 ? launch_kinds<true>(L, j1 != nullptr, b0 + b1, st) : launch_kinds<false>(L, j1 != nullptr, b0 + b1, st);
  if (!ok) return static_cast<int>(hipErrorNotSupported);  // a job kind the network does not launch
  return static_cast<int>(hipGetLastError());
}

// the split-K finish of up to 4 jobs (their slabs summed, their epilogues applied) in one launch
int det_cnn_finish(void* stream, const DetCnnJob* jobs, int32_t njobs) {
  if (njobs < 1 || njobs > kMaxFin) return static_cast<int>(hipErrorInvalidValue);
  FinishLaunch L;
  int64_t lanes = 0;
  for (int i = 0; i < njobs; ++i) {
    if (fill_job(jobs[i], &L.job[i]) <= 0 || L.job[i].splits < 2) return static_cast<int>(hipErrorInvalidValue);
    int T = 1;
    while (T < 32 && T * 8 < L.job[i].splits) T <<= 1;  // ~8 slabs per lane
    L.tpe[i] = T;
    L.lfirst[i] = lanes;
    const int64_t nel = (L.job[i].epi == E_BIAS_RELU_POOL ? L.job[i].M / 4 : L.job[i].M) * L.job[i].N;
    lanes += (nel * T + 63) / 64 * 64;
  }
  for (int i = njobs; i < kMaxFin; ++i) {
    L.job[i] = L.job[0];
    L.tpe[i] = 1;
  }
  for (int i = njobs; i <= kMaxFin; ++i) L.lfirst[i] = lanes;
  L.njobs = njobs;
  int64_t want = (lanes + NT - 1) / NT;
  const int blocks = static_cast<int>(want > 2048 ? 2048 : want);
  cnn_finish_kernel<<<blocks, NT, 0, static_cast<hipStream_t>(stream)>>>(L);
  return static_cast<int>(hipGetLastError());
}

int det_cnn_masks(void* stream, float* m0, int64_t n0, float p0, float* m1, int64_t n1, float p1, float* m2,
                  int64_t n2, float p2, uint64_t seed, uint64_t offset, const uint32_t* rng_base) {
  MaskLaunch L;
  L.out[0] = m0;
  L.out[1] = m1;
  L.out[2] = m2;
  L.n[0] = n0;
  L.n[1] = n1;
  L.n[2] = n2;
  L.p[0] = p0;
  L.p[1] = p1;
  L.p[2] = p2;
  L.seed = seed;
  L.offset = offset;
  L.rng_base = rng_base;
  int64_t mx = n0 > n1 ? n0 : n1;
  mx = mx > n2 ? mx : n2;
  int blocks = static_cast<int>((mx + NT - 1) / NT);
  blocks = blocks < 1 ? 1 : (blocks > 256 ? 256 : blocks);
  cnn_masks_kernel<<<blocks, NT, 0, static_cast<hipStream_t>(stream)>>>(L);
  return static_cast<int>(hipGetLastError());
}

int det_cnn_xent_fwd(void* stream, const float* z, const int64_t* y, int32_t N, int32_t C, float* loss,
                     float* acc, float* dz1) {
  if (N < 1 || C < 1) return static_cast<int>(hipErrorInvalidValue);
  cnn_xent_fwd_kernel<<<1, NT, 0, static_cast<hipStream_t>(stream)>>>(z, y, N, C, loss, acc, dz1);
  return static_cast<int>(hipGetLastError());
}

int det_cnn_xent_bwd(void* stream, const float* z, const int64_t* y, const float* g, int32_t N, int32_t C,
                     float* dz) {
  if (N < 1 || C < 1) return static_cast<int>(hipErrorInvalidValue);
  const int blocks = (N + NT - 1) / NT;
  cnn_xent_bwd_kernel<<<blocks, NT, 0, static_cast<hipStream_t>(stream)>>>(z, y, g, N, C, dz);
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
