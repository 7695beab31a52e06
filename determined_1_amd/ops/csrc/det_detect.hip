// det_detect.hip — detection ops for the two-stage detector (Faster R-CNN example):
//   * multi-level RoIAlign forward / backward over channels_last FPN maps, all levels in ONE launch;
//   * non-maximum suppression entirely on the device: a 64x64-tile IoU bitmask kernel and a
//     single-wave sweep that resolves suppression 64 boxes at a time.
//
// Reference behaviour: torchvision.ops.roi_align / MultiScaleRoIAlign (aligned=False,
// sampling_ratio 2) and torchvision.ops.nms, which the reference's
// examples/computer_vision/fasterrcnn_coco_pytorch/model_def.py:18,112 use through
// fasterrcnn_resnet50_fpn.  torchvision is not part of this image; these kernels are written for
// CDNA4 directly.
//
// RoIAlign layout choice: feature maps are NHWC (channels_last — what MIOpen's fastest convs
// produce on gfx950) and the pooled output is [K, PH, PW, C].  One thread owns one output channel
// of one bin, channels fastest, so a 64-lane wave reads 64 consecutive channels of the same pixel:
// every bilinear corner fetch is one contiguous 128-B (bf16) / 256-B (fp32) segment.  Torchvision's
// NCHW kernel instead strides H*W elements between lanes.  The box head consumes the [K, PH, PW, C]
// flattening (a fixed permutation of torchvision's [K, C, PH, PW]; same model up to fc6's column
// order).  Backward scatters with fp32 global atomics into an fp32 gradient map per level.
//
// NMS: the wavefront is 64 lanes wide, so a 64-bit word holds one box's suppression bits against a
// 64-box column block and a single wave can resolve a whole 64-box block with lane shuffles.  The
// sweep keeps the "removed" bitmap in LDS and only touches mask rows of boxes it keeps.  No host
// round-trip of the (n x n/64)-word mask (torchvision copies it to the CPU for the sweep).

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float load_f(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float load_f(const unsigned short* p, int64_t i) {
  return __uint_as_float(static_cast<uint32_t>(p[i]) << 16);
}
__device__ __forceinline__ void store_f(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void store_f(unsigned short* p, int64_t i, float v) {
  p[i] = __builtin_bit_cast(unsigned short, static_cast<__bf16>(v));
}

struct Levels {
  const void* feat[5];   // [N, H, W, C] per level
  float* grad[5];        // fp32 [N, H, W, C] per level (backward)
  int H[5], W[5];
  float scale[5];
  int n_levels;
};

struct RoiGeom {
  int K, C, PH, PW, sampling;
};

// torchvision's bilinear sampling rule (aligned=False): zero outside [-1, H] x [-1, W], clamp to
// the last row/column inside.
struct Bilinear {
  int64_t o1, o2, o3, o4;  // pixel offsets (in units of C) of the 4 corners
  float w1, w2, w3, w4;
  bool valid;
};

__device__ __forceinline__ Bilinear bilinear(float y, float x, int H, int W) {
  Bilinear b;
  b.valid = !(y < -1.0f || y > static_cast<float>(H) || x < -1.0f || x > static_cast<float>(W));
  if (!b.valid) {
    b.o1 = b.o2 = b.o3 = b.o4 = 0;
    b.w1 = b.w2 = b.w3 = b.w4 = 0.f;
    return b;
  }
  if (y <= 0.f) y = 0.f;
  if (x <= 0.f) x = 0.f;
  int yl = static_cast<int>(y), xl = static_cast<int>(x), yh, xh;
  if (yl >= H - 1) { yh = yl = H - 1; y = static_cast<float>(yl); } else { yh = yl + 1; }
  if (xl >= W - 1) { xh = xl = W - 1; x = static_cast<float>(xl); } else { xh = xl + 1; }
  const float ly = y - yl, lx = x - xl, hy = 1.f - ly, hx = 1.f - lx;
  b.o1 = static_cast<int64_t>(yl) * W + xl;
  b.o2 = static_cast<int64_t>(yl) * W + xh;
  b.o3 = static_cast<int64_t>(yh) * W + xl;
  b.o4 = static_cast<int64_t>(yh) * W + xh;
  b.w1 = hy * hx; b.w2 = hy * lx; b.w3 = ly * hx; b.w4 = ly * lx;
  return b;
}

struct BinGeom {
  float start_y, start_x, bin_h, bin_w;
  int gh, gw;
};

__device__ __forceinline__ BinGeom roi_bin(const float* roi, float scale, const RoiGeom& g) {
  // roi = (batch_index, x1, y1, x2, y2) in input-image coordinates
  BinGeom b;
  b.start_x = roi[1] * scale;
  b.start_y = roi[2] * scale;
  const float rw = fmaxf(roi[3] * scale - b.start_x, 1.f);
  const float rh = fmaxf(roi[4] * scale - b.start_y, 1.f);
  b.bin_h = rh / g.PH;
  b.bin_w = rw / g.PW;
  b.gh = g.sampling > 0 ? g.sampling : static_cast<int>(ceilf(rh / g.PH));
  b.gw = g.sampling > 0 ? g.sampling : static_cast<int>(ceilf(rw / g.PW));
  return b;
}

template <typename T>
__global__ void __launch_bounds__(kThreads) roi_align_fwd(const float* __restrict__ rois, const int* __restrict__ level,
                                                          Levels L, RoiGeom g, T* __restrict__ out, int64_t total) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * kThreads) {
    int64_t t = i;
    const int c = static_cast<int>(t % g.C); t /= g.C;
    const int pw = static_cast<int>(t % g.PW); t /= g.PW;
    const int ph = static_cast<int>(t % g.PH);
    const int k = static_cast<int>(t / g.PH);
    const float* roi = rois + 5 * static_cast<int64_t>(k);
    const int lv = level[k];
    const int H = L.H[lv], W = L.W[lv];
    const T* f = static_cast<const T*>(L.feat[lv]) + static_cast<int64_t>(roi[0]) * H * W * g.C + c;
    const BinGeom b = roi_bin(roi, L.scale[lv], g);
    float acc = 0.f;
    for (int iy = 0; iy < b.gh; ++iy) {
      const float y = b.start_y + ph * b.bin_h + (iy + 0.5f) * b.bin_h / b.gh;
      for (int ix = 0; ix < b.gw; ++ix) {
        const float x = b.start_x + pw * b.bin_w + (ix + 0.5f) * b.bin_w / b.gw;
        const Bilinear s = bilinear(y, x, H, W);
        if (!s.valid) continue;
        acc += s.w1 * load_f(f, s.o1 * g.C) + s.w2 * load_f(f, s.o2 * g.C) + s.w3 * load_f(f, s.o3 * g.C) +
               s.w4 * load_f(f, s.o4 * g.C);
      }
    }
    const int count = max(b.gh * b.gw, 1);
    store_f(out, i, acc / count);
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) roi_align_bwd(const float* __restrict__ rois, const int* __restrict__ level,
                                                          Levels L, RoiGeom g, const T* __restrict__ dy, int64_t total) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * kThreads) {
    int64_t t = i;
    const int c = static_cast<int>(t % g.C); t /= g.C;
    const int pw = static_cast<int>(t % g.PW); t /= g.PW;
    const int ph = static_cast<int>(t % g.PH);
    const int k = static_cast<int>(t / g.PH);
    const float* roi = rois + 5 * static_cast<int64_t>(k);
    const int lv = level[k];
    const int H = L.H[lv], W = L.W[lv];
    float* gr = L.grad[lv] + static_cast<int64_t>(roi[0]) * H * W * g.C + c;
    const BinGeom b = roi_bin(roi, L.scale[lv], g);
    const float go = load_f(dy, i) / max(b.gh * b.gw, 1);
    if (go == 0.f) continue;
    for (int iy = 0; iy < b.gh; ++iy) {
      const float y = b.start_y + ph * b.bin_h + (iy + 0.5f) * b.bin_h / b.gh;
      for (int ix = 0; ix < b.gw; ++ix) {
        const float x = b.start_x + pw * b.bin_w + (ix + 0.5f) * b.bin_w / b.gw;
        const Bilinear s = bilinear(y, x, H, W);
        if (!s.valid) continue;
        atomicAdd(gr + s.o1 * g.C, go * s.w1);
        atomicAdd(gr + s.o2 * g.C, go * s.w2);
        atomicAdd(gr + s.o3 * g.C, go * s.w3);
        atomicAdd(gr + s.o4 * g.C, go * s.w4);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// NMS
// ---------------------------------------------------------------------------------------------
constexpr int kBlk = 64;  // boxes per column block = wavefront width = bits per mask word

__device__ __forceinline__ float iou(const float4 a, const float4 b) {
  const float iw = fmaxf(fminf(a.z, b.z) - fmaxf(a.x, b.x), 0.f);
  const float ih = fmaxf(fminf(a.w, b.w) - fmaxf(a.y, b.y), 0.f);
  const float inter = iw * ih;
  const float ua = (a.z - a.x) * (a.w - a.y) + (b.z - b.x) * (b.w - b.y) - inter;
  return ua > 0.f ? inter / ua : 0.f;
}

// mask[r * cb + j] bit q = (IoU(box r, box 64j+q) > thr) and 64j+q > r; only tiles with j >= r/64
// are written (the sweep never reads the others).  Grid (cb, cb), one wave per tile.
__global__ void __launch_bounds__(kBlk) nms_mask(const float4* __restrict__ boxes, int n, float thr,
                                                 unsigned long long* __restrict__ mask, int cb) {
  const int rb = blockIdx.y, cbk = blockIdx.x;
  if (cbk < rb) return;
  __shared__ float4 cols[kBlk];
  const int lane = threadIdx.x;
  const int ci = cbk * kBlk + lane;
  cols[lane] = ci < n ? boxes[ci] : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  const int r = rb * kBlk + lane;
  if (r >= n) return;
  const float4 me = boxes[r];
  const int ncols = min(kBlk, n - cbk * kBlk);
  unsigned long long bits = 0ull;
  for (int q = 0; q < ncols; ++q) {
    const int col = cbk * kBlk + q;
    if (col > r && iou(me, cols[q]) > thr) bits |= 1ull << q;
  }
  mask[static_cast<int64_t>(r) * cb + cbk] = bits;
}

__device__ __forceinline__ unsigned long long shfl64(unsigned long long v, int src) {
  const int lo = __shfl(static_cast<int>(v & 0xffffffffull), src, kBlk);
  const int hi = __shfl(static_cast<int>(v >> 32), src, kBlk);
  return (static_cast<unsigned long long>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo);
}

// One wave. keep[i] = 1 if sorted box i survives.  removed bitmap (cb words) in LDS.
constexpr int kMaxWords = 4096;  // n <= 262144 boxes (32 KB of LDS)

__global__ void __launch_bounds__(kBlk) nms_sweep(const unsigned long long* __restrict__ mask, int n, int cb,
                                                  uint8_t* __restrict__ keep) {
  __shared__ unsigned long long removed[kMaxWords];
  const int lane = threadIdx.x;
  for (int j = lane; j < cb; j += kBlk) removed[j] = 0ull;
  __syncthreads();
  for (int b = 0; b < cb; ++b) {
    const int r = b * kBlk + lane;
    const unsigned long long diag = r < n ? mask[static_cast<int64_t>(r) * cb + b] : 0ull;
    unsigned long long rem = removed[b];
    unsigned long long kept = 0ull;
    const int nb = min(kBlk, n - b * kBlk);
    for (int q = 0; q < nb; ++q) {  // wave-uniform: every lane tracks the same rem / kept
      const unsigned long long row = shfl64(diag, q);
      if (!((rem >> q) & 1ull)) {
        kept |= 1ull << q;
        rem |= row;
      }
    }
    if (r < n) keep[r] = static_cast<uint8_t>((kept >> lane) & 1ull);
    for (int j = b + 1 + lane; j < cb; j += kBlk) {
      unsigned long long acc = removed[j];
      unsigned long long kb = kept;
      while (kb) {
        const int q = __builtin_ctzll(kb);
        kb &= kb - 1;
        acc |= mask[static_cast<int64_t>(b * kBlk + q) * cb + j];
      }
      removed[j] = acc;
    }
    __syncthreads();
  }
}

int grid_for(int64_t work) {
  int64_t b = (work + kThreads - 1) / kThreads;
  if (b > 65536) b = 65536;
  return static_cast<int>(b < 1 ? 1 : b);
}

Levels make_levels(int n_levels, const void* const* feats, float* const* grads, const int* hs, const int* ws,
                   const float* scales) {
  Levels L{};
  L.n_levels = n_levels;
  for (int l = 0; l < n_levels; ++l) {
    L.feat[l] = feats ? feats[l] : nullptr;
    L.grad[l] = grads ? grads[l] : nullptr;
    L.H[l] = hs[l];
    L.W[l] = ws[l];
    L.scale[l] = scales[l];
  }
  return L;
}

}  // namespace

extern "C" {

// rois [K, 5] fp32 (batch_idx, x1, y1, x2, y2); level [K] int32 in [0, n_levels); feats: n_levels
// NHWC maps of C channels (dtype 0 fp32 / 1 bf16); out [K, PH, PW, C] same dtype.
int det_roi_align_fwd(void* stream, int dtype, const float* rois, const int* level, int K, int n_levels,
                      const void* const* feats, const int* hs, const int* ws, const float* scales, int C, int PH,
                      int PW, int sampling, void* out) {
  if (n_levels < 1 || n_levels > 5 || K < 0 || C <= 0) return -1;
  if (K == 0) return 0;
  const Levels L = make_levels(n_levels, feats, nullptr, hs, ws, scales);
  const RoiGeom g{K, C, PH, PW, sampling};
  const int64_t total = static_cast<int64_t>(K) * PH * PW * C;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == 1)
    hipLaunchKernelGGL(roi_align_fwd<unsigned short>, dim3(grid_for(total)), dim3(kThreads), 0, st, rois, level, L, g,
                       static_cast<unsigned short*>(out), total);
  else
    hipLaunchKernelGGL(roi_align_fwd<float>, dim3(grid_for(total)), dim3(kThreads), 0, st, rois, level, L, g,
                       static_cast<float*>(out), total);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// dy [K, PH, PW, C] (dtype), grads: n_levels fp32 NHWC maps, accumulated into (caller zero-fills).
int det_roi_align_bwd(void* stream, int dtype, const float* rois, const int* level, int K, int n_levels,
                      float* const* grads, const int* hs, const int* ws, const float* scales, int C, int PH, int PW,
                      int sampling, const void* dy) {
  if (n_levels < 1 || n_levels > 5 || K < 0 || C <= 0) return -1;
  if (K == 0) return 0;
  const Levels L = make_levels(n_levels, nullptr, grads, hs, ws, scales);
  const RoiGeom g{K, C, PH, PW, sampling};
  const int64_t total = static_cast<int64_t>(K) * PH * PW * C;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == 1)
    hipLaunchKernelGGL(roi_align_bwd<unsigned short>, dim3(grid_for(total)), dim3(kThreads), 0, st, rois, level, L, g,
                       static_cast<const unsigned short*>(dy), total);
  else
    hipLaunchKernelGGL(roi_align_bwd<float>, dim3(grid_for(total)), dim3(kThreads), 0, st, rois, level, L, g,
                       static_cast<const float*>(dy), total);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int det_nms_mask_words(int n) { return (n + kBlk - 1) / kBlk; }
int det_nms_max_boxes() { return kMaxWords * kBlk; }

// boxes [n, 4] fp32 xyxy sorted by descending score; mask workspace n * cb uint64; keep [n] uint8.
int det_nms(void* stream, const float* boxes, int n, float thr, unsigned long long* mask, uint8_t* keep) {
  if (n < 0 || n > kMaxWords * kBlk) return -1;
  if (n == 0) return 0;
  const int cb = (n + kBlk - 1) / kBlk;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(nms_mask, dim3(cb, cb), dim3(kBlk), 0, st, reinterpret_cast<const float4*>(boxes), n, thr, mask,
                     cb);
  hipLaunchKernelGGL(nms_sweep, dim3(1), dim3(kBlk), 0, st, mask, n, cb, keep);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
