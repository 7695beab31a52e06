// det_stats.h — BatchNorm-statistics partials of a GEMM output tile, shared by the det_conv and
// det_igemm epilogues.  One pass over the accumulators: per wave, sums of (y - k) and (y - k)^2
// with a per-column shift k = the wave's first row (the shifted-data variance, no cancellation
// for |mean - k| ~ std), lane groups merged by shuffles, the WM waves of a column by the Chan
// formula from LDS; the statistics are of the bf16-rounded outputs (what the BN apply reads).
// Replaces a two-pass (mean, then M2) epilogue with three barriers: -25 % epilogue time on the
// write-bound expansion 1x1 convs (profiles/r2_igemm_microbench_4wave.jsonl: stats 0.237 vs 0.182 ms).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(4))) float det_f32x4;

__device__ __forceinline__ float det_stats_round_bf(float f) {
  return __uint_as_float(static_cast<uint32_t>(__builtin_bit_cast(unsigned short, static_cast<__bf16>(f))) << 16);
}

// acc[i][j][r] holds tile row wm*TM + i*16 + (lane>>4)*4 + r, column wn*TN + j*16 + (lane&15).
// red: 3 * WM * BN floats of LDS.  Writes pmean / pm2 [out_off + col] for the BN tile columns
// (threads tid < BN).  Contains one __syncthreads (every thread of the block must call it).
template <int FM, int FN, int WM, int TM, int TN, int BN>
__device__ __forceinline__ void det_block_bn_stats(const det_f32x4 (&acc)[FM][FN], float* red, int wm, int wn, int lane,
                                                   int tid, int nvalid, float* pmean, float* pm2, int64_t out_off) {
  float n = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) n += (wm * TM + i * 16 + (lane >> 4) * 4 + r) < nvalid ? 1.f : 0.f;
  n += __shfl_xor(n, 16, 64);
  n += __shfl_xor(n, 32, 64);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const float k = __shfl(det_stats_round_bf(acc[0][j][0]), lane & 15, 64);  // the wave's first row
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * TM + i * 16 + (lane >> 4) * 4 + r;
        const float d = det_stats_round_bf(acc[i][j][r]) - k;
        if (row < nvalid) {
          s += d;
          q += d * d;
        }
      }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    if (lane < 16) {
      float* e = red + (wm * BN + wn * TN + j * 16 + lane) * 3;
      const float inv = n > 0.f ? 1.f / n : 0.f;
      e[0] = n > 0.f ? k + s * inv : 0.f;
      e[1] = n > 0.f ? fmaxf(q - s * s * inv, 0.f) : 0.f;
      e[2] = n;
    }
  }
  __syncthreads();
  if (tid < BN) {
    float tot = 0.f, mu = 0.f;
#pragma unroll
    for (int w = 0; w < WM; ++w) {
      const float* e = red + (w * BN + tid) * 3;
      tot += e[2];
      mu += e[2] * e[0];
    }
    mu = tot > 0.f ? mu / tot : 0.f;
    float m2 = 0.f;
#pragma unroll
    for (int w = 0; w < WM; ++w) {
      const float* e = red + (w * BN + tid) * 3;
      const float dm = e[0] - mu;
      m2 += e[1] + e[2] * dm * dm;
    }
    pmean[out_off + tid] = mu;
    pm2[out_off + tid] = m2;
  }
}
