// det_stream.hip — HBM streaming yardsticks for the roofline (VERDICT r4 "roofline yardstick").
//
// Pure read, pure write and copy streams at the bandwidth the chip can actually sustain, so that
// "% of the streaming bound" rows of scripts/step_roofline.py are judged against a real ceiling
// (MI355X: 8 TB/s spec, ~6.3 TB/s achievable per MI355X_MICROARCH.md §HBM).  Design:
//   * 16 B per lane per access (dwordx4), UNROLL independent accesses in flight per lane before any
//     is consumed, so a CU keeps ~64-128 KiB outstanding (Little: 8 TB/s x ~2 us / 256 CUs);
//   * grid = a multiple of 256 CUs, chunked so each workgroup streams a contiguous span
//     (consecutive workgroups land on consecutive XCDs; every XCD's L2 sees its own spans);
//   * the read folds what it loads into one value per lane and stores it only when it equals an
//     impossible key, so nothing is dead-code-eliminated and nothing extra is written;
//   * nontemporal (slc/nt) variants for the write and copy, which skip L2 allocation.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kThreads = 256;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ void __launch_bounds__(kThreads) stream_read_kernel(const u32x4* __restrict__ p, int64_t n16,
                                                               uint32_t* __restrict__ sink) {
  const int64_t per_block = (n16 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per_block;
  const int64_t hi = lo + per_block < n16 ? lo + per_block : n16;
  uint32_t acc = 0;
  int64_t i = lo + threadIdx.x;
  for (; i + (UNROLL - 1) * kThreads < hi; i += UNROLL * kThreads) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = NT ? __builtin_nontemporal_load(p + i + u * kThreads) : p[i + u * kThreads];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < hi; i += kThreads) {
    u32x4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;  // never true for the buffers the benchmark fills
}

template <int UNROLL, bool NT>
__global__ void __launch_bounds__(kThreads) stream_write_kernel(u32x4* __restrict__ p, int64_t n16, uint32_t value) {
  const int64_t per_block = (n16 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per_block;
  const int64_t hi = lo + per_block < n16 ? lo + per_block : n16;
  const u32x4 v = u32x4{value, value, value, value};
  int64_t i = lo + threadIdx.x;
  for (; i + (UNROLL - 1) * kThreads < hi; i += UNROLL * kThreads) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (NT) __builtin_nontemporal_store(v, p + i + u * kThreads);
      else p[i + u * kThreads] = v;
    }
  }
  for (; i < hi; i += kThreads) p[i] = v;
}

template <int UNROLL, bool NT>
__global__ void __launch_bounds__(kThreads) stream_copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                               int64_t n16) {
  const int64_t per_block = (n16 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per_block;
  const int64_t hi = lo + per_block < n16 ? lo + per_block : n16;
  int64_t i = lo + threadIdx.x;
  for (; i + (UNROLL - 1) * kThreads < hi; i += UNROLL * kThreads) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(src + i + u * kThreads);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], dst + i + u * kThreads);
      else dst[i + u * kThreads] = v[u];
    }
  }
  for (; i < hi; i += kThreads) dst[i] = src[i];
}

int grid_for(int64_t n16, int blocks) {
  if (blocks <= 0) blocks = 256 * 8;
  int64_t max_useful = (n16 + kThreads - 1) / kThreads;
  if (max_useful < 1) max_useful = 1;
  return (int)(blocks < max_useful ? blocks : max_useful);
}

}  // namespace

// kind: 0 read (nontemporal loads), 1 write, 2 write nontemporal, 3 copy, 4 copy nontemporal-store,
// 5 read (plain loads).
// unroll: 1, 2, 4 or 8.  nbytes must be a multiple of 16 and the pointers 16-B aligned.
extern "C" int det_stream(void* stream, int kind, const void* src, void* dst, int64_t nbytes, int blocks,
                          int unroll, uint32_t value, uint32_t* sink) {
  if (nbytes <= 0 || (nbytes & 15) || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15)) return (int)hipErrorInvalidValue;
  const int64_t n16 = nbytes >> 4;
  const int g = grid_for(n16, blocks);
  hipStream_t s = (hipStream_t)stream;
  const u32x4* in = (const u32x4*)src;
  u32x4* out = (u32x4*)dst;
#define DET_STREAM_CASES(U)                                                                           \
  case U:                                                                                             \
    if (kind == 0) stream_read_kernel<U, true><<<g, kThreads, 0, s>>>(in, n16, sink);                 \
    else if (kind == 5) stream_read_kernel<U, false><<<g, kThreads, 0, s>>>(in, n16, sink);           \
    else if (kind == 1) stream_write_kernel<U, false><<<g, kThreads, 0, s>>>(out, n16, value);        \
    else if (kind == 2) stream_write_kernel<U, true><<<g, kThreads, 0, s>>>(out, n16, value);         \
    else if (kind == 3) stream_copy_kernel<U, false><<<g, kThreads, 0, s>>>(in, out, n16);            \
    else if (kind == 4) stream_copy_kernel<U, true><<<g, kThreads, 0, s>>>(in, out, n16);             \
    else return (int)hipErrorInvalidValue;                                                            \
    break;
  switch (unroll) {
    DET_STREAM_CASES(1)
    DET_STREAM_CASES(2)
    DET_STREAM_CASES(4)
    DET_STREAM_CASES(8)
    default:
      return (int)hipErrorInvalidValue;
  }
#undef DET_STREAM_CASES
  return (int)hipGetLastError();
}
