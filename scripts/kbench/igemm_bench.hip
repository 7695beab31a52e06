// Standalone A/B bench for det_igemm tile configurations on ResNet-50 (batch 512) conv shapes.
// Compiles the library source in (so it measures exactly the shipped kernels), checks every config
// against a naive fp32 GPU convolution, and times configs in interleaved rounds in one process
// (cdna_hip_programming.md §5.4 rule 24).  One JSON line per (shape, config).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/kbench/igemm_bench.hip -o /tmp/igemm_bench
//   /tmp/igemm_bench [batch] [cfg,cfg,...] [shape filter: r]
#include "../../determined_1_amd/ops/csrc/det_igemm.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void ref_conv(const unsigned short* X, const unsigned short* W, float* Y, int64_t M, int N, int Cin, int Hi,
                         int Wi, int Ho, int Wo, int R, int S, int st, int pad) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  const int64_t m = idx / N;
  const int n = static_cast<int>(idx - m * N);
  const int64_t hw = static_cast<int64_t>(Ho) * Wo;
  const int64_t b = m / hw;
  const int rem = static_cast<int>(m - b * hw), ho = rem / Wo, wo = rem - ho * Wo;
  float acc = 0.f;
  for (int r = 0; r < R; ++r)
    for (int s = 0; s < S; ++s) {
      const int hi = ho * st - pad + r, wi = wo * st - pad + s;
      if (hi < 0 || hi >= Hi || wi < 0 || wi >= Wi) continue;
      const unsigned short* x = X + ((b * Hi + hi) * Wi + wi) * static_cast<int64_t>(Cin);
      const unsigned short* w = W + (static_cast<int64_t>(n) * R * S + r * S + s) * Cin;
      for (int c = 0; c < Cin; ++c) acc += bf2f(x[c]) * bf2f(w[c]);
    }
  Y[idx] = acc;
}

__global__ void cmp(const unsigned short* Y, const float* R, int64_t n, float* maxerr, float* maxref) {
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  float e = 0.f, r = 0.f;
  for (; i < n; i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    e = fmaxf(e, fabsf(bf2f(Y[i]) - R[i]));
    r = fmaxf(r, fabsf(R[i]));
  }
  atomicMax(reinterpret_cast<int*>(maxerr), __float_as_int(e));
  atomicMax(reinterpret_cast<int*>(maxref), __float_as_int(r));
}

static unsigned short f2b(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return static_cast<unsigned short>((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}

struct Shape { int cin, cout, r, st, hin, mult; };

int main(int argc, char** argv) {
  const int NB = argc > 1 ? atoi(argv[1]) : 512;
  std::vector<int> cfgs = {1, 2, 3};
  if (argc > 2) {
    cfgs.clear();
    std::string s = argv[2];
    size_t p = 0;
    while (p < s.size()) { size_t q = s.find(',', p); if (q == std::string::npos) q = s.size(); cfgs.push_back(atoi(s.substr(p, q - p).c_str())); p = q + 1; }
  }
  const int rfilter = argc > 3 ? atoi(argv[3]) : 0;
  std::vector<Shape> shapes = {
      {64, 64, 3, 1, 56, 3},   {128, 128, 3, 2, 56, 1}, {128, 128, 3, 1, 28, 3}, {256, 256, 3, 2, 28, 1},
      {256, 256, 3, 1, 14, 5}, {512, 512, 3, 2, 14, 1}, {512, 512, 3, 1, 7, 2},
      {64, 64, 1, 1, 56, 1},   {64, 256, 1, 1, 56, 4},  {256, 64, 1, 1, 56, 2},  {256, 128, 1, 1, 56, 1},
      {128, 512, 1, 1, 28, 4}, {512, 128, 1, 1, 28, 3}, {256, 1024, 1, 1, 14, 6}, {1024, 256, 1, 1, 14, 5},
      {512, 2048, 1, 1, 7, 3}, {2048, 512, 1, 1, 7, 2}, {256, 512, 1, 2, 56, 1}, {1024, 2048, 1, 2, 14, 1}};
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  void* zero;
  CK(hipMalloc(&zero, 256));
  CK(hipMemset(zero, 0, 256));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& sh : shapes) {
    if (rfilter && sh.r != rfilter) continue;
    const int pad = sh.r / 2, ho = (sh.hin + 2 * pad - sh.r) / sh.st + 1;
    const int64_t M = static_cast<int64_t>(NB) * ho * ho;
    const int64_t nx = static_cast<int64_t>(NB) * sh.hin * sh.hin * sh.cin, nw = static_cast<int64_t>(sh.cout) * sh.r * sh.r * sh.cin;
    std::vector<unsigned short> hx(nx), hw(nw);
    for (auto& v : hx) v = f2b(U(rng));
    const float ws = 1.f / sqrtf(static_cast<float>(sh.cin * sh.r * sh.r));
    for (auto& v : hw) v = f2b(U(rng) * ws);
    unsigned short *dx, *dw, *dy;
    float *ref, *err;
    CK(hipMalloc(&dx, nx * 2));
    CK(hipMalloc(&dw, nw * 2));
    CK(hipMalloc(&dy, M * sh.cout * 2));
    CK(hipMalloc(&ref, M * sh.cout * 4));
    CK(hipMalloc(&err, 8));
    CK(hipMemcpy(dx, hx.data(), nx * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, hw.data(), nw * 2, hipMemcpyHostToDevice));
    const int64_t tot = M * sh.cout;
    ref_conv<<<static_cast<unsigned>((tot + 255) / 256), 256, 0, st>>>(dx, dw, ref, M, sh.cout, sh.cin, sh.hin, sh.hin, ho, ho,
                                                                     sh.r, sh.r, sh.st, pad);
    CK(hipStreamSynchronize(st));
    const double flops = 2.0 * M * sh.cout * sh.cin * sh.r * sh.r;
    std::vector<int> ok_cfgs;
    std::vector<float> errs;
    for (int c : cfgs) {
      CK(hipMemsetAsync(dy, 0xFF, M * sh.cout * 2, st));
      int rc = det_igemm_conv_cfg(st, dx, dw, dy, zero, M, sh.cout, sh.cin, sh.hin, sh.hin, ho, ho, sh.r, sh.r, sh.st, pad,
                                  nullptr, nullptr, c);
      if (rc != 0) { printf("{\"shape\":[%d,%d,%d,%d,%d],\"cfg\":%d,\"rc\":%d}\n", sh.cin, sh.cout, sh.r, sh.st, sh.hin, c, rc); continue; }
      CK(hipMemsetAsync(err, 0, 8, st));
      cmp<<<1024, 256, 0, st>>>(dy, ref, tot, err, err + 1);
      float he[2];
      CK(hipMemcpyAsync(he, err, 8, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      ok_cfgs.push_back(c);
      errs.push_back(he[0] / std::max(he[1], 1e-6f));
    }
    const int rounds = 7, iters = 5;
    std::vector<std::vector<float>> t(ok_cfgs.size());
    for (size_t i = 0; i < ok_cfgs.size(); ++i)  // warmup
      for (int w = 0; w < 3; ++w)
        det_igemm_conv_cfg(st, dx, dw, dy, zero, M, sh.cout, sh.cin, sh.hin, sh.hin, ho, ho, sh.r, sh.r, sh.st, pad, nullptr, nullptr, ok_cfgs[i]);
    for (int rd = 0; rd < rounds; ++rd)
      for (size_t i = 0; i < ok_cfgs.size(); ++i) {
        CK(hipEventRecord(e0, st));
        for (int it = 0; it < iters; ++it)
          det_igemm_conv_cfg(st, dx, dw, dy, zero, M, sh.cout, sh.cin, sh.hin, sh.hin, ho, ho, sh.r, sh.r, sh.st, pad, nullptr, nullptr, ok_cfgs[i]);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[i].push_back(ms / iters);
      }
    for (size_t i = 0; i < ok_cfgs.size(); ++i) {
      std::sort(t[i].begin(), t[i].end());
      const float med = t[i][t[i].size() / 2], mn = t[i][0];
      printf("{\"cin\":%d,\"cout\":%d,\"r\":%d,\"stride\":%d,\"hin\":%d,\"mult\":%d,\"M\":%ld,\"cfg\":%d,\"ms\":%.4f,\"min_ms\":%.4f,"
             "\"TFs\":%.1f,\"rel_err\":%.2e}\n",
             sh.cin, sh.cout, sh.r, sh.st, sh.hin, sh.mult, static_cast<long>(M), ok_cfgs[i], med, mn, flops / med / 1e9, errs[i]);
      fflush(stdout);
    }
    CK(hipFree(dx)); CK(hipFree(dw)); CK(hipFree(dy)); CK(hipFree(ref)); CK(hipFree(err));
  }
  return 0;
}
