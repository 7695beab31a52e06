// det_blaslt.hip -- the transformer Linear GEMMs on hipBLASLt without the per-call host cost of
// torch.mm / torch.addmm.
//
// Measured (r5s32 cProfile of the BERT-base eager step): every torch.mm / addmm / addmm_ into
// hipBLASLt costs 21-26 us of host time (dispatcher, tensor checks, descriptor and heuristic work
// per call), 108 calls per step = 2.6 ms of a ~9 ms host-bound step.  Here each GEMM shape gets its
// matmul descriptor, matrix layouts and heuristic-chosen algorithm once (a small cache keyed by the
// shape); a call then sets the bias pointer and issues hipblasLtMatmul.  Same library, same
// algorithm choice as torch's default path (the top heuristic result), so the GPU work is unchanged.
//
// hipBLASLt is the instance torch already loaded (its bundled libhipblaslt, opened by path with
// RTLD_NOLOAD and resolved with dlsym), so there is one hipBLASLt and one HIP runtime in the process.
//
// BLAS convention (column-major): D[m, n] = alpha * op(A) . op(B) + beta * C (C = D), optional
// per-row bias added in the epilogue (HIPBLASLT_EPILOGUE_BIAS: one rounding into D), or (bias_mode 2)
// the bias gradient of B written by the epilogue (HIPBLASLT_EPILOGUE_BGRADB: bias[n] = sum_k op(B)[k, n],
// a Linear's db from its weight-gradient GEMM instead of a separate column-sum pass).

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdint>
#include <map>
#include <mutex>
#include <tuple>

namespace {

struct Api {
  decltype(&hipblasLtCreate) create = nullptr;
  decltype(&hipblasLtMatmulDescCreate) desc_create = nullptr;
  decltype(&hipblasLtMatmulDescSetAttribute) desc_set = nullptr;
  decltype(&hipblasLtMatrixLayoutCreate) layout_create = nullptr;
  decltype(&hipblasLtMatmulPreferenceCreate) pref_create = nullptr;
  decltype(&hipblasLtMatmulPreferenceSetAttribute) pref_set = nullptr;
  decltype(&hipblasLtMatmulAlgoGetHeuristic) heuristic = nullptr;
  decltype(&hipblasLtMatmul) matmul = nullptr;
  hipblasLtHandle_t handle = nullptr;
  bool ok = false;
};

Api g_api;
std::mutex g_mu;

struct Plan {
  hipblasLtMatmulDesc_t desc;
  hipblasLtMatrixLayout_t a, b, d;
  hipblasLtMatmulAlgo_t algo;
  size_t ws;
  bool bias;
  int bias_mode;
};

// (device, transa, transb, m, n, k, lda, ldb, ldd, bias mode, beta != 0, dtype).  The plan is only
// used with 16-B aligned operands (ops/transformer.py _bl_ok), so alignment needs no key field.
typedef std::tuple<int, int, int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int, int> Key;
std::map<Key, Plan> g_plans;

template <typename F>
bool sym(void* lib, const char* name, F* out) {
  *out = reinterpret_cast<F>(dlsym(lib, name));
  return *out != nullptr;
}

hipDataType dtype_of(int code) { return code == 1 ? HIP_R_16BF : HIP_R_32F; }

}  // namespace

extern "C" {

// path: the hipBLASLt shared library torch loaded.  0 on success.
int det_blaslt_init(const char* path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_api.ok) return 0;
  void* lib = dlopen(path, RTLD_NOW | RTLD_NOLOAD);
  if (lib == nullptr) lib = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (lib == nullptr) return -1;
  Api a;
  if (!sym(lib, "hipblasLtCreate", &a.create) || !sym(lib, "hipblasLtMatmulDescCreate", &a.desc_create) ||
      !sym(lib, "hipblasLtMatmulDescSetAttribute", &a.desc_set) ||
      !sym(lib, "hipblasLtMatrixLayoutCreate", &a.layout_create) ||
      !sym(lib, "hipblasLtMatmulPreferenceCreate", &a.pref_create) ||
      !sym(lib, "hipblasLtMatmulPreferenceSetAttribute", &a.pref_set) ||
      !sym(lib, "hipblasLtMatmulAlgoGetHeuristic", &a.heuristic) || !sym(lib, "hipblasLtMatmul", &a.matmul))
    return -2;
  if (a.create(&a.handle) != HIPBLAS_STATUS_SUCCESS) return -3;
  a.ok = true;
  g_api = a;
  return 0;
}

// D = op(A) op(B) [+ bias per row of D] [+ beta * D].  transa / transb: 0 = N, 1 = T.  dtype 1 =
// bf16 operands and output (fp32 accumulate), 0 = fp32.  bias (nullable) has D's dtype; bias_mode
// 2 makes it an OUTPUT: the bias gradient of B (length n).  ws: device workspace of ws_bytes.
// Returns 0, or a negative code / hipblasStatus_t on failure (-14: no algorithm for this epilogue).
int det_blaslt_gemm(void* stream, int transa, int transb, int64_t m, int64_t n, int64_t k, const void* A, int64_t lda,
                    const void* B, int64_t ldb, void* D, int64_t ldd, const void* bias, float beta, int dtype, void* ws,
                    int64_t ws_bytes, int bias_mode) {
  if (!g_api.ok) return -10;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -16;
  const int bmode = bias == nullptr ? 0 : (bias_mode == 2 ? 2 : 1);
  const Key key{dev, transa, transb, m, n, k, lda, ldb, ldd, bmode, beta != 0.f, dtype};
  Plan p;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
      const hipDataType dt = dtype_of(dtype);
      if (g_api.desc_create(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return -11;
      const int32_t ta = transa ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = transb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
      g_api.desc_set(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
      g_api.desc_set(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
      p.bias = bias != nullptr;
      p.bias_mode = bmode;
      if (p.bias) {
        const uint32_t epi = bmode == 2 ? HIPBLASLT_EPILOGUE_BGRADB : HIPBLASLT_EPILOGUE_BIAS;
        const int32_t bt = dt;
        g_api.desc_set(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
        g_api.desc_set(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
        g_api.desc_set(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
      }
      // stored shapes (column-major): A is m x k (k x m when transposed), B is k x n (n x k)
      if (g_api.layout_create(&p.a, dt, transa ? k : m, transa ? m : k, lda) != HIPBLAS_STATUS_SUCCESS ||
          g_api.layout_create(&p.b, dt, transb ? n : k, transb ? k : n, ldb) != HIPBLAS_STATUS_SUCCESS ||
          g_api.layout_create(&p.d, dt, m, n, ldd) != HIPBLAS_STATUS_SUCCESS)
        return -12;
      hipblasLtMatmulPreference_t pref;
      if (g_api.pref_create(&pref) != HIPBLAS_STATUS_SUCCESS) return -13;
      const uint64_t wsb = static_cast<uint64_t>(ws_bytes);
      g_api.pref_set(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
      hipblasLtMatmulHeuristicResult_t res[1];
      int got = 0;
      if (g_api.heuristic(g_api.handle, p.desc, p.a, p.b, p.d, p.d, pref, 1, res, &got) != HIPBLAS_STATUS_SUCCESS ||
          got < 1)
        return -14;
      p.algo = res[0].algo;
      p.ws = res[0].workspaceSize;
      g_plans.emplace(key, p);
    } else {
      p = it->second;
    }
  }
  if (static_cast<int64_t>(p.ws) > ws_bytes) return -15;
  const float alpha = 1.f;
  hipblasStatus_t st;
  {
    // one handle for the process, used from the forward thread and autograd's backward thread: every
    // launch runs under the lock (the bias pointer also lives in the shared descriptor)
    std::lock_guard<std::mutex> lk(g_mu);
    if (p.bias) g_api.desc_set(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
    st = g_api.matmul(g_api.handle, p.desc, &alpha, A, p.a, B, p.b, &beta, D, p.d, D, p.d, &p.algo, ws, p.ws,
                      static_cast<hipStream_t>(stream));
  }
  return st == HIPBLAS_STATUS_SUCCESS ? 0 : static_cast<int>(st);
}

}  // extern "C"
