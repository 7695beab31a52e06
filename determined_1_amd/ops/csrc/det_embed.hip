// det_embed.hip — BERT's embedding layer (word + token-type + position lookup and sum) forward and a
// graph-safe, deterministic backward.
//
// Why native: torch's dense embedding backward for more than 3072 indices sorts the ids with rocprim
// and sizes later launches from a segment count it reads back to the host.  Captured in a hipGraph,
// those sizes are frozen at the capture batch's count, and a later batch with more distinct ids runs
// past its buffers: the BERT graph replay faulted (HSA memory aperture violation in rocprim's
// partition_kernel) after ~700 replays, every time (round-5 sessions 13/14).  Here every launch size
// depends only on the shapes: a one-block LDS bitonic sort of (id, position) keys, then one block per
// sorted position that sums its id's run if it starts one -- deterministic (fixed summation order),
// fp32 accumulation, one rounding into the gradient.
//
// Reference semantics: torch.nn.Embedding (padding_idx rows get no gradient), the three lookups
// summed in torch's order ((word + type) rounded, + position rounded) as models/bert.py does
// (reference examples/nlp/bert_squad_pytorch uses transformers' BertEmbeddings, same sum).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int NT = 256;
constexpr int SORT_MAX = 8192;  // tokens per step the one-block sort takes (B * S)
constexpr int POS_BITS = 13;    // key = id << 13 | token position

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}
template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
template <typename T>
__device__ __forceinline__ T cvt(float v);
template <>
__device__ __forceinline__ float cvt<float>(float v) { return v; }
template <>
__device__ __forceinline__ uint16_t cvt<uint16_t>(float v) { return f2bf(v); }
template <typename T>
__device__ __forceinline__ float rnd(float v);
template <>
__device__ __forceinline__ float rnd<float>(float v) { return v; }
template <>
__device__ __forceinline__ float rnd<uint16_t>(float v) { return bf2f(f2bf(v)); }

// out[t][c] = round(round(Ww[id[t]][c] + Wt[tt[t]][c]) + Wp[t % S][c])
template <typename T>
__global__ void __launch_bounds__(NT) embed_fwd_kernel(const int64_t* ids, const int64_t* tt, const T* ww, const T* wt,
                                                       const T* wp, T* out, int Tn, int S, int H) {
  const int t = blockIdx.x;
  const int64_t id = ids[t], ty = tt != nullptr ? tt[t] : 0;
  const int s = t % S;
  for (int c = threadIdx.x; c < H; c += NT) {
    const float a = rnd<T>(ldf<T>(ww, id * H + c) + ldf<T>(wt, ty * H + c));
    out[static_cast<int64_t>(t) * H + c] = cvt<T>(a + ldf<T>(wp, static_cast<int64_t>(s) * H + c));
  }
}

// one block: sort the (id << 13 | t) keys of the step's tokens ascending (bitonic, in LDS)
__global__ void __launch_bounds__(1024) embed_sort_kernel(const int64_t* ids, int Tn, int n2, uint32_t* keys_out) {
  __shared__ uint32_t k[SORT_MAX];
  for (int i = threadIdx.x; i < n2; i += 1024)
    k[i] = i < Tn ? (static_cast<uint32_t>(ids[i]) << POS_BITS) | static_cast<uint32_t>(i) : 0xffffffffu;
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < n2; i += 1024) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const uint32_t a = k[i], b = k[j];
          if ((a > b) == up) {
            k[i] = b;
            k[j] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < Tn; i += 1024) keys_out[i] = k[i];
}

// one block per sorted position p: if p starts a run of one id, sum the run's gradient rows in
// position order and add them into dW[id] (fp32, one rounding); padding_idx rows are skipped
template <typename T>
__global__ void __launch_bounds__(NT) embed_word_bwd_kernel(const uint32_t* keys, const T* g, T* dw, int Tn, int H,
                                                            int64_t pad, int accumulate) {
  const int p = blockIdx.x;
  const uint32_t id = keys[p] >> POS_BITS;
  if (p > 0 && (keys[p - 1] >> POS_BITS) == id) return;
  if (static_cast<int64_t>(id) == pad) return;
  int end = p + 1;
  while (end < Tn && (keys[end] >> POS_BITS) == id) ++end;
  for (int c = threadIdx.x; c < H; c += NT) {
    float acc = 0.f;
    for (int q = p; q < end; ++q) acc += ldf<T>(g, static_cast<int64_t>(keys[q] & ((1u << POS_BITS) - 1u)) * H + c);
    const int64_t e = static_cast<int64_t>(id) * H + c;
    dw[e] = cvt<T>(accumulate ? ldf<T>(dw, e) + acc : acc);
  }
}

// position rows: dWp[s][c] = sum_b g[b*S + s][c] (b ascending)
template <typename T>
__global__ void __launch_bounds__(NT) embed_pos_bwd_kernel(const T* g, T* dwp, int B, int S, int H, int accumulate) {
  const int s = blockIdx.x;
  for (int c = threadIdx.x; c < H; c += NT) {
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += ldf<T>(g, (static_cast<int64_t>(b) * S + s) * H + c);
    const int64_t e = static_cast<int64_t>(s) * H + c;
    dwp[e] = cvt<T>(accumulate ? ldf<T>(dwp, e) + acc : acc);
  }
}

constexpr int TYPE_MAX = 4;     // token-type vocabulary (BERT: 2)
constexpr int TYPE_CHUNK = 256;  // tokens per partial

// token-type rows, pass 1: partial[chunk][v][c] = sum over the chunk's tokens of type v
template <typename T>
__global__ void __launch_bounds__(NT) embed_type_part_kernel(const int64_t* tt, const T* g, float* part, int Tn, int H,
                                                             int Vt) {
  const int chunk = blockIdx.y;
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= H) return;
  float acc[TYPE_MAX] = {0.f, 0.f, 0.f, 0.f};
  const int t1 = (chunk + 1) * TYPE_CHUNK < Tn ? (chunk + 1) * TYPE_CHUNK : Tn;
  for (int t = chunk * TYPE_CHUNK; t < t1; ++t) {
    const int v = static_cast<int>(tt[t]);
    const float x = ldf<T>(g, static_cast<int64_t>(t) * H + c);
#pragma unroll
    for (int q = 0; q < TYPE_MAX; ++q) acc[q] += q == v ? x : 0.f;
  }
#pragma unroll
  for (int q = 0; q < TYPE_MAX; ++q)
    if (q < Vt) part[(static_cast<int64_t>(chunk) * Vt + q) * H + c] = acc[q];
}

// pass 2: dWt[v][c] (+)= sum over chunks (ascending)
template <typename T>
__global__ void __launch_bounds__(NT) embed_type_fin_kernel(const float* part, T* dwt, int nchunk, int Vt, int H,
                                                            int accumulate) {
  const int e = blockIdx.x * NT + threadIdx.x;
  if (e >= Vt * H) return;
  float acc = 0.f;
  for (int ch = 0; ch < nchunk; ++ch) acc += part[static_cast<int64_t>(ch) * Vt * H + e];
  dwt[e] = cvt<T>(accumulate ? ldf<T>(dwt, e) + acc : acc);
}

}  // namespace

extern "C" {

// out [T, H] = word[ids] + type[tt] + pos[t % S]; bf16 (bf16 = 1) or fp32 tables
int det_embed_fwd(void* stream, int32_t bf16, const int64_t* ids, const int64_t* tt, const void* ww, const void* wt,
                  const void* wp, void* out, int32_t Tn, int32_t S, int32_t H) {
  if (Tn < 1 || S < 1 || H < 1 || Tn % S) return static_cast<int>(hipErrorInvalidValue);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (bf16)
    embed_fwd_kernel<uint16_t><<<Tn, NT, 0, st>>>(ids, tt, static_cast<const uint16_t*>(ww), static_cast<const uint16_t*>(wt),
                                                  static_cast<const uint16_t*>(wp), static_cast<uint16_t*>(out), Tn, S, H);
  else
    embed_fwd_kernel<float><<<Tn, NT, 0, st>>>(ids, tt, static_cast<const float*>(ww), static_cast<const float*>(wt),
                                               static_cast<const float*>(wp), static_cast<float*>(out), Tn, S, H);
  return static_cast<int>(hipGetLastError());
}

// fp32 workspace floats det_embed_bwd needs: the sorted keys (as floats' storage) + type partials
int64_t det_embed_ws_floats(int32_t Tn, int32_t H, int32_t Vt) {
  const int64_t nchunk = (Tn + TYPE_CHUNK - 1) / TYPE_CHUNK;
  return Tn + nchunk * Vt * H;
}

// gradients of the three tables from g [T, H] (ids < 2^18, T <= 8192, Vt <= 4); dw* (+)= when
// accumulate, else overwritten -- dww must be zeroed by the caller when not accumulating (rows of
// ids not in the step are not written)
int det_embed_bwd(void* stream, int32_t bf16, const int64_t* ids, const int64_t* tt, const void* g, void* dww,
                  void* dwt, void* dwp, int32_t Tn, int32_t S, int32_t H, int32_t Vt, int64_t pad, float* ws,
                  int32_t accumulate) {
  if (Tn < 1 || Tn > SORT_MAX || S < 1 || Tn % S || H < 1 || Vt < 1 || Vt > TYPE_MAX)
    return static_cast<int>(hipErrorInvalidValue);
  hipStream_t st = static_cast<hipStream_t>(stream);
  int n2 = 1;
  while (n2 < Tn) n2 <<= 1;
  uint32_t* keys = reinterpret_cast<uint32_t*>(ws);
  float* part = ws + Tn;
  const int nchunk = (Tn + TYPE_CHUNK - 1) / TYPE_CHUNK;
  embed_sort_kernel<<<1, 1024, 0, st>>>(ids, Tn, n2, keys);
  const dim3 tgrid((H + NT - 1) / NT, nchunk);
  const int fin_blocks = (Vt * H + NT - 1) / NT;
  if (bf16) {
    const uint16_t* gb = static_cast<const uint16_t*>(g);
    embed_word_bwd_kernel<uint16_t><<<Tn, NT, 0, st>>>(keys, gb, static_cast<uint16_t*>(dww), Tn, H, pad, accumulate);
    embed_pos_bwd_kernel<uint16_t><<<S, NT, 0, st>>>(gb, static_cast<uint16_t*>(dwp), Tn / S, S, H, accumulate);
    if (dwt != nullptr) {
      embed_type_part_kernel<uint16_t><<<tgrid, NT, 0, st>>>(tt, gb, part, Tn, H, Vt);
      embed_type_fin_kernel<uint16_t><<<fin_blocks, NT, 0, st>>>(part, static_cast<uint16_t*>(dwt), nchunk, Vt, H, accumulate);
    }
  } else {
    const float* gf = static_cast<const float*>(g);
    embed_word_bwd_kernel<float><<<Tn, NT, 0, st>>>(keys, gf, static_cast<float*>(dww), Tn, H, pad, accumulate);
    embed_pos_bwd_kernel<float><<<S, NT, 0, st>>>(gf, static_cast<float*>(dwp), Tn / S, S, H, accumulate);
    if (dwt != nullptr) {
      embed_type_part_kernel<float><<<tgrid, NT, 0, st>>>(tt, gf, part, Tn, H, Vt);
      embed_type_fin_kernel<float><<<fin_blocks, NT, 0, st>>>(part, static_cast<float*>(dwt), nchunk, Vt, H, accumulate);
    }
  }
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
