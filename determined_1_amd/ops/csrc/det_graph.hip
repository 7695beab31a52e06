// hipGraph post-capture rewriting: memset nodes -> fill-kernel nodes.
//
// On this stack (HIP runtime 7.0.51831 bundled with torch 2.10+rocm7.0) a hipMemsetAsync captured
// into a graph writes the right value on the first launch of the executable graph and a stale,
// garbage byte pattern on every later launch when the memset is small (<= 4 KiB reproduced; 1 MiB
// is fine): scripts/dbg/memset_graph_repro.py, profiles/r6_graph_memset_root_cause.txt.  torch's
// cross-block reductions (e.g. the bias gradient of a Linear at batch >= 512, sum over dim 0)
// reset their semaphores that way, so their graphs replay stale from the second replay on.
//
// det_graph_fix_memsets walks a captured (not yet instantiated) hipGraph_t and replaces every
// memset node by a kernel node of det_graph_fill with the same parameters, dependencies and
// dependents.  Kernel nodes carry their arguments by value and replay correctly.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace {

// One thread per 4-byte word of a row (plus a byte tail): rows x width elements of esize bytes.
__global__ void det_graph_fill(unsigned char* dst, unsigned long long pitch, unsigned long long row_bytes,
                               unsigned long long rows, unsigned int value, unsigned int esize) {
  // the 4-byte pattern of the value replicated at the element size
  unsigned int pat = value;
  if (esize == 1) {
    pat = value & 0xFFu;
    pat |= pat << 8;
    pat |= pat << 16;
  } else if (esize == 2) {
    pat = value & 0xFFFFu;
    pat |= pat << 16;
  }
  const unsigned long long words = row_bytes / 4;
  const unsigned long long tail = row_bytes - words * 4;
  const unsigned long long per_row = words + tail;
  const unsigned long long total = per_row * rows;
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < total;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const unsigned long long r = i / per_row, c = i - r * per_row;
    unsigned char* row = dst + r * pitch;
    if (c < words) {
      // rows of a 2-D memset start at pitch multiples; word stores need 4-byte alignment
      if ((reinterpret_cast<uintptr_t>(row) & 3u) == 0) {
        reinterpret_cast<unsigned int*>(row)[c] = pat;
      } else {
        for (int b = 0; b < 4; ++b) row[c * 4 + b] = (unsigned char)(pat >> (8 * ((c * 4 + b) & 3)));
      }
    } else {
      const unsigned long long b = words * 4 + (c - words);
      row[b] = (unsigned char)(pat >> (8 * (b & 3)));
    }
  }
}

}  // namespace

extern "C" {

// mode 0: count memset nodes only; mode 1: replace them by fill-kernel nodes.
// Returns the number of memset nodes found (>= 0) or -(hipError) on a runtime failure.
int det_graph_fix_memsets(void* graph_handle, int mode) {
  hipGraph_t graph = reinterpret_cast<hipGraph_t>(graph_handle);
  size_t n = 0;
  if (hipGraphGetNodes(graph, nullptr, &n) != hipSuccess) return -1;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(graph, nodes.data(), &n) != hipSuccess) return -1;
  int found = 0;
  for (size_t k = 0; k < n; ++k) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[k], &t) != hipSuccess) return -2;
    if (t != hipGraphNodeTypeMemset) continue;
    ++found;
    if (mode == 0) continue;
    hipMemsetParams mp{};
    hipError_t e = hipGraphMemsetNodeGetParams(nodes[k], &mp);
    if (e != hipSuccess) return -(int)e;
    if (mp.elementSize != 1 && mp.elementSize != 2 && mp.elementSize != 4) return -1000;
    size_t nd = 0, nt = 0;
    if (hipGraphNodeGetDependencies(nodes[k], nullptr, &nd) != hipSuccess) return -3;
    std::vector<hipGraphNode_t> deps(nd);
    if (nd && hipGraphNodeGetDependencies(nodes[k], deps.data(), &nd) != hipSuccess) return -3;
    if (hipGraphNodeGetDependentNodes(nodes[k], nullptr, &nt) != hipSuccess) return -4;
    std::vector<hipGraphNode_t> outs(nt);
    if (nt && hipGraphNodeGetDependentNodes(nodes[k], outs.data(), &nt) != hipSuccess) return -4;

    unsigned char* dst = static_cast<unsigned char*>(mp.dst);
    unsigned long long rows = mp.height ? mp.height : 1;
    unsigned long long row_bytes = (unsigned long long)mp.width * mp.elementSize;
    unsigned long long pitch = rows > 1 ? (unsigned long long)mp.pitch : row_bytes;
    unsigned int value = mp.value;
    unsigned int esize = mp.elementSize;
    void* args[] = {&dst, &pitch, &row_bytes, &rows, &value, &esize};
    unsigned long long work = ((row_bytes + 3) / 4 + 3) * rows;
    unsigned int blocks = (unsigned int)((work + 255) / 256);
    if (blocks < 1) blocks = 1;
    if (blocks > 1024) blocks = 1024;
    hipKernelNodeParams kp{};
    kp.func = reinterpret_cast<void*>(&det_graph_fill);
    kp.gridDim = dim3(blocks);
    kp.blockDim = dim3(256);
    kp.sharedMemBytes = 0;
    kp.kernelParams = args;
    kp.extra = nullptr;
    hipGraphNode_t kn;
    e = hipGraphAddKernelNode(&kn, graph, deps.data(), nd, &kp);
    if (e != hipSuccess) return -(int)e;
    for (size_t j = 0; j < nt; ++j) {
      e = hipGraphAddDependencies(graph, &kn, &outs[j], 1);
      if (e != hipSuccess) return -(int)e;
    }
    e = hipGraphDestroyNode(nodes[k]);
    if (e != hipSuccess) return -(int)e;
  }
  return found;
}

}  // extern "C"
