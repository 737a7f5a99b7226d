// Graph surgery on captured HIP graphs (the train-step graph, gdino_amd.stepgraph).
#include <vector>

#include "gd_common.h"

// ---------------------------------------------------------------------------
// Memset nodes of a captured graph -> fill-kernel nodes.
//
// On ROCm 7.0 a replayed graph's memset nodes stop taking effect once eager
// device-to-device copies (hipMemcpyAsync) have run between replays
// (tools/graph_node_order_probe.py: fill Z -> memset Z to 0 -> Z += 1 ->
// count Z != 1 is 0 on back-to-back replays and ~8 M per replay with eager
// copies in between; memcpy and kernel nodes stay correct).  PyTorch's
// multi-block reductions zero their semaphores with such a memset, and the
// train-step graph then produced wrong bias gradients (tools/
// stepgraph_diag.py --flows).  Every memset node is replaced by a kernel
// node running the library's fill kernel with the same dependencies.
// -> the number of nodes replaced, or -1 (a memset this cannot express).
extern "C" int gd_graph_memsets_to_kernels(void* graph_ptr) {
  hipGraph_t graph = static_cast<hipGraph_t>(graph_ptr);
  size_t n = 0;
  if (hipGraphGetNodes(graph, nullptr, &n) != hipSuccess) return -1;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(graph, nodes.data(), &n) != hipSuccess) return -1;
  int replaced = 0;
  for (hipGraphNode_t nd : nodes) {
    hipGraphNodeType type;
    if (hipGraphNodeGetType(nd, &type) != hipSuccess) return -1;
    if (type != hipGraphNodeTypeMemset) continue;
    hipMemsetParams p;
    if (hipGraphMemsetNodeGetParams(nd, &p) != hipSuccess) return -1;
    const size_t es = p.elementSize, h = p.height ? p.height : 1;
    if (!(es == 1 || es == 2 || es == 4) || (h > 1 && p.pitch != p.width * es)) return -1;
    const size_t bytes = p.width * es * h;
    if (bytes % 4 != 0 || (reinterpret_cast<uintptr_t>(p.dst) & 3) != 0) return -1;
    uint32_t word = p.value;
    if (es == 1) word = (p.value & 0xffu) * 0x01010101u;
    if (es == 2) word = (p.value & 0xffffu) * 0x00010001u;
    size_t nd_in = 0, nd_out = 0;
    if (hipGraphNodeGetDependencies(nd, nullptr, &nd_in) != hipSuccess) return -1;
    if (hipGraphNodeGetDependentNodes(nd, nullptr, &nd_out) != hipSuccess) return -1;
    std::vector<hipGraphNode_t> deps(nd_in), outs(nd_out);
    if (nd_in && hipGraphNodeGetDependencies(nd, deps.data(), &nd_in) != hipSuccess) return -1;
    if (nd_out && hipGraphNodeGetDependentNodes(nd, outs.data(), &nd_out) != hipSuccess) return -1;
    uint32_t* dst = static_cast<uint32_t*>(p.dst);
    int64_t words = int64_t(bytes / 4);
    int vec = (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
    int64_t blocks = ((vec ? words / 4 : words) + 255) / 256;
    blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
    void* args[] = {&dst, &words, &word, &vec};
    hipKernelNodeParams kp = {};
    kp.func = reinterpret_cast<void*>(gd::fill_u32_kernel);
    kp.gridDim = dim3(unsigned(blocks));
    kp.blockDim = dim3(256);
    kp.sharedMemBytes = 0;
    kp.kernelParams = args;
    kp.extra = nullptr;
    hipGraphNode_t kn;
    if (hipGraphAddKernelNode(&kn, graph, deps.data(), deps.size(), &kp) != hipSuccess) return -1;
    for (hipGraphNode_t o : outs)
      if (hipGraphAddDependencies(graph, &kn, &o, 1) != hipSuccess) return -1;
    if (hipGraphDestroyNode(nd) != hipSuccess) return -1;
    ++replaced;
  }
  return replaced;
}
