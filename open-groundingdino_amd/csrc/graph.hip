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
// Every memset node is validated before any node is edited, so a graph with
// a memset this cannot express is left unchanged (-1).  Whole 4-byte words
// take the 16-byte-vector fill kernel; a byte count or destination that is
// not word-aligned (a bool / fp16 zero_) takes a byte-pattern fill kernel.
// -> the number of nodes replaced, or -1 (a memset this cannot express).
namespace {
__global__ void __launch_bounds__(256) fill_pattern_kernel(uint8_t* __restrict__ dst, int64_t n, uint32_t word) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256)
    dst[i] = uint8_t(word >> (8 * (i & 3)));
}

struct MemsetNode {
  hipGraphNode_t node;
  hipMemsetParams p;
  std::vector<hipGraphNode_t> deps, outs;
};
}  // namespace

extern "C" int gd_graph_memsets_to_kernels(void* graph_ptr) {
  hipGraph_t graph = static_cast<hipGraph_t>(graph_ptr);
  size_t n = 0;
  if (hipGraphGetNodes(graph, nullptr, &n) != hipSuccess) return -1;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(graph, nodes.data(), &n) != hipSuccess) return -1;
  // pass 1: collect and validate (no edits)
  std::vector<MemsetNode> ms;
  for (hipGraphNode_t nd : nodes) {
    hipGraphNodeType type;
    if (hipGraphNodeGetType(nd, &type) != hipSuccess) return -1;
    if (type != hipGraphNodeTypeMemset) continue;
    MemsetNode m;
    m.node = nd;
    if (hipGraphMemsetNodeGetParams(nd, &m.p) != hipSuccess) return -1;
    const size_t es = m.p.elementSize, h = m.p.height ? m.p.height : 1;
    if (!(es == 1 || es == 2 || es == 4) || (h > 1 && m.p.pitch != m.p.width * es)) return -1;
    if ((reinterpret_cast<uintptr_t>(m.p.dst) % es) != 0) return -1;
    size_t nd_in = 0, nd_out = 0;
    if (hipGraphNodeGetDependencies(nd, nullptr, &nd_in) != hipSuccess) return -1;
    if (hipGraphNodeGetDependentNodes(nd, nullptr, &nd_out) != hipSuccess) return -1;
    m.deps.resize(nd_in);
    m.outs.resize(nd_out);
    if (nd_in && hipGraphNodeGetDependencies(nd, m.deps.data(), &nd_in) != hipSuccess) return -1;
    if (nd_out && hipGraphNodeGetDependentNodes(nd, m.outs.data(), &nd_out) != hipSuccess) return -1;
    ms.push_back(std::move(m));
  }
  // pass 2: replace
  int replaced = 0;
  for (MemsetNode& m : ms) {
    const size_t es = m.p.elementSize, h = m.p.height ? m.p.height : 1;
    const size_t bytes = m.p.width * es * h;
    uint32_t word = m.p.value;
    if (es == 1) word = (m.p.value & 0xffu) * 0x01010101u;
    if (es == 2) word = (m.p.value & 0xffffu) * 0x00010001u;
    hipKernelNodeParams kp = {};
    kp.blockDim = dim3(256);
    kp.sharedMemBytes = 0;
    kp.extra = nullptr;
    uint32_t* dst32 = static_cast<uint32_t*>(m.p.dst);
    uint8_t* dst8 = static_cast<uint8_t*>(m.p.dst);
    int64_t words = int64_t(bytes / 4), nbytes = int64_t(bytes);
    int vec = (reinterpret_cast<uintptr_t>(dst32) & 15) == 0;
    void* args32[] = {&dst32, &words, &word, &vec};
    void* args8[] = {&dst8, &nbytes, &word};
    if (bytes % 4 == 0 && (reinterpret_cast<uintptr_t>(m.p.dst) & 3) == 0) {
      int64_t blocks = ((vec ? words / 4 : words) + 255) / 256;
      blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
      kp.func = reinterpret_cast<void*>(gd::fill_u32_kernel);
      kp.gridDim = dim3(unsigned(blocks));
      kp.kernelParams = args32;
    } else {
      int64_t blocks = (nbytes + 255) / 256;
      blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
      kp.func = reinterpret_cast<void*>(fill_pattern_kernel);
      kp.gridDim = dim3(unsigned(blocks));
      kp.kernelParams = args8;
    }
    hipGraphNode_t kn;
    if (hipGraphAddKernelNode(&kn, graph, m.deps.data(), m.deps.size(), &kp) != hipSuccess) return -1;
    for (hipGraphNode_t o : m.outs)
      if (hipGraphAddDependencies(graph, &kn, &o, 1) != hipSuccess) return -1;
    if (hipGraphDestroyNode(m.node) != hipSuccess) return -1;
    ++replaced;
  }
  return replaced;
}

// A capture that failed part-way (an operation the capture refused) leaves
// the stream capturing an invalidated graph; end it and drop the graph so
// the stream can run work again.  -> 1 when a capture was ended, 0 when the
// stream was not capturing, -1 on a HIP error.
extern "C" int gd_stream_abort_capture(void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  if (st == hipStreamCaptureStatusNone) return 0;
  hipGraph_t g = nullptr;
  (void)hipStreamEndCapture(s, &g);
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  return 1;
}
