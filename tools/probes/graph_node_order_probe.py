"""Are memset / memcpy nodes of a captured HIP graph ordered against the
kernel nodes around them on replay?  (The whole-step graph faulted on replay
while eager runs of the same work were clean; the HIP library's buffers that
need zeros were hipMemsetAsync'd inside the capture.)

Per replay, on one capturing stream:
  memset probe:  fill kernel Z := 7  ->  hipMemsetAsync(Z, 0)  ->  kernel Z += 1
                 ->  bad += count(Z != 1)
  memcpy probe:  kernel A := step    ->  hipMemcpyAsync(B <- A) ->  kernel
                 bad += count(B != step); step += 1
A long GEMM precedes each probe so that the node before the memset / memcpy
is still running when the next node could start.  No index is derived from
the probed data: a reordering shows as a nonzero count, never as a fault.

    python tools/probes/graph_node_order_probe.py [--replays 300] [--mb 64]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replays", type=int, default=300)
    ap.add_argument("--mb", type=float, default=64.0)
    a = ap.parse_args()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda")
    n = int(a.mb * 2 ** 20 / 4)
    z = torch.empty(n, dtype=torch.float32, device=dev)
    A = torch.empty(n, dtype=torch.float32, device=dev)
    B = torch.empty(n, dtype=torch.float32, device=dev)
    x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    y = torch.empty(4096, 4096, device=dev, dtype=torch.bfloat16)
    step = torch.zeros((), dtype=torch.float32, device=dev)
    bad_set = torch.zeros((), dtype=torch.int64, device=dev)
    bad_cpy = torch.zeros((), dtype=torch.int64, device=dev)

    def body():
        s = torch.cuda.current_stream().cuda_stream
        torch.mm(x, x, out=y)                      # a long kernel first
        z.fill_(7.0)
        assert hip.hipMemsetAsync(z.data_ptr(), 0, z.numel() * 4, s) == 0
        z.add_(1.0)
        bad_set.add_((z != 1.0).sum())
        torch.mm(x, x, out=y)
        A.copy_(step.expand_as(A))                 # a kernel (expand: not a memcpy)
        assert hip.hipMemcpyAsync(B.data_ptr(), A.data_ptr(), A.numel() * 4, 3, s) == 0  # D2D
        bad_cpy.add_((B != step).sum())
        step.add_(1.0)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        body()  # eager once
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    eager = (int(bad_set), int(bad_cpy))
    bad_set.zero_()
    bad_cpy.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        body()
    torch.cuda.synchronize()
    for i in range(a.replays):
        g.replay()
        if i % 50 == 49:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    back = (int(bad_set), int(bad_cpy))
    bad_set.zero_()
    bad_cpy.zero_()
    for i in range(a.replays):
        g.replay()
        torch.cuda.synchronize()
    synced = (int(bad_set), int(bad_cpy))
    # eager D2D memcpys between the replays (what corrupted the step graph)
    bad_set.zero_()
    bad_cpy.zero_()
    srcs = [torch.randn(4096, device=dev) for _ in range(64)]
    dsts = [torch.empty(4096, device=dev) for _ in range(64)]
    for i in range(a.replays // 10):
        g.replay()
        torch.cuda.synchronize()
        for _ in range(5):
            for d_, s_ in zip(dsts, srcs):
                d_.copy_(s_)
        torch.cuda.synchronize()
    interleaved = (int(bad_set), int(bad_cpy))
    # the same with the graph's memset nodes rewritten as fill kernels
    from gdino_amd.stepgraph import memsets_to_kernels
    g2 = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g2, stream=side):
        body()
    replaced = memsets_to_kernels(g2)
    g2.instantiate()
    bad_set.zero_()
    bad_cpy.zero_()
    for i in range(a.replays // 10):
        g2.replay()
        torch.cuda.synchronize()
        for _ in range(5):
            for d_, s_ in zip(dsts, srcs):
                d_.copy_(s_)
        torch.cuda.synchronize()
    rewritten = (int(bad_set), int(bad_cpy), replaced)
    print(json.dumps({"eager_bad": eager, "replays": a.replays, "back_to_back_bad(memset, memcpy)": back,
                      "synced_bad(memset, memcpy)": synced,
                      "eager_memcpys_between_bad(memset, memcpy)": interleaved,
                      "memsets_as_kernels_bad(memset, memcpy, replaced)": rewritten}), flush=True)
    small_memcpy_probe(a.replays // 10)
    sort_probe(a.replays // 10)
    reduce_probe(a.replays // 10)


def small_memcpy_probe(replays):
    """Small memcpy nodes (the step graph's are 4 B .. 5 MB) with eager
    small D2D copies issued between the replays."""
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda")
    res = {}
    for nbytes in (4, 1024, 8192, 614400):
        n = nbytes // 4
        A = torch.empty(n, device=dev)
        B = torch.empty(n, device=dev)
        step = torch.zeros((), device=dev)
        bad = torch.zeros((), dtype=torch.int64, device=dev)

        def body():
            s = torch.cuda.current_stream().cuda_stream
            A.copy_(step.expand_as(A))
            assert hip.hipMemcpyAsync(B.data_ptr(), A.data_ptr(), nbytes, 3, s) == 0
            bad.add_((B != step).sum())
            step.add_(1.0)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            body()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        bad.zero_()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            body()
        srcs = [torch.randn(2048, device=dev) for _ in range(64)]
        dsts = [torch.empty(2048, device=dev) for _ in range(64)]
        for i in range(replays):
            g.replay()
            torch.cuda.synchronize()
            for _ in range(5):
                for d_, s_ in zip(dsts, srcs):
                    d_.copy_(s_)
            torch.cuda.synchronize()
        res[nbytes] = int(bad)
    print(json.dumps({"small_memcpy_nodes_bad_with_eager_copies_between": res, "replays": replays}), flush=True)


def sort_probe(replays):
    """misc.topk_indices' capture path (a stable descending sort + slice) as
    a graph: on new scores each replay must return what eager topk returns
    (indices in range, same set).  The indices are only compared, never
    used to address memory."""
    from gdino_amd.misc import topk_indices
    dev = torch.device("cuda")
    res = {}
    for n, k in ((2550, 300), (22223, 900)):
        x = torch.randn(2, n, device=dev)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            topk_indices(x, k)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            idx = topk_indices(x, k)
        bad_range = bad_set = 0
        for i in range(replays):
            x.copy_(torch.randn(2, n, device=dev))
            g.replay()
            torch.cuda.synchronize()
            got = idx.clone()
            bad_range += int(((got < 0) | (got >= n)).sum())
            ref = torch.topk(x, k, dim=1)[1]
            bad_set += int((got.sort(1)[0] != ref.sort(1)[0]).sum())
        res[f"{n}/{k}"] = {"out_of_range": bad_range, "set_mismatch": bad_set}
    print(json.dumps({"sort_probe": res, "replays": replays}), flush=True)


def reduce_probe(replays):
    """PyTorch column sums (the bias gradient of a plain Linear: grad.sum(0))
    inside a graph against eager: the multi-block reductions zero their
    semaphores with a 4-byte hipMemsetAsync, a memset node in the graph."""
    dev = torch.device("cuda")
    res = {}
    for shape in ((600, 2048), (1800, 2048), (600, 256), (44446, 256), (2, 22223, 256)):
        x = torch.randn(*shape, device=dev)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            x.sum(0)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            y = x.sum(0)
        worst = 0.0
        for i in range(replays):
            x.copy_(torch.randn(*shape, device=dev))
            g.replay()
            torch.cuda.synchronize()
            ref = x.sum(0)
            worst = max(worst, float((y - ref).abs().max() / ref.abs().max()))
        res[str(shape)] = worst
    print(json.dumps({"reduce_probe_max_rel_err": res, "replays": replays}), flush=True)


if __name__ == "__main__":
    main()
