"""Capture the whole-step graph (gdino_amd.stepgraph) WITHOUT replaying it
and dump its node list (hipGraphDebugDotPrint through CUDAGraph.debug_dump):
node types (kernel / memcpy / memset / host / event), copy directions and
sizes -- the nodes a replay executes that the eager warm-ups did not show.

    python tools/probes/graph_dump.py [--full] [--out gpurun_out/graph.dot]
"""
import argparse
import collections
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true", help="the bench's shapes (default: the step-graph test's)")
    ap.add_argument("--ckpt", type=int, default=1)
    ap.add_argument("--out", default="gpurun_out/graph_nodes.txt")
    a = ap.parse_args()
    from gdino_amd.config import make_args
    from gdino_amd.stepgraph import TrainStepGraph
    from gdino_amd.train import build_training, set_activation_checkpointing, synthetic_batch
    dev = torch.device("cuda")
    torch.manual_seed(0)
    args = make_args(device="cuda") if a.full else make_args(device="cuda", enc_layers=2, dec_layers=2,
                                                               num_queries=300)
    model, crit, _, opt = build_training(args, dev)
    set_activation_checkpointing(model, bool(a.ckpt))
    model.train()
    b = (synthetic_batch(2, 800, 1333, n_boxes=8, n_tokens=256, seed=1000, device=dev) if a.full else
         synthetic_batch(2, 320, 384, n_boxes=5, n_tokens=40, seed=11, device=dev))
    g = TrainStepGraph(model, crit, opt, warmup=2)
    inputs = g._prepare(*b)
    key = g._signature(inputs) + (("padding_free", True),)
    # capture exactly as TrainStepGraph._capture, keeping the hipGraph_t
    orig_graph = torch.cuda.CUDAGraph
    import gdino_amd.stepgraph as sg
    sg.torch.cuda.CUDAGraph = lambda: orig_graph(keep_graph=True)
    try:
        c = g._capture(key, inputs, True)
    finally:
        sg.torch.cuda.CUDAGraph = orig_graph
    torch.cuda.synchronize()
    analyse(c.graph.raw_cuda_graph(), a.out)
    hip = ctypes.CDLL("libamdhip64.so")
    dot = os.path.abspath(a.out + ".dot").encode()
    r = hip.hipGraphDebugDotPrint(ctypes.c_void_p(c.graph.raw_cuda_graph()), ctypes.c_char_p(dot),
                                  ctypes.c_uint(0xFFFF))  # every verbose flag
    print(f"hipGraphDebugDotPrint -> {r}: {dot.decode()}", flush=True)
    if r == 0 and os.path.exists(dot):
        for line in open(dot, errors="replace"):
            low = line.lower()
            if ("memcpy" in low or "memset" in low) and "label" in low:
                print("DOT", line.strip()[:400])


_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "child_graph", 5: "empty", 6: "wait_event",
          7: "event_record", 8: "ext_sem_signal", 9: "ext_sem_wait", 10: "mem_alloc", 11: "mem_free",
          12: "memcpy_from_symbol", 13: "memcpy_to_symbol"}


class _Dim3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint), ("y", ctypes.c_uint), ("z", ctypes.c_uint)]


class _KParams(ctypes.Structure):  # hipKernelNodeParams
    _fields_ = [("blockDim", _Dim3), ("extra", ctypes.c_void_p), ("func", ctypes.c_void_p), ("gridDim", _Dim3),
                ("kernelParams", ctypes.c_void_p), ("sharedMemBytes", ctypes.c_uint)]


class _Pos(ctypes.Structure):
    _fields_ = [("x", ctypes.c_size_t), ("y", ctypes.c_size_t), ("z", ctypes.c_size_t)]


class _PPtr(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("pitch", ctypes.c_size_t), ("xsize", ctypes.c_size_t),
                ("ysize", ctypes.c_size_t)]


class _Ext(ctypes.Structure):
    _fields_ = [("width", ctypes.c_size_t), ("height", ctypes.c_size_t), ("depth", ctypes.c_size_t)]


class _M3D(ctypes.Structure):  # hipMemcpy3DParms
    _fields_ = [("srcArray", ctypes.c_void_p), ("srcPos", _Pos), ("srcPtr", _PPtr), ("dstArray", ctypes.c_void_p),
                ("dstPos", _Pos), ("dstPtr", _PPtr), ("extent", _Ext), ("kind", ctypes.c_int)]


class _MSet(ctypes.Structure):  # hipMemsetParams
    _fields_ = [("dst", ctypes.c_void_p), ("pitch", ctypes.c_size_t), ("value", ctypes.c_uint),
                ("elementSize", ctypes.c_uint), ("width", ctypes.c_size_t), ("height", ctypes.c_size_t)]


class _PAttr(ctypes.Structure):  # hipPointerAttribute_t (leading fields)
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def _ptr_kind(hip, p):
    a = _PAttr()
    r = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
    if r != 0:
        hip.hipGetLastError()
        return "unregistered-host"
    return {0: "unregistered", 1: "host", 2: "device", 3: "managed"}.get(a.type, str(a.type))


def _memcpy_desc(hip, nd):
    m = _M3D()
    if hip.hipGraphMemcpyNodeGetParams(ctypes.c_void_p(nd), ctypes.byref(m)) != 0:
        hip.hipGetLastError()
        return "(params?)"
    kind = {0: "HtoH", 1: "HtoD", 2: "DtoH", 3: "DtoD", 4: "default"}.get(m.kind, str(m.kind))
    nbytes = m.extent.width * max(m.extent.height, 1) * max(m.extent.depth, 1)
    return (f"{kind} {nbytes} B src={_ptr_kind(hip, m.srcPtr.ptr or 0)} dst={_ptr_kind(hip, m.dstPtr.ptr or 0)}")


def _memset_desc(hip, nd):
    m = _MSet()
    if hip.hipGraphMemsetNodeGetParams(ctypes.c_void_p(nd), ctypes.byref(m)) != 0:
        hip.hipGetLastError()
        return "(params?)"
    return f"{m.width * max(m.height, 1) * m.elementSize} B value={m.value} dst={_ptr_kind(hip, m.dst or 0)}"


def analyse(graph, out):
    """Node types, kernel names, and the graph's shape: a single stream's
    capture is a chain; a node with several predecessors / successors is a
    fork / join -- work a replay may run concurrently."""
    hip = ctypes.CDLL("libamdhip64.so")
    gp = ctypes.c_void_p(graph)
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(gp, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(gp, nodes, ctypes.byref(n)) == 0
    ne = ctypes.c_size_t(0)
    assert hip.hipGraphGetEdges(gp, None, None, ctypes.byref(ne)) == 0
    fr = (ctypes.c_void_p * max(ne.value, 1))()
    to = (ctypes.c_void_p * max(ne.value, 1))()
    assert hip.hipGraphGetEdges(gp, fr, to, ctypes.byref(ne)) == 0
    hip.hipKernelNameRefByPtr.restype = ctypes.c_char_p
    hip.hipKernelNameRefByPtr.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    kinds, names, info = collections.Counter(), collections.Counter(), {}
    for nd in nodes:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
        kind = _TYPES.get(t.value, str(t.value))
        kinds[kind] += 1
        label = kind
        if t.value == 0:
            kp = _KParams()
            if hip.hipGraphKernelNodeGetParams(ctypes.c_void_p(nd), ctypes.byref(kp)) == 0 and kp.func:
                nm = hip.hipKernelNameRefByPtr(ctypes.c_void_p(kp.func), None)
                label = (nm.decode(errors="replace") if nm else "?")[:110]
        if t.value == 1:
            label = "memcpy " + _memcpy_desc(hip, nd)
        elif t.value == 2:
            label = "memset " + _memset_desc(hip, nd)
        info[nd] = label
        if t.value != 0:
            names[label] += 1
    indeg, outdeg = collections.Counter(), collections.Counter()
    succ = collections.defaultdict(list)
    for i in range(ne.value):
        outdeg[fr[i]] += 1
        indeg[to[i]] += 1
        succ[fr[i]].append(to[i])
    forks = [nd for nd in nodes if outdeg[nd] > 1]
    joins = [nd for nd in nodes if indeg[nd] > 1]
    roots = [nd for nd in nodes if indeg[nd] == 0]
    lines = [f"nodes {n.value} edges {ne.value} roots {len(roots)} forks {len(forks)} joins {len(joins)}",
             "by kind: " + json.dumps(dict(kinds))]
    for k, v in names.most_common():
        lines.append(f"  non-kernel node {k}: {v}")
    for nd in forks[:40]:
        lines.append("FORK " + info[nd] + " -> " + " | ".join(info[x] for x in succ[nd]))
    for nd in joins[:40]:
        lines.append(f"JOIN (in {indeg[nd]}) " + info[nd])
    for nd in roots[:10]:
        lines.append("ROOT " + info[nd])
    txt = "\n".join(lines)
    print(txt, flush=True)
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        f.write(txt + "\n")
        order = list(nodes)
        for nd in order:
            f.write(f"{info[nd]}  in={indeg[nd]} out={outdeg[nd]}\n")


if __name__ == "__main__":
    main()
