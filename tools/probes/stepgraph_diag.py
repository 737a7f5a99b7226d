"""Which part of the captured train step makes a replayed gradient differ
from the eager step's?  The step-graph test's model and batch (lr 0), eager
vs graph, with pieces of the captured body switched off:

    python tools/probes/stepgraph_diag.py [--clip 0|1] [--opt 0|1] [--full]

Prints the parameters whose replayed gradient differs (relative norm > 1e-3)
and, for each, the first values of both.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clip", type=int, default=1)
    ap.add_argument("--opt", type=int, default=1)
    ap.add_argument("--ckpt", type=int, default=0)
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--replays", type=int, default=1)
    ap.add_argument("--batch", type=int, default=2, help="1: 5 targets (the capture batch), 2: 3 targets")
    a = ap.parse_args()
    import test_stepgraph_gpu as T
    from gdino_amd.stepgraph import TrainStepGraph
    from gdino_amd.train import train_step
    T.CKPT[0] = bool(a.ckpt)
    b1 = T._batch(11, 5) if a.batch == 1 else T._batch(12, 3)
    b0 = T._batch(11, 5)  # the capture batch (the test captures on 5 targets, replays 3)
    res = {}
    for mode in ("eager", "eager_seq", "body", "graph"):
        model, crit, opt = T._model()
        for g in opt.param_groups:
            g["lr"], g["weight_decay"] = 0.0, 0.0
        if mode == "eager":
            if not a.opt:
                opt.step = lambda *x, **k: None
            train_step(model, crit, opt, *b1, clip_max_norm=0.1 if a.clip else 0.0)
        elif mode == "eager_seq":  # the test's order: the capture batch first, then this one
            train_step(model, crit, opt, *b0, clip_max_norm=0.1 if a.clip else 0.0)
            train_step(model, crit, opt, *b1, clip_max_norm=0.1 if a.clip else 0.0)
        elif mode == "body":  # the captured body run eagerly on the padded inputs
            g = TrainStepGraph(model, crit, opt, clip_max_norm=0.1 if a.clip else 0.0, warmup=2)
            if not a.opt:
                opt.step = lambda *x, **k: None
            opt.zero_grad(set_to_none=True)
            g._body(g._prepare(*b1), True)
        else:
            g = TrainStepGraph(model, crit, opt, clip_max_norm=0.1 if a.clip else 0.0, warmup=2)
            if not a.opt:
                opt.step = lambda *x, **k: None
            g(*b0)
            for _ in range(a.replays):
                g(*b1)
        torch.cuda.synchronize()
        res[mode] = T._grads(model)
    for other in ("eager_seq", "body", "graph"):
        bad = []
        for n, ge in res["eager"].items():
            gg = res[other][n]
            d = float((gg - ge).norm() / ge.norm().clamp_min(1e-30))
            if d > 0.05:
                bad.append((n, d, gg.reshape(-1)[:4].tolist(), ge.reshape(-1)[:4].tolist()))
        print(f"batch={a.batch} clip={a.clip} opt={a.opt} ckpt={a.ckpt} {other} vs eager: {len(bad)} of "
              f"{len(res['eager'])} gradients differ by > 5%", flush=True)
        for row in bad[:10]:
            print("  ", row, flush=True)




def test_flow(skip_eager=False, grads_between=True, fresh=False, between=None):
    """tests/test_stepgraph_gpu._run's exact order; -> {param: relative
    difference} for the second batch (graph vs the eager reference)."""
    import test_stepgraph_gpu as T
    from gdino_amd.stepgraph import TrainStepGraph
    from gdino_amd.train import train_step
    b1, b2 = T._batch(11, 5), T._batch(12, 3)
    out = {}
    modes = ("graph", "eager") if skip_eager else ("eager", "eager2", "graph")
    for mode in modes:
        model, crit, opt = T._model()
        for g in opt.param_groups:
            g["lr"], g["weight_decay"] = 0.0, 0.0
        grads = []
        if mode.startswith("eager"):
            for b in (b1, b2):
                train_step(model, crit, opt, *b)
                grads.append(T._grads(model))
        else:
            g = TrainStepGraph(model, crit, opt, warmup=2)
            for b in ((T._batch(11, 5), T._batch(12, 3)) if fresh else (b1, b2)):
                float(g(*b))
                if b is not b2 and between is not None:
                    keep = between(model)  # noqa: F841  (held across the next replay)
                    grads.append(None)
                elif grads_between or b is b2:
                    grads.append(T._grads(model))
            if not grads_between:
                grads.insert(0, None)
        torch.cuda.synchronize()
        out[mode] = grads
    res = {}
    for n, ge in out["eager"][1].items():
        gg = out["graph"][1][n]
        res[n] = float((gg - ge).norm() / ge.norm().clamp_min(1e-30))
    return res


def flows():
    def big(model):
        return torch.empty(int(700e6) // 4, device="cuda")

    def norms(model):
        return [float(p.grad.norm()) for p in model.parameters() if p.grad is not None]

    def clones_freed(model):
        T_grads = [p.grad.clone() for p in model.parameters() if p.grad is not None]
        del T_grads
        return None

    def clone_named(pred):
        def f(model):
            keep = [p.grad.clone() for n, p in model.named_parameters() if p.grad is not None and pred(n, p)]
            return keep
        f.__name__ = pred.__name__
        return f

    def only_dec0_lin1_bias(n, p):
        return n == "transformer.decoder.layers.0.linear1.bias"

    def only_biases(n, p):
        return n.endswith("bias")

    def no_biases(n, p):
        return not n.endswith("bias")

    def small(n, p):
        return p.numel() * 4 < (1 << 20)

    def dec_only(n, p):
        return ".decoder." in n

    import test_stepgraph_gpu as T
    from gdino_amd.stepgraph import TrainStepGraph
    orig_capture = TrainStepGraph._capture
    stash = []

    def capture_keep(self, key, inputs, *x):
        stash.append(inputs)  # the first call's prepared (non-static) inputs stay alive
        return orig_capture(self, key, inputs, *x)
    TrainStepGraph._capture = capture_keep
    try:
        res = test_flow(skip_eager=True, between=T._grads)
    finally:
        TrainStepGraph._capture = orig_capture
    bad = sorted(((d, n) for n, d in res.items() if d > 0.05), reverse=True)
    print(f"(reference) first call's inputs kept alive: {len(bad)} gradients differ by > 5%: {bad[:4]}", flush=True)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")

    def raw_hipmalloc(model):
        ptrs = []
        for _ in range(8):
            p = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(2 << 20)) == 0
            ptrs.append(p)
        for p in ptrs:
            hip.hipFree(p)
        return None

    def raw_hipmalloc_keep(model):
        ptrs = []
        for _ in range(8):
            p = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(2 << 20)) == 0
            ptrs.append(p)
        return ptrs

    def small_tensors(model):
        return [torch.empty(2048, device="cuda") for _ in range(200)]

    def prewarm(model):
        return None

    src = [torch.randn(2048, device="cuda") for _ in range(200)]
    dst = [torch.empty(2048, device="cuda") for _ in range(200)]

    def memcpy_d2d(model):  # contiguous same-dtype copy_: hipMemcpyAsync
        for a_, b_ in zip(dst, src):
            a_.copy_(b_)
        return None

    def kernel_copies(model):  # strided source: an elementwise copy kernel
        for a_, b_ in zip(dst, src):
            a_.view(2, 1024).copy_(b_.view(1024, 2).t())
        return None

    def one_memcpy(model):
        dst[0].copy_(src[0])
        return None

    for kw in ({"skip_eager": True, "between": memcpy_d2d},
               {"skip_eager": True, "between": kernel_copies},
               {"skip_eager": True, "between": one_memcpy}):
        res = test_flow(**kw)
        bad = sorted(((d, n) for n, d in res.items() if d > 0.05), reverse=True)
        kw = {k: getattr(v, "__name__", v) for k, v in kw.items()}
        print(f"flow {kw}: {len(bad)} gradients differ by > 5%: {bad[:4]}", flush=True)



def pools():
    """After the first replay: which memory pool holds each parameter's
    .grad (the graph's private pool or the regular one), and which grads
    were not None when the capture began."""
    import test_stepgraph_gpu as T
    from gdino_amd import stepgraph
    from gdino_amd.stepgraph import TrainStepGraph
    model, crit, opt = T._model()
    for g in opt.param_groups:
        g["lr"], g["weight_decay"] = 0.0, 0.0
    names = {id(p): n for n, p in model.named_parameters()}
    orig = torch.cuda.graph.__enter__
    seen = {}

    def enter(self):
        seen["not_none"] = [names.get(id(p), "?") for p in model.parameters() if p.grad is not None]
        return orig(self)
    torch.cuda.graph.__enter__ = enter
    try:
        g = TrainStepGraph(model, crit, opt, warmup=2)
        g(*T._batch(11, 5))
    finally:
        torch.cuda.graph.__enter__ = orig
    torch.cuda.synchronize()
    segs = torch.cuda.memory_snapshot()
    ranges = [(s["address"], s["address"] + s["total_size"], tuple(s.get("segment_pool_id", (0, 0)))) for s in segs]

    def pool_of(ptr):
        for lo, hi, pid in ranges:
            if lo <= ptr < hi:
                return pid
        return None
    by_pool = {}
    for n, p in model.named_parameters():
        if p.grad is None:
            by_pool.setdefault("none", []).append(n)
            continue
        by_pool.setdefault(str(pool_of(p.grad.data_ptr())), []).append(n)
    print("grads not None at capture begin:", seen.get("not_none", [])[:10], flush=True)
    for k, v in by_pool.items():
        print(f"pool {k}: {len(v)} grads, e.g. {v[:3]}", flush=True)
    for n in ("transformer.decoder.layers.0.linear1.bias", "transformer.decoder.layers.0.linear1.weight"):
        p = dict(model.named_parameters())[n]
        print(n, "grad pool", pool_of(p.grad.data_ptr()), "is view", p.grad._base is not None,
              "dtype", p.grad.dtype, "stride", p.grad.stride(), flush=True)


def history():
    """Allocations made while the step graph was being captured that did NOT
    come from the graph's private pool (a capture allocates from the private
    pool only on the capturing stream): their blocks return to the regular
    pool when freed, and a later eager allocation can take memory the
    replays still read or write."""
    import collections
    import test_stepgraph_gpu as T
    from gdino_amd.stepgraph import TrainStepGraph
    model, crit, opt = T._model()
    for g in opt.param_groups:
        g["lr"], g["weight_decay"] = 0.0, 0.0
    torch.cuda.memory._record_memory_history(max_entries=400000)
    marks = {}
    orig_enter, orig_exit = torch.cuda.graph.__enter__, torch.cuda.graph.__exit__

    def count():
        return len(torch.cuda.memory._snapshot()["device_traces"][0])

    def enter(self):
        r = orig_enter(self)
        marks["begin"] = count()
        marks["stream"] = torch.cuda.current_stream().cuda_stream
        return r

    def exit_(self, *x):
        marks["end"] = count()
        return orig_exit(self, *x)
    torch.cuda.graph.__enter__, torch.cuda.graph.__exit__ = enter, exit_
    try:
        g = TrainStepGraph(model, crit, opt, warmup=2)
        g(*T._batch(11, 5))
    finally:
        torch.cuda.graph.__enter__, torch.cuda.graph.__exit__ = orig_enter, orig_exit
    import gc
    gc.collect()
    torch.cuda.synchronize()
    snap = torch.cuda.memory._snapshot()
    torch.cuda.memory._record_memory_history(enabled=None)
    allt = snap["device_traces"][0]
    # blocks allocated before the capture began and freed after it ended
    # (what a replay may still use while an eager allocation takes it)
    born = {}
    for e in allt[:marks["begin"]]:
        if e["action"] == "alloc":
            born[e["addr"]] = e
        elif e["action"] == "free_completed":
            born.pop(e["addr"], None)
    late = [e for e in allt[marks["end"]:] if e["action"] == "free_requested" and e["addr"] in born]
    print(f"{len(late)} blocks allocated before the capture and freed after it", flush=True)
    for e in late[:40]:
        a = born[e["addr"]]
        frames = [f"{f['filename'].split('/')[-1]}:{f['line']} {f['name']}" for f in a.get("frames", [])
                  if f["filename"].endswith(".py") and "site-packages" not in f["filename"]][:6]
        print("  size", a["size"], frames, flush=True)
    tr = allt[marks["begin"]:marks["end"]]
    streams = collections.Counter((e["action"], e.get("stream")) for e in tr)
    print("capture stream", marks["stream"], "trace events by (action, stream):", dict(streams), flush=True)
    odd = [e for e in tr if e["action"] == "alloc" and e.get("stream") != marks["stream"]]
    print(f"{len(odd)} allocations during capture on another stream", flush=True)
    for e in odd[:12]:
        frames = [f"{f['filename'].split('/')[-1]}:{f['line']} {f['name']}" for f in e.get("frames", [])
                  if "site-packages/torch" not in f["filename"] or "autograd" in f["filename"]][:6]
        print("  size", e["size"], "stream", e.get("stream"), frames, flush=True)



if __name__ == "__main__":
    if "--flows" in sys.argv:
        flows()
    elif "--pools" in sys.argv:
        pools()
    elif "--history" in sys.argv:
        history()
    else:
        main()
