"""Which ops of the captured train step become memcpy nodes?  PyTorch copies a
contiguous tensor into a contiguous one of the same dtype on the same device
with hipMemcpyAsync (a memcpy node when captured); every other copy is a
kernel.  On ROCm 7.0 eager hipMemcpyAsync calls issued between graph replays
corrupt the next replay when the graph holds memcpy nodes
(tools/probes/stepgraph_diag.py --flows: 200 eager D2D copies between two replays
change two decoder bias gradients; kernel copies do not), so the step graph
must hold none.  Logs every such copy of one eager step body, with its size
and the site (innermost package frame, or the autograd node).

    python tools/probes/memcpy_census.py [--full]
"""
import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402


def _site():
    node = torch._C._current_autograd_node()
    if node is not None:
        return "bwd " + node.name()
    for fr in reversed(traceback.extract_stack(limit=60)):
        if "open-groundingdino_amd" in fr.filename or "/tools/" in fr.filename:
            return "%s:%d %s" % (fr.filename.split("/")[-1], fr.lineno, fr.name)
    return "?"


def _memcpy_like(dst, src):
    return (isinstance(dst, torch.Tensor) and isinstance(src, torch.Tensor) and dst.is_cuda and src.is_cuda
            and dst.dtype == src.dtype and dst.is_contiguous() and src.is_contiguous()
            and dst.numel() == src.numel() and dst.numel() > 0)


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.hits = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        name = func.overloadpacket.__name__
        hit = None
        if name == "copy_" and _memcpy_like(args[0], args[1]):
            hit = args[0]
        elif name in ("clone", "_to_copy") and isinstance(out, torch.Tensor) and _memcpy_like(out, args[0]):
            hit = out
        if hit is not None:
            self.hits[(name, hit.numel() * hit.element_size(), _site())] += 1
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true")
    a = ap.parse_args()
    import test_stepgraph_gpu as T
    from gdino_amd.stepgraph import TrainStepGraph
    from gdino_amd.train import synthetic_batch
    T.CKPT[0] = False
    model, crit, opt = T._model()
    b = (synthetic_batch(2, 800, 1333, n_boxes=8, n_tokens=256, seed=1000, device="cuda") if a.full
         else T._batch(11, 5))
    g = TrainStepGraph(model, crit, opt, warmup=2)
    inputs = g._prepare(*b)
    opt.zero_grad(set_to_none=True)
    g._body(inputs, True)
    opt.zero_grad(set_to_none=True)
    c = Census()
    with c:
        g._body(inputs, True)
    torch.cuda.synchronize()
    print(f"{sum(c.hits.values())} memcpy-shaped copies in one step body", flush=True)
    for (name, nbytes, site), n in sorted(c.hits.items(), key=lambda kv: kv[0][2]):
        print(f"{n:4d} x {name:9s} {nbytes:10d} B  {site}", flush=True)


if __name__ == "__main__":
    main()
