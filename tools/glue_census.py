"""Census of the elementwise / copy / reduction ATen ops one eager train step
dispatches on large tensors: op, dtypes, shapes and the site that issued it
(the innermost package frame for forward ops, the running autograd node for
backward ops) -- the list of glue worth fusing away.

    python tools/glue_census.py [--min-numel 1000000] [--out gpurun_out/glue.txt]

Counts only (no timing): the kernel times per op family come from the
rocprofv3 kernel trace (tools/trace_steps.py); this names where they come from.
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

SKIP = ("mm", "addmm", "bmm", "_addmm_activation", "baddbmm", "view", "_unsafe_view", "t", "transpose",
        "permute", "expand", "select", "slice", "as_strided", "detach", "alias", "unsqueeze", "squeeze",
        "reshape", "split", "split_with_sizes", "unbind", "empty", "empty_like", "empty_strided", "new_empty",
        "new_empty_strided", "_to_copy_noop", "lift_fresh", "_reshape_alias", "set_", "record_stream")


GEMMS = ("mm", "addmm", "bmm", "_addmm_activation", "baddbmm")


def _site():
    node = torch._C._current_autograd_node()
    if node is not None:
        return "bwd " + node.name()
    for fr in reversed(traceback.extract_stack(limit=40)):
        if "open-groundingdino_amd" in fr.filename and "_python_dispatch" not in fr.filename:
            return "%s:%d %s" % (fr.filename.split("open-groundingdino_amd/")[-1], fr.lineno, fr.name)
    return "?"


class Census(TorchDispatchMode):
    def __init__(self, min_numel, gemms=False):
        super().__init__()
        self.min_numel = min_numel
        self.gemms = gemms
        self.count = collections.Counter()
        self.bytes = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.overloadpacket.__name__
        if name in SKIP and not (self.gemms and name in GEMMS):
            return out
        ts = [a for a in args if isinstance(a, torch.Tensor)]
        outs = out if isinstance(out, (tuple, list)) else (out,)
        outs = [o for o in outs if isinstance(o, torch.Tensor)]
        big = max([t.numel() for t in ts + outs] or [0])
        if big < self.min_numel or not any(t.is_cuda for t in ts + outs):
            return out
        desc = ",".join("%s%s" % (str(t.dtype).replace("torch.", ""), list(t.shape)) for t in ts[:3])
        odesc = ",".join(str(o.dtype).replace("torch.", "") for o in outs[:2])
        key = (name, desc + "->" + odesc, _site())
        self.count[key] += 1
        self.bytes[key] += sum(t.numel() * t.element_size() for t in ts + outs)
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-numel", type=int, default=1_000_000)
    ap.add_argument("--out", default="gpurun_out/glue.txt")
    ap.add_argument("--checkpointing", choices=("on", "off"), default="off")
    ap.add_argument("--gemms", action="store_true", help="also count the library GEMM ops")
    ap.add_argument("--by-count", type=int, default=0, help="also list the N most frequent op sites")
    a = ap.parse_args()
    from gdino_amd.config import make_args
    from gdino_amd.train import build_training, set_activation_checkpointing, synthetic_batch, train_step
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model, crit, _, opt = build_training(make_args(device="cuda"), dev)
    model.train()
    set_activation_checkpointing(model, a.checkpointing == "on")
    b = synthetic_batch(2, 800, 1333, n_boxes=8, n_tokens=256, seed=1000, device=dev)
    for _ in range(2):
        train_step(model, crit, opt, *b)
    torch.cuda.synchronize()
    c = Census(a.min_numel, a.gemms)
    with c:
        train_step(model, crit, opt, *b)
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    tot = sum(c.bytes.values())
    with open(a.out, "w") as f:
        f.write("glue ops on tensors >= %d elements: %d ops, %.2f GB operand bytes\n"
                % (a.min_numel, sum(c.count.values()), tot / 1e9))
        for k, v in c.bytes.most_common():
            f.write("%7.1f MB n=%3d  %-22s %-60s %s\n" % (v / 1e6, c.count[k], k[0], k[2][:60], k[1][:140]))
        if a.by_count:
            by_site = collections.Counter()
            for k, n in c.count.items():
                by_site[(k[0], k[2])] += n
            f.write("\n--- the %d most frequent (op, site) pairs, all shapes\n" % a.by_count)
            for (op, site), n in by_site.most_common(a.by_count):
                f.write("n=%4d  %-26s %s\n" % (n, op, site[:90]))
    print(open(a.out).read()[:6000])


if __name__ == "__main__":
    main()
