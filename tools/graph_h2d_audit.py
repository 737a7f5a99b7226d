"""Audit of the region bench.py --graphs captures (GroundingDINO.forward_core
and its backward): every op that builds a tensor from host data
(aten.lift_fresh*, i.e. torch.tensor / as_tensor of Python values), reads a
device value back (aten._local_scalar_dense: .item(), bool(t), int(t)) or
moves a tensor across devices (_to_copy / copy_ with a device change).

Inside a HIP-graph capture the first kind becomes a memcpy node whose host
source (a temporary staging buffer) does not outlive the capture -- a replay
then reads memory that is no longer mapped -- and the second kind is illegal.
On the CPU (default) the HIP-only ops are routed to their oracles, as the
CPU tests do: device changes cannot show there, host-data creation and
scalar reads can.  With --device cuda the HIP path itself runs under bf16
autocast, as bench.py's train step does.

    python tools/graph_h2d_audit.py [--device cuda] [--height H --width W] [--whole-step]

--whole-step audits the region gdino_amd.stepgraph captures instead: the
forward, SetCriterion.loss_prepared (device matching; on the CPU the solver
is scipy's, outside the audit), the weighted loss, the backward and the
gradient clipping (the captured fused AdamW is PyTorch's own capturable
kernel and is not run here).
"""
import argparse
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

FLAG = {"lift_fresh", "lift_fresh_copy", "_local_scalar_dense"}


def _site():
    for fr in reversed(traceback.extract_stack()[:-3]):
        if "open-groundingdino_amd" in fr.filename:
            return f"{os.path.relpath(fr.filename, ROOT)}:{fr.lineno} {fr.line}"
    return "?"


class Audit(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.hits = {}
        self.paused = False

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if self.paused:
            return func(*args, **kwargs)
        name = func._schema.name.split("::")[-1]
        hit = name in FLAG
        if name in ("_to_copy", "copy_"):
            src = args[1] if name == "copy_" else args[0]
            dst_dev = args[0].device if name == "copy_" else kwargs.get("device", src.device)
            hit = isinstance(src, torch.Tensor) and torch.device(dst_dev) != src.device
        if hit:
            key = (name, _site())
            self.hits[key] = self.hits.get(key, 0) + 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--whole-step", action="store_true")
    a = ap.parse_args()
    if a.whole_step:
        return whole_step(a)
    dev = torch.device(a.device)
    if dev.type == "cpu":
        from oracle_hooks import oracle_msda
        route = oracle_msda
    else:
        def route():
            return torch.autocast(device_type="cuda", dtype=torch.bfloat16)

    from gdino_amd.config import make_args
    from gdino_amd.train import build_training, synthetic_batch

    torch.manual_seed(0)
    args = make_args(device=str(dev))
    model, criterion, _, _ = build_training(args, dev)
    model.train()
    samples, targets, captions, cats = synthetic_batch(2, a.height, a.width, n_boxes=4, n_tokens=64, seed=0,
                                                       device=dev)
    with route():
        text, _ = model.prepare_text(captions, dev)
        inputs = (samples.tensors, samples.mask, text["input_ids"], text["token_type_ids"], text["text_token_mask"],
                  text["self_masks"], text["position_ids"])
        model.forward_core(*inputs)  # warm-up: device constants are built here, as in the capture's warm-up
        audit = Audit()
        with audit:
            outs = model.forward_core(*inputs)
            loss = sum(o.float().sum() for o in outs if isinstance(o, torch.Tensor) and o.requires_grad)
            loss.backward()
    if not audit.hits:
        print("graph_h2d_audit: forward_core + backward: no host-data tensors, scalar reads or device moves")
        return 0
    for (name, site), n in sorted(audit.hits.items(), key=lambda kv: kv[0][1]):
        print(f"{n:4d} x {name:22s} {site}")
    return 1


def whole_step(a):
    """The step graph's body (stepgraph.TrainStepGraph._body without the
    optimizer step) under the audit, on the CPU with the HIP-only ops routed
    to their oracles and the device LSA replaced by scipy (not audited)."""
    import numpy as np
    from scipy.optimize import linear_sum_assignment
    from oracle_hooks import oracle_msda
    from gdino_amd import lsap
    from gdino_amd.config import make_args
    from gdino_amd.stepgraph import TrainStepGraph
    from gdino_amd.train import build_training, synthetic_batch

    dev = torch.device(a.device)
    torch.manual_seed(0)
    model, criterion, _, _ = build_training(make_args(device=str(dev)), dev)
    model.train()
    audit = Audit()

    def host_lsa(cost, sizes, status=None):
        audit.paused = True
        try:
            p, q, k = cost.shape
            rows = torch.full((p, k), -1, dtype=torch.int64)
            cols = torch.full((p, k), -1, dtype=torch.int64)
            c = cost.detach().double().numpy()
            for i, n in enumerate(sizes.tolist()):
                r, cc = linear_sum_assignment(np.asarray(c[i, :, :n]))
                rows[i, :len(r)], cols[i, :len(r)] = torch.from_numpy(r), torch.from_numpy(cc)
            return rows.to(cost.device), cols.to(cost.device)
        finally:
            audit.paused = False

    class NoStep:
        def step(self):
            pass

        def zero_grad(self, set_to_none=True):
            model.zero_grad(set_to_none=set_to_none)

    on_gpu = dev.type == "cuda"
    # on the GPU the product path itself (bf16 autocast, the device LSA)
    g = TrainStepGraph(model, criterion, NoStep(), clip_max_norm=0.1, amp_dtype=torch.bfloat16 if on_gpu else None)
    samples, targets, captions, cats = synthetic_batch(2, a.height, a.width, n_boxes=4, n_tokens=64, seed=0,
                                                       device=dev)
    saved = lsap.linear_sum_assignment_batched
    if not on_gpu:
        lsap.linear_sum_assignment_batched = host_lsa
    import contextlib
    try:
        with (contextlib.nullcontext() if on_gpu else oracle_msda()):
            inputs, pf = g._prepare(samples, targets, captions, cats)
            g._body(inputs, pf)  # warm-up: device constants, caches
            with audit:
                g._body(inputs, pf)
    finally:
        lsap.linear_sum_assignment_batched = saved
    if not audit.hits:
        print("graph_h2d_audit: whole step body: no host-data tensors, scalar reads or device moves")
        return 0
    for (name, site), n in sorted(audit.hits.items(), key=lambda kv: kv[0][1]):
        print(f"{n:4d} x {name:22s} {site}")
    return 1


if __name__ == "__main__":
    sys.exit(main())
