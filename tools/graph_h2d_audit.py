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

    python tools/graph_h2d_audit.py [--device cuda] [--height H --width W]
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

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
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
    a = ap.parse_args()
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


if __name__ == "__main__":
    sys.exit(main())
