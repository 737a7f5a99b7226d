"""Count ATen dispatches (≈ device kernel launches) of one training step on
CPU, by op, with the HIP-only ops routed to the oracle (their own internals are
excluded from the count, each counts as one launch as on the GPU).

The count does not depend on the image size, so a small image gives the same
per-step launch profile as 800x1333.  CPU autocast (bf16) approximates CUDA
autocast's cast insertion.  Usage:
    python tools/probes/count_ops.py [--top 40] [--no-autocast]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

# ops that launch no device kernel (metadata / views / host-side)
_FREE = {"aten.view", "aten._unsafe_view", "aten.reshape", "aten.expand", "aten.permute", "aten.transpose",
         "aten.t", "aten.squeeze", "aten.unsqueeze", "aten.select", "aten.slice", "aten.as_strided",
         "aten.alias", "aten.detach", "aten.split", "aten.split_with_sizes", "aten.unbind", "aten.chunk",
         "aten.narrow", "aten.flatten", "aten.unflatten", "aten.empty", "aten.empty_like", "aten.empty_strided",
         "aten.lift_fresh", "aten._to_copy.no", "aten.size", "aten.stride", "aten.is_same_size",
         "aten.sym_size", "aten.numel", "aten.dim", "aten._reshape_alias", "aten.new_empty",
         "aten.new_empty_strided", "aten.view_as", "aten.movedim", "aten.diagonal", "aten.unfold",
         "aten.set_", "aten.resize_", "aten.item", "aten._local_scalar_dense", "aten.is_nonzero",
         "aten.equal", "aten.result_type"}


_OP_FILTER = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--op=")]


class Counter(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.counts = collections.Counter()
        self.paused = 0
        self.phase = "fwd"
        self.by_phase = collections.Counter()
        self.phase_ops = collections.defaultdict(collections.Counter)
        self.where = collections.Counter() if "--where" in sys.argv else None
        # --bytes: bytes touched per op (inputs + outputs) and per source line,
        # backward ops attributed to their forward line (anomaly-mode traceback)
        self.bytes = collections.Counter()
        self.where_bytes = collections.Counter()

    def _src(self):
        import traceback
        if self.phase == "backward":
            node = torch._C._current_autograd_node()
            tb = node.metadata.get("traceback_") if node is not None else None
            if tb:
                lines = "".join(tb).splitlines()
                for i in range(len(lines) - 1, -1, -1):
                    ln = lines[i].strip()
                    if ln.startswith("File") and "open-groundingdino_amd" in ln and "/torch/" not in ln:
                        f = ln.split('"')[1].split("open-groundingdino_amd/")[-1]
                        no = ln.split("line ")[1].split(",")[0]
                        code = lines[i + 1].strip()[:60] if i + 1 < len(lines) else ""
                        return f"bwd {f}:{no} {code} [{type(node).__name__}]"
                return f"bwd ? [{type(node).__name__}]"
            return "bwd ?"
        for fr in reversed(traceback.extract_stack()[:-2]):
            if "open-groundingdino_amd" in fr.filename and "torch" not in fr.filename:
                rel = fr.filename.split("open-groundingdino_amd/")[-1]
                return f"{rel}:{fr.lineno} {fr.line.strip()[:70]}"
        return "?"

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if "--bytes" in sys.argv and not self.paused and self.phase in ("forward", "criterion", "backward"):
            name = str(func.overloadpacket).replace("aten::", "aten.") if hasattr(func, "overloadpacket") else str(func)
            out = func(*args, **kwargs)
            if name not in _FREE:
                from torch.utils._pytree import tree_leaves
                nb = sum(t.nbytes for t in tree_leaves((args, kwargs, out)) if isinstance(t, torch.Tensor))
                if name == "aten._to_copy":
                    name = f"aten._to_copy[{args[0].dtype}->{kwargs.get('dtype')}]"
                self.counts[name] += 1
                self.bytes[name] += nb
                if not _OP_FILTER or any(f in name for f in _OP_FILTER):
                    self.where_bytes[self._src() + "  <" + name + ">"] += nb
            return out
        if not self.paused:
            name = str(func.overloadpacket) if hasattr(func, "overloadpacket") else str(func)
            name = name.replace("aten::", "aten.")
            if name not in _FREE:
                if name == "aten._to_copy":
                    dt = kwargs.get("dtype")
                    name = f"aten._to_copy[{args[0].dtype}->{dt}]"
                self.counts[name] += 1
                self.by_phase[self.phase] += 1
                self.phase_ops[self.phase][name] += 1
                if self.where is not None and self.phase in ("forward", "criterion", "backward") and (
                        not _OP_FILTER or any(f in name for f in _OP_FILTER)):
                    import traceback
                    for fr in reversed(traceback.extract_stack()[:-1]):
                        if "open-groundingdino_amd" in fr.filename and "torch" not in fr.filename:
                            rel = fr.filename.split("open-groundingdino_amd/")[-1]
                            self.where[f"{rel}:{fr.lineno} {fr.line.strip()[:70]}"] += 1
                            break
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--no-autocast", action="store_true")
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--where", action="store_true", help="attribute fwd/criterion dispatches to source lines")
    ap.add_argument("--bytes", action="store_true", help="bytes touched per op and per source line")
    ap.add_argument("--phase", action="store_true", help="top ops per phase")
    ap.add_argument("--op", action="append", default=[], help="with --where: only these ops (substring)")
    a = ap.parse_args()

    import oracle_hooks
    from gdino_amd import kernels, train
    from gdino_amd.config import make_args

    torch.manual_seed(0)
    args = make_args(device="cpu", num_queries=900)
    model, criterion, _, optimizer = train.build_training(args, "cpu")
    model.train()
    samples, targets, captions, cats = train.synthetic_batch(2, a.height, a.width, n_boxes=8, n_tokens=256,
                                                             seed=0, device="cpu")
    counter = Counter()

    # HIP-only ops: one launch each for forward and one for backward, as on
    # the GPU; the oracle restatements' own ops (forward and their autograd
    # backward) are not counted
    import models.GroundingDINO.ms_deform_attn as msda_mod
    from oracle.blocks import (attention_ref, bi_attention_ref, contrastive_ref, window_attention_image_ref,
                               window_attention_packed_ref)

    def counted(fn, tag):
        class Op(torch.autograd.Function):
            @staticmethod
            def forward(ctx, *args):
                ctx.args = args
                counter.paused += 1
                try:
                    with torch.no_grad():
                        out = fn(*args)
                finally:
                    counter.paused -= 1
                counter.counts[tag + "_fwd"] += 1
                ctx.tuple_out = isinstance(out, tuple)
                return out

            @staticmethod
            def backward(ctx, *grads):
                counter.paused += 1
                try:
                    with torch.enable_grad():
                        args = [a.detach().requires_grad_(True) if torch.is_tensor(a) and a.is_floating_point()
                                else a for a in ctx.args]
                        out = fn(*args)
                        outs = out if ctx.tuple_out else (out,)
                        ins = [a for a in args if torch.is_tensor(a) and a.requires_grad]
                        gs = iter(torch.autograd.grad(outs, ins, grads, allow_unused=True))
                finally:
                    counter.paused -= 1
                counter.counts[tag + "_bwd"] += 1
                return tuple(next(gs) if torch.is_tensor(a) and a.is_floating_point() else None
                             for a in ctx.args)
        return Op.apply

    msda_op = counted(lambda *x: oracle_hooks._OracleMSDA.apply(*x), "gd.msda")

    class CountedMSDA:
        @staticmethod
        def apply(*x):
            return msda_op(*x)

    bi_op = counted(lambda q, k, vv, vl, pv, pl: bi_attention_ref(q, k, vv, vl, pv, pl), "gd.biattn")

    def counted_bi(q, k, vv, vl, pv=None, pl=None, p=0.0):
        return bi_op(q, k, vv, vl, pv, pl)

    win_op = counted(lambda qkv, t, r, m, sc: window_attention_packed_ref(qkv.float(), t.float(), r, m, sc)
                     .to(qkv.dtype), "gd.window_attn")
    wimg_op = counted(lambda qkv, qb, t, r, m, hw, ws, sh, sc: window_attention_image_ref(
        qkv.float(), None if qb is None else qb.float(), t.float(), r, m, hw, ws, sh, sc).to(qkv.dtype),
        "gd.window_attn_image")
    attn_op = counted(lambda q, k, v, m, sc: attention_ref(q.float(), k.float(), v.float(), m, sc).to(q.dtype),
                      "gd.attn")

    def counted_attn(q, k, v, m=None, sc=None, p=0.0):
        return attn_op(q, k, v, m, sc)

    con_op = counted(lambda x, t, m, n: contrastive_ref(x.float(), t.float(), m, n), "gd.contrastive")

    def counted_rowmax(x, t, m):
        counter.counts["gd.contrastive_rowmax"] += 1
        counter.paused += 1
        try:
            with torch.no_grad():
                return contrastive_ref(x.float(), t.float(), m, t.shape[1]).max(-1)[0]
        finally:
            counter.paused -= 1

    # the MSDA prologue kernel (GPU-only, gdino_amd/msda_prologue.py): one
    # launch each way, computed here by the torch composition
    from gdino_amd import msda_prologue as pro_mod

    def pro_fn(off, logit, ref, shapes, m, l, p):
        n, lq, _ = off.shape
        loc = msda_mod.sampling_locations_from(ref, off.float().reshape(n, lq, m, l, p, 2), shapes, p)
        attn = logit.float().reshape(n, lq, m, l * p).softmax(-1).view(n, lq, m, l, p)
        return loc, attn

    pro_op = counted(pro_fn, "gd.msda_prologue")

    class CountedPrologue:
        @staticmethod
        def apply(*x):
            return pro_op(*x)

    # residual add + LayerNorm (GPU-only, gdino_amd/layernorm.py): one
    # launch forward, two backward (kernel + column reduction)
    from gdino_amd import layernorm as ln_mod
    ln_op = counted(lambda x, r, w, b, eps: torch.nn.functional.layer_norm(
        x.float() + (0 if r is None else r.float()), w.shape, w, b, eps),
                    "gd.add_layernorm")

    class CountedAddLN:
        @staticmethod
        def apply(*x):
            return ln_op(*x)

    prev_ln = (ln_mod.supported, ln_mod.AddLayerNormFunction)
    ln_mod.supported = lambda norm, x, r: x.shape[-1] in ln_mod.WIDTHS and norm.elementwise_affine
    ln_mod.AddLayerNormFunction = CountedAddLN
    prev_pro = (pro_mod.supported, pro_mod.MSDAPrologue)
    pro_mod.supported = lambda off, logit, ref, l, p: l * p == 16 and not ref.requires_grad
    pro_mod.MSDAPrologue = CountedPrologue
    prev = msda_mod.MSDeformAttnFunction
    msda_mod.MSDeformAttnFunction = CountedMSDA
    amp = None if a.no_autocast else torch.bfloat16

    def step(c):
        """train.train_step's phases, attributed separately (the optimizer is
        excluded from the total: CPU AdamW is the per-parameter loop, the GPU
        runs the fused multi-tensor kernel, ~25 launches)."""
        c.phase = "forward"
        with torch.autocast(device_type="cpu", dtype=amp or torch.bfloat16, enabled=amp is not None):
            outputs = model(samples, captions=captions)
            c.phase = "criterion"
            loss_dict = criterion(outputs, targets, cats, captions)
            loss = train.weighted_loss(loss_dict, criterion.weight_dict)
        optimizer.zero_grad(set_to_none=True)
        c.phase = "backward"
        loss.backward()
        c.phase = "clip"
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.1, foreach=True)
        c.phase = "optimizer"
        c.paused += 1
        optimizer.step()
        c.paused -= 1

    try:
        with kernels.override("bi_attention", counted_bi), \
                kernels.override("window_attention_packed", win_op), kernels.override("window_attention_image", wimg_op), \
                kernels.override("attention", counted_attn), \
                kernels.override("contrastive_logits", con_op), kernels.override("contrastive_rowmax", counted_rowmax):
            step(Counter())  # warm-up (caches)
            with counter, torch.autograd.set_detect_anomaly("--bytes" in sys.argv, check_nan=False):
                step(counter)
    finally:
        msda_mod.MSDeformAttnFunction = prev
        pro_mod.supported, pro_mod.MSDAPrologue = prev_pro
        ln_mod.supported, ln_mod.AddLayerNormFunction = prev_ln
    total = sum(counter.counts.values())
    casts = sum(v for k, v in counter.counts.items() if k.startswith("aten._to_copy"))
    print(f"dispatches/step={total} (+~25 fused AdamW on GPU)  casts={casts}  by phase: {dict(counter.by_phase)}")
    for k, v in counter.counts.most_common(a.top):
        print(f"  {v:6d}  {k}")
    if "--phase" in sys.argv:
        for ph, c in counter.phase_ops.items():
            print(f"--- {ph}")
            for k, v in c.most_common(a.top):
                print(f"  {v:6d}  {k}")
    if counter.bytes:
        tot = sum(counter.bytes.values())
        print(f"--- bytes touched (fwd + criterion + bwd): {tot / 1e9:.2f} GB")
        for k, v in counter.bytes.most_common(a.top):
            print(f"  {v / 1e6:10.1f} MB  {k}")
        print("--- by source line")
        for k, v in counter.where_bytes.most_common(a.top * 2):
            print(f"  {v / 1e6:10.1f} MB  {k}")
    if counter.where is not None:
        print("--- forward + criterion dispatches by source line")
        for k, v in counter.where.most_common(a.top):
            print(f"  {v:6d}  {k}")


if __name__ == "__main__":
    main()
