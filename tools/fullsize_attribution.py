"""Which HIP family moves the full-size bf16 outputs / gradients away from
the fp32 reference?  (in cfg5 the product P was
slightly worse than the torch bf16 composition C on pred_logits and the
decoder-layer-4 gradients.)

Runs tests/test_fullsize_gpu's comparison once for F (fp32 reference
composition) and C (bf16 reference composition), then the product P with ONE
family at a time replaced by its reference composition: GDINO_DISABLE=<fam>
for the families with a torch path, the oracle restatement for the MSDA core
and the BiAttention core (no torch path in the product), the cast cache /
fused projections switched off.  A variant whose error drops to C's names
the family responsible.  Matching and top-k selection are pinned as in the
tests.  Output: one JSON line per variant (gpurun_out/attribution.jsonl).

    python tools/fullsize_attribution.py [--cfg cfg5|cfg3]
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="cfg5", choices=("cfg5", "cfg3"))
    ap.add_argument("--out", default="gpurun_out/attribution.jsonl")
    a = ap.parse_args()
    import pytest
    import test_fullsize_gpu as T
    from gdino_amd import castcache, kernels
    from gdino_amd.misc import DropPath
    from gdino_amd.train import weighted_loss
    from oracle.blocks import bi_attention_ref
    from oracle_hooks import _OracleMSDA
    import models.GroundingDINO.ms_deform_attn as msda_mod

    backbone, hw, vg = (("swin_B_384_22k", (1024, 1024), 1) if a.cfg == "cfg5" else ("swin_T_224_1k", (800, 1333), 0))
    model, criterion, _ = T._build(backbone=backbone, perturb_offsets=True)
    model.train()
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
        if isinstance(m, DropPath):
            m.drop_prob = 0.0
    samples, targets, captions, cats = T._batch(2, hw[0], hw[1], vg_images=vg)
    params = {n: p for n, p in model.named_parameters() if p.requires_grad}
    pin, pm = T.PinnedTopk(), T.PinnedMatch(criterion.matcher)

    def run(amp=True):
        model.zero_grad(set_to_none=True)
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16, enabled=amp):
            out = model(samples, captions=captions)
            loss = weighted_loss(criterion(out, targets, cats, captions), criterion.weight_dict)
        loss.backward()
        torch.cuda.synchronize()
        outs = {k: v.detach().float() for k, v in T._outputs(out).items()}
        return outs, {n: p.grad.detach().clone() for n, p in params.items() if p.grad is not None}

    with pin.active("record"), pm.active("record"):
        p_out, p_g = run()
    with T.torch_composition(), pin.active("replay"), pm.active("replay"):
        c_out, c_g = run()
    with T.torch_composition(fp32=True), pin.active("replay"), pm.active("replay"):
        f_out, f_g = run(amp=False)

    def rl2(x, y):
        x, y = x.double(), y.double()
        return float((x - y).norm() / y.norm().clamp_min(1e-30))

    def summary(outs, grads):
        row = {k: T._rel(outs[k], f_out[k]) for k in f_out}
        errs = sorted((rl2(grads[n], f_g[n]), n) for n in f_g)
        row["grad_q0.5"] = errs[len(errs) // 2][0]
        row["grad_q0.95"] = errs[min(len(errs) - 1, int(0.95 * len(errs)))][0]
        row["worst"] = [(n, round(e, 4)) for e, n in errs[-4:]]
        return row

    @contextlib.contextmanager
    def env(fam):
        mp = pytest.MonkeyPatch()
        mp.setenv("GDINO_DISABLE", fam)
        try:
            yield
        finally:
            mp.undo()

    @contextlib.contextmanager
    def msda_oracle():
        prev = msda_mod.MSDeformAttnFunction
        msda_mod.MSDeformAttnFunction = _OracleMSDA
        try:
            yield
        finally:
            msda_mod.MSDeformAttnFunction = prev

    @contextlib.contextmanager
    def attr(obj, name, val):
        mp = pytest.MonkeyPatch()
        mp.setattr(obj, name, val)
        try:
            yield
        finally:
            mp.undo()

    variants = {
        "P (all HIP)": contextlib.nullcontext,
        "C (bf16 composition)": None,
        "msda -> oracle": msda_oracle,
        "biattn -> oracle": lambda: kernels.override("bi_attention", lambda q, k, vv, vl, pv=None, pl=None, p=0.0:
                                                     bi_attention_ref(q, k, vv, vl, pv, pl)),
        "cast cache off": lambda: attr(castcache, "ENABLED", False),
        "fused projections off": lambda: attr(castcache, "FUSE_SHARED_INPUT", False),
    }
    for fam in ("wattn", "attn", "contrastive", "prologue", "wgrad", "addln"):
        variants[f"no {fam}"] = (lambda f: lambda: env(f))(fam)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "a") as fo:
        for name, ctx in variants.items():
            if ctx is None:
                row = summary(c_out, c_g)
            elif name.startswith("P "):
                row = summary(p_out, p_g)
            else:
                with ctx(), pin.active("replay"), pm.active("replay"):
                    o, g = run()
                row = summary(o, g)
            row = {"cfg": a.cfg, "variant": name, **row}
            fo.write(json.dumps(row) + "\n")
            fo.flush()
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
