"""Generate MSDA golden vectors from the REFERENCE's own pure-PyTorch function.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py

It imports ``multi_scale_deformable_attn_pytorch`` from
/root/reference/models/GroundingDINO/ms_deform_attn.py:94-134 by file path
(bit-identical to ms_deform_attn_core_pytorch, ops/functions/
ms_deform_attn_func.py:41-61), evaluates it in fp64 with autograd for the
gradients, and writes data-only fixtures (inputs + outputs, .npz, no pickle)
next to this script.  Nothing from the reference is copied into the repo; the
GPU box only reads the .npz files.

Cases
  kat_*      ops/test.py shapes (N,M,D=1,2,2; Lq,L,P=2,2,2; levels (6,4),(3,2)),
             torch.manual_seed(3) and the same draw order as test.py:32-86
             (fwd double, fwd float, then D in {30, 32, 64, 71}).
  edge       locations on/around the -1 < h < H band edges, outside [0, 1],
             non-power-of-2 D=30, zero (pad-masked) value rows.
  cfg1       BASELINE config 1: N=1, levels 64^2/32^2/16^2/8^2 (S=5440), Lq=100,
             M=8, D=32, L=4, P=4; inputs regenerated from a CPU torch.Generator
             seed (stored), outputs stored as checksums + sampled elements.
"""
from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/models/GroundingDINO/ms_deform_attn.py"


def load_reference_core():
    spec = importlib.util.spec_from_file_location("_ref_ms_deform_attn", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.multi_scale_deformable_attn_pytorch


def shapes_lsi(levels):
    shapes = torch.as_tensor(levels, dtype=torch.long)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    return shapes, lsi


def run(core, value, shapes, loc, attn, grad_out):
    v = value.detach().clone().double().requires_grad_(True)
    l = loc.detach().clone().double().requires_grad_(True)
    a = attn.detach().clone().double().requires_grad_(True)
    out = core(v, shapes, l, a)
    (out * grad_out.double()).sum().backward()
    return out.detach(), v.grad, l.grad, a.grad


def kat_cases(core):
    N, M, D = 1, 2, 2
    Lq, L, P = 2, 2, 2
    shapes, lsi = shapes_lsi([(6, 4), (3, 2)])
    S = int(shapes.prod(1).sum())
    torch.manual_seed(3)
    cases = {}

    def draw(d):
        value = torch.rand(N, S, M, d) * 0.01
        loc = torch.rand(N, Lq, M, L, P, 2)
        attn = torch.rand(N, Lq, M, L, P) + 1e-5
        attn /= attn.sum(-1, keepdim=True).sum(-2, keepdim=True)
        return value, loc, attn

    for name, d in (("kat_fwd_double", D), ("kat_fwd_float", D), ("kat_grad_d30", 30),
                    ("kat_grad_d32", 32), ("kat_grad_d64", 64), ("kat_grad_d71", 71)):
        value, loc, attn = draw(d)
        g = torch.Generator().manual_seed(1000 + d)
        grad_out = torch.randn(N, Lq, M * d, generator=g, dtype=torch.float64)
        out, gv, gl, ga = run(core, value, shapes, loc, attn, grad_out)
        cases[name] = dict(value=value.double(), loc=loc.double(), attn=attn.double(),
                           shapes=shapes, lsi=lsi, grad_out=grad_out, out=out, grad_value=gv,
                           grad_loc=gl, grad_attn=ga)
    return cases


def edge_case(core):
    levels = [(5, 7), (3, 4)]
    shapes, lsi = shapes_lsi(levels)
    S = int(shapes.prod(1).sum())
    N, M, D, L, P = 2, 3, 30, 2, 4
    g = torch.Generator().manual_seed(7)
    value = torch.randn(N, S, M, D, generator=g, dtype=torch.float64)
    value[1, 3:9] = 0.0  # pad-masked rows
    # special coordinates: exactly on the excluded / included band edges
    specials = []
    for (h, w) in levels:
        specials += [
            (-0.5 / w, 0.3), (0.3, -0.5 / h),            # h_im or w_im == -1 -> excluded
            (-0.5 / w + 1e-9, 0.3),                      # just inside
            (1.0 + 0.5 / w, 0.4), (0.4, 1.0 + 0.5 / h),  # == W / == H -> excluded
            (1.0 + 0.5 / w - 1e-9, 0.6),                 # just inside
            (0.0, 0.0), (1.0, 1.0), (0.5 / w, 0.5 / h),  # corners / exact pixel centre
            (-0.25, 0.5), (1.3, 0.5), (0.5, -2.0),       # far outside
        ]
    Lq = len(specials)
    loc = torch.rand(N, Lq, M, L, P, 2, generator=g, dtype=torch.float64) * 1.4 - 0.2
    for qi, (x, y) in enumerate(specials):
        loc[:, qi, :, qi % L, qi % P, 0] = x
        loc[:, qi, :, qi % L, qi % P, 1] = y
    attn = torch.rand(N, Lq, M, L, P, generator=g, dtype=torch.float64) + 1e-5
    attn /= attn.sum(-1, keepdim=True).sum(-2, keepdim=True)
    grad_out = torch.randn(N, Lq, M * D, generator=g, dtype=torch.float64)
    out, gv, gl, ga = run(core, value, shapes, loc, attn, grad_out)
    return dict(value=value, loc=loc, attn=attn, shapes=shapes, lsi=lsi, grad_out=grad_out,
                out=out, grad_value=gv, grad_loc=gl, grad_attn=ga)


def cfg1_inputs(seed=0, dtype=torch.float64):
    """Regenerable on any host with this torch build (CPU generator)."""
    shapes, lsi = shapes_lsi([(64, 64), (32, 32), (16, 16), (8, 8)])
    N, S, M, D, L, P, Lq = 1, 5440, 8, 32, 4, 4, 100
    g = torch.Generator().manual_seed(seed)
    value = torch.rand(N, S, M, D, generator=g, dtype=dtype)
    loc = torch.rand(N, Lq, M, L, P, 2, generator=g, dtype=dtype)
    attn = torch.rand(N, Lq, M, L, P, generator=g, dtype=dtype) + 1e-5
    attn /= attn.sum(-1, keepdim=True).sum(-2, keepdim=True)
    grad_out = torch.randn(N, Lq, M * D, generator=g, dtype=dtype)
    return value, shapes, lsi, loc, attn, grad_out


def sample_idx(n, k, seed):
    return np.sort(np.random.default_rng(seed).choice(n, size=min(n, k), replace=False))


def cfg1_case(core):
    value, shapes, lsi, loc, attn, grad_out = cfg1_inputs()
    out, gv, gl, ga = run(core, value, shapes, loc, attn, grad_out)
    rec = dict(seed=np.int64(0), shapes=shapes, lsi=lsi)
    for name, t in (("out", out), ("grad_value", gv), ("grad_loc", gl), ("grad_attn", ga)):
        flat = t.reshape(-1).numpy()
        idx = sample_idx(flat.size, 256, {"out": 1, "grad_value": 2, "grad_loc": 3, "grad_attn": 4}[name])
        rec[f"{name}_idx"] = idx
        rec[f"{name}_val"] = flat[idx]
        rec[f"{name}_sum"] = np.float64(flat.sum())
        rec[f"{name}_abssum"] = np.float64(np.abs(flat).sum())
        rec[f"{name}_sqsum"] = np.float64((flat * flat).sum())
    # input checksum so a different torch RNG on the box is detected, not misread
    rec["value_sum"] = np.float64(value.sum())
    rec["loc_sum"] = np.float64(loc.sum())
    return rec


def to_np(d):
    return {k: (v.numpy() if isinstance(v, torch.Tensor) else v) for k, v in d.items()}


def main():
    core = load_reference_core()
    for name, case in kat_cases(core).items():
        np.savez_compressed(os.path.join(HERE, f"msda_{name}.npz"), **to_np(case))
    np.savez_compressed(os.path.join(HERE, "msda_edge.npz"), **to_np(edge_case(core)))
    np.savez_compressed(os.path.join(HERE, "msda_cfg1.npz"), **to_np(cfg1_case(core)))
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))


if __name__ == "__main__":
    sys.exit(main())
