"""Shared loaders for the MSDA golden fixtures (tests/golden/msda_*.npz)."""
import os

import numpy as np
import torch

from conftest import GOLDEN

KAT_NAMES = ["kat_fwd_double", "kat_fwd_float", "kat_grad_d30", "kat_grad_d32",
             "kat_grad_d64", "kat_grad_d71"]


def load_case(name):
    with np.load(os.path.join(GOLDEN, f"msda_{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def cfg1_inputs(dtype=torch.float64):
    """Regenerate BASELINE config 1 inputs (same recipe as make_golden.cfg1_inputs)."""
    shapes = torch.as_tensor([(64, 64), (32, 32), (16, 16), (8, 8)], dtype=torch.long)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    N, S, M, D, L, P, Lq = 1, 5440, 8, 32, 4, 4, 100
    g = torch.Generator().manual_seed(0)
    value = torch.rand(N, S, M, D, generator=g, dtype=dtype)
    loc = torch.rand(N, Lq, M, L, P, 2, generator=g, dtype=dtype)
    attn = torch.rand(N, Lq, M, L, P, generator=g, dtype=dtype) + 1e-5
    attn /= attn.sum(-1, keepdim=True).sum(-2, keepdim=True)
    grad_out = torch.randn(N, Lq, M * D, generator=g, dtype=dtype)
    return value, shapes, lsi, loc, attn, grad_out


def edge_excluded_mask(case):
    """Samples whose point lies exactly on a kink of the bilinear surface:
    on the excluded band edge (h_im == -1, w_im == -1, h_im == H, w_im == W)
    or on an integer pixel coordinate.  There the derivative is one-sided:
    the reference CUDA kernel (.cuh:288 strict band, .cuh:99-100 floor of
    loc*W-0.5) and grid_sample's autograd (which re-derives the coordinate as
    ((2*loc-1)+1)*W/2-1/2 and can land 1 ulp on the other side) pick
    different sides.  Values agree there; only grad_loc may differ."""
    loc = case["loc"]
    shapes = case["shapes"]
    mask = np.zeros(loc.shape[:-1], dtype=bool)
    for lvl, (h, w) in enumerate(shapes):
        y = loc[:, :, :, lvl, :, 1] * h - 0.5
        x = loc[:, :, :, lvl, :, 0] * w - 0.5
        mask[:, :, :, lvl, :] = (y == -1) | (x == -1) | (y == h) | (x == w) | (y == np.floor(y)) | (x == np.floor(x))
    return mask


def smooth_samples(loc, shapes, eps=1e-4):
    """[N, Lq, M, L, P, 1] bool: samples whose pixel coordinates are more than
    eps from a cell edge.  grad_loc (the derivative of the bilinear
    interpolation) jumps across cell edges, and fp32 vs fp64 rounding of
    loc * size - 0.5 may put a sample on different sides of one; grad_value
    and grad_attn are continuous there."""
    loc = torch.as_tensor(loc).double().cpu()
    hw = torch.as_tensor(shapes).double().cpu()  # [L, 2] (H, W)
    w_im = loc[..., 0] * hw[:, 1][None, None, None, :, None] - 0.5
    h_im = loc[..., 1] * hw[:, 0][None, None, None, :, None] - 0.5
    ok = ((w_im - w_im.round()).abs() > eps) & ((h_im - h_im.round()).abs() > eps)
    return ok[..., None].numpy()


def rel_err_grad_loc(gl, ref_gl, loc, shapes):
    keep = np.broadcast_to(smooth_samples(loc, shapes), np.shape(ref_gl))
    a = np.asarray(gl, np.float64)[keep]
    b = np.asarray(ref_gl, np.float64)[keep]
    return float(np.abs(a - b).max() / max(np.abs(np.asarray(ref_gl, np.float64)).max(), 1e-30))
