"""oracle/msda_torch.py — TEST INFRASTRUCTURE ONLY.

Pure-PyTorch restatements of the reference MSDA fallback, for CPU tests and
for bench.py's cpu_baseline leg (which times the reference's CPU algorithm on
the GPU box's host cores, since the reference itself never travels there).

* ``msda_grid_sample`` restates the reference fallback algorithm
  (ms_deform_attn_core_pytorch, /root/reference/models/GroundingDINO/ops/
  functions/ms_deform_attn_func.py:41-61, identical to
  multi_scale_deformable_attn_pytorch, ms_deform_attn.py:94-134): per level,
  F.grid_sample(bilinear, zeros, align_corners=False) over a [N*M, D, H, W]
  view of value, then an attention-weighted sum over (L, P).
* ``msda_gather`` is an explicit 4-corner gather restatement of the CUDA
  kernel semantics (.cuh:238-299) that runs on any dtype and is autograd-able.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def msda_grid_sample(value, spatial_shapes, sampling_locations, attention_weights):
    n, s, m, d = value.shape
    _, lq, _, n_levels, n_points, _ = sampling_locations.shape
    sizes = [int(h) * int(w) for h, w in spatial_shapes.tolist()]
    per_level = torch.split(value, sizes, dim=1)
    grids = sampling_locations * 2.0 - 1.0  # grid_sample wants [-1, 1]
    sampled = []
    for lvl, (h, w) in enumerate(spatial_shapes.tolist()):
        # [n, h*w, m, d] -> [n*m, d, h, w]
        img = per_level[lvl].permute(0, 2, 3, 1).reshape(n * m, d, int(h), int(w))
        # [n, lq, m, p, 2] -> [n*m, lq, p, 2]
        g = grids[:, :, :, lvl].permute(0, 2, 1, 3, 4).reshape(n * m, lq, n_points, 2)
        sampled.append(F.grid_sample(img, g, mode="bilinear", padding_mode="zeros",
                                     align_corners=False))  # [n*m, d, lq, p]
    stacked = torch.stack(sampled, dim=3).flatten(3)  # [n*m, d, lq, L*P]
    w = attention_weights.permute(0, 2, 1, 3, 4).reshape(n * m, 1, lq, n_levels * n_points)
    out = (stacked * w).sum(-1)  # [n*m, d, lq]
    return out.view(n, m * d, lq).transpose(1, 2).contiguous()


def msda_gather(value, spatial_shapes, level_start_index, sampling_locations, attention_weights):
    n, s, m, d = value.shape
    _, lq, _, n_levels, n_points, _ = sampling_locations.shape
    out = value.new_zeros((n, lq, m, d))
    bidx = torch.arange(n, device=value.device).view(n, 1, 1, 1)
    hidx = torch.arange(m, device=value.device).view(1, 1, m, 1)
    for lvl in range(n_levels):
        h, w = (int(x) for x in spatial_shapes[lvl].tolist())
        start = int(level_start_index[lvl])
        loc = sampling_locations[:, :, :, lvl]  # [n, lq, m, p, 2]
        y = loc[..., 1] * h - 0.5
        x = loc[..., 0] * w - 0.5
        inside = (y > -1) & (x > -1) & (y < h) & (x < w)
        y0 = torch.floor(y)
        x0 = torch.floor(x)
        fy, fx = y - y0, x - x0
        y0, x0 = y0.long(), x0.long()
        a = attention_weights[:, :, :, lvl] * inside.to(value.dtype)
        for dy, dx, wgt in ((0, 0, (1 - fy) * (1 - fx)), (0, 1, (1 - fy) * fx),
                            (1, 0, fy * (1 - fx)), (1, 1, fy * fx)):
            yy, xx = y0 + dy, x0 + dx
            ok = (yy >= 0) & (yy <= h - 1) & (xx >= 0) & (xx <= w - 1)
            pos = (start + yy.clamp(0, h - 1) * w + xx.clamp(0, w - 1))  # [n, lq, m, p]
            v = value[bidx, pos, hidx]  # [n, lq, m, p, d]
            coef = (wgt * a * ok.to(value.dtype)).unsqueeze(-1)
            out = out + (v * coef).sum(3)
    return out.reshape(n, lq, m * d)
