"""Convolutions of the hot path as GEMMs (no MIOpen).

The training step has exactly two kinds of convolution, both cheap but both
otherwise routed through MIOpen:

  * Swin's patch embedding, Conv2d(3, C, k=4, s=4): non-overlapping patches,
    i.e. one GEMM over [B*Ho*Wo, 3*4*4] patch rows
    (backbone/swin_transformer.py:464-497);
  * the input projections of GroundingDINO, Conv2d(C_l, 256, 1) per backbone
    level and Conv2d(C_last, 256, 3, s=2, p=1) for the extra level
    (groundingdino.py:142-163): a [256, C] x [B, C, HW] matmul, and im2col
    (F.unfold) + matmul.

On MI355X, MIOpen costs these three things per call:

  * host-side solver lookups;
  * NCHW<->NHWC transpose kernels around the implicit-GEMM kernel;
  * on the first call, find-mode benchmarking (about 0.7 s in the warm-up).

MIOpen also manages its own workspace. A GEMM through hipBLASLt on
torch-allocated memory is cheaper and safe to capture into a HIP graph.
Parameters are the nn.Conv2d ones (same state dict); set
``GemmConv2d.use_gemm = False`` to fall back to F.conv2d for A/B checks.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from . import castcache


def conv2d_gemm(x: torch.Tensor, weight: torch.Tensor, bias=None, stride=(1, 1), padding=(0, 0)):
    """F.conv2d(x, weight, bias, stride, padding) for dilation 1, groups 1,
    as a GEMM.  x [B, C, H, W] -> [B, O, Ho, Wo] (contiguous NCHW)."""
    o, c, kh, kw = weight.shape
    b, _, h, w = x.shape
    sh, sw = stride
    ph, pw = padding
    if (kh, kw) == (1, 1) and (sh, sw) == (1, 1) and (ph, pw) == (0, 0):
        ho, wo = h, w
        cols = x.reshape(b, c, h * w)
    elif (kh, kw) == (sh, sw) and (ph, pw) == (0, 0):
        # non-overlapping patches: the conv floors, so trailing rows/cols drop
        ho, wo = h // kh, w // kw
        xs = x[:, :, : ho * kh, : wo * kw]
        cols = xs.reshape(b, c, ho, kh, wo, kw).permute(0, 1, 3, 5, 2, 4).reshape(b, c * kh * kw, ho * wo)
    else:
        ho = (h + 2 * ph - kh) // sh + 1
        wo = (w + 2 * pw - kw) // sw + 1
        cols = F.unfold(x, (kh, kw), padding=(ph, pw), stride=(sh, sw))
    dt = castcache.autocast_dtype(x)
    if dt is not None:
        weight = castcache.cached_cast(weight, dt)
        bias = None if bias is None else castcache.cached_cast(bias, dt)
    out = torch.matmul(weight.reshape(o, c * kh * kw), cols)  # [B, O, Ho*Wo]
    if bias is not None:
        out = out + bias.to(out.dtype).view(1, o, 1)
    return out.view(b, o, ho, wo)


class GemmConv2d(nn.Conv2d):
    """nn.Conv2d whose forward runs as a GEMM (see module docstring)."""

    use_gemm = True

    def forward(self, x):
        if (not self.use_gemm or self.groups != 1 or self.dilation != (1, 1) or self.padding_mode != "zeros"
                or isinstance(self.padding, str)):
            return super().forward(x)
        return conv2d_gemm(x, self.weight, self.bias, self.stride, self.padding)
