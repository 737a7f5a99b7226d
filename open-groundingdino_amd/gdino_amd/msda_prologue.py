"""MSDA prologue on MI355X (csrc/msda_prologue.hip): the fused offsets /
attention-logits Linear output -> sampling locations and softmaxed attention
weights in one kernel, and the backward in one kernel.

Replaces, per MultiScaleDeformableAttention call (reference
ms_deform_attn.py:274-363), the attention-logit cast + softmax and the
offset cast + normalizer division + reference-point addition over
[N, Lq, M, L, P, 2] fp32 tensors, and their autograd backward.  Used when
L*P == 16, the projections are fp32 / bf16 device tensors and the reference
points need no gradient (the encoder's are constants and the decoder's are
detached, transformer.py:692-735); otherwise the torch composition runs.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

_p, _i, _i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
_lib.register("gd_msda_prologue_forward", [_i, _p, _i64, _p, _i64, _p, _i, _p, _i, _i, _i, _i, _i, _p, _p, _p])
_lib.register("gd_msda_prologue_backward", [_i, _p, _p, _p, _p, _i, _p, _i, _i, _i, _i, _i, _p, _p, _p])


def _rows_ok(t):
    """[N, Lq, C] with unit column stride and uniform row stride"""
    return t.dim() == 3 and t.stride(2) == 1 and t.stride(0) == t.shape[1] * t.stride(1)


def supported(offsets, logits, reference_points, num_levels, num_points) -> bool:
    return (_lib.enabled("prologue") and _lib.on_device(offsets) and num_levels * num_points == 16
            and offsets.dtype in (torch.float32, torch.bfloat16) and logits.dtype == offsets.dtype and _rows_ok(offsets) and _rows_ok(logits)
            and reference_points.shape[-1] in (2, 4) and not reference_points.requires_grad)


class MSDAPrologue(torch.autograd.Function):
    @staticmethod
    def forward(ctx, offsets, logits, reference_points, spatial_shapes, num_heads, num_levels, num_points):
        n, lq, _ = offsets.shape
        ref = reference_points.float().contiguous()
        loc = torch.empty(n, lq, num_heads, num_levels, num_points, 2, dtype=torch.float32, device=offsets.device)
        attn = torch.empty(n, lq, num_heads, num_levels, num_points, dtype=torch.float32, device=offsets.device)
        _lib.call("gd_msda_prologue_forward", _lib.dtype_code(offsets), offsets.data_ptr(), offsets.stride(1),
                  logits.data_ptr(), logits.stride(1), ref.data_ptr(), ref.shape[-1], spatial_shapes.data_ptr(),
                  n, lq, num_heads, num_levels, num_points, loc.data_ptr(), attn.data_ptr(),
                  _lib.stream_of(offsets))
        ctx.save_for_backward(attn, ref, spatial_shapes)
        ctx.meta = (offsets.dtype, offsets.shape, logits.shape, num_heads, num_levels, num_points)
        return loc, attn

    @staticmethod
    def backward(ctx, grad_loc, grad_attn):
        attn, ref, shapes = ctx.saved_tensors
        dt, oshape, lshape, m, l, p = ctx.meta
        n, lq = oshape[0], oshape[1]
        grad_loc = torch.zeros_like(attn).unsqueeze(-1).expand(*attn.shape, 2).contiguous() if grad_loc is None \
            else grad_loc.float().contiguous()
        grad_attn = torch.zeros_like(attn) if grad_attn is None else grad_attn.float().contiguous()
        g_off = torch.empty(oshape, dtype=dt, device=attn.device)
        g_log = torch.empty(lshape, dtype=dt, device=attn.device)
        _lib.call("gd_msda_prologue_backward", _lib.dtype_code(g_off), grad_loc.data_ptr(), grad_attn.data_ptr(),
                  attn.data_ptr(), ref.data_ptr(), ref.shape[-1], shapes.data_ptr(), n, lq, m, l, p,
                  g_off.data_ptr(), g_log.data_ptr(), _lib.stream_of(attn))
        return g_off, g_log, None, None, None, None, None
