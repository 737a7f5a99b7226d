"""ContrastiveEmbed on MI355X: csrc/contrastive.hip through the C-ABI.

``contrastive_logits(x, text, text_token_mask, max_text_len)`` (reference
utils.py:242-273): x [B, Q, C] . text [B, T, C]^T, -inf on padded tokens,
right-padded with -inf to max_text_len, fp32 -- one MFMA kernel writing the
final [B, Q, max_text_len] tensor (the reference: matmul, masked_fill, a -inf
fill and a slice copy).  Backward: the masked gradient through two hipBLASLt
GEMMs (dx = g.text, dtext = g^T.x).

``contrastive_rowmax(x, text, text_token_mask)``: max over tokens of the same
logits, the two-stage proposal score (transformer.py:292-296,
``enc_outputs_class_unselected.max(-1)[0]``), computed without materialising
the [B, S, 256] logits of every image token.  Only its top-k indices are used,
so it carries no gradient (as in the reference, where topk cuts the graph).

Under autocast the products run in the autocast dtype, like the reference's
autocast matmul; the kernel accumulates in fp32 either way.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, kernels

_p, _i = ctypes.c_void_p, ctypes.c_int
_lib.register("gd_contrastive_forward", [_i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p, _p, _p])


def _compute_dtype(x, text):
    dev = x.device.type
    if dev in ("cuda", "cpu") and torch.is_autocast_enabled(dev):
        return torch.get_autocast_dtype(dev)
    return x.dtype if x.dtype == text.dtype else torch.float32


def _prep(x, text, text_token_mask):
    _lib.require_device(x, text, text_token_mask, what="contrastive")
    dt = _compute_dtype(x, text)
    if dt not in (torch.float32, torch.bfloat16):
        dt = torch.float32
    xc, tc = x.to(dt), text.to(dt)
    if xc.stride(-1) != 1 or xc.data_ptr() % 16 or any(s % (16 // xc.element_size()) for s in xc.stride()[:2]):
        xc = xc.contiguous()
    if tc.stride(-1) != 1 or tc.data_ptr() % 16 or any(s % (16 // tc.element_size()) for s in tc.stride()[:2]):
        tc = tc.contiguous()
    keep = text_token_mask.contiguous().view(torch.uint8)
    return xc, tc, keep


def _launch(xc, tc, keep, tout, logits, rowmax):
    b, q, c = xc.shape
    t = tc.shape[1]
    _lib.call("gd_contrastive_forward", _lib.dtype_code(xc), xc.data_ptr(), (ctypes.c_int64 * 2)(*xc.stride()[:2]),
              tc.data_ptr(), (ctypes.c_int64 * 2)(*tc.stride()[:2]), keep.data_ptr(), b, q, t, c, tout,
              _lib.ptr(logits), _lib.ptr(rowmax), _lib.stream_of(xc), flops=2.0 * b * q * t * c)


def supported(x, text, max_text_len) -> bool:
    return (_lib.enabled("contrastive") and x.dim() == 3 and text.dim() == 3 and x.shape[-1] == text.shape[-1] and x.shape[-1] % 32 == 0
            and 0 < text.shape[1] <= max_text_len and x.shape[0] < 65536)


class ContrastiveFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, text, text_token_mask, max_text_len):
        xc, tc, keep = _prep(x, text, text_token_mask)
        b, q, _ = xc.shape
        out = torch.empty(b, q, max_text_len, dtype=torch.float32, device=x.device)
        _launch(xc, tc, keep, max_text_len, out, None)
        ctx.save_for_backward(xc, tc, text_token_mask)
        ctx.dtypes = (x.dtype, text.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        xc, tc, mask = ctx.saved_tensors
        t = tc.shape[1]
        gv = g[..., :t].masked_fill(~mask[:, None, :], 0.0).to(xc.dtype)
        dx = torch.matmul(gv, tc).to(ctx.dtypes[0]) if ctx.needs_input_grad[0] else None
        dtext = torch.matmul(gv.transpose(1, 2), xc).to(ctx.dtypes[1]) if ctx.needs_input_grad[1] else None
        return dx, dtext, None, None


def contrastive_logits_hip(x, text, text_token_mask, max_text_len):
    if not supported(x, text, max_text_len):
        return kernels._contrastive_torch(x, text, text_token_mask, max_text_len)
    return ContrastiveFunction.apply(x, text, text_token_mask, max_text_len)


def contrastive_rowmax_hip(x, text, text_token_mask):
    if not supported(x, text, text.shape[1]):
        return contrastive_rowmax_torch(x, text, text_token_mask)
    xc, tc, keep = _prep(x.detach(), text.detach(), text_token_mask)
    out = torch.empty(x.shape[0], x.shape[1], dtype=torch.float32, device=x.device)
    _launch(xc, tc, keep, tc.shape[1], None, out)
    return out


def contrastive_rowmax_torch(x, text, text_token_mask):
    with torch.no_grad():
        return kernels._contrastive_torch(x, text, text_token_mask, text.shape[1]).max(-1)[0]


kernels.register("contrastive_logits", "hip", contrastive_logits_hip, default=True)
kernels.register("contrastive_rowmax", "torch", contrastive_rowmax_torch)
kernels.register("contrastive_rowmax", "hip", contrastive_rowmax_hip, default=True)
