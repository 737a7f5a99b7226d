"""Masked multi-head attention core on MI355X: csrc/attn.hip (flash-style
MFMA kernels) through the C-ABI.

Backs ``kernels.attention(q, k, v, attn_mask, scale, dropout_p)`` for the
attention cores of the hot path:
  * BERT self-attention (bertwarper.py:31-166 via transformers'
    attention interface; T = 256, head_dim 64, block-diagonal phrase masks);
  * the text enhancer's self-attention (transformer_vanilla.py:83);
  * the decoder's self-attention and text cross-attention
    (transformer.py:839,844; 900 queries, head_dim 32).
The [B, H, Lq, Lk] score / probability tensors never reach HBM: per 64-query
block the softmax statistics live in registers and only lse [B, H, Lq] is
saved for the backward.

q [B, H, Lq, hd], k / v [B, H, Lk, hd] are read in place through their
(b, h, l) strides (the projections' permuted views; channels contiguous);
attn_mask is a bool keep-mask (True = attend) or an additive float mask
broadcastable to [B, H, Lq, Lk].  The output is stored [B, Lq, H, hd] (what
BERT's and the MHA's output projections read) and returned as the
[B, H, Lq, hd] view.  The kernels cover head_dim 32 / 64 in fp32 and bf16,
with attention-probability dropout (BERT's attention dropout 0.1 in training)
drawn from a counter-based hash of (seed, b*H+h, q, k) that the backward
regenerates -- the same distribution as torch's dropout, not its RNG stream.
The seed is a 1-element device tensor drawn by torch's CUDA generator and
read by the kernels from memory, so a captured step graph draws a new mask
per replay (a host seed would be frozen into the graph).
Anything else uses PyTorch SDPA (ROCm flash / mem-efficient kernels).  CPU
tensors raise.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F

from . import _lib, kernels

_p, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
_u32 = ctypes.c_uint32
_lib.register("gd_attn_forward", [_i] * 6 + [_p] * 7 + [_i, _p, _f, _f, _u32, _p, _p, _p, _p])
_lib.register("gd_attn_backward", [_i] * 6 + [_p] * 7 + [_i, _p, _f, _f, _u32] + [_p] * 13)
_lib.register("gd_attn_forward_dev", [_i] * 6 + [_p] * 7 + [_i, _p, _f, _f, _u32, _p, _p, _p, _p, _p])
_lib.register("gd_attn_backward_dev", [_i] * 6 + [_p] * 7 + [_i, _p, _f, _f, _u32, _p] + [_p] * 13)


def _st3(t):
    return (ctypes.c_int64 * 3)(*t.stride()[:3])


def _rows(t):
    """channels contiguous and rows 16-byte aligned (else a contiguous copy)"""
    align = 16 // t.element_size()
    if t.stride(-1) != 1 or any(s % align for s in t.stride()[:3]) or t.data_ptr() % 16:
        t = t.contiguous()
    return t


def _mask_args(mask, b, h, lq, lk):
    """-> (tensor kept alive for the call, kind, (b, h, q) strides)"""
    if mask is None:
        return None, 0, None
    m = mask if mask.dtype == torch.bool else mask.float()
    while m.dim() < 4:
        m = m.unsqueeze(0)
    m = m.expand(b, h, lq, lk)
    if m.stride(-1) != 1:
        m = m.contiguous()
    if m.dtype == torch.bool:
        m, kind = m.view(torch.uint8), 1
    else:
        kind = 2
    return m, kind, (ctypes.c_int64 * 3)(*m.stride()[:3])


def supported(q, k, v, dropout_p) -> bool:
    hd = q.shape[-1]
    return (_lib.enabled("attn") and 0.0 <= dropout_p < 1.0 and q.dtype in (torch.float32, torch.bfloat16) and q.dtype == k.dtype == v.dtype
            and hd in (32, 64) and k.shape[-1] == hd and v.shape[-1] == hd and q.shape[2] > 0 and k.shape[2] > 0
            and q.shape[0] * q.shape[1] < 65536)


class AttnFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, mask, scale, dropout_p=0.0, seed=None):
        """seed: None, or a 1-element int32 device tensor -- the dropout mask
        seed, read by the kernels from device memory (graph-safe: a captured
        step refills it every replay; the backward reads the same word)."""
        _lib.require_device(q, k, v, mask, what="attention")
        q, k, v = _rows(q), _rows(k), _rows(v)
        b, h, lq, hd = q.shape
        lk = k.shape[2]
        m, kind, ms = _mask_args(mask, b, h, lq, lk)
        out = torch.empty(b, lq, h, hd, dtype=q.dtype, device=q.device).transpose(1, 2)
        lse = torch.empty(b, h, lq, dtype=torch.float32, device=q.device)
        _lib.call("gd_attn_forward_dev", _lib.dtype_code(q), b, h, lq, lk, hd, q.data_ptr(), _st3(q), k.data_ptr(),
                  _st3(k), v.data_ptr(), _st3(v), _lib.ptr(m), kind, ms, float(scale), float(dropout_p), 0,
                  _lib.ptr(seed), out.data_ptr(), _st3(out), lse.data_ptr(), _lib.stream_of(q),
                  flops=4.0 * b * h * lq * lk * hd)  # S = QK^T, O = PV
        ctx.save_for_backward(q, k, v, m, out, lse, seed)
        ctx.kind, ctx.ms, ctx.scale = kind, tuple(ms) if ms is not None else None, float(scale)
        ctx.dropout_p = float(dropout_p)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, m, out, lse, seed = ctx.saved_tensors
        b, h, lq, hd = q.shape
        lk = k.shape[2]
        dout = _rows(dout.to(q.dtype))
        ms = None if ctx.ms is None else (ctypes.c_int64 * 3)(*ctx.ms)
        dsum = torch.empty(b, h, lq, dtype=torch.float32, device=q.device)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        dq, dk, dv = _rows(dq), _rows(dk), _rows(dv)
        _lib.call("gd_attn_backward_dev", _lib.dtype_code(q), b, h, lq, lk, hd, q.data_ptr(), _st3(q),
                  k.data_ptr(), _st3(k), v.data_ptr(), _st3(v), _lib.ptr(m), ctx.kind, ms, ctx.scale, ctx.dropout_p,
                  0, _lib.ptr(seed), out.data_ptr(), _st3(out), dout.data_ptr(), _st3(dout), lse.data_ptr(),
                  dsum.data_ptr(), dq.data_ptr(), _st3(dq), dk.data_ptr(), _st3(dk), dv.data_ptr(), _st3(dv),
                  _lib.stream_of(q), flops=10.0 * b * h * lq * lk * hd)  # S recompute, dP, dV, dQ, dK (2.5x fwd)
        return dq, dk, dv, None, None, None, None


def attention_hip(q, k, v, attn_mask=None, scale=None, dropout_p=0.0):
    """Same contract as kernels._attention_torch."""
    if not supported(q, k, v, dropout_p):
        return F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask, dropout_p=dropout_p, scale=scale)
    scale = q.shape[-1] ** -0.5 if scale is None else scale
    if dropout_p > 0.0:
        # the mask seed drawn on the device by torch's generator (graph-safe:
        # inside a captured step each replay draws a new one) and read by the
        # kernels from memory; torch.manual_seed reproduces it
        seed = torch.randint(0, 2 ** 31 - 1, (1,), dtype=torch.int32, device=q.device)
        return AttnFunction.apply(q, k, v, attn_mask, scale, dropout_p, seed)
    return AttnFunction.apply(q, k, v, attn_mask, scale)


kernels.register("attention", "hip", attention_hip, default=True)
