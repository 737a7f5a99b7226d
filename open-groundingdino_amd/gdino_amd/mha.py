"""Multi-head attention with nn.MultiheadAttention's parameter layout
(``in_proj_weight``, ``in_proj_bias``, ``out_proj``) and call contract
(sequence-first by default, bool masks True = "not allowed", float masks
additive, ``attn_mask`` [L, S] or [B*H, L, S] in batch-major (b*H + h) order,
``key_padding_mask`` [B, S] True = pad), whose core runs through
``gdino_amd.kernels.attention``.  Used where the reference instantiates
nn.MultiheadAttention on the hot path: the text enhancer
(transformer_vanilla.py:83) and the decoder self / text-cross attention
(transformer.py:839,844).  Returns (output, None): attention weights are never
requested on the hot path."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from . import castcache
from .misc import inverted, mask_cache_key, split_last
from .wgrad import _dx


def merge_masks(attn_mask: Optional[Tensor], key_padding_mask: Optional[Tensor], b: int, h: int,
                lq: int, lk: int, dtype) -> Optional[Tensor]:
    """-> bool keep-mask or float additive mask broadcastable to [B, H, Lq, Lk]."""
    if attn_mask is None and key_padding_mask is None:
        return None
    def am_view(m):
        return m.view(1, 1, lq, lk) if m.dim() == 2 else (m.view(b, h, lq, lk) if m.dim() == 3 else m)
    am = None if attn_mask is None else am_view(attn_mask)
    kp = None if key_padding_mask is None else key_padding_mask.view(b, 1, 1, lk)
    if all(m is None or m.dtype == torch.bool for m in (am, kp)):
        # bool masks: the inversions and their AND once per mask objects and
        # step (the layers pass the same masks; misc.inverted caches on them)
        if am is None:
            return inverted(key_padding_mask).view(b, 1, 1, lk)
        if kp is None:
            return am_view(inverted(attn_mask))
        key = mask_cache_key(attn_mask, key_padding_mask) + (b, h, lq, lk)
        c = getattr(attn_mask, "_gd_merged", None)
        if c is not None and c[0] is key_padding_mask and c[1] == key:
            return c[2]
        keep = am_view(inverted(attn_mask)) & inverted(key_padding_mask).view(b, 1, 1, lk)
        attn_mask._gd_merged = (key_padding_mask, key, keep)
        return keep
    add = torch.zeros((), dtype=dtype, device=(am if am is not None else kp).device)
    for m in (am, kp):
        if m is None:
            continue
        if m.dtype == torch.bool:
            add = add + torch.zeros_like(m, dtype=dtype).masked_fill(m, float("-inf"))
        else:
            add = add + m.to(dtype)
    return add


PACKED_INPROJ = True


def _low(x, dt):
    """x in dtype dt: the bf16 twin written beside x by its producer when it
    is current (misc.add_with_twins, layernorm), else a cast."""
    if x.dtype == dt:
        return x
    tw = getattr(x, "_gd_bf16", None)
    if tw is not None and tw[1] == x._version and tw[0].dtype == dt and tw[0].shape == x.shape:
        return tw[0]
    return x.to(dt)


class _PackedInProj(torch.autograd.Function):
    """Two row blocks of a packed projection: ya = xa W[:split]^T + b[:split],
    yb = xb W[split:]^T + b[split:].  Same GEMMs as two F.linear calls on
    weight slices; the backward fills one packed dW / db with mm(out=) /
    sum(out=) instead of autograd's zero-filled slice gradients + add."""

    @staticmethod
    def forward(ctx, w, b, xa, xb, split):
        # xa / xb in their own dtype (the decoder's fp32 stream): the
        # low-precision copy is the bf16 twin a producer wrote beside the
        # tensor (misc.add_with_twins) or a cast here, and the backward
        # writes dX in x's dtype straight from the GEMM (wgrad._dx) -- no
        # cast kernel and no ToCopy backward per input
        ctx.x_dtypes = (xa.dtype, xb.dtype)
        xa, xb = _low(xa, w.dtype), _low(xb, w.dtype)
        ctx.save_for_backward(w, xa, xb)
        ctx.split = split
        return castcache.linear2d(xa, w[:split], b[:split]), castcache.linear2d(xb, w[split:], b[split:])

    @staticmethod
    def backward(ctx, dya, dyb):
        w, xa, xb = ctx.saved_tensors
        sp = ctx.split
        e = w.shape[1]
        if dya is None:
            dya = torch.zeros(*xa.shape[:-1], sp, dtype=w.dtype, device=w.device)
        if dyb is None:
            dyb = torch.zeros(*xb.shape[:-1], w.shape[0] - sp, dtype=w.dtype, device=w.device)
        ga, gb = dya.reshape(-1, sp), dyb.reshape(-1, w.shape[0] - sp)
        dxa = _dx(ga, w[:sp], ctx.x_dtypes[0]).view(xa.shape) if ctx.needs_input_grad[2] else None
        dxb = _dx(gb, w[sp:], ctx.x_dtypes[1]).view(xb.shape) if ctx.needs_input_grad[3] else None
        dw = db = None
        if ctx.needs_input_grad[0]:
            dw = torch.empty_like(w)
            torch.mm(ga.t(), xa.reshape(-1, e), out=dw[:sp])
            torch.mm(gb.t(), xb.reshape(-1, e), out=dw[sp:])
        if ctx.needs_input_grad[1]:
            db = torch.empty(w.shape[0], dtype=w.dtype, device=w.device)
            torch.sum(ga, 0, out=db[:sp])
            torch.sum(gb, 0, out=db[sp:])
        return dw, db, dxa, dxb, None


class MultiheadAttention(nn.Module):
    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=True, batch_first=False):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        assert self.head_dim * num_heads == embed_dim, "embed_dim must be divisible by num_heads"
        self.dropout = dropout
        self.batch_first = batch_first
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim)) if bias else None
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=bias)
        self._reset_parameters()

    def _reset_parameters(self):
        nn.init.xavier_uniform_(self.in_proj_weight)
        if self.in_proj_bias is not None:
            nn.init.constant_(self.in_proj_bias, 0.0)
            nn.init.constant_(self.out_proj.bias, 0.0)

    def _project(self, query, key, value):
        """q/k/v in-projections (nn.MultiheadAttention's in_proj layout).
        Inputs that are the same tensor share one GEMM: q = k = x + pos in
        the text enhancer and decoder self-attention, k = v = text in the
        decoder's text cross-attention.  Under autocast the packed weight is
        cast once per step (castcache) and the two GEMMs run in
        _PackedInProj, whose backward writes the packed [3E, E] gradient
        directly (no zero-filled gradient per weight slice)."""
        e = self.embed_dim
        w, bias = self.in_proj_weight, self.in_proj_bias
        if query is key and key is value:
            return split_last(castcache.linear(query, w, bias), (e, e, e))
        dt = castcache.autocast_dtype(query)
        if dt is not None:
            w = castcache.cached_cast(w, dt)
            bias = None if bias is None else castcache.cached_cast(bias, dt)
            if bias is not None and PACKED_INPROJ and (query is key or key is value):
                split = 2 * e if query is key else e
                xa, xb = (query, value) if query is key else (query, key)
                ya, yb = _PackedInProj.apply(w, bias, xa, xb, split)
                if query is key:
                    q, k = split_last(ya, (e, e))
                    return q, k, yb
                k, v = split_last(yb, (e, e))
                return ya, k, v

        def lin(x, r0, r1):
            return castcache.linear2d(x, w[r0:r1], None if bias is None else bias[r0:r1])

        if query is key:
            q, k = split_last(lin(query, 0, 2 * e), (e, e))
            return q, k, lin(value, 2 * e, 3 * e)
        if key is value:
            k, v = split_last(lin(key, e, 3 * e), (e, e))
            return lin(query, 0, e), k, v
        return lin(query, 0, e), lin(key, e, 2 * e), lin(value, 2 * e, 3 * e)

    def forward(self, query, key, value, key_padding_mask=None, need_weights=False, attn_mask=None,
                average_attn_weights=True, is_causal=False):
        from . import kernels
        if self.batch_first:
            query, key, value = (x.transpose(0, 1) for x in (query, key, value))
        lq, b, e = query.shape
        lk = key.shape[0]
        q, k, v = self._project(query, key, value)
        h, hd = self.num_heads, self.head_dim
        # [L, B, E] -> [B, H, L, hd]
        q = q.view(lq, b, h, hd).permute(1, 2, 0, 3)
        k = k.view(lk, b, h, hd).permute(1, 2, 0, 3)
        v = v.view(lk, b, h, hd).permute(1, 2, 0, 3)
        mask = merge_masks(attn_mask, key_padding_mask, b, h, lq, lk, q.dtype)
        out = kernels.attention(q, k, v, mask, None, self.dropout if self.training else 0.0)
        out = out.permute(2, 0, 1, 3).reshape(lq, b, e)
        out = self.out_proj(out)
        if self.batch_first:
            out = out.transpose(0, 1)
        return out, None
