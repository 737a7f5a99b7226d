"""BiMultiHeadAttention core on MI355X: one shared score GEMM + the fused
bidirectional softmax kernels of csrc/biattn.hip + two output GEMMs.

    s    = q . k^T                         [B, H, S, T]   (hipBLASLt, MFMA)
    P_v, P_l = gd_biattn_softmax_fwd(s)    row softmax over T / column
                                           softmax over S, one pass over s
    out_v = P_v . v_l                      [B, H, S, hd]  (hipBLASLt)
    out_l = P_l^T . v_v                    [B, H, T, hd]  (hipBLASLt)

Backward: the GEMM grads come from autograd; the softmax backward
dS = P_v (dP_v - rowsum(dP_v P_v)) + P_l (dP_l - colsum(dP_l P_l)) is one
fused kernel pass (gd_biattn_softmax_bwd).  Replaces the reference's
materialise -> global max -> clamp -> transpose -> column max -> clamp ->
mask -> softmax x2 chain (fuse_modules.py:174-217) and PyTorch SDPA, whose
256-query text-side call leaves most of the chip idle at head_dim 256.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, kernels, wgrad

_p, _i = ctypes.c_void_p, ctypes.c_int
_lib.register("gd_biattn_softmax_fwd", [_i, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p])
_lib.register("gd_biattn_softmax_bwd", [_i, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])


def _workspace(b, h, s, t, device):
    fn = _lib.lib().gd_biattn_workspace_bytes
    fn.restype = ctypes.c_size_t
    fn.argtypes = [_i, _i, _i, _i]
    n = int(fn(b, h, s, t))
    return torch.empty((n + 3) // 4, dtype=torch.float32, device=device)


def _u8(mask):
    if mask is None:
        return None
    return mask.contiguous().view(torch.uint8)


class BiSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, pad_v, pad_l):
        _lib.require_device(s, pad_v, pad_l, what="biattn")
        if s.dtype not in (torch.float32, torch.bfloat16):
            s = s.float()
        s = s.contiguous()
        b, h, n, t = s.shape
        pv = torch.empty_like(s)
        pl = torch.empty_like(s)
        ws = _workspace(b, h, n, t, s.device)
        mv, ml = _u8(pad_v), _u8(pad_l)
        _lib.call("gd_biattn_softmax_fwd", _lib.dtype_code(s), s.data_ptr(), _lib.ptr(mv), _lib.ptr(ml),
                  b, h, n, t, pv.data_ptr(), pl.data_ptr(), ws.data_ptr(), _lib.stream_of(s),
                  nbytes=3.0 * s.numel() * s.element_size())  # read S, write P_v and P_l
        ctx.save_for_backward(pv, pl)
        return pv, pl

    @staticmethod
    def backward(ctx, dpv, dpl):
        pv, pl = ctx.saved_tensors
        dpv = torch.zeros_like(pv) if dpv is None else dpv.to(pv.dtype).contiguous()
        dpl = torch.zeros_like(pl) if dpl is None else dpl.to(pl.dtype).contiguous()
        b, h, n, t = pv.shape
        ds = torch.empty_like(pv)
        ws = _workspace(b, h, n, t, pv.device)
        _lib.call("gd_biattn_softmax_bwd", _lib.dtype_code(pv), pv.data_ptr(), pl.data_ptr(), dpv.data_ptr(),
                  dpl.data_ptr(), b, h, n, t, ds.data_ptr(), ws.data_ptr(), _lib.stream_of(pv),
                  nbytes=5.0 * pv.numel() * pv.element_size())  # read P_v, P_l, dP_v, dP_l; write dS
        return ds, None, None


class _QKt(torch.autograd.Function):
    """s = q k^T; dk = dS^T q is the long-K (S image tokens) product."""

    @staticmethod
    def forward(ctx, q, k):
        ctx.save_for_backward(q, k)
        return torch.matmul(q, k.transpose(-1, -2))

    @staticmethod
    def backward(ctx, ds):
        q, k = ctx.saved_tensors
        ds = ds.to(q.dtype).contiguous()
        return torch.matmul(ds, k), wgrad.tn_matmul(ds, q.contiguous())


class _PV(torch.autograd.Function):
    """out_v = P_v v_l; dv_l = P_v^T dout_v is the long-K product."""

    @staticmethod
    def forward(ctx, pv, vl):
        ctx.save_for_backward(pv, vl)
        return torch.matmul(pv, vl)

    @staticmethod
    def backward(ctx, dout):
        pv, vl = ctx.saved_tensors
        dout = dout.to(pv.dtype).contiguous()
        return torch.matmul(dout, vl.transpose(-1, -2)), wgrad.tn_matmul(pv, dout)


class _PlTV(torch.autograd.Function):
    """out_l = P_l^T v_v (long-K forward); its gradients are ordinary GEMMs."""

    @staticmethod
    def forward(ctx, pl, vv):
        ctx.save_for_backward(pl, vv)
        return wgrad.tn_matmul(pl, vv.contiguous())

    @staticmethod
    def backward(ctx, dout):
        pl, vv = ctx.saved_tensors
        dout = dout.to(pl.dtype)
        return torch.matmul(vv, dout.transpose(-1, -2)), torch.matmul(pl, dout)


def _long_k_ok(q, k, v_v, v_l):
    """the three S-long products on the split-K kernel (gdino_amd/wgrad.py)"""
    return (q.dtype == k.dtype == v_v.dtype == v_l.dtype and wgrad.tn_eligible(q, q)
            and k.shape[-2] % 64 == 0 and q.shape[-1] % 64 == 0)


def bi_attention_hip(q, k, v_v, v_l, pad_v=None, pad_l=None, dropout_p=0.0):
    """Same contract as kernels._bi_attention_torch (q pre-scaled)."""
    if dropout_p > 0.0:
        # attention-probability dropout (fusion_dropout > 0) is not fused;
        # the SDPA composition implements it.
        return kernels._bi_attention_torch(q, k, v_v, v_l, pad_v, pad_l, dropout_p)
    if _long_k_ok(q, k, v_v, v_l):
        s = _QKt.apply(q, k)
        pv, pl = BiSoftmax.apply(s, pad_v, pad_l)
        return _PV.apply(pv, v_l), _PlTV.apply(pl, v_v)
    s = torch.matmul(q, k.transpose(-1, -2))
    pv, pl = BiSoftmax.apply(s, pad_v, pad_l)
    out_v = torch.matmul(pv.to(v_l.dtype) if pv.dtype != v_l.dtype else pv, v_l)
    out_l = torch.matmul(pl.transpose(-1, -2).to(v_v.dtype) if pl.dtype != v_v.dtype else pl.transpose(-1, -2),
                         v_v)
    return out_v, out_l


kernels.register("bi_attention", "hip", bi_attention_hip, default=True)
