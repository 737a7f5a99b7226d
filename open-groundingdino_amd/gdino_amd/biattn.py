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


def _softmax_fwd(s, pad_v, pad_l):
    b, h, n, t = s.shape
    pv = torch.empty_like(s)
    pl = torch.empty_like(s)
    ws = _workspace(b, h, n, t, s.device)
    mv, ml = _u8(pad_v), _u8(pad_l)
    _lib.call("gd_biattn_softmax_fwd", _lib.dtype_code(s), s.data_ptr(), _lib.ptr(mv), _lib.ptr(ml),
              b, h, n, t, pv.data_ptr(), pl.data_ptr(), ws.data_ptr(), _lib.stream_of(s),
              nbytes=3.0 * s.numel() * s.element_size())  # read S, write P_v and P_l
    return pv, pl


def _softmax_bwd(pv, pl, dpv, dpl):
    b, h, n, t = pv.shape
    ds = torch.empty_like(pv)
    ws = _workspace(b, h, n, t, pv.device)
    _lib.call("gd_biattn_softmax_bwd", _lib.dtype_code(pv), pv.data_ptr(), pl.data_ptr(), dpv.data_ptr(),
              dpl.data_ptr(), b, h, n, t, ds.data_ptr(), ws.data_ptr(), _lib.stream_of(pv),
              nbytes=5.0 * pv.numel() * pv.element_size())  # read P_v, P_l, dP_v, dP_l; write dS
    return ds


def _hv(x2, nh):
    """[L, E] token rows (any row stride, unit channel stride) -> the [nh, L, hd]
    per-head view (strides hd, row stride, 1): what the library's strided
    batched GEMM reads in place."""
    return x2.unflatten(-1, (nh, x2.shape[-1] // nh)).transpose(0, 1)


def _tn_ok(a, b, o, i) -> bool:
    """What gd_wgrad_batched accepts: o and i multiples of 16 (bf16) / 64
    (fp32), unit channel stride, 16-B aligned rows and bases.  o is the text
    length T when a is P_l / P_v / dS: captions pad to the longest in the
    batch (groundingdino.py:56), so T is often not a multiple of 16."""
    gran = 16 if a.dtype == torch.bfloat16 else 64
    align = 16 // a.element_size()
    return (a.dtype == b.dtype and a.dtype in (torch.float32, torch.bfloat16) and o % gran == 0 and i % gran == 0
            and all(x.stride(-1) == 1 and x.stride(1) % align == 0 and x.stride(0) % align == 0
                    and x.data_ptr() % 16 == 0 for x in (a, b)))


def _tn(a, b, out):
    """out[h] = a[h]^T b[h] for [nh, L, o] / [nh, L, i] views contracting
    over the L image tokens (the long-K products): the split-K kernel of
    csrc/wgrad.hip reading both operands through their strides, or the
    library GEMM below its token threshold."""
    nh, t, o = a.shape
    i = b.shape[-1]
    if t >= wgrad.TN_MIN_TOKENS and _lib.enabled("wgrad") and _tn_ok(a, b, o, i):
        s = int(_lib.lib().gd_wgrad_splits_batched(t, o, i, nh))
        ws = wgrad._workspace(o, i, s * nh, a.device)
        _lib.call("gd_wgrad_batched", _lib.dtype_code(a), a.data_ptr(), a.stride(1), a.stride(0), b.data_ptr(),
                  b.stride(1), b.stride(0), t, o, i, nh, s, ws.data_ptr(), _lib.dtype_code(out), out.data_ptr(),
                  out.stride(0), None, _lib.stream_of(a), flops=2.0 * nh * t * o * i)
    else:
        torch.bmm(a.transpose(1, 2), b, out=out)


class BiAttnTokens(torch.autograd.Function):
    """The BiMultiHeadAttention core on token-major operands (reference
    fuse_modules.py:162-232, from the projections to the output reshape):
    qvv [B, S, 2E] = (q | v_v) and klv [B, T, 2E] = (k | v_l), the joint
    outputs of the shared-input projections (E = nh * hd), read in place ->
    out_v [B, S, E], out_l [B, T, E].  ``scale`` multiplies k (256 text
    tokens) instead of q (22 223 image tokens); for a power-of-two scale
    (hd = 256: 1/16) that is exact in any dtype.  Per image the head split is
    a strided batched GEMM view (batch stride hd, row stride 2E), not a copy,
    and the gradients of (q | v_v) and (k | v_l) are written into one tensor
    each: the [B, H, S, hd] transposes of q / v_v / out_v and their
    gradients, the q scaling pass and the split backward's concatenation
    (about 1 GB of copies per fusion layer and step) are gone.  The scores,
    P_v and P_l are the [B, H, S, T] tensors of gd_biattn_softmax_fwd / _bwd."""

    @staticmethod
    def forward(ctx, qvv, klv, pad_v, pad_l, nh, scale):
        B, S, E2 = qvv.shape
        E, T = E2 // 2, klv.shape[1]
        hd = E // nh
        q, vv = qvv[..., :E], qvv[..., E:]
        k, vl = (klv[..., :E] * scale).contiguous(), klv[..., E:]
        s = torch.empty(B, nh, S, T, dtype=qvv.dtype, device=qvv.device)
        for b in range(B):
            torch.bmm(_hv(q[b], nh), _hv(k[b], nh).transpose(1, 2), out=s[b])
        pv, pl = _softmax_fwd(s, pad_v, pad_l)
        del s
        out_v = torch.empty(B, S, E, dtype=qvv.dtype, device=qvv.device)
        out_l = torch.empty(B, nh, T, hd, dtype=qvv.dtype, device=qvv.device)
        for b in range(B):
            torch.bmm(pv[b], _hv(vl[b], nh), out=_hv(out_v[b], nh))
            _tn(pl[b], _hv(vv[b], nh), out_l[b])
        ctx.save_for_backward(qvv, k, vl, pv, pl)
        ctx.nh, ctx.scale = nh, scale
        return out_v, out_l.transpose(1, 2).reshape(B, T, E)

    @staticmethod
    def backward(ctx, dout_v, dout_l):
        qvv, k, vl, pv, pl = ctx.saved_tensors
        nh = ctx.nh
        B, S, E2 = qvv.shape
        E, T = E2 // 2, k.shape[1]
        hd = E // nh
        q, vv = qvv[..., :E], qvv[..., E:]
        dt = qvv.dtype
        dout_v = torch.zeros(B, S, E, dtype=dt, device=qvv.device) if dout_v is None else dout_v.to(dt)
        dout_l = torch.zeros(B, T, E, dtype=dt, device=qvv.device) if dout_l is None else dout_l.to(dt)
        if dout_v.stride(-1) != 1 or dout_v.stride(-2) % 8 or dout_v.data_ptr() % 16:
            dout_v = dout_v.contiguous()
        dout_l = dout_l.contiguous()
        dpv = torch.empty_like(pv)
        dpl = torch.empty_like(pl)
        for b in range(B):
            torch.bmm(_hv(dout_v[b], nh), _hv(vl[b], nh).transpose(1, 2), out=dpv[b])
            torch.bmm(_hv(vv[b], nh), _hv(dout_l[b], nh).transpose(1, 2), out=dpl[b])
        ds = _softmax_bwd(pv, pl, dpv, dpl)
        del dpv, dpl
        dqvv = torch.empty(B, S, E2, dtype=dt, device=qvv.device)
        dk = torch.empty(B, nh, T, hd, dtype=dt, device=qvv.device)
        dvl = torch.empty(B, nh, T, hd, dtype=dt, device=qvv.device)
        for b in range(B):
            torch.bmm(ds[b], _hv(k[b], nh), out=_hv(dqvv[b, :, :E], nh))   # dq = dS k
            torch.bmm(pl[b], _hv(dout_l[b], nh), out=_hv(dqvv[b, :, E:], nh))  # dv_v = P_l dout_l
            _tn(ds[b], _hv(q[b], nh), dk[b])            # dk = dS^T q
            _tn(pv[b], _hv(dout_v[b], nh), dvl[b])      # dv_l = P_v^T dout_v
        dklv = torch.cat([dk.transpose(1, 2).reshape(B, T, E) * ctx.scale, dvl.transpose(1, 2).reshape(B, T, E)],
                         -1)
        return dqvv, dklv, None, None, None, None


def _tunableop_tuning() -> bool:
    t = getattr(torch.cuda, "tunable", None)
    try:
        return bool(t is not None and t.is_enabled() and t.tuning_is_enabled())
    except (RuntimeError, AttributeError):
        return False


def tokens_ok(qvv, klv, nh) -> bool:
    """Token-major core applicable: ROCm device, one dtype (fp32 / bf16), the
    joint projection outputs [B, L, 2E] with unit channel stride and 16-B
    aligned rows, hd a multiple of 16 (bf16) / 64 (fp32)."""
    if qvv is None or klv is None:
        return False
    if _tunableop_tuning():
        # PyTorch TunableOp, while TUNING, runs each candidate GEMM on copies
        # of the operands sized max(stride * batch, m * k * batch) elements
        # (GemmStridedBatchedParams::GetSizeA/B, ATen/cuda/tunable/
        # GemmCommon.h): it assumes non-overlapping batches.  The per-head
        # views below have batch stride hd = 256 < row stride 2E, so their
        # true extent is ~2x that -- the candidates read past the copies
        # (the round-3 hipErrorIllegalAddress of tools/tune_gemms.py).  While
        # tuning, take the head-major path (contiguous per-head operands).
        return False
    ts = (qvv, klv)
    if not (all(_lib.on_device(t) for t in ts) and qvv.dtype == klv.dtype
            and qvv.dtype in (torch.float32, torch.bfloat16) and kernels.IMPL.get("bi_attention") == "hip"):
        return False
    e2 = qvv.shape[-1]
    gran = 16 if qvv.dtype == torch.bfloat16 else 64
    align = 8 if qvv.dtype == torch.bfloat16 else 4
    return (e2 % 2 == 0 and (e2 // 2) % nh == 0 and (e2 // 2 // nh) % gran == 0 and klv.shape[-1] == e2
            and all(t.dim() == 3 and t.stride(-1) == 1 and t.stride(-2) % align == 0 and t.data_ptr() % 16 == 0
                    for t in ts))


def bi_attention_tokens(qvv, klv, pad_v, pad_l, nh, scale):
    """(out_v, out_l) of the BiMultiHeadAttention core from the joint
    projection outputs (q | v_v), (k | v_l); q unscaled, ``scale`` applied
    to k."""
    _lib.require_device(qvv, klv, pad_v, pad_l, what="biattn")
    return BiAttnTokens.apply(qvv, klv, pad_v, pad_l, nh, float(scale))


kernels.register("bi_attention", "hip", bi_attention_hip, default=True)
