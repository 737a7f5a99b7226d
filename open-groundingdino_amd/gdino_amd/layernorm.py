"""Residual add + LayerNorm on MI355X (csrc/layernorm.hip).

``add_norm(norm, x, r)`` = ``norm(x + r)`` for an nn.LayerNorm ``norm``: the
post-norm sublayer ending of the deformable encoder / decoder layers and the
text enhancer (reference transformer.py:789-808, 877-936,
transformer_vanilla.py:83-110).  On the GPU it is one kernel forward (the add,
the row statistics and the affine output in fp32, as autocast's fp32
LayerNorm) and one kernel + a column reduction backward (the input gradient
written once for the residual in x's dtype and once for the sublayer in r's
dtype, gamma / beta gradients in fp32).  Elsewhere (CPU, other widths) it is
the plain composition.
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from . import _lib

_p, _i, _i64, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
_lib.register("gd_add_layernorm_forward", [_i, _p, _i, _p, _p, _p, _i64, _i, _f, _p, _p, _p, _p])
_lib.register("gd_add_layernorm_forward2", [_i, _p, _i, _p, _p, _p, _i64, _i, _f, _p, _p, _p, _p, _p])


def _bf16_twin_wanted(x, wanted: bool = True) -> bool:
    """Under bf16 autocast the fp32 LayerNorm output is cast again by every
    GEMM that reads it; the forward kernel writes that bf16 copy itself
    (``y._gd_bf16``, read by wgrad.TokenLinear) for one extra 2-byte store
    per element instead of a cast kernel per consumer."""
    return (wanted and TWIN and x.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16)


TWIN = True
_lib.register("gd_add_layernorm_backward", [_i, _p, _i, _p, _p, _p, _p, _p, _i64, _i, _p, _p, _p, _p, _p, _p])
_lib.register("gd_add_layernorm_backward2", [_i, _p, _i, _p, _p, _p, _p, _p, _p, _i64, _i, _p, _p, _p, _p, _p, _p])

WIDTHS = (64, 96, 128, 192, 256, 384, 512, 768, 1024, 1536, 2048)
ENABLED = True


def supported(norm: nn.LayerNorm, x: torch.Tensor, r) -> bool:
    c = x.shape[-1]
    return (ENABLED and _lib.enabled("addln") and _lib.on_device(x) and len(norm.normalized_shape) == 1
            and norm.normalized_shape[0] == c and c in WIDTHS and norm.elementwise_affine and norm.weight is not None and norm.bias is not None
            and norm.weight.dtype == torch.float32 and norm.bias.dtype == torch.float32
            and x.dtype in (torch.float32, torch.bfloat16)
            and (r is None or (r.dtype in (torch.float32, torch.bfloat16) and x.shape == r.shape)))


def _workspace(c, device):
    fn = _lib.lib().gd_add_layernorm_workspace_bytes
    fn.restype, fn.argtypes = ctypes.c_size_t, [_i]
    return torch.empty((int(fn(c)) + 3) // 4, dtype=torch.float32, device=device)


def _with_taps(y, y16, taps):
    """y, or (y, a view of y) for an output read by two consumers: autograd
    then hands the two gradients to the backward separately, whose kernel
    sums them (no accumulation add).  Both carry the bf16 twin."""
    if y16 is not None:
        y._gd_bf16 = (y16, y._version)  # stale once y is modified in place
    if taps == 1:
        return y
    t = y.view(y.shape)
    if y16 is not None:
        t._gd_bf16 = (y16, t._version)
    return y, t


class AddLayerNormFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, weight, bias, eps, twin=True, taps=1):
        c = x.shape[-1]
        rows = x.numel() // c
        y = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        rd = x if r is None else r  # r None: LayerNorm(x) alone (NULL residual)
        y16 = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if _bf16_twin_wanted(x, twin) else None
        _lib.call("gd_add_layernorm_forward2", _lib.dtype_code(x), x.data_ptr(), _lib.dtype_code(rd), _lib.ptr(r),
                  weight.data_ptr(), bias.data_ptr(), rows, c, float(eps), y.data_ptr(), _lib.ptr(y16),
                  mean.data_ptr(), rstd.data_ptr(), _lib.stream_of(x),
                  nbytes=rows * (c * (x.element_size() + (0 if r is None else r.element_size()) + 4
                                      + (0 if y16 is None else 2)) + 8))
        ctx.save_for_backward(x, r, weight, mean, rstd)
        return _with_taps(y, y16, taps)

    @staticmethod
    def backward(ctx, dy, dy2=None):
        x, r, weight, mean, rstd = ctx.saved_tensors
        c = x.shape[-1]
        rows = x.numel() // c
        if dy is None:
            dy, dy2 = dy2, None
        dy = dy.float().contiguous()
        dy2 = None if dy2 is None else dy2.float().contiguous()
        dx = torch.empty_like(x)
        dr = torch.empty_like(r) if r is not None and ctx.needs_input_grad[1] else None
        want_wb = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        dw = torch.empty(c, dtype=torch.float32, device=x.device) if want_wb else None
        db = torch.empty(c, dtype=torch.float32, device=x.device) if want_wb else None
        ws = _workspace(c, x.device) if want_wb else None
        _lib.call("gd_add_layernorm_backward2", _lib.dtype_code(x), x.data_ptr(),
                  _lib.dtype_code(x if r is None else r), _lib.ptr(r), weight.data_ptr(), dy.data_ptr(), _lib.ptr(dy2),
                  mean.data_ptr(), rstd.data_ptr(), rows, c, dx.data_ptr(),
                  _lib.ptr(dr), _lib.ptr(dw), _lib.ptr(db), _lib.ptr(ws), _lib.stream_of(x),
                  nbytes=rows * (c * (2 * x.element_size() + (0 if r is None else r.element_size()) + 4
                                      + (r.element_size() if dr is not None else 0)) + 8))
        return (dx if ctx.needs_input_grad[0] else None, dr, dw if ctx.needs_input_grad[2] else None,
                db if ctx.needs_input_grad[3] else None, None, None, None)


_u32 = ctypes.c_uint32
_lib.register("gd_add_layernorm3_forward", [_p, _p, _p, _p, _p, _i64, _i, _f, _f, _u32, _p, _p, _p, _p, _p, _p])
_lib.register("gd_add_layernorm3_backward", [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _f, _u32, _p, _p, _p, _p,
                                              _p, _p, _p])


class AddLayerNorm3Function(torch.autograd.Function):
    """y = LayerNorm(x + (r + dropout_p(r2))): x, r fp32, r2 bf16, C = 256
    (csrc/layernorm.hip addln3_*).  seed: None (p = 0) or a 1-element int32
    device tensor the kernels read (a captured step draws a new mask per
    replay); the backward regenerates the mask from it."""

    @staticmethod
    def forward(ctx, x, r, r2, weight, bias, eps, p, seed, twin=True, taps=1):
        rows = x.numel() // 256
        y = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        y16 = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if _bf16_twin_wanted(x, twin) else None
        _lib.call("gd_add_layernorm3_forward", x.data_ptr(), r.data_ptr(), r2.data_ptr(), weight.data_ptr(),
                  bias.data_ptr(), rows, 256, float(eps), float(p), 0, _lib.ptr(seed), y.data_ptr(), _lib.ptr(y16),
                  mean.data_ptr(), rstd.data_ptr(), _lib.stream_of(x),
                  nbytes=rows * (256 * (4 + 4 + 2 + 4 + (0 if y16 is None else 2)) + 8))
        ctx.save_for_backward(x, r, r2, weight, mean, rstd, seed)
        ctx.p = float(p)
        return _with_taps(y, y16, taps)

    @staticmethod
    def backward(ctx, dy, dy2=None):
        x, r, r2, weight, mean, rstd, seed = ctx.saved_tensors
        rows = x.numel() // 256
        if dy is None:
            dy, dy2 = dy2, None
        dy = dy.float().contiguous()
        dy2 = None if dy2 is None else dy2.float().contiguous()
        dx = torch.empty_like(x)
        dr2 = torch.empty_like(r2) if ctx.needs_input_grad[2] else None
        dw = torch.empty(256, dtype=torch.float32, device=x.device)
        db = torch.empty(256, dtype=torch.float32, device=x.device)
        ws = _workspace(256, x.device)
        _lib.call("gd_add_layernorm3_backward", x.data_ptr(), r.data_ptr(), r2.data_ptr(), weight.data_ptr(),
                  dy.data_ptr(), _lib.ptr(dy2), mean.data_ptr(), rstd.data_ptr(), rows, 256, ctx.p, 0, _lib.ptr(seed),
                  dx.data_ptr(), _lib.ptr(dr2), dw.data_ptr(), db.data_ptr(), ws.data_ptr(), _lib.stream_of(x),
                  nbytes=rows * (256 * (4 + 4 + 4 + 2 + 4 + (2 if dr2 is not None else 0)) + 8))
        # x and r receive the same gradient (one tensor: autograd never
        # accumulates into a gradient it does not own alone)
        return (dx if ctx.needs_input_grad[0] else None, dx if ctx.needs_input_grad[1] else None, dr2,
                dw if ctx.needs_input_grad[3] else None, db if ctx.needs_input_grad[4] else None, None, None, None,
                None, None)


def add_norm3(norm: nn.LayerNorm, x: torch.Tensor, r: torch.Tensor, r2: torch.Tensor, dropout: nn.Module,
              bf16_twin: bool = True, taps: int = 1):
    """norm(x + (r + dropout(r2))): the deformable layers' attention sublayer
    with the MSDA module's identity add and output dropout folded in (one
    kernel each way instead of dropout, a mixed bf16 + fp32 add and
    add + LayerNorm).  x, r fp32 [..., 256], r2 bf16 of the same shape,
    ``dropout`` an nn.Dropout (its rate and mode) or nn.Identity; None when
    not applicable (the caller runs the composition).  taps=2 as in add_norm."""
    p = float(getattr(dropout, "p", 0.0)) if dropout.training else 0.0
    if not (supported(norm, x, r) and x.shape[-1] == 256 and x.dtype == r.dtype == torch.float32
            and r2.dtype == torch.bfloat16 and r2.shape == x.shape and (p == 0.0 or isinstance(dropout, nn.Dropout))
            and 0.0 <= p < 1.0):
        return None
    seed = torch.randint(0, 2 ** 31 - 1, (1,), dtype=torch.int32, device=x.device) if p > 0 else None
    return AddLayerNorm3Function.apply(x.contiguous(), r.contiguous(), r2.contiguous(), norm.weight, norm.bias,
                                       norm.eps, p, seed, bool(bf16_twin), int(taps))


_lib.register("gd_add_scaled_layernorm_forward", [_p, _i, _p, _p, _i64, _i, _p, _p, _i64, _i, _f, _p, _p, _p, _p,
                                                   _p, _p])
_lib.register("gd_add_scaled_layernorm_backward", [_p, _p, _p, _i, _p, _i64, _i, _p, _p, _p, _i64, _i, _p, _p, _p,
                                                    _p, _p, _p])
SLN_WIDTHS = (96, 192, 256, 384, 768)


class AddScaledNormFunction(torch.autograd.Function):
    """(sum, y) = (x + branch * scale, LayerNorm(x + branch * scale)) with a
    per-sample (or single) fp32 scale that carries no gradient
    (csrc/layernorm.hip addsln_*).  The backward receives both gradients and
    sums them inside the kernel."""

    @staticmethod
    def forward(ctx, x, branch, scale, per_sample, weight, bias, eps, twin=True):
        c = x.shape[-1]
        rows = x.numel() // c
        n_per = rows // x.shape[0] if per_sample else 1
        s = torch.empty_like(x)
        y = torch.empty_like(x)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        y16 = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if _bf16_twin_wanted(x, twin) else None
        _lib.call("gd_add_scaled_layernorm_forward", x.data_ptr(), _lib.dtype_code(branch), branch.data_ptr(),
                  scale.data_ptr(), n_per, int(per_sample), weight.data_ptr(), bias.data_ptr(), rows, c, float(eps),
                  s.data_ptr(), y.data_ptr(), _lib.ptr(y16), mean.data_ptr(), rstd.data_ptr(), _lib.stream_of(x),
                  nbytes=rows * (c * (4 + branch.element_size() + 4 + 4 + (0 if y16 is None else 2)) + 8))
        if y16 is not None:
            y._gd_bf16 = (y16, y._version)
        ctx.save_for_backward(s, scale, weight, mean, rstd)
        ctx.meta = (per_sample, n_per, branch.dtype)
        return s, y

    @staticmethod
    def backward(ctx, g_s, g_y):
        s, scale, weight, mean, rstd = ctx.saved_tensors
        per_sample, n_per, bdt = ctx.meta
        c = s.shape[-1]
        rows = s.numel() // c
        g_y = torch.zeros_like(s) if g_y is None else g_y.float().contiguous()
        g_s = None if g_s is None else g_s.float().contiguous()
        dx = torch.empty_like(s)
        db_ = torch.empty(s.shape, dtype=bdt, device=s.device) if ctx.needs_input_grad[1] else None
        dw = torch.empty(c, dtype=torch.float32, device=s.device)
        dbias = torch.empty(c, dtype=torch.float32, device=s.device)
        ws = _workspace(c, s.device)
        _lib.call("gd_add_scaled_layernorm_backward", _lib.ptr(g_s), g_y.data_ptr(), s.data_ptr(),
                  _lib._DTYPE_CODE[bdt], scale.data_ptr(), n_per, int(per_sample),
                  weight.data_ptr(), mean.data_ptr(), rstd.data_ptr(), rows, c, dx.data_ptr(), _lib.ptr(db_),
                  dw.data_ptr(), dbias.data_ptr(), ws.data_ptr(), _lib.stream_of(s),
                  nbytes=rows * (c * (4 * 4 + (2 if db_ is not None else 0)) + 8))
        return (dx if ctx.needs_input_grad[0] else None, db_, None, None,
                dw if ctx.needs_input_grad[4] else None, dbias if ctx.needs_input_grad[5] else None, None, None)


def add_scaled_norm(norm: nn.LayerNorm, x: torch.Tensor, branch: torch.Tensor, drop_prob: float = 0.0,
                    training: bool = False, bf16_twin: bool = True):
    """(x + drop_path(branch), norm(x + drop_path(branch))) as one kernel
    each way (the Swin blocks' attention residual and norm2, reference
    swin_transformer.py:295-296), the per-sample drop-path mask drawn as
    misc.add_drop_path draws it.  None when not applicable (the caller runs
    add_drop_path + layer_norm)."""
    c = x.shape[-1]
    if not (supported(norm, x, None) and c in SLN_WIDTHS and x.dtype == torch.float32 and x.shape == branch.shape
            and branch.dtype in (torch.float32, torch.bfloat16) and x.dim() == 3):
        return None
    from .misc import device_const
    if drop_prob > 0.0 and training:
        keep = 1.0 - drop_prob
        mask = torch.empty((branch.shape[0], 1, 1), dtype=branch.dtype, device=branch.device).bernoulli_(keep)
        scale, per_sample = mask.div_(keep).float().reshape(-1), True
    else:
        scale = device_const(("unit_scale",), lambda: torch.ones(1, dtype=torch.float32), x.device)
        per_sample = False
    return AddScaledNormFunction.apply(x.contiguous(), branch.contiguous(), scale, per_sample, norm.weight,
                                       norm.bias, norm.eps, bool(bf16_twin))


def layer_norm(norm: nn.LayerNorm, x: torch.Tensor, bf16_twin: bool = True) -> torch.Tensor:
    """norm(x) with no residual (Swin's pre-norms and patch-merging norm,
    swin_transformer.py:245, 296, 357): the same kernels with a NULL residual,
    fp32 output as autocast's LayerNorm; elsewhere nn.LayerNorm.
    ``bf16_twin``: the output feeds a GEMM (TokenLinear reads the twin);
    False where it does not (a permute / copy), to skip the extra store."""
    if supported(norm, x, None):
        return AddLayerNormFunction.apply(x.contiguous(), None, norm.weight, norm.bias, norm.eps, bool(bf16_twin))
    return norm(x)


def add_norm(norm: nn.LayerNorm, x: torch.Tensor, r: torch.Tensor, bf16_twin: bool = True, taps: int = 1):
    """norm(x + r); ``bf16_twin`` as in layer_norm.  taps=2: (y, y') for an
    output read by two consumers -- hand one to each; their gradients are
    summed inside the backward kernel."""
    if supported(norm, x, r):
        # (the decoder's MSDA output arrives transposed: one copy, which the
        # unfused add would pay as well)
        return AddLayerNormFunction.apply(x.contiguous(), r.contiguous(), norm.weight, norm.bias, norm.eps,
                                          bool(bf16_twin), int(taps))
    y = norm(x + r)
    return y if taps == 1 else (y, y)
