"""Token-heavy Linear layers with a split-K weight-gradient kernel
(csrc/wgrad.hip) on MI355X.

For a Linear over T tokens with a small O x I weight (the encoder's
value / output / sampling projections: T = 44 446 at 800x1333 bs=2, 256 x 256
to 384 x 256; Swin stage 2: T = 33 400, 192-wide), the library GEMM for
dW = dY^T X tiles only the O x I output (16-24 tiles of 64 x 64 on 256 CUs).
``token_linear`` keeps the forward and dX GEMMs on hipBLASLt and computes dW
and db with the split-K kernel, in fp32, straight into the fp32 master
parameters' gradients (no bf16 weight-gradient rounding, no bf16 -> fp32
cast kernel per weight).  Numerically it is the same product with fp32
accumulation; tested against the fp64 reference in tests/test_kernels_gpu.py.

Used by castcache.linear / linear_shared_input under autocast on the GPU
when the shape qualifies (``eligible``); everything else is unchanged.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn.functional as F

from . import _lib

_p, _i, _i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
_lib.register("gd_wgrad", [_i, _p, _i64, _p, _i64, _i, _i, _i, _i, _p, _p, _p, _p])
_lib.register("gd_wgrad_splits", [_i, _i, _i])  # returns int (the registered restype)
_lib.register("gd_wgrad_splits_batched", [_i, _i, _i, _i])
_lib.register("gd_wgrad_batched", [_i, _p, _i64, _i64, _p, _i64, _i64, _i, _i, _i, _i, _i, _p, _i, _p, _i64, _p,
                                   _p])

# split-K weight gradient from 512 tokens up: the decoder's Linears (1 800
# query tokens) and the text side (512) included -- measured 2x faster than
# the library GEMM + fp32 bias sum there too (15-19 vs 28-34 us,
# tools/wgrad_microbench.py); the long-K BiAttention products keep 4096
MIN_TOKENS = 512
TN_MIN_TOKENS = 4096
ENABLED = True
# Linears below the split-K kernel's token threshold (decoder: 1 800 query
# tokens, text: 512): dW through the library's bf16 x bf16 -> fp32 GEMM
# (aten::mm.dtype) and db as an fp32-accumulated sum, straight into the fp32
# parameters' gradients -- instead of autocast's bf16 dW / db plus a
# bf16 -> fp32 cast kernel for each (GDINO_FP32_WGRAD=0: autocast's path)
FP32_OUT_GEMM = os.environ.get("GDINO_FP32_WGRAD", "1") != "0"

# the forward GEMM of TokenLinear on csrc/tlin.hip (GD_TLIN=0: the library
# GEMM, A/B); from this many tokens on (below, the library's small-M tiles win)
_lib.register("gd_token_linear_forward", [_p, _i64, _p, _p, _i, _i, _i, _i, _p, _i64, _p])
TLIN = os.environ.get("GD_TLIN", "1") != "0"
TLIN_MIN_TOKENS = 2048


def tlin_wins(k: int, n: int) -> bool:
    """The shapes where the kernel beats the library GEMM, device time from
    graph replays (tools/tlin_microbench.py, profiles/r06f_tlin_shapes.jsonl):
    a narrow reduction (Swin-T stage 0, K = 96: 41 vs 69 us at 96 -> 288,
    19 vs 34 at 96 -> 96) or output (stage 0's fc2, N = 96), and the wide
    expansions of the 192- / 384-channel stages (192 -> 576: 25 vs 29 us,
    192 -> 768: 30 vs 36, 384 -> 1152: 21 vs 25).  Everywhere else the
    library's tiles are faster (K = 256: 18 vs 14 us at 256 -> 256, 54 vs
    45 at 256 -> 1024; square 192 / 384 shapes; K >= 768)."""
    return k <= TLIN_MAX_NARROW or n <= 96 or (k in (192, 384) and n >= 3 * k)


TLIN_MAX_NARROW = 128


def tlin_ok(x2: torch.Tensor, wc: torch.Tensor, bc) -> bool:
    """x2 [M, K] bf16 rows (unit column stride, 16-B aligned), wc [N, K] bf16
    contiguous, bc None or bf16 [N]; K, N multiples of 8; a winning shape."""
    m, k = x2.shape
    n = wc.shape[0]
    return (TLIN and _lib.enabled("tlin") and _lib.on_device(x2) and m >= TLIN_MIN_TOKENS and tlin_wins(k, n)
            and x2.dtype == wc.dtype == torch.bfloat16 and (bc is None or (bc.dtype == torch.bfloat16
                                                                           and bc.is_contiguous()
                                                                           and bc.data_ptr() % 8 == 0))
            and wc.is_contiguous() and k % 8 == 0 and n % 8 == 0 and x2.stride(1) == 1 and x2.stride(0) % 8 == 0
            and x2.data_ptr() % 16 == 0 and wc.data_ptr() % 16 == 0)


def tlin_forward(x2: torch.Tensor, wc: torch.Tensor, bc=None, relu: bool = False) -> torch.Tensor:
    """y [M, N] bf16 = x2 . wc^T (+ bc) (ReLU) on the token-linear kernel."""
    m, k = x2.shape
    n = wc.shape[0]
    y = torch.empty(m, n, dtype=torch.bfloat16, device=x2.device)
    _lib.call("gd_token_linear_forward", x2.data_ptr(), x2.stride(0), wc.data_ptr(), _lib.ptr(bc), m, k, n,
              int(relu), y.data_ptr(), y.stride(0), _lib.stream_of(x2), flops=2.0 * m * k * n)
    return y


# the input gradient of a Linear fed by a relu TokenLinear's output, with the
# ReLU's backward in the store (csrc/tlin.hip MASK): replaces the library dX
# GEMM + a threshold pass over [tokens, d_ffn] (the encoder FFN: 6 x 546 MB
# of threshold traffic per step, profiles/r05t_glue_census.txt).
# GD_TLIN_MASKED=0: the unfused path (A/B)
_lib.register("gd_token_linear_forward_masked", [_p, _i64, _p, _i, _i, _i, _p, _i64, _p, _i64, _p])
TLIN_MASKED = os.environ.get("GD_TLIN_MASKED", "1") != "0"
TLIN_MASKED_MIN_TOKENS = 8192


def masked_dx_ok(x: torch.Tensor, wc: torch.Tensor) -> bool:
    """Route this Linear's dX to gd_token_linear_forward_masked: x is the
    output of a relu TokenLinear (tagged ``_gd_relu_box``; its only consumer),
    bf16 contiguous rows, both feature counts multiples of 8, enough tokens."""
    if not (TLIN_MASKED and TLIN and getattr(x, "_gd_relu_box", None) is not None and _lib.enabled("tlin")
            and _lib.on_device(x) and x.dtype == wc.dtype == torch.bfloat16 and x.is_contiguous()
            and wc.is_contiguous() and x.data_ptr() % 16 == 0):
        return False
    n_out, k_in = wc.shape
    return x.numel() // max(k_in, 1) >= TLIN_MASKED_MIN_TOKENS and n_out % 8 == 0 and k_in % 8 == 0


def masked_dx(dy2: torch.Tensor, wc: torch.Tensor, mask2: torch.Tensor) -> torch.Tensor:
    """dX [M, K_in] bf16 = (dy2 [M, N_out] . wc [N_out, K_in]) where
    mask2 [M, K_in] > 0, else 0."""
    m, n_out = dy2.shape
    k_in = wc.shape[1]
    wt = wc.t().contiguous()  # [K_in, N_out]: the kernel's K-contiguous W
    y = torch.empty(m, k_in, dtype=torch.bfloat16, device=dy2.device)
    _lib.call("gd_token_linear_forward_masked", dy2.data_ptr(), dy2.stride(0), wt.data_ptr(), m, n_out, k_in,
              mask2.data_ptr(), mask2.stride(0), y.data_ptr(), y.stride(0), _lib.stream_of(dy2),
              flops=2.0 * m * n_out * k_in)
    return y


def eligible(x: torch.Tensor, out_features: int, dtype=None) -> bool:
    """Route a Linear's weight gradient to the split-K kernel: GPU, T >= MIN_TOKENS
    tokens, O and I multiples of 16 (bf16, the 128 x 128 transposed-read
    kernel) or of 64 (fp32); ``dtype``: the dtype the GEMM runs in (the
    autocast dtype), default x's.  Measured 2.4-6x faster than the library GEMM
    on every token-heavy Linear of the train step, 256 x 256 to 2048 x 256
    and the Swin MLPs (tools/wgrad_microbench.py)."""
    in_features = x.shape[-1]
    gran = 16 if (dtype or x.dtype) == torch.bfloat16 else 64
    if not (ENABLED and _lib.enabled("wgrad") and _lib.on_device(x) and out_features % gran == 0
            and in_features % gran == 0):
        return False
    return x.numel() // max(in_features, 1) >= MIN_TOKENS


def _splits(t, o, i):
    return int(_lib.lib().gd_wgrad_splits(t, o, i))


def _workspace(o, i, s, device):
    fn = _lib.lib().gd_wgrad_workspace_bytes
    fn.restype, fn.argtypes = ctypes.c_size_t, [_i, _i, _i]
    return torch.empty((int(fn(o, i, s)) + 3) // 4, dtype=torch.float32, device=device)


def weight_grad(dy2: torch.Tensor, x2: torch.Tensor, want_bias: bool):
    """dy2 [T, O], x2 [T, I] (same dtype, contiguous rows) -> dW [O, I] fp32,
    db [O] fp32 or None."""
    t, o = dy2.shape
    i = x2.shape[1]
    s = _splits(t, o, i)
    ws = _workspace(o, i, s, dy2.device)
    dw = torch.empty(o, i, dtype=torch.float32, device=dy2.device)
    db = torch.empty(o, dtype=torch.float32, device=dy2.device) if want_bias else None
    _lib.call("gd_wgrad", _lib.dtype_code(dy2), dy2.data_ptr(), dy2.stride(0), x2.data_ptr(), x2.stride(0), t, o, i,
              s, ws.data_ptr(), dw.data_ptr(), _lib.ptr(db), _lib.stream_of(dy2), flops=2.0 * t * o * i)
    return dw, db


def lib_eligible(x: torch.Tensor, dtype) -> bool:
    """Route a (non split-K) Linear's weight gradient to weight_grad_lib."""
    # a library GEMM (aten::mm.dtype exists for the ROCm device only): x.is_cuda,
    # not _lib.on_device, which the host-side emulator tests redirect
    # honours the same kill switches as the split-K route (ENABLED,
    # GDINO_DISABLE=wgrad), so the documented A/B off-switch covers both
    return (ENABLED and _lib.enabled("wgrad") and FP32_OUT_GEMM and dtype == torch.bfloat16
            and x.is_cuda)


_MM_DTYPE_OK = True


def weight_grad_lib(dy2: torch.Tensor, x2: torch.Tensor, want_bias: bool):
    """dy2 [T, O], x2 [T, I] bf16 -> dW [O, I] fp32 (library GEMM with fp32
    output), db [O] fp32 or None.  If this torch build's ROCm backend
    rejects aten::mm.dtype, dW is the bf16 GEMM cast to fp32 -- autocast's
    own numerics -- for the rest of the process."""
    global _MM_DTYPE_OK
    dw = None
    if _MM_DTYPE_OK:
        try:
            dw = torch.mm(dy2.t(), x2, out_dtype=torch.float32)
        except (RuntimeError, NotImplementedError, TypeError):
            _MM_DTYPE_OK = False
    if dw is None:
        dw = torch.mm(dy2.t(), x2).float()
    db = dy2.sum(0, dtype=torch.float32) if want_bias else None
    return dw, db


def tn_eligible(a: torch.Tensor, b: torch.Tensor) -> bool:
    """a^T b over the token dimension (-2) with the split-K kernel?"""
    gran = 16 if a.dtype == torch.bfloat16 else 64
    return (_lib.enabled("wgrad") and _lib.on_device(a) and a.dtype == b.dtype
            and a.dtype in (torch.float32, torch.bfloat16) and a.shape[:-1] == b.shape[:-1]
            and a.shape[-2] >= TN_MIN_TOKENS and a.shape[-1] % gran == 0 and b.shape[-1] % gran == 0)


def tn_matmul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a [..., T, O], b [..., T, I] -> a^T b [..., O, I] in a's dtype (fp32
    accumulation), batched over the leading dims: the long-K products whose
    K (= T tokens) dwarfs the O x I output."""
    t, o, i = a.shape[-2], a.shape[-1], b.shape[-1]
    lead = a.shape[:-2]
    a2 = a.reshape(-1, t, o).contiguous()
    b2 = b.reshape(-1, t, i).contiguous()
    nb = a2.shape[0]
    s = int(_lib.lib().gd_wgrad_splits_batched(t, o, i, nb))
    ws = _workspace(o, i, s * nb, a.device)
    out = torch.empty(nb, o, i, dtype=a.dtype, device=a.device)
    _lib.call("gd_wgrad_batched", _lib.dtype_code(a2), a2.data_ptr(), a2.stride(1), a2.stride(0), b2.data_ptr(),
              b2.stride(1), b2.stride(0), t, o, i, nb, s, ws.data_ptr(), _lib.dtype_code(out), out.data_ptr(),
              out.stride(0), None, _lib.stream_of(a2), flops=2.0 * nb * t * o * i)
    return out.reshape(*lead, o, i)


def _dx(dy, wc, x_dtype):
    """dX = dY . W for an fp32 input: the library GEMM writes fp32 directly
    (aten::mm.dtype, fp32 accumulation) instead of a bf16 result plus a
    cast kernel; other dtypes, or a torch without mm.dtype, the plain
    product."""
    global _MM_DTYPE_OK
    if x_dtype == torch.float32 and dy.dtype == torch.bfloat16 and _MM_DTYPE_OK and dy.is_cuda:
        try:
            return torch.mm(dy.reshape(-1, dy.shape[-1]), wc, out_dtype=torch.float32).view(*dy.shape[:-1],
                                                                                         wc.shape[-1])
        except (RuntimeError, NotImplementedError, TypeError):
            _MM_DTYPE_OK = False
    return torch.matmul(dy, wc).to(x_dtype)


class TokenLinear(torch.autograd.Function):
    """y = x . wc^T + bc with wc / bc the low-precision copies of the fp32
    parameters ``params`` (one or several row blocks of the weight, then the
    matching bias blocks); gradients go to ``params`` in fp32."""

    @staticmethod
    def forward(ctx, x, wc, bc, nw, lib_wgrad, relu, fold, *params):
        # the bf16 copy a producer wrote beside x (layernorm: ``_gd_bf16``)
        # instead of a cast kernel
        tw = getattr(x, "_gd_bf16", None)
        if tw is not None and tw[1] == x._version and tw[0].dtype == wc.dtype and tw[0].shape == x.shape:
            xc = tw[0]
        else:
            xc = x if x.dtype == wc.dtype else x.to(wc.dtype)
        if relu:
            # relu(x wc^T + bc) in the GEMM's epilogue (hipBLASLt bias + ReLU):
            # no separate activation pass over the [tokens, d_ffn] output;
            # relu commutes with the bf16 rounding, so the result equals the
            # unfused F.relu(F.linear(...))
            x2 = xc.reshape(-1, xc.shape[-1])
            if tlin_ok(x2, wc, bc):
                y = tlin_forward(x2, wc, bc, relu=True)
            else:
                y = torch._addmm_activation(bc, x2, wc.t(), use_gelu=False)
            y = y.view(*xc.shape[:-1], wc.shape[0])
            # set by the consumer Linear when it folds this ReLU's backward
            # into its own dX (masked_dx): the gradient arrives masked
            ctx.relu_box = [False]
            if fold:  # the caller owns y's only consumer (castcache.ffn / MLP)
                y._gd_relu_box = ctx.relu_box
            # x2: the rows the weight gradient reads (already copied once
            # when xc could not be viewed 2-D -- not again in the backward)
            ctx.save_for_backward(x2, wc, y)
        else:
            # one 2-D GEMM over the flattened tokens: F.linear on a 3-D input
            # that cannot be viewed 2-D (the decoder's [nq, bs, C] transposes)
            # dispatches a bmm against the weight expanded to [nq, C, C]
            x2 = xc.reshape(-1, xc.shape[-1])
            if tlin_ok(x2, wc, bc):
                y2 = tlin_forward(x2, wc, bc)
            else:
                y2 = torch.mm(x2, wc.t()) if bc is None else torch.addmm(bc, x2, wc.t())
            y = y2.view(*xc.shape[:-1], wc.shape[0])
            ctx.save_for_backward(x2, wc)
            ctx.mask_dx = xc is x and masked_dx_ok(x, wc)
            if ctx.mask_dx:
                x._gd_relu_box[0] = True
                del x._gd_relu_box  # claimed: no second consumer may fold it
        ctx.relu = relu
        ctx.lib_wgrad = lib_wgrad
        ctx.x_dtype = x.dtype
        ctx.rows = [p.shape[0] for p in params[:nw]]
        ctx.nw = nw
        ctx.has_bias = len(params) > nw
        return y

    @staticmethod
    def backward(ctx, dy):
        if ctx.relu:
            x2, wc, y = ctx.saved_tensors
            if not ctx.relu_box[0]:  # (else dy was masked by the consumer's dX kernel)
                dy = torch.ops.aten.threshold_backward(dy.to(wc.dtype), y, 0)
        else:
            x2, wc = ctx.saved_tensors
        dy = dy.to(wc.dtype)
        # one row-major copy of dy at most, shared by dX and dW
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        if not ctx.needs_input_grad[0]:
            dx = None
        elif not ctx.relu and ctx.mask_dx:
            dx = masked_dx(dy2, wc, x2).view(*dy.shape[:-1], wc.shape[1])
        else:
            dx = _dx(dy2, wc, ctx.x_dtype).view(*dy.shape[:-1], wc.shape[1])
        wg = weight_grad_lib if ctx.lib_wgrad else weight_grad
        dw, db = wg(dy2, x2.contiguous(), ctx.has_bias)
        grads = list(dw.split(ctx.rows, 0))
        if ctx.has_bias:
            grads += list(db.split(ctx.rows, 0))
        return (dx, None, None, None, None, None, None, *grads)


def token_linear(x, wc, bc, weights, biases, lib_wgrad=False, relu=False, fold=False):
    """F.linear(x, wc, bc) whose weight / bias gradients reach the fp32
    ``weights`` / ``biases`` (row blocks of wc / bc) through the split-K
    kernel (or, lib_wgrad, the library GEMM with fp32 output); ``relu``:
    relu(F.linear(...)) with the activation in the GEMM epilogue; ``fold``
    (relu only): the caller guarantees the output's only consumer is the next
    Linear, which may then fold the ReLU backward into its dX kernel."""
    params = list(weights) + (list(biases) if bc is not None else [])
    relu = bool(relu and bc is not None)
    return TokenLinear.apply(x, wc.detach(), None if bc is None else bc.detach(), len(weights), bool(lib_wgrad),
                             relu, bool(fold and relu), *params)
