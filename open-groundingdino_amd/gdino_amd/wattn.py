"""Swin W-MSA / SW-MSA core on MI355X: csrc/wattn.hip through the C-ABI.

    out = softmax(q.scale.k^T + table[rel_index] (+ shift mask)) . v

for every (window, head), as ONE MFMA kernel per direction, replacing the
eager chain of the reference's WindowAttention.forward
(backbone/swin_transformer.py:134-174): the [nH, N, N] bias gather +
permute copy, q.k^T, two broadcast adds, softmax and attn.v, and in the
backward their gradients plus the index_put scatter into
relative_position_bias_table.

Contract of ``window_attention_packed(qkv, table, rel_index, mask, scale)``:
  qkv        [B_, N, 3, nH, hd]  the qkv Linear output, read in place
  table      [(2Wh-1)(2Ww-1), nH] relative_position_bias_table (fp32 param)
  rel_index  [N*N] int64          relative_position_index
  mask       [nW, N, N] or None   0 / -100 shift mask, windows of one image
                                  consecutive (window b uses mask[b % nW])
  -> [B_, N, nH*hd]               the layout the proj Linear reads

``window_attention_image(qkv, qkv_bias, table, rel_index, mask, hw, ws,
shift, scale)`` is the same on the qkv Linear output of the unpartitioned
image [B, H*W, 3C] -> [B, H*W, C]: SwinTransformerBlock.forward's zero pad,
cyclic shift, window partition, window reverse, roll back and crop
(swin_transformer.py:250-290) are the kernel's row map, so none of those
copies (nor their backward) is launched.  A pad position's q/k/v is the qkv
bias (the Linear of the zero pad row); its gradient is returned as the bias
gradient, which autograd adds to the Linear's own.

The HIP kernel covers N <= 144 (windows up to 12x12: Swin-T/S/B/L at 224 and
Swin-B/L at 384) and hd = 32 (every Swin-T/S/B/L head) in fp32 and bf16.
Other shapes and dtypes use the torch composition (ROCm library kernels);
CPU tensors raise, like every HIP op of this package.

When relative_position_index is the reference's (swin_transformer.py:104-115;
checked once per buffer) the kernel is given NULL and computes the index
itself, and a shift mask made by ``shifted_window_mask`` (the reference's
region mask, :402-426) is passed as NULL to the image entry points, which then
compute it from the geometry: neither the [N*N] int64 index nor the
[nW, N, N] fp32 mask is read per window.
"""
from __future__ import annotations

import ctypes
import weakref

import torch

from . import _lib, kernels

_p, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
_lib.register("gd_window_attn_forward", [_i, _p, _p, _p, _p, _i, _i, _i, _i, _i, _f, _p, _p, _p])
_lib.register("gd_window_attn_backward", [_i, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _f, _p, _p, _p])
_lib.register("gd_window_attn_image_forward", [_i] + [_p] * 5 + [_i] * 7 + [_f, _p, _p, _p])
_lib.register("gd_window_attn_image_backward", [_i] + [_p] * 8 + [_i] * 7 + [_f, _p, _p, _p, _p])

MAX_TOKENS = 144

_STD_INDEX = {}  # id(base tensor) -> (weakref to it, (version, numel, offset), is the reference index)


def _kernel_index(rel_index: torch.Tensor, n: int):
    """None (the kernel computes the index) when rel_index is the reference's
    for a square window, else the int64 tensor; the comparison is made once
    per buffer object and version (a host sync on first use only).  Keyed by
    the base tensor (the module buffer behind the per-call .view(-1)), held
    weakly, so a freed buffer's address reused by another tensor never hits."""
    ws = int(round(n ** 0.5))
    if ws * ws != n:
        return rel_index.to(torch.int64).contiguous()
    base = rel_index._base if rel_index._base is not None else rel_index
    key = (base._version, rel_index.numel(), rel_index.storage_offset())
    hit = _STD_INDEX.get(id(base))
    if hit is None or hit[0]() is not base or hit[1] != key:
        from models.GroundingDINO.backbone.swin_transformer import relative_position_index
        std = bool(torch.equal(rel_index.detach().reshape(-1).cpu(), relative_position_index(ws, ws).reshape(-1)))
        for k in [k for k, v in _STD_INDEX.items() if v[0]() is None]:
            del _STD_INDEX[k]
        hit = _STD_INDEX[id(base)] = (weakref.ref(base), key, std)
    return None if hit[2] else rel_index.to(torch.int64).contiguous()


def _is_region_mask(mask, hw, ws, shift) -> bool:
    """mask is shifted_window_mask's region mask for this geometry"""
    hp, wp = -(-hw[0] // ws) * ws, -(-hw[1] // ws) * ws
    return getattr(mask, "_gd_region_mask", None) == (hp, wp, ws, shift)


def supported(qkv: torch.Tensor) -> bool:
    _, n, _, _, hd = qkv.shape
    return _lib.enabled("wattn") and qkv.dtype in (torch.float32, torch.bfloat16) and n <= MAX_TOKENS and hd == 32


class WindowAttnFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, table, rel_index, mask, scale):
        _lib.require_device(qkv, table, rel_index, mask, what="window_attention")
        qkv = qkv.contiguous()
        table32 = table.detach().float().contiguous()
        b_, n, _, nh, hd = qkv.shape
        ridx = _kernel_index(rel_index, n)
        mask32 = None if mask is None else mask.float().contiguous()
        nw = 1 if mask32 is None else mask32.shape[0]
        out = torch.empty(b_, n, nh * hd, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(b_, nh, n, dtype=torch.float32, device=qkv.device)
        _lib.call("gd_window_attn_forward", _lib.dtype_code(qkv), qkv.data_ptr(), table32.data_ptr(),
                  _lib.ptr(ridx), _lib.ptr(mask32), b_, n, nh, hd, nw, float(scale), out.data_ptr(),
                  lse.data_ptr(), _lib.stream_of(qkv), flops=4.0 * b_ * nh * n * n * hd)
        ctx.save_for_backward(qkv, table32, ridx, mask32, out, lse)
        ctx.scale = float(scale)
        ctx.table_dtype = table.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, table32, ridx, mask32, out, lse = ctx.saved_tensors
        b_, n, _, nh, hd = qkv.shape
        nw = 1 if mask32 is None else mask32.shape[0]
        dout = dout.to(qkv.dtype).contiguous()
        dqkv = torch.empty_like(qkv)
        dtable = torch.zeros_like(table32)
        _lib.call("gd_window_attn_backward", _lib.dtype_code(qkv), qkv.data_ptr(), table32.data_ptr(),
                  _lib.ptr(ridx), _lib.ptr(mask32), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), b_, n, nh,
                  hd, nw, ctx.scale, dqkv.data_ptr(), dtable.data_ptr(), _lib.stream_of(qkv),
                  flops=10.0 * b_ * nh * n * n * hd)
        return dqkv, dtable.to(ctx.table_dtype), None, None, None


def window_attention_packed_hip(qkv, table, rel_index, mask, scale):
    if not supported(qkv):
        return window_attention_packed_torch(qkv, table, rel_index, mask, scale)
    return WindowAttnFunction.apply(qkv, table, rel_index, mask, scale)


def window_attention_packed_torch(qkv, table, rel_index, mask, scale):
    """The same op composed from ROCm library kernels (shapes the HIP kernel
    does not cover)."""
    b_, n, _, nh, hd = qkv.shape
    q, k, v = qkv.permute(2, 0, 3, 1, 4)
    bias = table[rel_index.view(-1)].view(n, n, nh).permute(2, 0, 1).contiguous()
    out = kernels._window_attention_torch(q, k, v, bias, mask, scale)
    return out.transpose(1, 2).reshape(b_, n, nh * hd)


class WindowAttnImageFunction(torch.autograd.Function):
    """gd_window_attn_image_*: the window attention of one SwinTransformerBlock
    on the qkv Linear output of the unpartitioned image; the block's pad,
    roll, partition, reverse, roll back and crop are the kernel's row map."""

    @staticmethod
    def forward(ctx, qkv, qkv_bias, table, rel_index, mask, hw, ws, shift, scale):
        _lib.require_device(qkv, qkv_bias, table, rel_index, mask, what="window_attention_image")
        qkv = qkv.contiguous()
        bias = None if qkv_bias is None else qkv_bias.detach().to(qkv.dtype).contiguous()
        table32 = table.detach().float().contiguous()
        ridx = _kernel_index(rel_index, ws * ws)
        # the region mask is computed by the kernel (NULL with shift > 0) --
        # only in its computed-index variant: with a given rel_index tensor the
        # kernel runs its generic mode, which reads the mask tensor
        mask32 = (None if (mask is None or shift == 0 or (ridx is None and _is_region_mask(mask, hw, ws, shift)))
                  else mask.float().contiguous())
        b, _, c3 = qkv.shape
        nh = table.shape[1]
        hd = c3 // (3 * nh)
        hp, wp = -(-hw[0] // ws) * ws, -(-hw[1] // ws) * ws
        out = torch.empty(b, hw[0] * hw[1], c3 // 3, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(b * (hp // ws) * (wp // ws), nh, ws * ws, dtype=torch.float32, device=qkv.device)
        _lib.call("gd_window_attn_image_forward", _lib.dtype_code(qkv), qkv.data_ptr(), _lib.ptr(bias),
                  table32.data_ptr(), _lib.ptr(ridx), _lib.ptr(mask32), b, hw[0], hw[1], ws, shift, nh, hd,
                  float(scale), out.data_ptr(), lse.data_ptr(), _lib.stream_of(qkv),
                  flops=4.0 * lse.numel() * ws * ws * hd)  # windows x heads x N^2 x hd
        ctx.save_for_backward(qkv, bias, table32, ridx, mask32, out, lse)
        ctx.geo = (hw, ws, shift, float(scale))
        ctx.dtypes = (None if qkv_bias is None else qkv_bias.dtype, table.dtype)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, bias, table32, ridx, mask32, out, lse = ctx.saved_tensors
        hw, ws, shift, scale = ctx.geo
        b, _, c3 = qkv.shape
        nh = table32.shape[1]
        dout = dout.to(qkv.dtype).contiguous()
        dqkv = torch.empty_like(qkv)
        # the two atomically accumulated gradients zeroed by ONE fill kernel
        nb = 0 if bias is None else c3
        zbuf = torch.zeros(nb + table32.numel(), dtype=torch.float32, device=qkv.device)
        dbias = None if bias is None else zbuf[:c3]
        dtable = zbuf[nb:].view(table32.shape)
        _lib.call("gd_window_attn_image_backward", _lib.dtype_code(qkv), qkv.data_ptr(), _lib.ptr(bias),
                  table32.data_ptr(), _lib.ptr(ridx), _lib.ptr(mask32), out.data_ptr(), dout.data_ptr(),
                  lse.data_ptr(), b, hw[0], hw[1], ws, shift, nh, c3 // (3 * nh), scale, dqkv.data_ptr(),
                  _lib.ptr(dbias), dtable.data_ptr(), _lib.stream_of(qkv),
                  flops=10.0 * lse.numel() * ws * ws * c3 // (3 * nh))
        bias_dt, table_dt = ctx.dtypes
        return (dqkv, None if dbias is None else dbias.to(bias_dt), dtable.to(table_dt),
                None, None, None, None, None, None)


def image_supported(qkv, table, ws):
    return (_lib.enabled("wattn") and qkv.dtype in (torch.float32, torch.bfloat16) and ws * ws <= MAX_TOKENS
            and qkv.shape[-1] == 3 * 32 * table.shape[1])


def window_attention_image_hip(qkv, qkv_bias, table, rel_index, mask, hw, ws, shift, scale):
    if not image_supported(qkv, table, ws):
        return window_attention_image_torch(qkv, qkv_bias, table, rel_index, mask, hw, ws, shift, scale)
    return WindowAttnImageFunction.apply(qkv, qkv_bias, table, rel_index, mask, tuple(hw), ws, shift, scale)


def window_attention_image_torch(qkv, qkv_bias, table, rel_index, mask, hw, ws, shift, scale):
    """The same op composed from ROCm library kernels: pad (the qkv of a zero
    row is the Linear bias), roll, partition, window attention, reverse, roll
    back, crop."""
    b, _, c3 = qkv.shape
    h, w = hw
    nh = table.shape[1]
    hp, wp = -(-h // ws) * ws, -(-w // ws) * ws
    x = qkv.view(b, h, w, c3)
    if hp != h or wp != w:
        fill = qkv.new_zeros(()) if qkv_bias is None else qkv_bias.to(qkv.dtype)
        pad = fill.expand(b, hp, wp, c3)
        x = torch.cat([torch.cat([x, pad[:, :h, w:]], 2), pad[:, h:]], 1)
    if shift > 0:
        x = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2))
    win = x.view(b, hp // ws, ws, wp // ws, ws, c3).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws, 3, nh,
                                                                                     c3 // (3 * nh))
    out = kernels.window_attention_packed(win, table, rel_index, mask if shift > 0 else None, scale)
    x = out.view(b, hp // ws, wp // ws, ws, ws, -1).permute(0, 1, 3, 2, 4, 5).reshape(b, hp, wp, -1)
    if shift > 0:
        x = torch.roll(x, shifts=(shift, shift), dims=(1, 2))
    if hp != h or wp != w:
        x = x[:, :h, :w]
    return x.reshape(b, h * w, -1)


kernels.register("window_attention_packed", "torch", window_attention_packed_torch)
kernels.register("window_attention_packed", "hip", window_attention_packed_hip, default=True)
kernels.register("window_attention_image", "torch", window_attention_image_torch)
kernels.register("window_attention_image", "hip", window_attention_image_hip, default=True)
