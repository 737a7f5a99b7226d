"""ctypes front-end of the host-side SIMT emulator (tests/emu): the product's
csrc/*.hip compiled as host C++ against tests/emu/include/hip/hip_runtime.h,
exporting the same C ABI as libgdino_amd.so (include/gdino_amd.h) on host
pointers.  Test infrastructure only: it lets the CPU suite execute the exact
kernel sources (indexing, LDS, barriers, DPP/swizzle exchanges, launch
geometry) against the oracle when no GPU is available."""
import ctypes
import os
import subprocess

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU_DIR = os.path.join(ROOT, "tests", "emu")
_LIB = None

F32, F64, BF16 = 0, 1, 2
_p, _i = ctypes.c_void_p, ctypes.c_int


def lib():
    global _LIB
    if _LIB is None:
        # GD_EMU_ASAN=1: the AddressSanitizer build (the process must preload
        # the clang ASan runtime; see tests/test_emu_kernels.py)
        asan = os.environ.get("GD_EMU_ASAN") == "1"
        subprocess.run(["make", "-s", "-j8", "-C", EMU_DIR] + (["asan"] if asan else []), check=True)
        _LIB = ctypes.CDLL(os.path.join(EMU_DIR, "_build", "libgd_emu_asan.so" if asan else "libgd_emu.so"))
        _LIB.gd_msda_forward.argtypes = [_i, _p, _p, _p, _p, _p] + [_i] * 7 + [_p, _p]
        _LIB.gd_msda_backward.argtypes = [_i, _p, _p, _p, _p, _p, _p] + [_i] * 7 + [_p, _p, _p, _p]
        _LIB.gd_msda_backward_geom.argtypes = [_i, _p, _p, _p, _p, _p, _p] + [_i] * 7 + [_p, _p, _p, _p, _p]
        _LIB.gd_msda_backward_workspace_bytes.argtypes = [_i] * 8 + [_p, _i]
        _LIB.gd_msda_backward_workspace_bytes.restype = ctypes.c_size_t
        _LIB.gd_msda_backward_sorted.argtypes = ([_i, _p, _p, _p, _p, _p, _p] + [_i] * 7 +
                                                 [_p, _i, _p, _p, _p, _p, ctypes.c_size_t, _i, _p])
        _LIB.gd_biattn_workspace_bytes.argtypes = [_i] * 4
        _LIB.gd_biattn_workspace_bytes.restype = ctypes.c_size_t
        _LIB.gd_biattn_softmax_fwd.argtypes = [_i, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p]
        _LIB.gd_biattn_softmax_bwd.argtypes = [_i, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p]
        _LIB.gd_window_attn_forward.argtypes = [_i, _p, _p, _p, _p] + [_i] * 5 + [ctypes.c_float, _p, _p, _p]
        _LIB.gd_window_attn_backward.argtypes = ([_i, _p, _p, _p, _p, _p, _p, _p] + [_i] * 5 +
                                                 [ctypes.c_float, _p, _p, _p])
        _f, _u = ctypes.c_float, ctypes.c_uint32
        _LIB.gd_window_attn_image_forward.argtypes = [_i] + [_p] * 5 + [_i] * 7 + [_f, _p, _p, _p]
        _LIB.gd_window_attn_image_backward.argtypes = [_i] + [_p] * 8 + [_i] * 7 + [_f, _p, _p, _p, _p]
        _LIB.gd_attn_forward.argtypes = [_i] * 6 + [_p] * 7 + [_i, _p, _f, _f, _u, _p, _p, _p, _p]
        _LIB.gd_attn_backward.argtypes = [_i] * 6 + [_p] * 7 + [_i, _p, _f, _f, _u] + [_p] * 13
        _LIB.gd_contrastive_forward.argtypes = [_i] + [_p] * 5 + [_i] * 5 + [_p, _p, _p]
        _i64 = ctypes.c_int64
        _LIB.gd_msda_prologue_forward.argtypes = [_i, _p, _i64, _p, _i64, _p, _i, _p] + [_i] * 5 + [_p, _p, _p]
        _LIB.gd_msda_prologue_backward.argtypes = [_i, _p, _p, _p, _p, _i, _p] + [_i] * 5 + [_p, _p, _p]
        _LIB.gd_wgrad.argtypes = [_i, _p, _i64, _p, _i64, _i, _i, _i, _i, _p, _p, _p, _p]
        _LIB.gd_wgrad_splits.argtypes = [_i, _i, _i]
        _LIB.gd_wgrad_workspace_bytes.argtypes = [_i, _i, _i]
        _LIB.gd_wgrad_workspace_bytes.restype = ctypes.c_size_t
        _LIB.gd_add_layernorm_forward.argtypes = [_i, _p, _i, _p, _p, _p, _i64, _i, ctypes.c_float, _p, _p, _p, _p]
        _LIB.gd_add_layernorm_backward.argtypes = [_i, _p, _i, _p, _p, _p, _p, _p, _i64, _i] + [_p] * 6
        _LIB.gd_linear_sum_assignment.argtypes = [_p, _i, _i, _i, _i64, _p, _p, _p, _p, _p]
        _LIB.gd_add_layernorm_workspace_bytes.argtypes = [_i]
        _LIB.gd_add_layernorm_workspace_bytes.restype = ctypes.c_size_t
        _LIB.gd_last_error.restype = ctypes.c_char_p
        _LIB.gd_runtime_info.restype = ctypes.c_char_p
    return _LIB


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _check(rc):
    if rc != 0:
        raise RuntimeError(lib().gd_last_error().decode())


def _code(t):
    return {torch.float32: F32, torch.float64: F64, torch.bfloat16: BF16}[t.dtype]


def msda_forward(value, shapes, lsi, loc, attn):
    """value [N,S,M,D] (f32/f64/bf16), loc/attn f32 (f64 for f64 value) -> out [N,Lq,M*D]."""
    N, S, M, D = value.shape
    _, Lq, _, L, P, _ = loc.shape
    value, loc, attn = value.contiguous(), loc.contiguous(), attn.contiguous()
    shapes, lsi = shapes.to(torch.int64).contiguous(), lsi.to(torch.int64).contiguous()
    out = torch.empty(N, Lq, M * D, dtype=value.dtype)
    _check(lib().gd_msda_forward(_code(value), _ptr(value), _ptr(shapes), _ptr(lsi), _ptr(loc), _ptr(attn),
                                 N, S, M, D, L, Lq, P, _ptr(out), None))
    return out


def msda_backward(value, shapes, lsi, loc, attn, grad_out, host_shapes=None):
    """-> grad_value (f32, or f64 for f64 value), grad_loc, grad_attn.
    host_shapes: [(H, W)] -> gd_msda_backward_geom (pixel-block tiles)."""
    N, S, M, D = value.shape
    _, Lq, _, L, P, _ = loc.shape
    acc = torch.float64 if value.dtype == torch.float64 else torch.float32
    value, loc, attn, grad_out = (t.contiguous() for t in (value, loc, attn, grad_out))
    shapes, lsi = shapes.to(torch.int64).contiguous(), lsi.to(torch.int64).contiguous()
    gv = torch.empty(N, S, M, D, dtype=acc)
    gl = torch.empty(N, Lq, M, L, P, 2, dtype=acc)
    ga = torch.empty(N, Lq, M, L, P, dtype=acc)
    if host_shapes is None:
        _check(lib().gd_msda_backward(_code(value), _ptr(value), _ptr(shapes), _ptr(lsi), _ptr(loc), _ptr(attn),
                                      _ptr(grad_out), N, S, M, D, L, Lq, P, _ptr(gv), _ptr(gl), _ptr(ga), None))
    else:
        hs = (ctypes.c_int64 * (2 * L))(*[int(v) for hw in host_shapes for v in hw])
        _check(lib().gd_msda_backward_geom(_code(value), _ptr(value), _ptr(shapes), _ptr(lsi), _ptr(loc),
                                           _ptr(attn), _ptr(grad_out), N, S, M, D, L, Lq, P, _ptr(gv), _ptr(gl),
                                           _ptr(ga), hs, None))
    return gv, gl, ga


def msda_backward_sorted(value, shapes, lsi, loc, attn, grad_out, host_shapes, gv_dtype=torch.float32,
                         deterministic=False):
    """gd_msda_backward_sorted -> grad_value (gv_dtype), grad_loc, grad_attn
    (f32); None when the sorted backward does not apply."""
    N, S, M, D = value.shape
    _, Lq, _, L, P, _ = loc.shape
    value, loc, attn, grad_out = (t.contiguous() for t in (value, loc, attn, grad_out))
    shapes, lsi = shapes.to(torch.int64).contiguous(), lsi.to(torch.int64).contiguous()
    hs = (ctypes.c_int64 * (2 * L))(*[int(v) for hw in host_shapes for v in hw])
    flags = 1 if deterministic else 0
    nb = lib().gd_msda_backward_workspace_bytes(_code(value), N, S, M, D, L, Lq, P, hs, flags)
    if nb == 0:
        return None
    ws = torch.empty(nb, dtype=torch.uint8)
    gv = torch.full((N, S, M, D), float("nan"), dtype=gv_dtype)  # every row must be written
    gl = torch.full((N, Lq, M, L, P, 2), float("nan"), dtype=torch.float32)
    ga = torch.full((N, Lq, M, L, P), float("nan"), dtype=torch.float32)
    _check(lib().gd_msda_backward_sorted(_code(value), _ptr(value), _ptr(shapes), _ptr(lsi), _ptr(loc), _ptr(attn),
                                         _ptr(grad_out), N, S, M, D, L, Lq, P, _ptr(gv), _code(gv), _ptr(gl),
                                         _ptr(ga), hs, _ptr(ws), nb, flags, None))
    return gv, gl, ga


def _u8(m):
    return None if m is None else m.to(torch.uint8).contiguous()


def biattn_softmax_fwd(s, pad_v=None, pad_l=None):
    B, H, S, T = s.shape
    s = s.contiguous()
    pv, pl = torch.empty_like(s), torch.empty_like(s)
    ws = torch.empty((int(lib().gd_biattn_workspace_bytes(B, H, S, T)) + 3) // 4, dtype=torch.float32)
    mv, ml = _u8(pad_v), _u8(pad_l)
    _check(lib().gd_biattn_softmax_fwd(_code(s), _ptr(s), _ptr(mv), _ptr(ml), B, H, S, T, _ptr(pv), _ptr(pl),
                                       _ptr(ws), None))
    return pv, pl


def biattn_softmax_bwd(pv, pl, dpv, dpl):
    B, H, S, T = pv.shape
    pv, pl, dpv, dpl = (t.contiguous() for t in (pv, pl, dpv, dpl))
    ds = torch.empty_like(pv)
    ws = torch.empty((int(lib().gd_biattn_workspace_bytes(B, H, S, T)) + 3) // 4, dtype=torch.float32)
    _check(lib().gd_biattn_softmax_bwd(_code(pv), _ptr(pv), _ptr(pl), _ptr(dpv), _ptr(dpl), B, H, S, T, _ptr(ds),
                                       _ptr(ws), None))
    return ds


def window_attn_forward(qkv, table, ridx, mask, scale):
    """qkv [B_, N, 3, nH, hd] (f32/bf16), table [R, nH] f32, ridx [N*N] int64,
    mask [nW, N, N] f32 or None -> out [B_, N, nH*hd], lse [B_, nH, N]."""
    B_, N, _, nH, hd = qkv.shape
    nW = 1 if mask is None else mask.shape[0]
    qkv, table = qkv.contiguous(), table.float().contiguous()
    ridx = None if ridx is None else ridx.to(torch.int64).contiguous()
    mask = None if mask is None else mask.float().contiguous()
    out = torch.empty(B_, N, nH * hd, dtype=qkv.dtype)
    lse = torch.empty(B_, nH, N, dtype=torch.float32)
    _check(lib().gd_window_attn_forward(_code(qkv), _ptr(qkv), _ptr(table), _ptr(ridx), _ptr(mask), B_, N, nH, hd,
                                        nW, scale, _ptr(out), _ptr(lse), None))
    return out, lse


def window_attn_backward(qkv, table, ridx, mask, scale, out, lse, grad_out):
    """-> grad_qkv (qkv dtype), grad_table (f32, [R, nH])."""
    B_, N, _, nH, hd = qkv.shape
    nW = 1 if mask is None else mask.shape[0]
    qkv, table = qkv.contiguous(), table.float().contiguous()
    ridx = None if ridx is None else ridx.to(torch.int64).contiguous()
    mask = None if mask is None else mask.float().contiguous()
    out, lse, grad_out = out.contiguous(), lse.contiguous(), grad_out.contiguous()
    gq = torch.full_like(qkv, float("nan"))
    gt = torch.zeros_like(table)
    _check(lib().gd_window_attn_backward(_code(qkv), _ptr(qkv), _ptr(table), _ptr(ridx), _ptr(mask), _ptr(out),
                                         _ptr(grad_out), _ptr(lse), B_, N, nH, hd, nW, scale, _ptr(gq), _ptr(gt),
                                         None))
    return gq, gt


def window_attn_image_forward(qkv, qkv_bias, table, ridx, mask, hw, ws, shift, scale):
    """qkv [B, H*W, 3C] (f32/bf16), qkv_bias [3C] or None -> out [B, H*W, C],
    lse [B*nW, nH, ws*ws] (gd_window_attn_image_forward)."""
    b, _, c3 = qkv.shape
    nh = table.shape[1]
    hd = c3 // (3 * nh)
    qkv, table = qkv.contiguous(), table.float().contiguous()
    ridx = None if ridx is None else ridx.to(torch.int64).contiguous()
    bias = None if qkv_bias is None else qkv_bias.to(qkv.dtype).contiguous()
    mask = None if mask is None else mask.float().contiguous()
    hp, wp = -(-hw[0] // ws) * ws, -(-hw[1] // ws) * ws
    out = torch.full((b, hw[0] * hw[1], c3 // 3), float("nan"), dtype=qkv.dtype)
    lse = torch.empty(b * (hp // ws) * (wp // ws), nh, ws * ws, dtype=torch.float32)
    _check(lib().gd_window_attn_image_forward(_code(qkv), _ptr(qkv), _ptr(bias), _ptr(table), _ptr(ridx),
                                              _ptr(mask), b, hw[0], hw[1], ws, shift, nh, hd, scale, _ptr(out),
                                              _ptr(lse), None))
    return out, lse


def window_attn_image_backward(qkv, qkv_bias, table, ridx, mask, hw, ws, shift, scale, out, lse, grad_out):
    """-> grad_qkv (qkv dtype), grad_qkv_bias (f32 [3C], pad rows only; None
    without a bias), grad_table (f32)."""
    b, _, c3 = qkv.shape
    nh = table.shape[1]
    hd = c3 // (3 * nh)
    qkv, table = qkv.contiguous(), table.float().contiguous()
    ridx = None if ridx is None else ridx.to(torch.int64).contiguous()
    bias = None if qkv_bias is None else qkv_bias.to(qkv.dtype).contiguous()
    mask = None if mask is None else mask.float().contiguous()
    gq = torch.full_like(qkv, float("nan"))
    gb = None if bias is None else torch.zeros(c3, dtype=torch.float32)
    gt = torch.zeros_like(table)
    _check(lib().gd_window_attn_image_backward(_code(qkv), _ptr(qkv), _ptr(bias), _ptr(table), _ptr(ridx),
                                               _ptr(mask), _ptr(out.contiguous()), _ptr(grad_out.contiguous()),
                                               _ptr(lse), b, hw[0], hw[1], ws, shift, nh, hd, scale, _ptr(gq),
                                               _ptr(gb), _ptr(gt), None))
    return gq, gb, gt


def _st3(t):
    return (ctypes.c_int64 * 3)(*t.stride()[:3])


def _mask_args(mask):
    """mask broadcastable to [B, H, Lq, Lk] (bool keep or additive float) ->
    (tensor, kind, strides)"""
    if mask is None:
        return None, 0, None
    m = mask if mask.dtype == torch.bool else mask.float()
    while m.dim() < 4:
        m = m.unsqueeze(0)
    if m.stride(-1) != 1:
        m = m.contiguous()
    if m.dtype == torch.bool:
        m = m.view(torch.uint8)
        kind = 1
    else:
        kind = 2
    st = [0 if m.shape[i] == 1 else m.stride(i) for i in range(3)]
    return m, kind, (ctypes.c_int64 * 3)(*st)


def attn_forward(q, k, v, mask, scale, dropout_p=0.0, seed=0):
    """q [B,H,Lq,hd], k/v [B,H,Lk,hd] (any (b,h,l) strides, contiguous hd)
    -> out [B,H,Lq,hd] (stored [B,Lq,H,hd]), lse [B,H,Lq]"""
    B, H, Lq, hd = q.shape
    Lk = k.shape[2]
    m, kind, ms = _mask_args(mask)
    out = torch.empty(B, Lq, H, hd, dtype=q.dtype).transpose(1, 2)
    lse = torch.empty(B, H, Lq, dtype=torch.float32)
    _check(lib().gd_attn_forward(_code(q), B, H, Lq, Lk, hd, _ptr(q), _st3(q), _ptr(k), _st3(k), _ptr(v), _st3(v),
                                 _ptr(m), kind, ms, scale, dropout_p, seed, _ptr(out), _st3(out), _ptr(lse), None))
    return out, lse


def attn_backward(q, k, v, mask, scale, out, lse, grad_out, dropout_p=0.0, seed=0):
    B, H, Lq, hd = q.shape
    Lk = k.shape[2]
    m, kind, ms = _mask_args(mask)
    dsum = torch.empty(B, H, Lq, dtype=torch.float32)
    dq = torch.full_like(q, float("nan"))
    dk = torch.full_like(k, float("nan"))
    dv = torch.full_like(v, float("nan"))
    _check(lib().gd_attn_backward(_code(q), B, H, Lq, Lk, hd, _ptr(q), _st3(q), _ptr(k), _st3(k), _ptr(v), _st3(v),
                                  _ptr(m), kind, ms, scale, dropout_p, seed, _ptr(out), _st3(out), _ptr(grad_out),
                                  _st3(grad_out),
                                  _ptr(lse), _ptr(dsum), _ptr(dq), _st3(dq), _ptr(dk), _st3(dk), _ptr(dv), _st3(dv),
                                  None))
    return dq, dk, dv


def contrastive_forward(x, text, mask, tout, want_logits=True, want_rowmax=True):
    """x [B, Q, C], text [B, T, C] (f32/bf16), mask [B, T] bool keep ->
    (logits [B, Q, tout] f32 or None, rowmax [B, Q] f32 or None)"""
    B, Q, C = x.shape
    T = text.shape[1]
    keep = mask.to(torch.uint8).contiguous()
    logits = torch.full((B, Q, tout), float("nan")) if want_logits else None
    rowmax = torch.full((B, Q), float("nan")) if want_rowmax else None
    _check(lib().gd_contrastive_forward(_code(x), _ptr(x), (ctypes.c_int64 * 2)(*x.stride()[:2]), _ptr(text),
                                        (ctypes.c_int64 * 2)(*text.stride()[:2]), _ptr(keep), B, Q, T, C, tout,
                                        _ptr(logits), _ptr(rowmax), None))
    return logits, rowmax


def msda_prologue_forward(offsets, logits, ref, shapes, M, L, P):
    """offsets [N, Lq, M*L*P*2], logits [N, Lq, M*L*P] (row-strided views
    allowed), ref [N, Lq, L, 2|4] f32 -> loc [N, Lq, M, L, P, 2], attn"""
    N, Lq, _ = offsets.shape
    ref = ref.float().contiguous()
    shapes = shapes.to(torch.int64).contiguous()
    loc = torch.full((N, Lq, M, L, P, 2), float("nan"))
    attn = torch.full((N, Lq, M, L, P), float("nan"))
    _check(lib().gd_msda_prologue_forward(_code(offsets), _ptr(offsets), offsets.stride(1), _ptr(logits),
                                          logits.stride(1), _ptr(ref), ref.shape[-1], _ptr(shapes), N, Lq, M, L, P,
                                          _ptr(loc), _ptr(attn), None))
    return loc, attn


def msda_prologue_backward(grad_loc, grad_attn, attn, ref, shapes, dtype):
    N, Lq, M, L, P = attn.shape
    ref = ref.float().contiguous()
    shapes = shapes.to(torch.int64).contiguous()
    g_off = torch.full((N, Lq, M * L * P * 2), float("nan")).to(dtype)
    g_log = torch.full((N, Lq, M * L * P), float("nan")).to(dtype)
    _check(lib().gd_msda_prologue_backward(_code(g_off), _ptr(grad_loc.contiguous()), _ptr(grad_attn.contiguous()),
                                           _ptr(attn), _ptr(ref), ref.shape[-1], _ptr(shapes), N, Lq, M, L, P,
                                           _ptr(g_off), _ptr(g_log), None))
    return g_off, g_log


def wgrad(dy, x, bias=True, splits=None):
    """dy [T, O], x [T, I] (f32/bf16, row-major) -> dW [O, I] f32, db [O] f32"""
    T, O = dy.shape
    I = x.shape[1]
    s = int(lib().gd_wgrad_splits(T, O, I)) if splits is None else splits
    ws = torch.empty((int(lib().gd_wgrad_workspace_bytes(O, I, s)) + 3) // 4, dtype=torch.float32)
    dw = torch.full((O, I), float("nan"))
    db = torch.full((O,), float("nan")) if bias else None
    _check(lib().gd_wgrad(_code(dy), _ptr(dy), dy.stride(0), _ptr(x), x.stride(0), T, O, I, s, _ptr(ws), _ptr(dw),
                          _ptr(db), None))
    return dw, db


def add_layernorm_forward(x, r, w, b, eps):
    C = x.shape[-1]
    rows = x.numel() // C
    y = torch.full(x.shape, float("nan"))
    mean = torch.full((rows,), float("nan"))
    rstd = torch.full((rows,), float("nan"))
    _check(lib().gd_add_layernorm_forward(_code(x), _ptr(x), _code(r) if r is not None else 0, _ptr(r), _ptr(w),
                                          _ptr(b), rows, C, eps, _ptr(y), _ptr(mean), _ptr(rstd), None))
    return y, mean, rstd


def add_layernorm_backward(x, r, w, dy, mean, rstd):
    C = x.shape[-1]
    rows = x.numel() // C
    dx = torch.full_like(x, float("nan"))
    dr = None if r is None else torch.full_like(r, float("nan"))
    dw = torch.full((C,), float("nan"))
    db = torch.full((C,), float("nan"))
    ws = torch.empty((int(lib().gd_add_layernorm_workspace_bytes(C)) + 3) // 4)
    _check(lib().gd_add_layernorm_backward(_code(x), _ptr(x), _code(r) if r is not None else 0, _ptr(r), _ptr(w),
                                           _ptr(dy.contiguous()), _ptr(mean), _ptr(rstd), rows, C, _ptr(dx),
                                           _ptr(dr), _ptr(dw), _ptr(db), _ptr(ws), None))
    return dx, dr, dw, db


def attn_dropout_keep(B, H, Lq, Lk, p, seed):
    """The kernels' dropout mask (include/gdino_amd.h, gd_attn_forward):
    keep[b, h, q, k] = lowbias32(k*0x9E3779B1 ^ q*0x85EBCA77 ^ (b*H+h)*0xC2B2AE3D
    ^ seed) >= p * 2^32, restated in numpy uint32 arithmetic."""
    M = np.uint32(0xFFFFFFFF)
    k = np.arange(Lk, dtype=np.uint64)[None, None, :]
    q = np.arange(Lq, dtype=np.uint64)[None, :, None]
    bh = np.arange(B * H, dtype=np.uint64)[:, None, None]
    x = ((k * 0x9E3779B1) & 0xFFFFFFFF) ^ ((q * 0x85EBCA77) & 0xFFFFFFFF) ^ ((bh * 0xC2B2AE3D) & 0xFFFFFFFF) ^ seed
    x = x.astype(np.uint64)
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    thresh = min(int(p * 4294967296.0), int(M))
    return torch.from_numpy((x >= thresh).reshape(B, H, Lq, Lk))


def rel_err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def linear_sum_assignment(cost, sizes):
    """cost [P, Q, K] f32, sizes [P] int -> (rows, cols, status) as the device
    gd_linear_sum_assignment writes them"""
    cost = cost.float().contiguous()
    P, Q, K = cost.shape
    sizes = torch.as_tensor(sizes, dtype=torch.int32).contiguous()
    rows = torch.full((P, K), 7777, dtype=torch.int64)
    cols = torch.full((P, K), 7777, dtype=torch.int64)
    status = torch.full((P,), 7, dtype=torch.int32)
    _check(lib().gd_linear_sum_assignment(_ptr(cost), P, Q, K, Q * K, _ptr(sizes), _ptr(rows), _ptr(cols),
                                          _ptr(status), None))
    return rows, cols, status
