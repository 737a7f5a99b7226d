"""Op-level MSDA API: a drop-in for the reference extension module
``MultiScaleDeformableAttention`` (models/GroundingDINO/ops/src/vision.cpp:13-16),
backed by the HIP kernels of csrc/msda.hip through the C-ABI.

Contract kept from ops/src/cuda/ms_deform_attn_cuda.cu:20-153:
  * inputs must be contiguous device tensors, else RuntimeError;
  * ``batch % min(batch, im2col_step) == 0`` else RuntimeError;
  * outputs are freshly allocated and owned by the caller;
  * work is enqueued on the current stream.
Device dispatch as the reference's ops/src/ms_deform_attn.h:20-61: device
tensors run the gfx950 kernels, HOST tensors the C++ CPU backend
(libgdino_cpu.so, same C-ABI, NULL stream) where the reference raises "Not
implemented on the CPU"; mixing devices raises.
Differences (documented in DESIGN.md): the whole batch is one launch (no
im2col_step chunking — it only bounded the reference's column buffer), bf16
``value`` is accepted (fp32 accumulate; sampling locations / weights stay
fp32), and launch errors raise instead of being printed.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib

_p, _i = ctypes.c_void_p, ctypes.c_int
_lib.register("gd_msda_backward_sorted", [_i, _p, _p, _p, _p, _p, _p] + [_i] * 7 +
              [_p, _i, _p, _p, _p, _p, ctypes.c_size_t, _i, _p])
_lib.register("gd_device_status", [_p])
GD_MSDA_DETERMINISTIC = 1


def check_device_status(device=None) -> None:
    """Synchronise the current stream and raise GdError when a device-side
    check of the MSDA kernels fired since the last call (the sorted
    backward's record-slot guard: a record it refused to store out of
    bounds).  The check word is cleared by the read."""
    dev = torch.device(device or "cuda")
    _lib.call("gd_device_status", torch.cuda.current_stream(dev).cuda_stream)


def _workspace_bytes(dt, N, S, M, D, L, Lq, P, hs, flags) -> int:
    fn = _lib.lib().gd_msda_backward_workspace_bytes
    fn.restype = ctypes.c_size_t
    fn.argtypes = [_i] * 8 + [_p, _i]
    return int(fn(dt, N, S, M, D, L, Lq, P, hs, flags))


def deterministic() -> bool:
    """Deterministic MSDA backward (GD_MSDA_DETERMINISTIC flag of the sorted
    kernel): torch.use_deterministic_algorithms(True) or GD_MSDA_DETERMINISTIC=1."""
    return torch.are_deterministic_algorithms_enabled() or os.environ.get("GD_MSDA_DETERMINISTIC") == "1"


def backward_variant() -> str:
    """GD_MSDA_BWD: sorted (default: the atomic-free csrc/msda_sorted.inc for
    the encoder shape, lane32 for the decoder), sorted-all (sorted for every
    call), or the round-1/2 kernels for A/B runs: enc / lane32 / tiled."""
    return os.environ.get("GD_MSDA_BWD", "sorted")


class LaunchTimer:
    """Optional HIP-event bracketing of every MSDA launch (bench.py's live
    roofline measurement).  Events are recorded on the launch stream (torch's
    current stream, which is where the C-ABI call enqueues the kernel).  Not
    inside a HIP-graph capture: ROCm refuses timing events there (torch's
    ``external`` events are disallowed), so launches replayed from a graph are
    timed in an eager step instead (bench.py)."""

    def __init__(self):
        self.records = []  # (kind, lq, bytes, start_event, end_event)

    def begin(self):
        if torch.cuda.is_current_stream_capturing():
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def end(self, kind, lq, nbytes, start):
        if start is None:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.records.append((kind, lq, nbytes, start, ev))

    def summary(self):
        if self.records:
            torch.cuda.synchronize()
        out = {}
        for kind, lq, nbytes, s, e in self.records:
            d = out.setdefault((kind, lq), {"n": 0, "ms": 0.0, "bytes": nbytes})
            d["n"] += 1
            d["ms"] += s.elapsed_time(e)
        return out


timer = None  # set to a LaunchTimer to measure


def algorithmic_bytes(kind, N, S, M, D, L, Lq, P, sv, sf=4, so=None, sg=4):
    """SURVEY §8d per-launch algorithmic traffic.  fwd: value + (loc, attn) +
    out.  bwd: value + grad_value (sg bytes per element: fp32 for the atomic
    kernels' accumulation buffer, the value dtype when the sorted kernel
    writes it directly) + 2x(loc, attn, grads) + grad_out."""
    so = sv if so is None else so
    if kind == "fwd":
        return sv * N * S * M * D + 3 * sf * N * Lq * M * L * P + so * N * Lq * M * D
    return sv * N * S * M * D + sg * N * S * M * D + 6 * sf * N * Lq * M * L * P + so * N * Lq * M * D


def _acc_dtype(value: torch.Tensor) -> torch.dtype:
    return torch.float64 if value.dtype == torch.float64 else torch.float32


def _on_host(*tensors) -> bool:
    """True when every tensor is a host tensor (the CPU backend), False when
    every one is on the ROCm device; raise on a mix."""
    devs = {t.is_cuda for t in tensors if t is not None}
    if len(devs) > 1:
        raise RuntimeError("ms_deform_attn: tensors must all be on one device, the CPU (host backend) or the ROCm device")
    return devs == {False}


def _check(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, im2col_step, extra=()):
    if not _on_host(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, *extra):
        _lib.require_device(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, *extra,
                            what="ms_deform_attn")
    _lib.require_contiguous("ms_deform_attn", value=value, spatial_shapes=spatial_shapes,
                            level_start_index=level_start_index, sampling_loc=sampling_loc,
                            attn_weight=attn_weight)
    if value.dim() != 4:
        raise RuntimeError(f"value must be [N, S, M, D], got {tuple(value.shape)}")
    N, S, M, D = value.shape
    if sampling_loc.dim() != 6 or sampling_loc.size(-1) != 2:
        raise RuntimeError(f"sampling_loc must be [N, Lq, M, L, P, 2], got {tuple(sampling_loc.shape)}")
    L = spatial_shapes.size(0)
    _, Lq, M2, L2, P, _ = sampling_loc.shape
    if sampling_loc.size(0) != N or M2 != M or L2 != L:
        raise RuntimeError("sampling_loc shape does not match value / spatial_shapes")
    if tuple(attn_weight.shape) != (N, Lq, M, L, P):
        raise RuntimeError(f"attn_weight must be {(N, Lq, M, L, P)}, got {tuple(attn_weight.shape)}")
    if spatial_shapes.dtype != torch.int64 or level_start_index.dtype != torch.int64:
        raise RuntimeError("spatial_shapes / level_start_index must be int64")
    step = min(N, int(im2col_step)) if N > 0 else 1
    if step <= 0 or N % step != 0:
        raise RuntimeError(f"batch({N}) must divide im2col_step({step})")
    acc = _acc_dtype(value)
    if sampling_loc.dtype != acc:
        sampling_loc = sampling_loc.to(acc).contiguous()
    if attn_weight.dtype != acc:
        attn_weight = attn_weight.to(acc).contiguous()
    return (N, S, M, D, L, Lq, P), sampling_loc, attn_weight


def ms_deform_attn_forward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight,
                           im2col_step: int = 64) -> torch.Tensor:
    """-> output [N, Lq, M*D] (value dtype)."""
    (N, S, M, D, L, Lq, P), loc, attn = _check(value, spatial_shapes, level_start_index,
                                               sampling_loc, attn_weight, im2col_step)
    out = torch.empty((N, Lq, M * D), dtype=value.dtype, device=value.device)
    if not value.is_cuda:  # C++ CPU backend, same C-ABI, NULL stream
        _lib.call_cpu("gd_msda_forward", _lib.dtype_code(value), value.data_ptr(), spatial_shapes.data_ptr(),
                      level_start_index.data_ptr(), loc.data_ptr(), attn.data_ptr(), N, S, M, D, L, Lq, P,
                      out.data_ptr(), None)
        return out
    nbytes = algorithmic_bytes("fwd", N, S, M, D, L, Lq, P, value.element_size())
    t0 = timer.begin() if timer is not None else None
    _lib.call("gd_msda_forward", _lib.dtype_code(value), value.data_ptr(), spatial_shapes.data_ptr(),
              level_start_index.data_ptr(), loc.data_ptr(), attn.data_ptr(), N, S, M, D, L, Lq, P,
              out.data_ptr(), _lib.stream_of(value), nbytes=nbytes)
    if t0 is not None:
        timer.end("fwd", Lq, nbytes, t0)
    return out


def host_level_shapes(spatial_shapes):
    """The host copy of the level shapes the model attaches to its cached
    spatial_shapes tensor (``gd_host_shapes``), or None.  Never syncs."""
    return getattr(spatial_shapes, "gd_host_shapes", None)


def ms_deform_attn_backward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight,
                            grad_output, im2col_step: int = 64, grad_value_dtype=None, host_shapes=None):
    """-> [grad_value, grad_sampling_loc, grad_attn_weight].

    grad_value is accumulated in fp32 (fp64 for fp64 value); it is returned in
    ``grad_value_dtype`` (default: value.dtype, as the reference).
    ``host_shapes`` ([(H, W)] per level, host ints) lets the encoder-shape
    backward tile by pixel blocks (gd_msda_backward_geom)."""
    (N, S, M, D, L, Lq, P), loc, attn = _check(value, spatial_shapes, level_start_index,
                                               sampling_loc, attn_weight, im2col_step,
                                               extra=(grad_output,))
    if grad_output.dtype != value.dtype:
        grad_output = grad_output.to(value.dtype)
    grad_output = grad_output.contiguous()
    if grad_output.numel() != N * Lq * M * D:
        raise RuntimeError("grad_output must be [N, Lq, M*D]")
    acc = _acc_dtype(value)
    hs = None
    if host_shapes is not None and len(host_shapes) == L:
        hs = (ctypes.c_int64 * (2 * L))(*[int(v) for hw in host_shapes for v in hw])
    variant = backward_variant()
    # sorted: the encoder shape (Lq == S) by default; the decoder's 900
    # score-sorted queries crowd a few cells (the lane-group walk then has a
    # long tail: 173 us in the train step vs 114 us for the direct-atomic
    # kernel), so it keeps msda_bwd_lane32 unless determinism is asked for
    if value.is_cuda and hs is not None and (variant == "sorted" and (Lq == S or deterministic())
                                             or variant == "sorted-all"):
        out = _backward_sorted(value, spatial_shapes, level_start_index, loc, attn, grad_output,
                               (N, S, M, D, L, Lq, P), hs, grad_value_dtype)
        if out is not None:
            return _finish_grads(value, sampling_loc, attn_weight, *out, grad_value_dtype)
    grad_value = torch.empty((N, S, M, D), dtype=acc, device=value.device)
    grad_loc = torch.empty((N, Lq, M, L, P, 2), dtype=acc, device=value.device)
    grad_attn = torch.empty((N, Lq, M, L, P), dtype=acc, device=value.device)
    if not value.is_cuda:  # C++ CPU backend, same C-ABI, NULL stream
        _lib.call_cpu("gd_msda_backward", _lib.dtype_code(value), value.data_ptr(), spatial_shapes.data_ptr(),
                      level_start_index.data_ptr(), loc.data_ptr(), attn.data_ptr(), grad_output.data_ptr(),
                      N, S, M, D, L, Lq, P, grad_value.data_ptr(), grad_loc.data_ptr(), grad_attn.data_ptr(), None)
        return _finish_grads(value, sampling_loc, attn_weight, grad_value, grad_loc, grad_attn, grad_value_dtype)
    nbytes = algorithmic_bytes("bwd", N, S, M, D, L, Lq, P, value.element_size())
    t0 = timer.begin() if timer is not None else None
    _lib.call("gd_msda_backward_geom", _lib.dtype_code(value), value.data_ptr(), spatial_shapes.data_ptr(),
              level_start_index.data_ptr(), loc.data_ptr(), attn.data_ptr(), grad_output.data_ptr(),
              N, S, M, D, L, Lq, P, grad_value.data_ptr(), grad_loc.data_ptr(), grad_attn.data_ptr(),
              hs, _lib.stream_of(value), nbytes=nbytes)
    if t0 is not None:
        timer.end("bwd", Lq, nbytes, t0)
    return _finish_grads(value, sampling_loc, attn_weight, grad_value, grad_loc, grad_attn, grad_value_dtype)


def _backward_sorted(value, shapes, lsi, loc, attn, grad_output, dims, hs, grad_value_dtype):
    """gd_msda_backward_sorted (no float atomics; bitwise deterministic when
    deterministic()): grad_value written once per row, directly in
    grad_value_dtype when that is value.dtype or fp32.  None when the kernel
    does not apply to these sizes (the caller then runs gd_msda_backward_geom)."""
    N, S, M, D, L, Lq, P = dims
    out_dtype = value.dtype if grad_value_dtype is None else grad_value_dtype
    if out_dtype not in (value.dtype, torch.float32):
        return None
    flags = GD_MSDA_DETERMINISTIC if deterministic() else 0
    dt = _lib.dtype_code(value)
    nws = _workspace_bytes(dt, N, S, M, D, L, Lq, P, hs, flags)
    if nws == 0:
        return None
    ws = torch.empty(nws, dtype=torch.uint8, device=value.device)
    grad_value = torch.empty((N, S, M, D), dtype=out_dtype, device=value.device)
    grad_loc = torch.empty((N, Lq, M, L, P, 2), dtype=torch.float32, device=value.device)
    grad_attn = torch.empty((N, Lq, M, L, P), dtype=torch.float32, device=value.device)
    nbytes = algorithmic_bytes("bwd", N, S, M, D, L, Lq, P, value.element_size(), sg=grad_value.element_size())
    t0 = timer.begin() if timer is not None else None
    _lib.call("gd_msda_backward_sorted", dt, value.data_ptr(), shapes.data_ptr(), lsi.data_ptr(), loc.data_ptr(),
              attn.data_ptr(), grad_output.data_ptr(), N, S, M, D, L, Lq, P, grad_value.data_ptr(),
              _lib.dtype_code(grad_value), grad_loc.data_ptr(), grad_attn.data_ptr(), hs, ws.data_ptr(), nws, flags,
              _lib.stream_of(value), nbytes=nbytes)
    if t0 is not None:
        timer.end("bwd", Lq, nbytes, t0)
    return [grad_value, grad_loc, grad_attn]


def _finish_grads(value, sampling_loc, attn_weight, grad_value, grad_loc, grad_attn, grad_value_dtype):
    out_dtype = value.dtype if grad_value_dtype is None else grad_value_dtype
    if grad_value.dtype != out_dtype:
        grad_value = grad_value.to(out_dtype)
    if grad_loc.dtype != sampling_loc.dtype:
        grad_loc = grad_loc.to(sampling_loc.dtype)
        grad_attn = grad_attn.to(attn_weight.dtype)
    return [grad_value, grad_loc, grad_attn]
