"""ctypes binding of libgdino_amd.so (the C-ABI declared in include/gdino_amd.h).

This is the only door from Python into the HIP kernels.  There is no CPU or
eager-PyTorch fallback behind it: if the library is missing, or a tensor is
not on a ROCm device, the call raises — mirroring the reference extension,
whose CPU backend raises "Not implemented on the CPU"
(models/GroundingDINO/ops/src/ms_deform_attn.h:38,60).

The one exception is the op the reference dispatches by device: MSDA on
HOST tensors runs libgdino_cpu.so (csrc/cpu/msda_cpu.cpp), a C++/OpenMP
implementation exported under the same C-ABI with a NULL stream, where the
reference has its AT_ERROR stub.  Device tensors never reach it.
"""
from __future__ import annotations

import ctypes
import functools
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GDINO_AMD_LIB", os.path.join(_HERE, "lib", "libgdino_amd.so"))

GD_OK, GD_ERR_INVALID, GD_ERR_UNSUPPORTED, GD_ERR_LAUNCH = 0, 1, 2, 3
GD_F32, GD_F64, GD_BF16, GD_F16 = 0, 1, 2, 3

_DTYPE_CODE = {
    torch.float32: GD_F32,
    torch.float64: GD_F64,
    torch.bfloat16: GD_BF16,
    torch.float16: GD_F16,
}

_lock = threading.Lock()
_lib = None

_p = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float

# name -> (argtypes) ; every function returns gd_status (int)
_SIGNATURES = {
    "gd_msda_forward": [_i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p],
    "gd_msda_backward": [_i, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p],
    "gd_msda_backward_geom": [_i, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p],
}


class GdError(RuntimeError):
    """A C-ABI call returned a non-OK gd_status."""


def lib() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raise if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"gdino_amd: HIP library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (make -C "
                "open-groundingdino_amd/csrc)"
            )
        # torch must own the HIP runtime first so the library binds to it
        # (same soname libamdhip64.so.7) and torch's streams stay valid.
        import torch.cuda  # noqa: F401

        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        handle.gd_last_error.restype = ctypes.c_char_p
        handle.gd_runtime_info.restype = ctypes.c_char_p
        handle.gd_abi_version.restype = ctypes.c_int
        if handle.gd_abi_version() != 1:
            raise RuntimeError("gdino_amd: ABI version mismatch")
        _lib = handle
        return _lib


def register(name: str, argtypes) -> None:
    """Declare the signature of an additional entry point (used by kernel
    modules that extend the ABI)."""
    _SIGNATURES[name] = argtypes
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int


class CallTimer:
    """HIP events around every C-ABI call, recorded on torch's current stream
    (the stream every entry point is handed): launches and device time per
    entry point.  bench.py runs one extra step after the timed region with
    it, so the per-kernel figures cost the measured step nothing."""

    def __init__(self):
        self.records = []  # (entry point, start event, end event, algorithmic flops, algorithmic bytes)

    def begin(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def end(self, name, start, flops=None, nbytes=None):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.records.append((name, start, ev, flops, nbytes))

    def summary(self):
        """{entry point: {"calls": n, "total_ms": t, "avg_us": t / n}}, plus
        for the MFMA entry points (those given algorithmic flops) "tflops" and
        "mfma_frac" against the dense bf16 MFMA peak, and for the HBM-bound
        ones (given algorithmic bytes) "GBps" and "hbm_frac" against 8 TB/s."""
        if self.records:
            torch.cuda.synchronize()
        out = {}
        for name, s, e, flops, nbytes in self.records:
            d = out.setdefault(name, {"calls": 0, "total_ms": 0.0, "flops": 0.0 if flops is not None else None,
                                      "bytes": 0.0 if nbytes is not None else None})
            d["calls"] += 1
            d["total_ms"] += s.elapsed_time(e)
            for key, v in (("flops", flops), ("bytes", nbytes)):
                d[key] = d[key] + v if (v is not None and d[key] is not None) else None
        for d in out.values():
            d["avg_us"] = d["total_ms"] / d["calls"] * 1e3
            fl, nb = d.pop("flops"), d.pop("bytes")
            sec = d["total_ms"] * 1e-3
            if fl is not None and sec > 0:
                d["tflops"] = fl / sec / 1e12
                d["mfma_frac"] = fl / sec / MFMA_BF16_PEAK
            if nb is not None and sec > 0:
                d["GBps"] = nb / sec / 1e9
                d["hbm_frac"] = nb / sec / HBM_PEAK
        return out


call_timer = None  # set to a CallTimer to time every entry point
MFMA_BF16_PEAK = 2.5e15  # FLOP/s, dense bf16 (MI355X_MICROARCH.md chip table)
HBM_PEAK = 8.0e12  # B/s, same table


CPU_LIB_PATH = os.environ.get("GDINO_CPU_LIB", os.path.join(_HERE, "lib", "libgdino_cpu.so"))
_cpu_lib = None
# the MSDA core: the only entry points the CPU backend exports
_CPU_ENTRY_POINTS = ("gd_msda_forward", "gd_msda_backward", "gd_msda_backward_geom")


def cpu_lib() -> ctypes.CDLL:
    """Load (once) the CPU backend of the MSDA op (same C-ABI, host pointers,
    NULL stream); raise if it is not built."""
    global _cpu_lib
    if _cpu_lib is not None:
        return _cpu_lib
    with _lock:
        if _cpu_lib is None:
            if not os.path.exists(CPU_LIB_PATH):
                raise RuntimeError(f"gdino_amd: CPU backend not found at {CPU_LIB_PATH}; build it with "
                                   "make -C open-groundingdino_amd/csrc")
            handle = ctypes.CDLL(CPU_LIB_PATH, mode=ctypes.RTLD_LOCAL)
            for name in _CPU_ENTRY_POINTS:
                fn = getattr(handle, name)
                fn.argtypes = _SIGNATURES[name]
                fn.restype = ctypes.c_int
            handle.gd_last_error.restype = ctypes.c_char_p
            handle.gd_runtime_info.restype = ctypes.c_char_p
            if handle.gd_abi_version() != 1:
                raise RuntimeError("gdino_amd: CPU backend ABI version mismatch")
            _cpu_lib = handle
    return _cpu_lib


def call_cpu(name: str, *args) -> None:
    """Run MSDA entry point ``name`` of the CPU backend (stream argument NULL)."""
    status = getattr(cpu_lib(), name)(*args)
    if status != GD_OK:
        msg = cpu_lib().gd_last_error().decode(errors="replace")
        raise GdError(f"{name} (CPU backend): status {status}: {msg}")


def call(name: str, *args, flops: float | None = None, nbytes: float | None = None) -> None:
    """Run entry point ``name``; raise GdError on a non-OK status.  ``flops``
    (MFMA entry points) and ``nbytes`` (HBM-bound ones), both algorithmic,
    feed CallTimer's TFLOP/s and GB/s."""
    timer = call_timer
    start = timer.begin() if timer is not None else None
    status = getattr(lib(), name)(*args)
    if status != GD_OK:
        msg = lib().gd_last_error().decode(errors="replace")
        raise GdError(f"{name}: status {status}: {msg}")
    if timer is not None:
        timer.end(name, start, flops, nbytes)


def runtime_info() -> str:
    return lib().gd_runtime_info().decode()


def dtype_code(t: torch.Tensor) -> int:
    try:
        return _DTYPE_CODE[t.dtype]
    except KeyError:
        raise TypeError(f"gdino_amd: unsupported dtype {t.dtype}") from None


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def on_device(t: torch.Tensor) -> bool:
    """Whether t lives where the HIP library operates (a ROCm device)."""
    return t.is_cuda


def require_device(*tensors: torch.Tensor, what: str = "op") -> None:
    for t in tensors:
        if t is None:
            continue
        if not on_device(t):
            raise RuntimeError(f"gdino_amd {what}: Not implemented on the CPU (tensor on {t.device})")


def require_contiguous(what: str, **tensors: torch.Tensor) -> None:
    for name, t in tensors.items():
        if t is not None and not t.is_contiguous():
            raise RuntimeError(f"{name} tensor has to be contiguous ({what})")


@functools.lru_cache(maxsize=8)
def _disabled(spec: str) -> frozenset:
    return frozenset(x.strip() for x in spec.split(",") if x.strip())


def enabled(family: str) -> bool:
    """False when ``family`` is listed in GDINO_DISABLE (comma-separated:
    wattn, attn, contrastive, prologue, wgrad, addln).  A disabled family runs
    its torch composition (ROCm library kernels) instead -- for A/B runs and
    bisection on the box; the MSDA core and BiAttention kernels have no such
    switch (GD_MSDA_BWD=lane32 selects the round-1 MSDA backward)."""
    spec = os.environ.get("GDINO_DISABLE")
    return not spec or family not in _disabled(spec)


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()
