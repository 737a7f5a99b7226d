"""oracle — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference algorithms on the hot path, used as the
parity checker for the HIP kernels.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import this package; the product
path (``open-groundingdino_amd/``) never does.

Parity pinning: the MSDA restatements here are checked against golden vectors
generated from the reference's own pure-PyTorch function
``ms_deform_attn_core_pytorch`` (/root/reference/models/GroundingDINO/ops/
functions/ms_deform_attn_func.py:41-61) by ``tests/golden/make_golden.py``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        lp = ctypes.POINTER(ctypes.c_int64)
        i = ctypes.c_int
        _lib.oracle_msda_forward.argtypes = [dp, lp, lp, dp, dp, i, i, i, i, i, i, i, dp]
        _lib.oracle_msda_backward.argtypes = [dp, lp, lp, dp, dp, dp, i, i, i, i, i, i, i, dp, dp, dp]
    return _lib


def _d(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _cp(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def msda_forward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight):
    """C oracle forward. numpy/torch-CPU inputs -> numpy fp64 [N, Lq, M*D]."""
    value, loc, attn = _d(value), _d(sampling_loc), _d(attn_weight)
    shapes = np.ascontiguousarray(spatial_shapes, dtype=np.int64)
    lsi = np.ascontiguousarray(level_start_index, dtype=np.int64)
    N, S, M, D = value.shape
    _, Lq, _, L, P, _ = loc.shape
    out = np.zeros((N, Lq, M * D), dtype=np.float64)
    _load().oracle_msda_forward(_cp(value, ctypes.c_double), _cp(shapes, ctypes.c_int64),
                                _cp(lsi, ctypes.c_int64), _cp(loc, ctypes.c_double),
                                _cp(attn, ctypes.c_double), N, S, M, D, L, Lq, P,
                                _cp(out, ctypes.c_double))
    return out


def msda_backward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, grad_output):
    """C oracle backward -> (grad_value, grad_loc, grad_attn) numpy fp64."""
    value, loc, attn, go = _d(value), _d(sampling_loc), _d(attn_weight), _d(grad_output)
    shapes = np.ascontiguousarray(spatial_shapes, dtype=np.int64)
    lsi = np.ascontiguousarray(level_start_index, dtype=np.int64)
    N, S, M, D = value.shape
    _, Lq, _, L, P, _ = loc.shape
    gv = np.zeros_like(value)
    gl = np.zeros_like(loc)
    ga = np.zeros_like(attn)
    _load().oracle_msda_backward(_cp(value, ctypes.c_double), _cp(shapes, ctypes.c_int64),
                                 _cp(lsi, ctypes.c_int64), _cp(loc, ctypes.c_double),
                                 _cp(attn, ctypes.c_double), _cp(go, ctypes.c_double),
                                 N, S, M, D, L, Lq, P, _cp(gv, ctypes.c_double),
                                 _cp(gl, ctypes.c_double), _cp(ga, ctypes.c_double))
    return gv, gl, ga
