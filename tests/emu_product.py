"""Run the PRODUCT's HIP path on the CPU: the model's autograd functions and
ctypes calls exactly as on the box, with libgdino_amd.so swapped for the
host-side SIMT emulator build of the same kernel sources (tests/emu) and
host tensors accepted as "device" tensors.

TEST INFRASTRUCTURE ONLY.  It checks the integration of the kernels into the
model -- strides, dtypes, views, autograd wiring, which kernel each call
reaches -- when no GPU is reachable; it says nothing about speed.
"""
import contextlib
import ctypes

import emu_lib


@contextlib.contextmanager
def emulated_product(min_tokens=None):
    from gdino_amd import _lib, wgrad
    emu = emu_lib.lib()
    for name, argtypes in _lib._SIGNATURES.items():
        if name.startswith(("gd_graph_", "gd_stream_")):  # HIP graph / capture runtime API: no emulator twin
            continue
        fn = getattr(emu, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    saved = (_lib._lib, _lib.on_device, _lib.stream_of, wgrad.MIN_TOKENS, wgrad.TN_MIN_TOKENS)
    _lib._lib = emu
    _lib.on_device = lambda t: True
    _lib.stream_of = lambda t: None
    if min_tokens is not None:  # the split-K thresholds (weight gradients, long-K products)
        wgrad.MIN_TOKENS = min_tokens
        wgrad.TN_MIN_TOKENS = min_tokens
    try:
        yield
    finally:
        _lib._lib, _lib.on_device, _lib.stream_of, wgrad.MIN_TOKENS, wgrad.TN_MIN_TOKENS = saved
