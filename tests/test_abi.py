"""CPU-side checks of the C-ABI boundary: the shared library exists, loads,
and exports every entry point declared in include/gdino_amd.h (no compute
calls — there is no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "gdino_amd.h")
LIB = os.path.join(PKG, "gdino_amd", "lib", "libgdino_amd.so")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gd_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_core_entry_points():
    syms = declared_symbols()
    for s in ("gd_msda_forward", "gd_msda_backward", "gd_last_error", "gd_runtime_info",
              "gd_abi_version"):
        assert s in syms


def test_library_built_and_exports_header():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    lib.gd_abi_version.restype = ctypes.c_int
    assert lib.gd_abi_version() == 1


def test_library_targets_gfx950_only():
    blob = open(LIB, "rb").read()
    assert b"gfx950" in blob
    for other in (b"gfx942", b"gfx90a", b"gfx1100"):
        assert other not in blob


def test_python_binding_signatures_cover_header():
    from gdino_amd import _lib
    import gdino_amd.kernels  # noqa: F401  (kernel modules register their signatures)
    import gdino_amd.msda  # noqa: F401
    import gdino_amd.misc  # noqa: F401
    import gdino_amd.stepgraph  # noqa: F401
    compute = [s for s in declared_symbols()
               if s not in ("gd_last_error", "gd_runtime_info", "gd_abi_version") and not s.endswith("_bytes")]
    missing = [s for s in compute if s not in _lib._SIGNATURES]
    assert not missing, missing


def test_product_refuses_cpu_tensors():
    """The HIP-only ops raise on host tensors (as the reference's CPU stub);
    MSDA, which the reference dispatches by device, runs its C++ CPU backend
    (tests/test_msda_cpu_backend.py)."""
    import torch
    from gdino_amd.wattn import WindowAttnFunction
    with pytest.raises(RuntimeError, match="Not implemented on the CPU"):
        WindowAttnFunction.apply(torch.zeros(2, 49, 3, 1, 32), torch.zeros(169, 1),
                                 torch.zeros(49 * 49, dtype=torch.long), None, 1.0)
    from gdino_amd import msda
    v = torch.ones(1, 4, 1, 2)
    shapes = torch.tensor([[2, 2]])
    lsi = torch.tensor([0])
    loc = torch.full((1, 1, 1, 1, 1, 2), 0.5)
    attn = torch.ones(1, 1, 1, 1, 1)
    out = msda.ms_deform_attn_forward(v, shapes, lsi, loc, attn, 64)
    assert torch.allclose(out, torch.ones(1, 1, 2))


def test_msda_module_is_a_drop_in_for_the_reference_extension():
    """replacing `import MultiScaleDeformableAttention as
    MSDA` (ops/functions/ms_deform_attn_func.py:18) with `from gdino_amd
    import msda as MSDA` works because the call shapes of :25-26 and :35-36
    are accepted positionally."""
    import inspect
    from gdino_amd import msda
    fwd = list(inspect.signature(msda.ms_deform_attn_forward).parameters.values())
    bwd = list(inspect.signature(msda.ms_deform_attn_backward).parameters.values())
    # reference passes 6 (fwd) / 7 (bwd) positional arguments, nothing else
    assert len([p for p in fwd if p.default is inspect.Parameter.empty]) <= 6 <= len(fwd)
    assert len([p for p in bwd if p.default is inspect.Parameter.empty]) <= 7 <= len(bwd)
    assert [p.name for p in bwd[5:7]] == ["grad_output", "im2col_step"]


def test_call_timer_brackets_every_entry_point(monkeypatch):
    """_lib.CallTimer (bench.py's per-entry-point pass): events recorded
    before and after each C-ABI call, summed per entry point; a failing call
    still raises and records nothing."""
    import itertools

    import torch

    from gdino_amd import _lib

    clock = itertools.count()

    class FakeEvent:
        def __init__(self, enable_timing=False):
            assert enable_timing

        def record(self):
            self.t = next(clock)

        def elapsed_time(self, other):
            return float(other.t - self.t)

    class FakeLib:
        def gd_a(self, *args):
            return _lib.GD_OK

        def gd_hbm(self, *args):
            return _lib.GD_OK

        def gd_mfma(self, *args):
            return _lib.GD_OK

        def gd_bad(self, *args):
            return _lib.GD_OK + 1

        def gd_last_error(self):
            return b"boom"

    fake = FakeLib()
    monkeypatch.setattr(torch.cuda, "Event", FakeEvent)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(_lib, "lib", lambda: fake)
    monkeypatch.setattr(_lib, "call_timer", _lib.CallTimer())
    for _ in range(3):
        _lib.call("gd_a", 1, 2)
    with pytest.raises(_lib.GdError, match="boom"):
        _lib.call("gd_bad")
    _lib.call("gd_mfma", flops=1e12)
    _lib.call("gd_mfma", flops=2e12)
    _lib.call("gd_a", nbytes=1e9)  # bytes given on some calls only: no GB/s
    _lib.call("gd_hbm", nbytes=4e9)
    s = _lib.call_timer.summary()
    assert set(s) == {"gd_a", "gd_mfma", "gd_hbm"}
    assert "GBps" not in s["gd_a"] and "GBps" not in s["gd_mfma"]
    assert s["gd_hbm"]["GBps"] == pytest.approx(4000.0) and s["gd_hbm"]["hbm_frac"] == pytest.approx(0.5)
    assert s["gd_a"]["calls"] == 4 and s["gd_a"]["total_ms"] == 4.0 and s["gd_a"]["avg_us"] == 1000.0
    assert "tflops" not in s["gd_a"]
    # 3e12 flops in 2 ms = 1500 TFLOP/s, 0.6 of the 2.5 PFLOP/s dense bf16 peak
    assert s["gd_mfma"]["tflops"] == pytest.approx(1500.0) and s["gd_mfma"]["mfma_frac"] == pytest.approx(0.6)
