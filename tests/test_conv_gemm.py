"""GEMM formulation of the hot path's convolutions (gdino_amd/conv.py) vs
F.conv2d: outputs and input / weight / bias gradients, fp64 (tight) and
under bf16 autocast (bf16 tolerance), for every conv shape the model has:
Swin patch embedding (k=s=4), 1x1 input projections, the 3x3/s2 extra
level; odd spatial sizes included."""
import pytest
import torch
import torch.nn.functional as F

from gdino_amd.conv import GemmConv2d, conv2d_gemm

CASES = [  # (C, O, k, s, p, H, W)
    (3, 96, 4, 4, 0, 32, 48),
    (3, 96, 4, 4, 0, 30, 45),      # floors like the conv
    (192, 256, 1, 1, 0, 13, 21),
    (768, 256, 3, 2, 1, 13, 21),
    (768, 256, 3, 2, 1, 25, 42),
]


@pytest.mark.parametrize("case", CASES)
def test_matches_conv2d_fp64(case):
    c, o, k, s, p, h, w = case
    g = torch.Generator().manual_seed(sum(case))
    x = torch.randn(2, c, h, w, generator=g, dtype=torch.float64, requires_grad=True)
    wt = torch.randn(o, c, k, k, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(o, generator=g, dtype=torch.float64, requires_grad=True)
    ref = F.conv2d(x, wt, b, stride=s, padding=p)
    out = conv2d_gemm(x, wt, b, (s, s), (p, p))
    assert out.shape == ref.shape and out.is_contiguous()
    assert torch.allclose(out, ref, rtol=1e-12, atol=1e-12)
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    gr = torch.autograd.grad(ref, (x, wt, b), gy)
    gm = torch.autograd.grad(out, (x, wt, b), gy)
    for a, r in zip(gm, gr):
        assert torch.allclose(a, r, rtol=1e-11, atol=1e-11)


@pytest.mark.parametrize("case", CASES[:1] + CASES[2:4])
def test_module_under_bf16_autocast(case):
    c, o, k, s, p, h, w = case
    torch.manual_seed(0)
    m = GemmConv2d(c, o, k, stride=s, padding=p)
    x = torch.randn(2, c, h, w)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        out = m(x)
        GemmConv2d.use_gemm = False
        try:
            ref = m(x)
        finally:
            GemmConv2d.use_gemm = True
    assert out.dtype == ref.dtype == torch.bfloat16
    err = (out.float() - ref.float()).abs().max() / ref.float().abs().max()
    assert err < 1e-2
    assert set(m.state_dict()) == {"weight", "bias"}
