"""GPU parity of the fused attention-family kernels against the oracle's
literal restatements of the reference math (oracle/blocks.py), forward and
gradients.  Tolerances: fp32 1e-3, bf16 1e-2 (north_star), relative to the
largest reference magnitude."""
import pytest
import torch

from oracle.blocks import bi_attention_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _bi_inputs(b, h, s, t, hd, dtype, seed=0, pad=True):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(b, h, s, hd, generator=g) * hd ** -0.5
    k = torch.randn(b, h, t, hd, generator=g)
    vv = torch.randn(b, h, s, hd, generator=g)
    vl = torch.randn(b, h, t, hd, generator=g)
    pad_v = torch.zeros(b, s, dtype=torch.bool)
    pad_l = torch.zeros(b, t, dtype=torch.bool)
    if pad:
        pad_v[-1, s * 3 // 4:] = True
        pad_l[0, t // 2:] = True
    return [x.to(dtype) for x in (q, k, vv, vl)], pad_v, pad_l


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 1e-2)])
# T = 40 / 100: strided lane slots (T not a multiple of 64); T = 64 / 128 / 256:
# contiguous vector slots (E = 1 / 2 / 4 elements per lane)
@pytest.mark.parametrize("shape", [(2, 4, 300, 40, 64), (1, 2, 700, 100, 32), (1, 2, 333, 64, 16),
                                   (2, 2, 500, 128, 32), (1, 2, 1000, 256, 32), (2, 4, 2048, 256, 256)])
def test_bi_attention_fwd_bwd(dtype, tol, shape):
    from gdino_amd.biattn import bi_attention_hip
    b, h, s, t, hd = shape
    (q, k, vv, vl), pad_v, pad_l = _bi_inputs(b, h, s, t, hd, dtype)
    ref_in = [x.double().requires_grad_(True) for x in (q, k, vv, vl)]
    rv, rl = bi_attention_ref(*ref_in, pad_v, pad_l)
    gv = torch.randn_like(rv)
    gl = torch.randn_like(rl)
    (rv * gv).sum().backward(retain_graph=True)
    (rl * gl).sum().backward()
    dev_in = [x.to(DEV).requires_grad_(True) for x in (q, k, vv, vl)]
    ov, ol = bi_attention_hip(*dev_in, pad_v.to(DEV), pad_l.to(DEV), 0.0)
    ((ov.float() * gv.to(DEV, torch.float32)).sum() + (ol.float() * gl.to(DEV, torch.float32)).sum()).backward()
    assert _rel(ov.cpu(), rv.detach()) < tol
    assert _rel(ol.cpu(), rl.detach()) < tol
    for name, mine, ref in zip(("dq", "dk", "dvv", "dvl"), dev_in, ref_in):
        assert _rel(mine.grad.cpu(), ref.grad) < tol * 3, name


def test_bi_attention_production_shape_bf16():
    """800x1333 bs=2 fusion layer: S=22223 image tokens, T=256, 4 heads of 256."""
    from gdino_amd.biattn import bi_attention_hip
    from gdino_amd import kernels
    b, h, s, t, hd = 2, 4, 22223, 256, 256
    (q, k, vv, vl), pad_v, pad_l = _bi_inputs(b, h, s, t, hd, torch.bfloat16, seed=3)
    args = [x.to(DEV) for x in (q, k, vv, vl)] + [pad_v.to(DEV), pad_l.to(DEV)]
    ov, ol = bi_attention_hip(*args, 0.0)
    # SDPA composition in fp32 as the on-device reference at this size
    rv, rl = kernels._bi_attention_torch(*[a.float() for a in args[:4]], args[4], args[5], 0.0)
    assert _rel(ov, rv) < 1e-2
    assert _rel(ol, rl) < 1e-2


# --------------------------------------------- Swin window attention (HIP)
def _wattn_inputs(ws, nh, b_, nw, masked, dtype, seed=0):
    from models.GroundingDINO.backbone.swin_transformer import relative_position_index
    g = torch.Generator().manual_seed(seed)
    n = ws * ws
    qkv = torch.randn(b_, n, 3, nh, 32, generator=g).to(dtype)
    table = torch.randn((2 * ws - 1) ** 2, nh, generator=g) * 0.5
    ridx = relative_position_index(ws, ws).reshape(-1)
    mask = torch.where(torch.rand(nw, n, n, generator=g) < 0.3, -100.0, 0.0) if masked else None
    return qkv, table, ridx, mask


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("ws,nh,b_,nw,masked", [
    (7, 3, 2784, 1392, True),   # Swin-T stage 0 at 800x1333 bs=2, shifted blocks
    (7, 12, 192, 96, False),    # stage 2
    (7, 5, 22, 1, False),       # tail blocks
    (3, 2, 6, 3, True),         # N = 9 (mostly padded tokens)
    (8, 4, 16, 4, True),        # N = 64 (no padding)
])
def test_window_attention_fwd_bwd(dtype, tol, ws, nh, b_, nw, masked):
    from gdino_amd.wattn import WindowAttnFunction
    from oracle.blocks import window_attention_packed_ref
    qkv, table, ridx, mask = _wattn_inputs(ws, nh, b_, nw, masked, dtype, seed=ws + nh + b_)
    scale = 32 ** -0.5
    qd = qkv.double().requires_grad_(True)
    td = table.double().requires_grad_(True)
    ref = window_attention_packed_ref(qd, td, ridx, None if mask is None else mask.double(), scale)
    grad = torch.randn(ref.shape, generator=torch.Generator().manual_seed(1)).to(dtype)
    ref.backward(grad.double())
    qg = qkv.to(DEV).requires_grad_(True)
    tg = table.to(DEV).requires_grad_(True)
    out = WindowAttnFunction.apply(qg, tg, ridx.to(DEV), None if mask is None else mask.to(DEV), scale)
    out.backward(grad.to(DEV))
    torch.cuda.synchronize()
    assert _rel(out.cpu(), ref.detach()) < tol
    assert _rel(qg.grad.cpu(), qd.grad) < tol * 3
    assert _rel(tg.grad.cpu(), td.grad) < tol * 3


def test_window_attention_op_dispatch_and_fallback():
    """window_attention_packed runs the HIP kernel for N <= 64 and the torch
    composition for Swin-B/384's 12x12 windows; both agree with the oracle."""
    from gdino_amd import kernels
    from oracle.blocks import window_attention_packed_ref
    for ws in (7, 12):
        qkv, table, ridx, mask = _wattn_inputs(ws, 4, 8, 4, True, torch.float32, seed=ws)
        out = kernels.window_attention_packed(qkv.to(DEV), table.to(DEV), ridx.to(DEV), mask.to(DEV), 32 ** -0.5)
        ref = window_attention_packed_ref(qkv.double(), table.double(), ridx, mask.double(), 32 ** -0.5)
        assert _rel(out.cpu(), ref) < 1e-3, ws


def test_window_attention_rejects_host_tensors():
    from gdino_amd.wattn import WindowAttnFunction
    qkv, table, ridx, mask = _wattn_inputs(7, 2, 4, 2, True, torch.float32)
    with pytest.raises(RuntimeError, match="Not implemented on the CPU"):
        WindowAttnFunction.apply(qkv, table, ridx, mask, 1.0)
