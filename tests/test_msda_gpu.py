"""MSDA parity on the GPU: the HIP kernels (through the C-ABI) vs the oracle.

Mirrors the reference's ops/test.py checks (fwd fp64 allclose, fwd fp32
rtol 1e-2/atol 1e-3, fp64 gradcheck for D in {30, 32, 64, 71}) and adds the
BASELINE shapes: config-1 (512x512) and the 800x1333 encoder/decoder shapes,
fp32 (tolerance 1e-3 per north_star) and bf16 value (tolerance 1e-2).
"""
import numpy as np
import pytest
import torch

import oracle
from msda_cases import KAT_NAMES, cfg1_inputs, edge_excluded_mask, load_case, rel_err_grad_loc as _rel_err_gl

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _msda():
    from gdino_amd import msda
    return msda


def _func():
    from models.GroundingDINO.ops.functions.ms_deform_attn_func import MSDeformAttnFunction
    return MSDeformAttnFunction


def _t(a, dtype=torch.float64):
    return torch.as_tensor(np.asarray(a)).to(DEV, dtype)


def _shapes(c):
    return (torch.as_tensor(c["shapes"]).to(DEV, torch.int64),
            torch.as_tensor(c["lsi"]).to(DEV, torch.int64))


def _rel_err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


# --------------------------------------------------------------------- KATs
def test_library_loads_on_gpu():
    from gdino_amd import _lib
    info = _lib.runtime_info()
    assert "gfx950" in info, info


@pytest.mark.parametrize("name", KAT_NAMES + ["edge"])
def test_forward_fp64_matches_golden(name):
    c = load_case(name)
    shapes, lsi = _shapes(c)
    out = _msda().ms_deform_attn_forward(_t(c["value"]), shapes, lsi, _t(c["loc"]), _t(c["attn"]), 2)
    np.testing.assert_allclose(out.cpu().numpy(), c["out"], rtol=1e-10, atol=1e-13)


def test_forward_float_kat_reference_tolerance():
    # ops/test.py:48-60: fp32, torch.allclose(rtol=1e-2, atol=1e-3)
    c = load_case("kat_fwd_float")
    shapes, lsi = _shapes(c)
    out = _func().apply(_t(c["value"], torch.float32), shapes, lsi, _t(c["loc"], torch.float32),
                        _t(c["attn"], torch.float32), 2)
    assert torch.allclose(out.double().cpu(), torch.from_numpy(c["out"]), rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("name", KAT_NAMES + ["edge"])
def test_backward_fp64_matches_golden(name):
    c = load_case(name)
    shapes, lsi = _shapes(c)
    gv, gl, ga = _msda().ms_deform_attn_backward(_t(c["value"]), shapes, lsi, _t(c["loc"]), _t(c["attn"]),
                                                 _t(c["grad_out"]), 2)
    np.testing.assert_allclose(gv.cpu().numpy(), c["grad_value"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(ga.cpu().numpy(), c["grad_attn"], rtol=1e-9, atol=1e-12)
    # grad_loc is one-sided on kink points (band edges, integer pixel
    # coordinates); which side depends on FMA contraction of loc*W-0.5 (the
    # reference's nvcc build contracts too).  Compare everywhere else.
    keep = ~np.repeat(edge_excluded_mask(c)[..., None], 2, axis=-1)
    np.testing.assert_allclose(gl.cpu().numpy()[keep], c["grad_loc"][keep], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("channels", [30, 32, 64, 71])
def test_gradcheck_fp64(channels):
    # ops/test.py:63-86 — gradcheck of MSDeformAttnFunction in fp64
    c = load_case(f"kat_grad_d{channels}")
    shapes, lsi = _shapes(c)
    value = _t(c["value"]).requires_grad_(True)
    loc = _t(c["loc"]).requires_grad_(True)
    attn = _t(c["attn"]).requires_grad_(True)
    assert torch.autograd.gradcheck(_func().apply, (value, shapes, lsi, loc, attn, 2))


# ------------------------------------------------------- BASELINE config 1
def _cfg1(dtype):
    value, shapes, lsi, loc, attn, grad_out = cfg1_inputs()
    return value, shapes, lsi, loc, attn, grad_out


@pytest.mark.parametrize("vdtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 1e-2)])
def test_cfg1_forward_backward(vdtype, tol):
    value, shapes, lsi, loc, attn, grad_out = _cfg1(vdtype)
    v_dev = value.to(DEV, vdtype)
    go_dev = grad_out.to(DEV, vdtype)
    # oracle on exactly the values the kernel sees (bf16-rounded inputs)
    v_ref = v_dev.double().cpu().numpy()
    go_ref = go_dev.double().cpu().numpy()
    loc32, attn32 = loc.float(), attn.float()
    ref_out = oracle.msda_forward(v_ref, shapes, lsi, loc32.double(), attn32.double())
    ref_gv, ref_gl, ref_ga = oracle.msda_backward(v_ref, shapes, lsi, loc32.double(), attn32.double(), go_ref)
    sh, ls = shapes.to(DEV), lsi.to(DEV)
    out = _msda().ms_deform_attn_forward(v_dev, sh, ls, loc32.to(DEV), attn32.to(DEV), 64)
    assert out.dtype == vdtype
    assert _rel_err(out.double().cpu(), ref_out) < tol
    gv, gl, ga = _msda().ms_deform_attn_backward(v_dev, sh, ls, loc32.to(DEV), attn32.to(DEV), go_dev, 64,
                                                 grad_value_dtype=torch.float32)
    assert _rel_err(gv.cpu(), ref_gv) < 1e-3 if vdtype == torch.float32 else _rel_err(gv.cpu(), ref_gv) < tol
    assert _rel_err(ga.cpu(), ref_ga) < tol
    assert _rel_err_gl(gl.cpu(), ref_gl, loc, shapes) < tol


def test_cfg1_fp32_matches_reference_golden():
    z = load_case("cfg1")
    value, shapes, lsi, loc, attn, grad_out = cfg1_inputs()
    sh, ls = shapes.to(DEV), lsi.to(DEV)
    out = _msda().ms_deform_attn_forward(value.float().to(DEV), sh, ls, loc.float().to(DEV),
                                         attn.float().to(DEV), 64).double().cpu().numpy().reshape(-1)
    np.testing.assert_allclose(out[z["out_idx"]], z["out_val"], rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(out.sum(), z["out_sum"], rtol=1e-5)


def test_forward_is_deterministic_and_linear():
    value, shapes, lsi, loc, attn, _ = _cfg1(torch.float32)
    sh, ls = shapes.to(DEV), lsi.to(DEV)
    v1 = value.float().to(DEV)
    v2 = torch.randn_like(v1)
    l, a = loc.float().to(DEV), attn.float().to(DEV)
    f = lambda v: _msda().ms_deform_attn_forward(v, sh, ls, l, a, 64)  # noqa: E731
    o1 = f(v1)
    assert torch.equal(o1, f(v1))
    lin = f(2.0 * v1 - 3.0 * v2)
    torch.testing.assert_close(lin, 2.0 * o1 - 3.0 * f(v2), rtol=1e-5, atol=1e-5)


# ------------------------------------------------ 800x1333 encoder / decoder
LEVELS_800 = [(100, 167), (50, 84), (25, 42), (13, 21)]


def _big_inputs(lq, seed, n=2, vdtype=torch.float32):
    shapes = torch.as_tensor(LEVELS_800, dtype=torch.long)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    S = int(shapes.prod(1).sum())
    g = torch.Generator(device=DEV).manual_seed(seed)
    M, D, L, P = 8, 32, 4, 4
    value = torch.randn(n, S, M, D, generator=g, device=DEV).to(vdtype)
    # encoder-like: points near their query, occasionally outside the map
    loc = torch.rand(n, lq, M, L, P, 2, generator=g, device=DEV) * 1.1 - 0.05
    attn = torch.rand(n, lq, M, L, P, generator=g, device=DEV) + 1e-5
    attn = attn / attn.sum((-1, -2), keepdim=True)
    grad_out = torch.randn(n, lq, M * D, generator=g, device=DEV).to(vdtype)
    return value, shapes, lsi, loc, attn, grad_out


@pytest.mark.parametrize("lq,vdtype,tol", [(900, torch.float32, 1e-3), (900, torch.bfloat16, 1e-2),
                                           (22223, torch.float32, 1e-3), (22223, torch.bfloat16, 1e-2)])
def test_800x1333_shapes(lq, vdtype, tol):
    """Decoder (900 queries) and encoder (Lq = S = 22 223) shapes at bs=2
    800x1333 against the oracle in fp64: fp32 1e-3, bf16 1e-2 (north_star),
    forward and every gradient (the bf16 encoder row is the product's own
    path: bf16 value, sorted backward)."""
    value, shapes, lsi, loc, attn, grad_out = _big_inputs(lq, seed=lq, vdtype=vdtype)
    sh, ls = shapes.to(DEV), lsi.to(DEV)
    out = _msda().ms_deform_attn_forward(value, sh, ls, loc, attn, 64)
    gv, gl, ga = _msda().ms_deform_attn_backward(value, sh, ls, loc, attn, grad_out, 64,
                                                 grad_value_dtype=torch.float32)
    torch.cuda.synchronize()
    v = value.double().cpu().numpy()
    ref_out = oracle.msda_forward(v, shapes, lsi, loc.double().cpu(), attn.double().cpu())
    ref_gv, ref_gl, ref_ga = oracle.msda_backward(v, shapes, lsi, loc.double().cpu(), attn.double().cpu(),
                                                  grad_out.double().cpu().numpy())
    assert _rel_err(out.double().cpu(), ref_out) < tol
    assert _rel_err(gv.cpu(), ref_gv) < tol
    assert _rel_err(ga.cpu(), ref_ga) < tol
    assert _rel_err_gl(gl.cpu(), ref_gl, loc, shapes) < tol


# ------------------------------- encoder self-attention: tiled LDS backward
def _encoder_inputs(levels, n, seed, vdtype, spread_px=2.0, outlier_frac=0.0):
    """Lq == S (every value position is a query, in value order): points
    within ~spread_px pixels of each query's own position on every level, as
    the encoder samples (transformer.py:471-485 reference points + offsets);
    outlier_frac of the points are redrawn uniformly (boxes too large for the
    LDS accumulator -> the kernel's global-atomic fallback)."""
    shapes = torch.as_tensor(levels, dtype=torch.long)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    S = int(shapes.prod(1).sum())
    M, D, L, P = 8, 32, len(levels), 4
    g = torch.Generator().manual_seed(seed)
    refs = []
    for (h, w) in levels:
        yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
        refs.append(torch.stack([(xx.reshape(-1) + 0.5) / w, (yy.reshape(-1) + 0.5) / h], -1))
    ref = torch.cat(refs).double()  # [S, 2]
    wh = torch.as_tensor([(w, h) for (h, w) in levels], dtype=torch.float64)
    off = torch.randn(n, S, M, L, P, 2, generator=g, dtype=torch.float64) * spread_px / wh[None, None, None, :, None, :]
    loc = ref[None, :, None, None, None, :] + off
    if outlier_frac > 0:
        pick = torch.rand(n, S, M, L, P, 1, generator=g) < outlier_frac
        loc = torch.where(pick, torch.rand(loc.shape, generator=g, dtype=torch.float64) * 1.2 - 0.1, loc)
    value = torch.randn(n, S, M, D, generator=g)
    attn = torch.rand(n, S, M, L, P, generator=g) + 1e-5
    attn = attn / attn.sum((-1, -2), keepdim=True)
    grad_out = torch.randn(n, S, M * D, generator=g)
    return (value.to(vdtype), shapes, lsi, loc.float(), attn.float(), grad_out.to(vdtype))


def _check_bwd_vs_oracle(inputs, tol, host_shapes=None):
    value, shapes, lsi, loc, attn, grad_out = inputs
    dev = [t.to(DEV) for t in inputs]
    gv, gl, ga = _msda().ms_deform_attn_backward(*dev, 64, grad_value_dtype=torch.float32,
                                                 host_shapes=host_shapes)
    torch.cuda.synchronize()
    v = value.double().numpy()
    ref_gv, ref_gl, ref_ga = oracle.msda_backward(v, shapes, lsi, loc.double(), attn.double(),
                                                  grad_out.double().numpy())
    assert _rel_err(gv.cpu(), ref_gv) < tol
    assert _rel_err(ga.cpu(), ref_ga) < tol
    assert _rel_err_gl(gl.cpu(), ref_gl, loc, shapes) < tol
    return gv, gl, ga


@pytest.mark.parametrize("levels,n", [([(6, 9), (3, 5), (2, 3), (1, 2)], 1),     # S=76: tiles cross levels
                                      ([(13, 21), (7, 11), (4, 6), (2, 3)], 2),  # tail tile, n boundary
                                      ([(40, 67), (20, 34), (10, 17), (5, 9)], 2)])
@pytest.mark.parametrize("outliers", [0.0, 0.05])
def test_encoder_tiled_backward_small(levels, n, outliers, monkeypatch):
    monkeypatch.setenv("GD_MSDA_BWD", "tiled")
    _check_bwd_vs_oracle(_encoder_inputs(levels, n, seed=len(levels) + n, vdtype=torch.float32,
                                         outlier_frac=outliers), 1e-3)


@pytest.mark.parametrize("vdtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 1e-2)])
def test_encoder_tiled_backward_800x1333(vdtype, tol, monkeypatch):
    monkeypatch.setenv("GD_MSDA_BWD", "tiled")
    _check_bwd_vs_oracle(_encoder_inputs(LEVELS_800, 2, seed=7, vdtype=vdtype, outlier_frac=0.01), tol)


@pytest.mark.parametrize("vdtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("variant", ["tiled", "auto", "enc", "sorted"])
def test_encoder_pixel_block_backward_800x1333(vdtype, tol, variant, monkeypatch):
    """gd_msda_backward_geom (host level shapes -> 4 x 8 pixel-block tiles
    with GD_MSDA_BWD=tiled), the path the model's encoder takes."""
    monkeypatch.setenv("GD_MSDA_BWD", variant)
    _check_bwd_vs_oracle(_encoder_inputs(LEVELS_800, 2, seed=8, vdtype=vdtype, outlier_frac=0.01), tol,
                         host_shapes=LEVELS_800)


@pytest.mark.parametrize("levels", [[(6, 9), (3, 5), (2, 3), (1, 2)], [(13, 21), (7, 11), (4, 6), (2, 3)]])
@pytest.mark.parametrize("variant", ["tiled", "enc", "sorted"])
def test_encoder_pixel_block_backward_small(levels, variant, monkeypatch):
    monkeypatch.setenv("GD_MSDA_BWD", variant)
    _check_bwd_vs_oracle(_encoder_inputs(levels, 2, seed=3, vdtype=torch.float32, outlier_frac=0.05), 1e-3,
                         host_shapes=levels)


def test_encoder_tiled_matches_direct_atomic_kernel(monkeypatch):
    """Same sums, different order: the LDS-aggregated kernel against the
    round-1 direct-atomic kernel (GD_MSDA_BWD=lane32) on one input."""
    inputs = [t.to(DEV) for t in _encoder_inputs(LEVELS_800, 2, seed=11, vdtype=torch.float32)]
    monkeypatch.setenv("GD_MSDA_BWD", "tiled")
    tiled = _msda().ms_deform_attn_backward(*inputs, 64)
    monkeypatch.setenv("GD_MSDA_BWD", "lane32")
    direct = _msda().ms_deform_attn_backward(*inputs, 64)
    for a, b in zip(tiled, direct):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    # grad_loc / grad_attn do not involve atomics: the same expressions, so
    # they agree to fp32 rounding -- the compiler's FMA contraction differs
    # between the kernels (the round-2 direct kernel selects zeroed corners
    # instead of branching around them), which moves sums that nearly
    # cancel by a few ulp of their terms (2.9e-6 at most on this input)
    torch.testing.assert_close(tiled[1], direct[1], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(tiled[2], direct[2], rtol=1e-5, atol=1e-5)


ENC_TILINGS = [None, "8x16,8x8,4x4,2x4", "4x16,3x8,2x4,1x4", "5x7,3x3,2x2,1x1"]


@pytest.mark.parametrize("tiles", ENC_TILINGS)
@pytest.mark.parametrize("cap,rmax", [("224,96,64,64", 8), ("40,16,8,0", 4), ("500,300,100,100", 0)])
@pytest.mark.parametrize("spread,outliers", [(2.0, 0.01), (6.0, 0.05)])
def test_encoder_enc_backward_tilings_800x1333(tiles, cap, rmax, spread, outliers, monkeypatch):
    """msda_bwd_enc (2-D query tiles per level, one LDS box per sampled
    level): any tile extents, region sizes and clip radius give the oracle's
    sums, including wide offsets whose boxes overflow their region (global
    fallback)."""
    monkeypatch.setenv("GD_MSDA_BWD", "enc")
    monkeypatch.setenv("GD_MSDA_ENC_CAP", cap)
    monkeypatch.setenv("GD_MSDA_ENC_RMAX", str(rmax))
    if tiles:
        monkeypatch.setenv("GD_MSDA_ENC_TILE", tiles)
    _check_bwd_vs_oracle(_encoder_inputs(LEVELS_800, 2, seed=31, vdtype=torch.float32, spread_px=spread,
                                         outlier_frac=outliers), 1e-3, host_shapes=LEVELS_800)


def _init_geometry_loc(levels, n):
    """The reference initialisation's encoder sampling locations
    (ms_deform_attn.py:198-221: zero offset weights, per-head direction x
    (point + 1) pixel biases): every point lands (up to fp32 rounding) on an
    integer pixel coordinate, so floor() sits on a cell edge -- the geometry
    the train-step bench runs at."""
    import math
    M, P = 8, 4
    refs = []
    for (h, w) in levels:
        yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
        refs.append(torch.stack([(xx.reshape(-1) + 0.5) / w, (yy.reshape(-1) + 0.5) / h], -1))
    ref = torch.cat(refs)
    ang = torch.arange(M, dtype=torch.float32) * (2 * math.pi / M)
    d = torch.stack([ang.cos(), ang.sin()], -1)
    d = d / d.abs().max(-1, keepdim=True).values
    off = d[:, None, :] * torch.arange(1, P + 1, dtype=torch.float32)[None, :, None]
    wh = torch.as_tensor([(w, h) for (h, w) in levels], dtype=torch.float32)
    loc = ref[:, None, None, None, :] + off[None, :, None, :, :] / wh[None, None, :, None, :]
    return loc[None].expand(n, -1, -1, -1, -1, -1).contiguous()


@pytest.mark.parametrize("variant", ["lane32", "tiled", "enc", "sorted"])
@pytest.mark.parametrize("vdtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 1e-2)])
def test_encoder_backward_init_geometry_800x1333(variant, vdtype, tol, monkeypatch):
    """Sampling points on cell edges (the reference init): a kernel that
    evaluates loc * W - 0.5 twice (e.g. for a pipelined gather and again for
    the weights) can floor the two results to different cells."""
    monkeypatch.setenv("GD_MSDA_BWD", variant)
    value, shapes, lsi, _, attn, grad_out = _encoder_inputs(LEVELS_800, 2, seed=41, vdtype=vdtype)
    loc = _init_geometry_loc(LEVELS_800, 2)
    _check_bwd_vs_oracle((value, shapes, lsi, loc, attn, grad_out), tol, host_shapes=LEVELS_800)


@pytest.mark.parametrize("vdtype", [torch.float32, torch.bfloat16])
def test_encoder_enc_matches_direct_atomic_kernel(vdtype, monkeypatch):
    """Same sums, different order: msda_bwd_enc against msda_bwd_lane32 on
    one input (fp32 accumulation in both)."""
    inputs = [t.to(DEV) for t in _encoder_inputs(LEVELS_800, 2, seed=13, vdtype=vdtype)]
    monkeypatch.setenv("GD_MSDA_BWD", "enc")
    enc = _msda().ms_deform_attn_backward(*inputs, 64, grad_value_dtype=torch.float32, host_shapes=LEVELS_800)
    monkeypatch.setenv("GD_MSDA_BWD", "lane32")
    direct = _msda().ms_deform_attn_backward(*inputs, 64, grad_value_dtype=torch.float32, host_shapes=LEVELS_800)
    torch.testing.assert_close(enc[0], direct[0], rtol=1e-4, atol=1e-5)
    # grad_attn: per-lane dot products summed in a different order
    torch.testing.assert_close(enc[2], direct[2], rtol=1e-4, atol=1e-5)
    assert _rel_err_gl(enc[1].cpu(), direct[1].double().cpu().numpy(), inputs[3].cpu(), inputs[1].cpu()) < 1e-5


# ------------------------------ sorted backward (no float atomics, round 3)
@pytest.mark.parametrize("lq,vdtype,tol", [(900, torch.float32, 1e-3), (900, torch.bfloat16, 1e-2)])
def test_sorted_backward_decoder_shape_800x1333(lq, vdtype, tol, monkeypatch):
    """The decoder's cross-attention (900 queries sampling anywhere, also
    outside the levels) through the sorted backward (host shapes given, as the
    model passes them; GD_MSDA_BWD=sorted-all: by default the decoder shape
    keeps the direct-atomic kernel)."""
    monkeypatch.setenv("GD_MSDA_BWD", "sorted-all")
    value, shapes, lsi, loc, attn, grad_out = _big_inputs(lq, seed=lq + 1, vdtype=vdtype)
    inputs = (value.cpu(), shapes, lsi, loc.cpu(), attn.cpu(), grad_out.cpu())
    _check_bwd_vs_oracle(inputs, tol, host_shapes=LEVELS_800)


@pytest.mark.parametrize("vdtype", [torch.float32, torch.bfloat16])
def test_sorted_matches_direct_atomic_kernel(vdtype, monkeypatch):
    """Same sums, different order: the destination-sorted backward against
    msda_bwd_lane32 (float atomics) on one encoder-shape input."""
    inputs = [t.to(DEV) for t in _encoder_inputs(LEVELS_800, 2, seed=17, vdtype=vdtype, outlier_frac=0.02)]
    monkeypatch.setenv("GD_MSDA_BWD", "sorted")
    srt = _msda().ms_deform_attn_backward(*inputs, 64, grad_value_dtype=torch.float32, host_shapes=LEVELS_800)
    monkeypatch.setenv("GD_MSDA_BWD", "lane32")
    direct = _msda().ms_deform_attn_backward(*inputs, 64, grad_value_dtype=torch.float32, host_shapes=LEVELS_800)
    torch.testing.assert_close(srt[0], direct[0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(srt[2], direct[2], rtol=1e-4, atol=1e-5)
    assert _rel_err_gl(srt[1].cpu(), direct[1].double().cpu().numpy(), inputs[3].cpu(), inputs[1].cpu()) < 1e-5


@pytest.mark.parametrize("lq", [22223, 900])
def test_sorted_backward_deterministic_mode_is_bitwise_reproducible(lq, monkeypatch):
    """GD_MSDA_DETERMINISTIC=1 (or torch.use_deterministic_algorithms): each
    cell's sample list is sorted by sample id before the per-destination sums,
    so two runs give bitwise-equal grad_value (and grad_loc / grad_attn, which
    never use atomics).  bf16 value, grad_value written in bf16 as autograd
    takes it."""
    monkeypatch.setenv("GD_MSDA_BWD", "sorted-all")
    monkeypatch.setenv("GD_MSDA_DETERMINISTIC", "1")
    if lq == 900:
        inputs = [t.to(DEV) for t in _big_inputs(900, seed=5, vdtype=torch.bfloat16)]
    else:
        inputs = [t.to(DEV) for t in _encoder_inputs(LEVELS_800, 2, seed=19, vdtype=torch.bfloat16,
                                                     outlier_frac=0.02)]
    runs = [_msda().ms_deform_attn_backward(*inputs, 64, host_shapes=LEVELS_800) for _ in range(3)]
    torch.cuda.synchronize()
    assert runs[0][0].dtype == torch.bfloat16
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)
    monkeypatch.setenv("GD_MSDA_DETERMINISTIC", "0")
    fast = _msda().ms_deform_attn_backward(*inputs, 64, host_shapes=LEVELS_800)
    torch.testing.assert_close(fast[0].float(), runs[0][0].float(), rtol=1e-2, atol=1e-3)
    assert torch.equal(fast[1], runs[0][1]) and torch.equal(fast[2], runs[0][2])


@pytest.mark.parametrize("geometry", ["init", "spread"])
def test_sorted_level_loaded_locations_are_bitwise_the_default(geometry, monkeypatch):
    """The default per-sample pass (locations loaded level by level,
    reloaded for the owned samples) does the same arithmetic as
    GD_MSDA_SORTED_LL=0 (all held from the start): in deterministic mode all
    three gradients are bitwise equal."""
    monkeypatch.setenv("GD_MSDA_BWD", "sorted")
    monkeypatch.setenv("GD_MSDA_DETERMINISTIC", "1")
    monkeypatch.setenv("GD_MSDA_SORTED_GS", "0")  # the two per-lane-geometry variants
    value, shapes, lsi, loc, attn, grad_out = _encoder_inputs(LEVELS_800, 2, seed=43, vdtype=torch.bfloat16,
                                                              outlier_frac=0.02)
    if geometry == "init":
        loc = _init_geometry_loc(LEVELS_800, 2)
    inputs = [t.to(DEV) for t in (value, shapes, lsi, loc, attn, grad_out)]
    runs = []
    for ll in ("0", "1"):
        monkeypatch.setenv("GD_MSDA_SORTED_LL", ll)
        runs.append(_msda().ms_deform_attn_backward(*inputs, 64, host_shapes=LEVELS_800))
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("geometry", ["init", "spread"])
def test_geometry_shared_kernels_match_the_per_lane_kernels(geometry, monkeypatch):
    """Round 5: msda_fwd_gs and msda_bwd_samples_gs (one lane's geometry per
    sample, DPP quad broadcasts, packed / dot2 arithmetic) against the
    per-lane kernels on the 800x1333 encoder shape: forward and grad_value
    within bf16 rounding, grad_loc / grad_attn within fp32 summation order
    (deterministic mode, so grad_value's order is fixed)."""
    monkeypatch.setenv("GD_MSDA_BWD", "sorted")
    monkeypatch.setenv("GD_MSDA_DETERMINISTIC", "1")
    value, shapes, lsi, loc, attn, grad_out = _encoder_inputs(LEVELS_800, 2, seed=47, vdtype=torch.bfloat16,
                                                              outlier_frac=0.02)
    if geometry == "init":
        loc = _init_geometry_loc(LEVELS_800, 2)
    inputs = [t.to(DEV) for t in (value, shapes, lsi, loc, attn, grad_out)]
    res = {}
    for gs in ("0", "1"):
        monkeypatch.setenv("GD_MSDA_FWD_GS", gs)
        monkeypatch.setenv("GD_MSDA_SORTED_GS", gs)
        out = _msda().ms_deform_attn_forward(*inputs[:5], 64)
        res[gs] = (out,) + tuple(_msda().ms_deform_attn_backward(*inputs, 64, host_shapes=LEVELS_800))
    for i, (a, b) in enumerate(zip(res["0"], res["1"])):
        a, b = a.float(), b.float()
        rel = float((a - b).abs().max() / a.abs().max())
        assert torch.isfinite(b).all()
        assert rel < (1e-2 if i in (0, 1) else 1e-4), (i, rel)
    _msda().check_device_status()  # the record-slot guard of the sorted backward stayed quiet


def test_sorted_backward_bf16_grad_value_is_the_rounded_fp32_sum(monkeypatch):
    """grad_value in bf16 straight from the kernel equals the kernel's fp32
    result rounded to bf16 (same sums, deterministic mode)."""
    monkeypatch.setenv("GD_MSDA_BWD", "sorted")
    monkeypatch.setenv("GD_MSDA_DETERMINISTIC", "1")
    inputs = [t.to(DEV) for t in _encoder_inputs(LEVELS_800, 2, seed=23, vdtype=torch.bfloat16)]
    g16 = _msda().ms_deform_attn_backward(*inputs, 64, grad_value_dtype=torch.bfloat16, host_shapes=LEVELS_800)
    g32 = _msda().ms_deform_attn_backward(*inputs, 64, grad_value_dtype=torch.float32, host_shapes=LEVELS_800)
    assert g16[0].dtype == torch.bfloat16 and g32[0].dtype == torch.float32
    assert torch.equal(g16[0], g32[0].to(torch.bfloat16))


# ------------------------------------------------------------- edge/contract
def test_empty_inputs():
    shapes = torch.as_tensor([(4, 4), (2, 2)], dtype=torch.long, device=DEV)
    lsi = torch.as_tensor([0, 16], dtype=torch.long, device=DEV)
    value = torch.randn(2, 20, 8, 32, device=DEV)
    loc = torch.rand(2, 0, 8, 2, 4, 2, device=DEV)
    attn = torch.rand(2, 0, 8, 2, 4, device=DEV)
    out = _msda().ms_deform_attn_forward(value, shapes, lsi, loc, attn, 64)
    assert out.shape == (2, 0, 256)
    gv, gl, ga = _msda().ms_deform_attn_backward(value, shapes, lsi, loc, attn, out, 64)
    assert torch.count_nonzero(gv) == 0 and gl.shape == loc.shape


def test_contract_errors():
    c = load_case("kat_fwd_float")
    shapes, lsi = _shapes(c)
    v = _t(c["value"], torch.float32)
    l = _t(c["loc"], torch.float32)
    a = _t(c["attn"], torch.float32)
    with pytest.raises(RuntimeError, match="contiguous"):
        _msda().ms_deform_attn_forward(v.transpose(2, 3), shapes, lsi, l, a, 2)
    with pytest.raises(RuntimeError, match="CPU"):
        _msda().ms_deform_attn_forward(v.cpu(), shapes, lsi, l, a, 2)
    v3 = torch.cat([v, v, v])
    with pytest.raises(RuntimeError, match="im2col_step"):
        _msda().ms_deform_attn_forward(v3, shapes, lsi, torch.cat([l, l, l]), torch.cat([a, a, a]), 2)


def test_module_runs_and_backprops():
    from models.GroundingDINO.ms_deform_attn import MultiScaleDeformableAttention
    torch.manual_seed(0)
    m = MultiScaleDeformableAttention(embed_dims=256, num_levels=4, num_heads=8, num_points=4,
                                      batch_first=True).to(DEV)
    shapes = torch.as_tensor([(16, 20), (8, 10), (4, 5), (2, 3)], dtype=torch.long, device=DEV)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    S = int(shapes.prod(1).sum())
    src = torch.randn(2, S, 256, device=DEV, requires_grad=True)
    ref = torch.rand(2, S, 4, 2, device=DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(query=src, value=src, reference_points=ref, spatial_shapes=shapes, level_start_index=lsi)
    out.float().sum().backward()
    assert out.shape == src.shape and torch.isfinite(src.grad).all()
    assert m.sampling_offsets.weight.grad is not None and m.value_proj.weight.grad.abs().sum() > 0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_forward_nonfinite_locations_add_zero(dtype):
    """A NaN or +-Inf sampling location is skipped (adds 0) as in the
    reference kernel's bounds test (.cuh:238-299, NaN compares false); the
    vectorised forward's branchless gathers must not turn it into NaN * 0.
    Against the C oracle on the same inputs (fp64)."""
    g = torch.Generator().manual_seed(5)
    shapes = torch.as_tensor([(16, 20), (8, 10), (4, 5), (2, 3)], dtype=torch.long)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    S = int(shapes.prod(1).sum())
    value = torch.rand(2, S, 8, 32, generator=g).to(dtype).double()
    loc = torch.rand(2, 37, 8, 4, 4, 2, generator=g, dtype=torch.float64)
    bad = torch.rand(loc.shape[:-1], generator=g) < 0.2
    kinds = torch.randint(0, 3, loc.shape[:-1], generator=g)
    fill = torch.where(kinds == 0, float("nan"), torch.where(kinds == 1, float("inf"), float("-inf"))).double()
    axis = torch.randint(0, 2, loc.shape[:-1], generator=g)
    for a in (0, 1):
        loc[..., a] = torch.where(bad & (axis == a), fill, loc[..., a])
    attn = torch.rand(2, 37, 8, 4, 4, generator=g, dtype=torch.float64) + 1e-5
    attn /= attn.sum((-1, -2), keepdim=True)
    ref = oracle.msda_forward(value, shapes, lsi, loc, attn)
    assert np.isfinite(ref).all()
    out = _msda().ms_deform_attn_forward(value.to(DEV, dtype), shapes.to(DEV), lsi.to(DEV), loc.to(DEV, torch.float32),
                                         attn.to(DEV, torch.float32), 64)
    torch.cuda.synchronize()
    o = out.double().cpu().numpy()
    assert np.isfinite(o).all(), "non-finite location leaked NaN into the output"
    assert _rel_err(o, ref) < (1e-3 if dtype == torch.float32 else 1e-2)
