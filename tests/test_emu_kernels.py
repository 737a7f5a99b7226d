"""The HIP kernels' own sources, executed on the CPU by the host-side SIMT
emulator (tests/emu, test infrastructure), against the oracle.

Why: when no GPU is reachable, this is how kernel changes are checked before
they ship -- the exact csrc/*.hip code with its indexing, LDS accumulator,
barriers, DPP / ds_swizzle butterflies and launch geometry.  It does not
replace the GPU parity tests (tests/test_msda_gpu.py, test_kernels_gpu.py),
which run the gfx950 build on the box.

The emulator itself is pinned by the kernels that passed the GPU tests in
round 1 (msda_fwd_vec, msda_bwd_lane32): they must match the oracle here too.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import emu_lib as E
import oracle

HERE = os.path.dirname(os.path.abspath(__file__))


def _levels_inputs(levels, n, lq, seed, vdtype=torch.float32, local=False, spread_px=2.0, outlier_frac=0.0):
    shapes = torch.as_tensor(levels, dtype=torch.long)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    S = int(shapes.prod(1).sum())
    M, D, L, P = 8, 32, len(levels), 4
    g = torch.Generator().manual_seed(seed)
    if local:  # encoder: Lq == S, points near each query's own position
        assert lq == S
        refs = []
        for (h, w) in levels:
            yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
            refs.append(torch.stack([(xx.reshape(-1) + 0.5) / w, (yy.reshape(-1) + 0.5) / h], -1))
        ref = torch.cat(refs).double()
        wh = torch.as_tensor([(w, h) for (h, w) in levels], dtype=torch.float64)
        off = torch.randn(n, S, M, L, P, 2, generator=g, dtype=torch.float64) * spread_px
        loc = ref[None, :, None, None, None, :] + off / wh[None, None, None, :, None, :]
        if outlier_frac:
            pick = torch.rand(n, S, M, L, P, 1, generator=g) < outlier_frac
            loc = torch.where(pick, torch.rand(loc.shape, generator=g, dtype=torch.float64) * 1.2 - 0.1, loc)
        loc = loc.float()
    else:
        loc = torch.rand(n, lq, M, L, P, 2, generator=g) * 1.1 - 0.05
    value = torch.randn(n, S, M, D, generator=g).to(vdtype)
    attn = torch.rand(n, lq, M, L, P, generator=g) + 1e-5
    attn = attn / attn.sum((-1, -2), keepdim=True)
    grad_out = torch.randn(n, lq, M * D, generator=g).to(vdtype)
    return value, shapes, lsi, loc, attn, grad_out


def _oracle_bwd(value, shapes, lsi, loc, attn, grad_out):
    return oracle.msda_backward(value.double().numpy(), shapes, lsi, loc.double(), attn.double(),
                                grad_out.double().numpy())


def _check_bwd(inputs, tol, host_shapes=None):
    from msda_cases import rel_err_grad_loc
    gv, gl, ga = E.msda_backward(*inputs, host_shapes=host_shapes)
    rgv, rgl, rga = _oracle_bwd(*inputs)
    assert E.rel_err(gv, rgv) < tol
    assert rel_err_grad_loc(gl, rgl, inputs[3], inputs[1]) < tol  # away from cell edges
    assert E.rel_err(ga, rga) < tol
    return gv, gl, ga


SMALL = [(6, 9), (3, 5), (2, 3), (1, 2)]               # S = 76
MEDIUM = [(13, 21), (7, 11), (4, 6), (2, 3)]           # S = 380 (tail tiles, tiles across levels)
WIDE = [(20, 67), (10, 34), (5, 17), (3, 9)]           # level-0 boxes of 32-query tiles overflow LDS


# ------------------------------------------------- emulator pinned by round-1
@pytest.mark.parametrize("vdtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-5)])
def test_emulated_verified_kernels_match_oracle(vdtype, tol):
    """msda_fwd_vec / msda_bwd_lane32 passed the GPU parity tests in round 1;
    the emulator must reproduce them (inputs are bf16-exact, so the oracle on
    the same values is tight)."""
    value, shapes, lsi, loc, attn, grad_out = _levels_inputs(MEDIUM, 2, 50, seed=1, vdtype=vdtype)
    out = E.msda_forward(value, shapes, lsi, loc, attn)
    ref = oracle.msda_forward(value.double().numpy(), shapes, lsi, loc.double(), attn.double())
    assert E.rel_err(out.double(), ref) < (1e-5 if vdtype == torch.float32 else 1e-2)
    _check_bwd((value, shapes, lsi, loc, attn, grad_out), tol)


@pytest.mark.parametrize("vdtype", [torch.float32, torch.bfloat16])
def test_emulated_forward_nonfinite_locations_add_zero(vdtype):
    """NaN / +-Inf sampling locations are skipped samples (the reference's
    bounds test is false for them), so the vectorised forward's output stays
    finite and equals the oracle's (NaN fractions times a zero
    corner gave NaN)."""
    value, shapes, lsi, loc, attn, _ = _levels_inputs(MEDIUM, 2, 50, seed=3, vdtype=vdtype)
    g = torch.Generator().manual_seed(3)
    bad = torch.rand(loc.shape[:-1], generator=g) < 0.25
    kinds = torch.randint(0, 3, loc.shape[:-1], generator=g)
    fill = torch.where(kinds == 0, float("nan"), torch.where(kinds == 1, float("inf"), float("-inf")))
    axis = torch.randint(0, 2, loc.shape[:-1], generator=g)
    loc = loc.clone()
    for a in (0, 1):
        loc[..., a] = torch.where(bad & (axis == a), fill.to(loc.dtype), loc[..., a])
    out = E.msda_forward(value, shapes, lsi, loc, attn)
    ref = oracle.msda_forward(value.double().numpy(), shapes, lsi, loc.double(), attn.double())
    assert np.isfinite(ref).all() and torch.isfinite(out).all()
    assert E.rel_err(out.double(), ref) < (1e-5 if vdtype == torch.float32 else 1e-2)


# ------------------------------- sorted backward (no float atomics, round 3)
def _check_sorted(inputs, levels, tol, gv_dtype=torch.float32, deterministic=False):
    from msda_cases import rel_err_grad_loc
    res = E.msda_backward_sorted(*inputs, host_shapes=levels, gv_dtype=gv_dtype, deterministic=deterministic)
    assert res is not None
    gv, gl, ga = res
    assert torch.isfinite(gv).all() and torch.isfinite(gl).all() and torch.isfinite(ga).all()
    rgv, rgl, rga = _oracle_bwd(*inputs)
    assert E.rel_err(gv.double(), rgv) < (tol if gv_dtype == torch.float32 else 1e-2)
    assert rel_err_grad_loc(gl, rgl, inputs[3], inputs[1]) < tol  # away from cell edges
    assert E.rel_err(ga, rga) < tol
    return gv, gl, ga


@pytest.mark.parametrize("levels,n,lq,local,outliers,vdtype", [
    (SMALL, 1, None, True, 0.0, torch.float32),      # encoder shape, Lq == S
    (MEDIUM, 2, None, True, 0.1, torch.float32),     # + outliers, batch of 2
    (MEDIUM, 2, None, True, 0.05, torch.bfloat16),   # bf16 value / grad_out
    (MEDIUM, 2, 37, False, 0.0, torch.float32),      # decoder shape: Lq != S, points anywhere (and outside)
    (WIDE, 1, 23, False, 0.0, torch.bfloat16),
])
@pytest.mark.parametrize("k4", ["sweep", "cellsum"])
def test_emulated_sorted_backward_matches_oracle(levels, n, lq, local, outliers, vdtype, k4, monkeypatch):
    """grad_value by the column sweep (default) and by the per-cell partial +
    per-pixel sum pair (GD_MSDA_SORTED_K4=1)."""
    monkeypatch.setenv("GD_MSDA_SORTED_K4", "1" if k4 == "cellsum" else "0")
    S = sum(h * w for h, w in levels)
    inputs = _levels_inputs(levels, n, S if lq is None else lq, seed=11, vdtype=vdtype, local=local,
                            outlier_frac=outliers)
    _check_sorted(inputs, levels, 1e-5)


@pytest.mark.parametrize("vdtype", [torch.float32, torch.bfloat16])
def test_emulated_sorted_backward_level_by_level_per_sample_pass(vdtype, monkeypatch):
    """GD_MSDA_SORTED_K1=2: the level-by-level per-sample pass (one level's
    partials live at a time, its owned sample's record stored per level; the
    A/B alternative to the default that holds all four levels)."""
    monkeypatch.setenv("GD_MSDA_SORTED_K1", "2")
    S = sum(h * w for h, w in MEDIUM)
    inputs = _levels_inputs(MEDIUM, 2, S, seed=17, vdtype=vdtype, local=True, outlier_frac=0.05)
    _check_sorted(inputs, MEDIUM, 1e-5)


@pytest.mark.parametrize("priv", ["0", "2"])
def test_emulated_sorted_backward_lds_histograms(priv, monkeypatch):
    """GD_MSDA_COUNT_PRIV=0: every count / slot a global atomic; =2: the
    per-sample pass reserves the coarse levels' slots through its LDS
    histogram whatever the run statistics say (the default decides on the
    device), with both (n, m) and head-pair slots in play (batch of 2)."""
    monkeypatch.setenv("GD_MSDA_COUNT_PRIV", priv)
    S = sum(h * w for h, w in MEDIUM)
    for vd in (torch.float32, torch.bfloat16):
        inputs = _levels_inputs(MEDIUM, 2, S, seed=29, vdtype=vd, local=True, outlier_frac=0.1)
        _check_sorted(inputs, MEDIUM, 1e-5)


@pytest.mark.parametrize("rounds,levels", [("1", MEDIUM), ("4", MEDIUM), ("8", WIDE)])
def test_emulated_sorted_backward_count_rounds(rounds, levels, monkeypatch):
    """The count pass with 4 rounds of 64 units per workgroup (the default
    when Lq >= 256: MEDIUM's 380 queries, a ragged last workgroup, units of
    two (n, m) in one histogram), with one round (GD_MSDA_COUNT_R=1) and
    with eight (=8, Lq >= 512: WIDE's 1 792 queries); the cells of a batch
    of 2 span several scan blocks."""
    monkeypatch.setenv("GD_MSDA_COUNT_R", rounds)
    S = sum(h * w for h, w in levels)
    inputs = _levels_inputs(levels, 2, S, seed=31, vdtype=torch.bfloat16, local=True, outlier_frac=0.05)
    _check_sorted(inputs, levels, 1e-5)


def test_emulated_sorted_backward_sweep_record_prefetch(monkeypatch):
    """GD_MSDA_SWEEP_PF=1: the sweep loads a row's first records during the
    previous row's exchange."""
    monkeypatch.setenv("GD_MSDA_SWEEP_PF", "1")
    S = sum(h * w for h, w in MEDIUM)
    inputs = _levels_inputs(MEDIUM, 2, S, seed=23, vdtype=torch.bfloat16, local=True, outlier_frac=0.05)
    _check_sorted(inputs, MEDIUM, 1e-5)


@pytest.mark.parametrize("vdtype", [torch.float32, torch.bfloat16])
def test_emulated_sorted_backward_locations_held(vdtype, monkeypatch):
    """GD_MSDA_SORTED_LL=0: the per-sample pass holds all 48 location /
    weight floats from the start (the default loads them level by level and
    reloads the owned samples'), head pairs, batch of 2."""
    monkeypatch.setenv("GD_MSDA_SORTED_LL", "0")
    S = sum(h * w for h, w in MEDIUM)
    inputs = _levels_inputs(MEDIUM, 2, S, seed=23, vdtype=vdtype, local=True, outlier_frac=0.05)
    _check_sorted(inputs, MEDIUM, 1e-5)


def test_emulated_sorted_backward_one_head_per_wave(monkeypatch):
    """GD_MSDA_SORTED_HP=1: per-sample pass and sweep with one head per wave
    (the default pairs heads m, m + 1 for value / grad_out line reuse)."""
    monkeypatch.setenv("GD_MSDA_SORTED_HP", "1")
    S = sum(h * w for h, w in MEDIUM)
    inputs = _levels_inputs(MEDIUM, 2, S, seed=19, vdtype=torch.bfloat16, local=True, outlier_frac=0.05)
    _check_sorted(inputs, MEDIUM, 1e-5)


def test_emulated_sorted_backward_bf16_grad_value_and_determinism():
    """grad_value written directly in bf16 (the autograd dtype of a bf16
    value) equals the fp32 result rounded; the deterministic mode sorts each
    cell segment by sample id, so two runs agree bit for bit, and the sums
    agree with the arrival-order mode to fp32 rounding."""
    inputs = _levels_inputs(MEDIUM, 2, 380, seed=12, vdtype=torch.bfloat16, local=True, outlier_frac=0.1)
    gv32, gl, ga = _check_sorted(inputs, MEDIUM, 1e-5)
    gv16, gl2, ga2 = _check_sorted(inputs, MEDIUM, 1e-5, gv_dtype=torch.bfloat16)
    assert torch.equal(gv16, gv32.to(torch.bfloat16))
    assert torch.equal(gl, gl2) and torch.equal(ga, ga2)  # no atomics in grad_loc / grad_attn
    d1 = _check_sorted(inputs, MEDIUM, 1e-5, deterministic=True)
    d2 = _check_sorted(inputs, MEDIUM, 1e-5, deterministic=True)
    for a, b in zip(d1, d2):
        assert torch.equal(a, b)
    assert E.rel_err(d1[0].double(), gv32.double().numpy()) < 1e-6


@pytest.mark.parametrize("lq", [90, 300])
def test_emulated_sorted_backward_long_cell_segments(lq):
    """Cells holding > 64 samples take the deterministic mode's LDS bitonic
    sort (<= 1024: 90 queries x 4 points) or its wave radix sort (> 1024:
    300 x 4): every query samples the same few points."""
    levels = [(3, 4), (2, 2), (1, 2), (1, 1)]
    value, shapes, lsi, loc, attn, grad_out = _levels_inputs(levels, 1, lq, seed=13)
    g = torch.Generator().manual_seed(3)
    loc = (torch.rand(1, lq, 8, 4, 4, 2, generator=g) * 0.05 + 0.3)  # all in one cell per level
    _check_sorted((value, shapes, lsi, loc, attn, grad_out), levels, 1e-5, deterministic=True)


# ------------------------------------------- tiled (LDS) encoder backward
@pytest.mark.parametrize("levels,n,local,outliers", [
    (SMALL, 1, False, 0.0),     # every level box fits: all-LDS path
    (MEDIUM, 2, True, 0.0),     # encoder geometry, batch boundary inside the grid
    (MEDIUM, 2, True, 0.1),     # + outliers: mixed LDS / global atomics
    (MEDIUM, 1, False, 0.0),    # uniform points: boxes overflow, global fallback
    (WIDE, 1, True, 0.02),
])
def test_emulated_tiled_backward_matches_oracle(levels, n, local, outliers, monkeypatch):
    monkeypatch.setenv("GD_MSDA_BWD", "tiled")
    S = sum(h * w for h, w in levels)
    inputs = _levels_inputs(levels, n, S, seed=S + n, local=local, outlier_frac=outliers)
    _check_bwd(inputs, 1e-5)


@pytest.mark.parametrize("levels,n,local,outliers", [
    (SMALL, 1, False, 0.0),
    (MEDIUM, 2, True, 0.0),     # partial 4 x 8 blocks at every level's right / bottom edge
    (MEDIUM, 2, True, 0.1),
    (WIDE, 1, True, 0.02),
])
def test_emulated_pixel_block_tiles_match_oracle(levels, n, local, outliers, monkeypatch):
    monkeypatch.setenv("GD_MSDA_BWD", "tiled")
    """gd_msda_backward_geom: 4 x 8 pixel-block tiles of each level (host
    level shapes given) -- same sums as the oracle and the strip tiling."""
    S = sum(h * w for h, w in levels)
    inputs = _levels_inputs(levels, n, S, seed=S + 7 * n, local=local, outlier_frac=outliers)
    blocks = _check_bwd(inputs, 1e-5, host_shapes=levels)
    strips = E.msda_backward(*inputs)
    torch.testing.assert_close(blocks[0], strips[0], rtol=1e-5, atol=1e-6)
    assert torch.equal(blocks[1], strips[1]) and torch.equal(blocks[2], strips[2])


def test_emulated_geom_falls_back_when_levels_do_not_tile_the_queries(monkeypatch):
    monkeypatch.setenv("GD_MSDA_BWD", "tiled")
    S = sum(h * w for h, w in MEDIUM)
    inputs = _levels_inputs(MEDIUM, 1, S, seed=21, local=True)
    wrong = [(h, w + 1) for h, w in MEDIUM]  # covers more than S: strip tiling
    _check_bwd(inputs, 1e-5, host_shapes=wrong)


def test_emulated_tiled_backward_bf16(monkeypatch):
    monkeypatch.setenv("GD_MSDA_BWD", "tiled")
    S = sum(h * w for h, w in MEDIUM)
    inputs = _levels_inputs(MEDIUM, 2, S, seed=5, vdtype=torch.bfloat16, local=True, outlier_frac=0.05)
    _check_bwd(inputs, 1e-5)  # bf16-exact inputs, fp32 accumulation


# ------------------------------ encoder backward: 2-D tiles, packed LDS boxes
ENC_TILES = ["16x16,8x8,4x4,2x4", "4x16,3x8,2x4,1x4", "5x7,3x3,2x2,1x1"]


@pytest.mark.parametrize("levels,n,local,outliers,spread", [
    (SMALL, 1, True, 0.0, 2.0),     # every level box fits
    (MEDIUM, 2, True, 0.0, 2.0),    # tail tiles on every level, batch boundary inside the grid
    (MEDIUM, 2, True, 0.1, 2.0),    # + outliers: clipped boxes, mixed LDS / global atomics
    (MEDIUM, 1, False, 0.0, 2.0),   # uniform points: boxes clipped to the footprint window
    (WIDE, 1, True, 0.02, 6.0),     # wide spread: boxes overflow the accumulator
])
@pytest.mark.parametrize("vdtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("depth", ["1", "2"])
def test_emulated_enc_backward_matches_oracle(levels, n, local, outliers, spread, vdtype, depth, monkeypatch):
    """depth: units whose gathers are in flight (GD_MSDA_ENC_DEPTH; 1 is the
    default, 2 the two-deep pipeline variant)."""
    monkeypatch.setenv("GD_MSDA_BWD", "enc")
    monkeypatch.setenv("GD_MSDA_ENC_DEPTH", depth)
    S = sum(h * w for h, w in levels)
    inputs = _levels_inputs(levels, n, S, seed=S + 3 * n, vdtype=vdtype, local=local, spread_px=spread,
                            outlier_frac=outliers)
    _check_bwd(inputs, 1e-5, host_shapes=levels)  # bf16-exact inputs, fp32 accumulation


@pytest.mark.parametrize("tiles", ENC_TILES)
@pytest.mark.parametrize("cap,rmax", [("224,96,64,64", 8), ("40,16,8,0", 2), ("500,300,100,100", 0)])
def test_emulated_enc_backward_tilings(tiles, cap, rmax, monkeypatch):
    """Any tile extents, LDS region sizes and clip radius give the same sums."""
    monkeypatch.setenv("GD_MSDA_BWD", "enc")
    monkeypatch.setenv("GD_MSDA_ENC_TILE", tiles)
    monkeypatch.setenv("GD_MSDA_ENC_CAP", cap)
    monkeypatch.setenv("GD_MSDA_ENC_RMAX", str(rmax))
    S = sum(h * w for h, w in MEDIUM)
    inputs = _levels_inputs(MEDIUM, 2, S, seed=17, local=True, outlier_frac=0.05)
    _check_bwd(inputs, 1e-5, host_shapes=MEDIUM)


def test_emulated_enc_without_host_shapes_uses_direct_kernel(monkeypatch):
    """gd_msda_backward (no level shapes on the host): the direct kernel."""
    monkeypatch.setenv("GD_MSDA_BWD", "enc")
    S = sum(h * w for h, w in MEDIUM)
    inputs = _levels_inputs(MEDIUM, 1, S, seed=23, local=True)
    _check_bwd(inputs, 1e-5)


def test_emulated_tiled_equals_direct_atomic_kernel(monkeypatch):
    S = sum(h * w for h, w in MEDIUM)
    inputs = _levels_inputs(MEDIUM, 2, S, seed=9, local=True, outlier_frac=0.05)
    monkeypatch.setenv("GD_MSDA_BWD", "tiled")
    tiled = E.msda_backward(*inputs)
    monkeypatch.setenv("GD_MSDA_BWD", "lane32")
    direct = E.msda_backward(*inputs)
    torch.testing.assert_close(tiled[0], direct[0], rtol=1e-5, atol=1e-6)
    assert torch.equal(tiled[1], direct[1]) and torch.equal(tiled[2], direct[2])


# --------------------------------------------------- BiAttention softmax
def _softmax_ref(s, pad_v, pad_l):
    s = s.double()
    pv = torch.softmax(s.masked_fill(pad_l[:, None, None, :], float("-inf")), -1).nan_to_num(0.0)
    pl = torch.softmax(s.masked_fill(pad_v[:, None, :, None], float("-inf")), -2).nan_to_num(0.0)
    return pv, pl


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("shape", [(2, 2, 300, 40), (1, 2, 200, 100), (1, 1, 333, 64), (2, 1, 260, 128),
                                   (1, 1, 130, 256), (1, 1, 70, 600)])
def test_emulated_biattn_softmax(dtype, tol, shape):
    b, h, s_len, t = shape
    g = torch.Generator().manual_seed(sum(shape))
    s = (torch.randn(b, h, s_len, t, generator=g) * 2).to(dtype)
    pad_v = torch.zeros(b, s_len, dtype=torch.bool)
    pad_l = torch.zeros(b, t, dtype=torch.bool)
    pad_v[-1, s_len * 3 // 4:] = True
    pad_l[0, t // 2:] = True
    pv, pl = E.biattn_softmax_fwd(s, pad_v, pad_l)
    sd = s.double().requires_grad_(True)
    rpv, rpl = _softmax_ref(sd, pad_v, pad_l)
    assert E.rel_err(pv.double(), rpv.detach()) < tol
    assert E.rel_err(pl.double(), rpl.detach()) < tol
    dpv = torch.randn(pv.shape, generator=g).to(dtype)
    dpl = torch.randn(pl.shape, generator=g).to(dtype)
    ds = E.biattn_softmax_bwd(pv, pl, dpv, dpl)
    # the kernel's backward uses its own P_v / P_l: compare with the exact
    # Jacobian products evaluated at those probabilities
    pvd, pld = pv.double(), pl.double()
    r = (dpv.double() * pvd).sum(-1, keepdim=True)
    c = (dpl.double() * pld).sum(-2, keepdim=True)
    ref = pvd * (dpv.double() - r) + pld * (dpl.double() - c)
    assert E.rel_err(ds.double(), ref) < tol
    # and with autograd of the reference softmaxes
    ((rpv * dpv.double()).sum() + (rpl * dpl.double()).sum()).backward()
    assert E.rel_err(ds.double(), sd.grad) < (1e-5 if dtype == torch.float32 else 3e-2)


# ------------------------------------------------- scheduling perturbation
_SCHED_SCRIPT = r"""
import sys
sys.path[:0] = {paths!r}
import torch
import test_emu_kernels as t
S = sum(h * w for h, w in t.MEDIUM)
t._check_bwd(t._levels_inputs(t.MEDIUM, 2, S, seed=11, local=True, outlier_frac=0.1), 1e-5)
t._check_bwd(t._levels_inputs(t.SMALL, 1, sum(h * w for h, w in t.SMALL), seed=12), 1e-5)
t._check_bwd(t._levels_inputs(t.MEDIUM, 1, 29, seed=13), 1e-5)
t._check_bwd(t._levels_inputs(t.MEDIUM, 2, S, seed=14, local=True, outlier_frac=0.1), 1e-5, host_shapes=t.MEDIUM)
t.test_emulated_biattn_softmax(torch.float32, 1e-5, (2, 2, 300, 40))
t.test_emulated_biattn_softmax(torch.bfloat16, 1e-2, (1, 1, 130, 256))
t.test_emulated_window_attention(7, 3, 8, 4, True, torch.float32, 1e-5, True)
t.test_emulated_window_attention(3, 4, 6, 3, True, torch.bfloat16, 1.5e-2, False)
t.test_emulated_window_attention(12, 1, 3, 1, False, torch.bfloat16, 1.5e-2, True)
t.test_emulated_window_attention_image(1, 9, 11, 7, 3, 3, True, torch.float32, 1e-5, True)
t.test_emulated_attention(2, 2, 100, 130, 64, "bool", torch.float32, 1e-5, "lbh")
print("sched-ok")
"""


@pytest.mark.parametrize("sched", ["rev", "shuffle:7"])
def test_emulated_kernels_under_other_schedules(sched):
    """Work-items resumed in descending / shuffled order between
    synchronisation points, with LDS poisoned before every workgroup: a
    missing barrier or a read of LDS the workgroup never wrote changes the
    results (the default ascending order could hide either)."""
    paths = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "open-groundingdino_amd")]
    env = dict(os.environ, GD_EMU_SCHED=sched)
    r = subprocess.run([sys.executable, "-c", _SCHED_SCRIPT.format(paths=paths)], env=env, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0 and "sched-ok" in r.stdout, r.stderr[-4000:]


# ------------------------------------------------------ AddressSanitizer
_ASAN_HEAD = r"""
import sys
sys.path[:0] = {paths!r}
import torch
import test_emu_kernels as t
S = sum(h * w for h, w in t.MEDIUM)
"""
# four groups, run as concurrent processes (the ASan build is ~10x slower)
_ASAN_GROUPS = [
    r"""
t._check_bwd(t._levels_inputs(t.MEDIUM, 2, S, seed=3, local=True, outlier_frac=0.1), 1e-5)
t._check_bwd(t._levels_inputs(t.MEDIUM, 1, 37, seed=6), 1e-5)
t._check_bwd(t._levels_inputs(t.WIDE, 1, sum(h * w for h, w in t.WIDE), seed=8, local=True, outlier_frac=0.02), 1e-5,
             host_shapes=t.WIDE)
import os
for v in ("enc", "tiled"):  # the round-1/2 encoder kernels (A/B only since round 3)
    os.environ["GD_MSDA_BWD"] = v
    t._check_bwd(t._levels_inputs(t.MEDIUM, 2, S, seed=5, local=True, outlier_frac=0.1), 1e-5, host_shapes=t.MEDIUM)
del os.environ["GD_MSDA_BWD"]
""",
    r"""
# the sorted backward (the encoder default): both per-sample passes, both
# grad_value kernels, the coarse-level chunks, the deterministic sort
import os
inp = t._levels_inputs(t.MEDIUM, 2, S, seed=21, vdtype=torch.bfloat16, local=True, outlier_frac=0.1)
t._check_sorted(inp, t.MEDIUM, 1e-5)
t._check_sorted(inp, t.MEDIUM, 1e-5, deterministic=True)
os.environ["GD_MSDA_SORTED_K1"] = "2"
os.environ["GD_MSDA_SORTED_K4"] = "1"
t._check_sorted(t._levels_inputs(t.WIDE, 1, 23, seed=22, vdtype=torch.float32, local=False), t.WIDE, 1e-5)
del os.environ["GD_MSDA_SORTED_K1"], os.environ["GD_MSDA_SORTED_K4"]
t.test_emulated_sorted_backward_long_cell_segments(300)
t.test_emulated_add_layernorm(41, 96, torch.float32, None)
""",
    r"""
t._check_bwd(t._levels_inputs(t.WIDE, 1, sum(h * w for h, w in t.WIDE), seed=4, local=True, outlier_frac=0.02), 1e-5)
t.test_emulated_biattn_softmax(torch.bfloat16, 1e-2, (1, 2, 200, 100))
t.test_emulated_biattn_softmax(torch.float32, 1e-5, (2, 1, 260, 128))
import os


class _Env:  # the monkeypatch argument of the contrastive test
    @staticmethod
    def setenv(k, v):
        os.environ[k] = v


for wide in ("0", "1"):
    t.test_emulated_contrastive(2, 100, 37, 64, 256, torch.float32, 1e-5, wide, _Env)
os.environ.pop("GD_CONTRASTIVE_WIDE", None)
t.test_emulated_msda_prologue(2, torch.bfloat16)
t.test_emulated_msda_prologue(4, torch.float32)
t.test_emulated_window_attention_image(1, 9, 11, 7, 3, 3, True, torch.bfloat16, 1.5e-2, True)
t.test_emulated_window_attention_image(1, 14, 17, 12, 6, 1, True, torch.bfloat16, 1.5e-2, False)
""",
    r"""
t.test_emulated_window_attention(7, 2, 22, 1, False, torch.float32, 1e-5, True)
t.test_emulated_wgrad(2000, 128, 144, 2, torch.bfloat16, 1e-6)  # the LDS-DMA ring, column clamp, token tail
t.test_emulated_wgrad(333, 48, 80, 2, torch.bfloat16, 1e-6)
t.test_emulated_window_attention(3, 4, 6, 3, True, torch.bfloat16, 1.5e-2, False)
t.test_emulated_window_attention(12, 2, 4, 2, True, torch.float32, 1e-5, True)
t.test_emulated_attention(2, 2, 130, 40, 32, "keypad", torch.float32, 1e-5, "lbh")
t.test_emulated_attention(1, 1, 33, 300, 32, "add", torch.float32, 1e-5, "blh")
t.test_emulated_attention_dropout(torch.float32, 1e-5)
t.test_emulated_wgrad(777, 64, 192, 3, torch.float32, 1e-6)
t.test_emulated_add_layernorm(50, 192, torch.float32, torch.float32)
""",
]


def test_emulated_kernels_under_address_sanitizer():
    """Out-of-bounds global or LDS accesses of the kernels (the usual cause
    of a GPU memory fault) abort the ASan build of the emulator."""
    clang = "/opt/rocm/lib/llvm/bin/clang++"
    if not os.path.exists(clang):
        pytest.skip("host clang++ not available")
    rt = subprocess.run([clang, "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True,
                        text=True).stdout.strip()
    if not os.path.exists(rt):
        pytest.skip("clang ASan runtime not available")
    paths = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "open-groundingdino_amd")]
    env = dict(os.environ, GD_EMU_ASAN="1", LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0", OMP_NUM_THREADS="1")
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(HERE, "emu"), "asan"], check=True)
    procs = [subprocess.Popen([sys.executable, "-c", _ASAN_HEAD.format(paths=paths) + g + 'print("asan-clean")'],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for g in _ASAN_GROUPS]
    for p in procs:
        out, err = p.communicate(timeout=900)
        assert p.returncode == 0 and "asan-clean" in out, err[-4000:]


# ------------------------------------------- Swin window attention (MFMA)
def _wattn_case(ws, nH, B_, nW, masked, seed, dtype):
    from models.GroundingDINO.backbone.swin_transformer import relative_position_index
    g = torch.Generator().manual_seed(seed)
    N, hd = ws * ws, 32
    qkv = torch.randn(B_, N, 3, nH, hd, generator=g).to(dtype)
    table = torch.randn((2 * ws - 1) ** 2, nH, generator=g) * 0.5
    ridx = relative_position_index(ws, ws).reshape(-1)
    mask = torch.where(torch.rand(nW, N, N, generator=g) < 0.3, -100.0, 0.0) if masked else None
    grad = torch.randn(B_, N, nH * hd, generator=g).to(dtype)
    return qkv, table, ridx, mask, hd ** -0.5, grad


def _wattn_ref(qkv, table, ridx, mask, scale):
    """reference WindowAttention.forward core (swin_transformer.py:134-174), fp64"""
    B_, N, _, nH, hd = qkv.shape
    q, k, v = qkv.permute(2, 0, 3, 1, 4)
    attn = (q * scale) @ k.transpose(-1, -2) + table[ridx].view(N, N, nH).permute(2, 0, 1)
    if mask is not None:
        nW = mask.shape[0]
        attn = (attn.view(B_ // nW, nW, nH, N, N) + mask[None, :, None]).view(B_, nH, N, N)
    return (attn.softmax(-1) @ v).transpose(1, 2).reshape(B_, N, nH * hd)


@pytest.mark.parametrize("ws,nH,B_,nW,masked,dtype,tol", [
    (7, 3, 8, 4, True, torch.float32, 1e-5),     # Swin-T stage 0 heads, shifted windows
    (7, 2, 22, 1, False, torch.float32, 1e-5),   # tail blocks (B_ not a multiple of 16)
    (8, 1, 4, 2, True, torch.float32, 1e-5),     # N = 64: no padded tokens
    (3, 4, 6, 3, True, torch.float32, 1e-5),     # N = 9: mostly padding
    (7, 3, 8, 4, True, torch.bfloat16, 1.5e-2),  # the training dtype
    (5, 2, 20, 5, False, torch.bfloat16, 1.5e-2),
    (12, 2, 4, 2, True, torch.float32, 1e-5),    # Swin-B/384: 12x12 windows, N = 144 (9 tiles)
    (12, 1, 3, 1, False, torch.bfloat16, 1.5e-2),
    (11, 1, 2, 1, False, torch.float32, 1e-5),   # N = 121: padded keys in the 9-tile kernel
])
@pytest.mark.parametrize("std_index", [False, True], ids=["rel_index", "computed_index"])
def test_emulated_window_attention(ws, nH, B_, nW, masked, dtype, tol, std_index):
    """gd_window_attn_*: with the rel_index tensor, and with rel_index NULL
    (the kernel computes the reference's index, swin_transformer.py:104-115)."""
    qkv, table, ridx, mask, scale, grad = _wattn_case(ws, nH, B_, nW, masked, seed=ws * 100 + B_, dtype=dtype)
    kidx = None if std_index else ridx
    out, lse = E.window_attn_forward(qkv, table, kidx, mask, scale)
    qd = qkv.double().requires_grad_(True)
    td = table.double().requires_grad_(True)
    ref = _wattn_ref(qd, td, ridx, None if mask is None else mask.double(), scale)
    assert E.rel_err(out.double(), ref.detach()) < tol
    ref.backward(grad.double())
    gq, gt = E.window_attn_backward(qkv, table, kidx, mask, scale, out, lse, grad)
    assert torch.isfinite(gq).all()
    assert E.rel_err(gq.double(), qd.grad) < tol * 2
    assert E.rel_err(gt.double(), td.grad) < tol * 2


def test_emulated_window_attention_rejects_bad_shapes():
    qkv, table, ridx, mask, scale, _ = _wattn_case(7, 2, 8, 4, True, 0, torch.float32)
    with pytest.raises(RuntimeError, match="multiple of nW"):
        E.window_attn_forward(qkv[:6], table, ridx, mask, scale)
    big = torch.zeros(2, 169, 3, 1, 32)
    with pytest.raises(RuntimeError, match="bad sizes"):
        E.window_attn_forward(big, torch.zeros(625, 1), torch.zeros(169 * 169, dtype=torch.long), None, 1.0)
    with pytest.raises(RuntimeError, match="square window"):  # computed index needs N = ws^2
        E.window_attn_forward(torch.zeros(2, 10, 3, 1, 32), torch.zeros(49, 1), None, None, 1.0)


@pytest.mark.parametrize("b,h,w,ws,shift,nH,bias,dtype,tol", [
    (1, 9, 11, 7, 3, 3, True, torch.float32, 1e-5),    # shifted + padded both ways (Swin-T stage 0)
    (2, 14, 14, 7, 0, 2, True, torch.float32, 1e-5),   # exact tiling, no shift: pure row map
    (2, 14, 14, 7, 3, 2, False, torch.float32, 1e-5),  # shifted, no pad, no qkv bias
    (1, 5, 9, 4, 2, 1, False, torch.float32, 1e-5),    # pad reads zeros (qkv_bias=False)
    (1, 9, 11, 7, 3, 3, True, torch.bfloat16, 1.5e-2),
    (2, 3, 10, 7, 0, 2, True, torch.bfloat16, 1.5e-2),  # H < window: one window row, mostly pad
    (1, 14, 17, 12, 6, 2, True, torch.float32, 1e-5),   # Swin-B/384 12x12 windows, shifted + padded
    (1, 14, 17, 12, 6, 1, True, torch.bfloat16, 1.5e-2),
])
@pytest.mark.parametrize("computed", [False, True], ids=["given_mask_index", "computed_mask_index"])
def test_emulated_window_attention_image(b, h, w, ws, shift, nH, bias, dtype, tol, computed):
    """gd_window_attn_image_*: the pad / roll / partition / reverse / crop of
    SwinTransformerBlock.forward fused into the kernel's row map, against
    oracle.blocks.window_attention_image_ref in fp64 (the shift mask of
    models' shifted_window_mask, i.e. the reference's :402-426 mask)."""
    from models.GroundingDINO.backbone.swin_transformer import relative_position_index, shifted_window_mask
    from oracle.blocks import window_attention_image_ref
    g = torch.Generator().manual_seed(b * 1000 + h * 10 + w)
    C = nH * 32
    qkv = torch.randn(b, h * w, 3 * C, generator=g).to(dtype)
    qb = (torch.randn(3 * C, generator=g) * 0.5).to(dtype) if bias else None
    table = torch.randn((2 * ws - 1) ** 2, nH, generator=g) * 0.5
    ridx = relative_position_index(ws, ws).reshape(-1)
    hp, wp = -(-h // ws) * ws, -(-w // ws) * ws
    mask = shifted_window_mask(hp, wp, ws, shift, "cpu") if shift else None
    grad = torch.randn(b, h * w, C, generator=g).to(dtype)
    scale = 32 ** -0.5
    # computed: rel_index and mask NULL -- the kernel derives the reference's
    # index and region mask (:402-426) from the geometry
    kidx, kmask = (None, None) if computed else (ridx, mask)
    out, lse = E.window_attn_image_forward(qkv, qb, table, kidx, kmask, (h, w), ws, shift, scale)
    qd = qkv.double().requires_grad_(True)
    bd = qb.double().requires_grad_(True) if bias else None
    td = table.double().requires_grad_(True)
    ref = window_attention_image_ref(qd, bd, td, ridx, None if mask is None else mask.double(), (h, w), ws, shift,
                                     scale)
    assert torch.isfinite(out.double()).all()  # every real token row written
    assert E.rel_err(out.double(), ref.detach()) < tol
    ref.backward(grad.double())
    gq, gb, gt = E.window_attn_image_backward(qkv, qb, table, kidx, kmask, (h, w), ws, shift, scale, out, lse,
                                              grad)
    assert torch.isfinite(gq.double()).all()
    assert E.rel_err(gq.double(), qd.grad) < tol * 2
    assert E.rel_err(gt.double(), td.grad) < tol * 2
    if bias:
        assert E.rel_err(gb.double(), bd.grad) < tol * 2


def test_emulated_window_attention_image_rejects_bad_geometry():
    qkv = torch.zeros(1, 81, 96 * 3)
    table, ridx = torch.zeros(169, 3), torch.zeros(49 * 49, dtype=torch.long)
    with pytest.raises(RuntimeError, match="shift"):
        E.window_attn_image_forward(qkv, None, table, ridx, None, (9, 9), 7, 7, 1.0)
    with pytest.raises(RuntimeError, match="window 13"):
        E.window_attn_image_forward(torch.zeros(1, 169, 96 * 3), None, torch.zeros(625, 3),
                                    torch.zeros(169 * 169, dtype=torch.long), None, (13, 13), 13, 0, 1.0)


# ------------------------------- masked multi-head attention (flash, MFMA)
def _attn_case(B, H, Lq, Lk, hd, mask_kind, dtype, seed, layout="lbh"):
    g = torch.Generator().manual_seed(seed)

    def proj(L):  # the MHA / BERT projection layouts, read in place
        if layout == "lbh":
            return torch.randn(L, B, H, hd, generator=g).to(dtype).permute(1, 2, 0, 3)
        return torch.randn(B, L, H, hd, generator=g).to(dtype).transpose(1, 2)

    q, k, v = proj(Lq), proj(Lk), proj(Lk)
    if mask_kind == "none":
        mask = None
    elif mask_kind == "keypad":  # [B, 1, 1, Lk] bool, the decoder's text cross-attention
        mask = torch.ones(B, 1, 1, Lk, dtype=torch.bool)
        mask[-1, ..., Lk // 2:] = False
    elif mask_kind == "bool":  # [B, H, Lq, Lk] (text enhancer / BERT phrase blocks)
        mask = torch.rand(B, H, Lq, Lk, generator=g) < 0.7
        mask[..., 0] = True
    elif mask_kind == "dead_rows":  # some rows attend nothing
        mask = torch.rand(B, 1, Lq, Lk, generator=g) < 0.7
        mask[:, :, 3] = False
    else:  # additive float [B, 1, Lq, Lk] (BERT extended mask)
        mask = torch.where(torch.rand(B, 1, Lq, Lk, generator=g) < 0.2, -1e4, 0.0)
    grad = torch.randn(B, H, Lq, hd, generator=g).to(dtype)
    return q, k, v, mask, hd ** -0.5, grad


@pytest.mark.parametrize("B,H,Lq,Lk,hd,mask_kind,dtype,tol,layout", [
    (1, 2, 70, 50, 32, "none", torch.float32, 1e-5, "lbh"),
    (2, 2, 100, 130, 64, "bool", torch.float32, 1e-5, "lbh"),
    (1, 1, 33, 300, 32, "add", torch.float32, 1e-5, "blh"),
    (2, 2, 130, 40, 32, "keypad", torch.float32, 1e-5, "lbh"),   # decoder text cross-attention shape class
    (1, 2, 64, 64, 64, "bool", torch.bfloat16, 1.5e-2, "blh"),   # BERT shape class
    (2, 1, 90, 70, 32, "keypad", torch.bfloat16, 1.5e-2, "lbh"),
])
def test_emulated_attention(B, H, Lq, Lk, hd, mask_kind, dtype, tol, layout):
    from oracle.blocks import attention_ref
    q, k, v, mask, scale, grad = _attn_case(B, H, Lq, Lk, hd, mask_kind, dtype, seed=Lq + Lk, layout=layout)
    out, lse = E.attn_forward(q, k, v, mask, scale)
    qd, kd, vd = (t.double().requires_grad_(True) for t in (q, k, v))
    md = None if mask is None else (mask if mask.dtype == torch.bool else mask.double())
    ref = attention_ref(qd, kd, vd, md, scale)
    assert E.rel_err(out.double(), ref.detach()) < tol
    ref.backward(grad.double())
    dq, dk, dv = E.attn_backward(q, k, v, mask, scale, out, lse, grad)
    for name, mine, r in (("dq", dq, qd.grad), ("dk", dk, kd.grad), ("dv", dv, vd.grad)):
        assert torch.isfinite(mine).all(), name
        assert E.rel_err(mine.double(), r) < tol * 2, name


@pytest.mark.parametrize("qt,kt,split", [("4", "2", "0"), ("1", "1", "0"), ("4", "1", "0"), ("1", "2", "0"),
                                          ("0", "0", "1")])
def test_emulated_attention_wave_tilings(qt, kt, split, monkeypatch):
    """Both query-tile widths of the one-walk forward / dQ kernels (64 or 16
    queries per wave) and both key-tile widths of their dK / dV kernel (32 or
    16 keys per wave), forced with GD_ATTN_QT / GD_ATTN_KT under
    GD_ATTN_SPLIT=0, and the split kernels (attn_ks.inc, the default at
    these sizes): identical math, ragged lengths on both sides."""
    from oracle.blocks import attention_ref
    monkeypatch.setenv("GD_ATTN_QT", qt)
    monkeypatch.setenv("GD_ATTN_KT", kt)
    monkeypatch.setenv("GD_ATTN_SPLIT", split)
    q, k, v, mask, scale, grad = _attn_case(2, 2, 150, 90, 32, "bool", torch.float32, seed=11, layout="blh")
    out, lse = E.attn_forward(q, k, v, mask, scale)
    qd, kd, vd = (t.double().requires_grad_(True) for t in (q, k, v))
    ref = attention_ref(qd, kd, vd, mask, scale)
    assert E.rel_err(out.double(), ref.detach()) < 1e-5
    ref.backward(grad.double())
    dq, dk, dv = E.attn_backward(q, k, v, mask, scale, out, lse, grad)
    for name, mine, r in (("dq", dq, qd.grad), ("dk", dk, kd.grad), ("dv", dv, vd.grad)):
        assert E.rel_err(mine.double(), r) < 2e-5, name


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1.5e-2)])
def test_emulated_attention_growing_logits(dtype, tol):
    """Logits that grow along the keys by far more than the split forward's
    lazy-rescale margin (2^8 in p): the reference max moves several times
    inside one wave's key chunk and the merged states stay exact."""
    from oracle.blocks import attention_ref
    g = torch.Generator().manual_seed(5)
    B, H, Lq, Lk, hd = 1, 2, 40, 700, 32
    q = torch.randn(B, H, Lq, hd, generator=g).abs()
    ramp = torch.linspace(0.1, 6.0, Lk)[None, None, :, None]
    k = (torch.rand(B, H, Lk, hd, generator=g) * ramp)
    v = torch.randn(B, H, Lk, hd, generator=g)
    q, k, v = (t.to(dtype) for t in (q, k, v))
    scale = hd ** -0.5
    out, lse = E.attn_forward(q, k, v, None, scale)
    qd, kd, vd = (t.double().requires_grad_(True) for t in (q, k, v))
    ref = attention_ref(qd, kd, vd, None, scale)
    assert E.rel_err(out.double(), ref.detach()) < tol
    grad = torch.randn(B, H, Lq, hd, generator=g).to(dtype)
    ref.backward(grad.double())
    dq, dk, dv = E.attn_backward(q, k, v, None, scale, out, lse, grad)
    for name, mine, r in (("dq", dq, qd.grad), ("dk", dk, kd.grad), ("dv", dv, vd.grad)):
        assert E.rel_err(mine.double(), r) < tol * 2, name


def test_emulated_attention_fully_masked_rows_are_zero():
    """A query row whose keys are all masked gives 0 output and 0 gradients
    (the reference's softmax would give NaN there; no caller produces such
    rows: every caption keeps its [CLS] token)."""
    from oracle.blocks import attention_ref
    q, k, v, mask, scale, grad = _attn_case(1, 2, 20, 30, 32, "dead_rows", torch.float32, seed=3)
    out, lse = E.attn_forward(q, k, v, mask, scale)
    assert torch.equal(out[:, :, 3], torch.zeros_like(out[:, :, 3]))
    live = torch.ones(20, dtype=torch.bool)
    live[3] = False
    ref = attention_ref(q.double(), k.double(), v.double(), mask, scale)
    assert E.rel_err(out[:, :, live].double(), ref[:, :, live]) < 1e-5
    dq, dk, dv = E.attn_backward(q, k, v, mask, scale, out, lse, grad)
    assert torch.isfinite(dq).all() and torch.isfinite(dk).all() and torch.isfinite(dv).all()
    assert torch.equal(dq[:, :, 3], torch.zeros_like(dq[:, :, 3]))


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1.5e-2)])
def test_emulated_attention_dropout(dtype, tol):
    """Attention-probability dropout (BERT's 0.1 in training): output and
    gradients equal the reference math with the kernels' counter-based mask
    Z applied after the softmax normaliser, O = (softmax(S) . Z / (1-p)) V;
    the backward regenerates Z from the same seed."""
    p, seed = 0.25, 12345
    B, H, Lq, Lk, hd = 2, 2, 70, 90, 64
    q, k, v, mask, scale, grad = _attn_case(B, H, Lq, Lk, hd, "add", dtype, seed=7, layout="blh")
    out, lse = E.attn_forward(q, k, v, mask, scale, p, seed)
    keep = E.attn_dropout_keep(B, H, Lq, Lk, p, seed)
    assert abs(keep.float().mean().item() - (1 - p)) < 0.01
    qd, kd, vd = (t.double().requires_grad_(True) for t in (q, k, v))
    prob = torch.softmax((qd @ kd.transpose(-1, -2)) * scale + mask.double(), -1)
    ref = (prob * keep / (1 - p)) @ vd
    assert E.rel_err(out.double(), ref.detach()) < tol
    ref.backward(grad.double())
    dq, dk, dv = E.attn_backward(q, k, v, mask, scale, out, lse, grad, p, seed)
    for name, mine, r in (("dq", dq, qd.grad), ("dk", dk, kd.grad), ("dv", dv, vd.grad)):
        assert E.rel_err(mine.double(), r) < tol * 2, name


# --------------------------------------------------- contrastive head
@pytest.mark.parametrize("B,Q,T,C,tout,dtype,tol", [
    (2, 100, 37, 64, 256, torch.float32, 1e-5),    # padded to max_text_len
    (1, 70, 256, 256, 256, torch.float32, 1e-5),   # full caption, hidden 256
    (2, 130, 90, 256, 256, torch.bfloat16, 1e-5),  # bf16-exact inputs, fp32 accumulation
])
@pytest.mark.parametrize("wide", ["0", "1"])
def test_emulated_contrastive(B, Q, T, C, tout, dtype, tol, wide, monkeypatch):
    """both workgroup shapes of the v2 kernel (16 rows, 64 rows per
    workgroup; GD_CONTRASTIVE_WIDE forces one)"""
    from oracle.blocks import contrastive_ref
    monkeypatch.setenv("GD_CONTRASTIVE_WIDE", wide)
    g = torch.Generator().manual_seed(Q + T)
    x = torch.randn(B, Q, C, generator=g).to(dtype)
    text = torch.randn(B, T, C, generator=g).to(dtype)
    mask = torch.rand(B, T, generator=g) < 0.8
    mask[:, 0] = True
    logits, rowmax = E.contrastive_forward(x, text, mask, tout)
    ref = contrastive_ref(x.double(), text.double(), mask, tout).double()
    fin = torch.isfinite(ref)
    assert torch.equal(torch.isfinite(logits), fin) and (logits[~fin] == float("-inf")).all()
    assert E.rel_err(logits[fin], ref[fin]) < tol
    assert E.rel_err(rowmax, ref.max(-1)[0]) < tol
    _, only_max = E.contrastive_forward(x, text, mask, T, want_logits=False)
    assert torch.equal(only_max, rowmax)


# ------------------------------------------------------ MSDA prologue
@pytest.mark.parametrize("ref_dim", [2, 4])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_emulated_msda_prologue(ref_dim, dtype):
    """softmax + sampling-location math (ms_deform_attn.py:274-363) against
    the product's torch composition (itself pinned by the Transformer
    goldens): loc bit-identical, attn and both gradients to fp32 rounding."""
    from models.GroundingDINO.ms_deform_attn import sampling_locations_from
    g = torch.Generator().manual_seed(ref_dim)
    N, Lq, M, L, P = 2, 37, 8, 4, 4
    shapes = torch.as_tensor([(13, 21), (7, 11), (4, 6), (2, 3)])
    proj = (torch.randn(N, Lq, M * L * P * 3, generator=g) * 3).to(dtype)  # the fused Linear output
    off, logit = proj[..., :M * L * P * 2], proj[..., M * L * P * 2:]   # row-strided views, read in place
    ref = torch.rand(N, Lq, L, ref_dim, generator=g)
    loc, attn = E.msda_prologue_forward(off, logit, ref, shapes, M, L, P)
    offd = off.float().requires_grad_(True)
    logd = logit.float().requires_grad_(True)
    rl = sampling_locations_from(ref, offd.reshape(N, Lq, M, L, P, 2), shapes, P)
    ra = logd.reshape(N, Lq, M, L * P).softmax(-1).view(N, Lq, M, L, P)
    assert torch.equal(loc, rl.detach())
    torch.testing.assert_close(attn, ra.detach(), rtol=1e-6, atol=1e-7)
    gl = torch.randn(loc.shape, generator=g)
    ga = torch.randn(attn.shape, generator=g)
    (rl * gl).sum().backward()
    (ra * ga).sum().backward()
    g_off, g_log = E.msda_prologue_backward(gl, ga, attn, ref, shapes, dtype)
    if dtype == torch.float32:
        assert torch.equal(g_off, offd.grad)
        torch.testing.assert_close(g_log, logd.grad, rtol=1e-5, atol=1e-6)
    else:  # the reference returns these grads through the bf16 cast as well
        assert torch.equal(g_off, offd.grad.to(dtype))
        torch.testing.assert_close(g_log.float(), logd.grad.to(dtype).float(), rtol=1e-2, atol=1e-3)


# ------------------------------------------- split-K weight gradient
@pytest.mark.parametrize("T,O,I,splits,dtype,tol", [
    (1000, 128, 64, None, torch.float32, 1e-6),   # token tail inside the last split
    (777, 64, 192, 3, torch.float32, 1e-6),       # splits not dividing T, 3 column tiles
    (300, 192, 128, 1, torch.bfloat16, 1e-6),     # bf16-exact inputs, fp32 accumulation
    (64, 64, 64, 5, torch.float32, 1e-6),         # more splits than token chunks: empty splits
    (333, 48, 80, 2, torch.bfloat16, 1e-6),       # bf16 128-tile kernel: O, I multiples of 16, partial tiles
    (700, 384, 256, 3, torch.bfloat16, 1e-6),     # bf16: 3 x 2 tiles, token tail
    (96, 16, 16, 7, torch.bfloat16, 1e-6),        # bf16: empty splits, one 16-wide column
    (2000, 128, 144, 2, torch.bfloat16, 1e-6),    # bf16: 31 whole chunks per split through the 4-slot DMA ring
])
def test_emulated_wgrad(T, O, I, splits, dtype, tol):
    g = torch.Generator().manual_seed(T + O)
    dy = torch.randn(T, O, generator=g).to(dtype)
    x = torch.randn(T, I, generator=g).to(dtype)
    dw, db = E.wgrad(dy, x, splits=splits)
    ref_w = dy.double().t() @ x.double()
    ref_b = dy.double().sum(0)
    assert E.rel_err(dw, ref_w) < tol * 10
    assert E.rel_err(db, ref_b) < tol * 10
    dw2, none = E.wgrad(dy, x, bias=False, splits=splits)
    assert none is None and torch.equal(dw, dw2)


# ------------------------------------------------ residual add + LayerNorm
@pytest.mark.parametrize("rows,C,xd,rd", [
    (37, 256, torch.float32, torch.bfloat16),   # fp32 residual + bf16 sublayer output (autocast)
    (50, 192, torch.float32, torch.float32),
    (9, 768, torch.bfloat16, torch.bfloat16),
    (3000, 64, torch.float32, torch.float32),   # more rows than the backward grid's waves
    (41, 96, torch.float32, None),              # Swin-T stage 0: C not a multiple of 64, no residual
    (7, 1536, torch.bfloat16, None),            # patch-merging width, no residual
    (5, 2048, torch.float32, torch.bfloat16),
])
def test_emulated_add_layernorm(rows, C, xd, rd):
    g = torch.Generator().manual_seed(rows + C)
    x = (torch.randn(rows, C, generator=g) * 2 + 0.5).to(xd)
    r = torch.randn(rows, C, generator=g).to(rd) if rd is not None else None
    w = torch.randn(C, generator=g)
    b = torch.randn(C, generator=g)
    y, mean, rstd = E.add_layernorm_forward(x, r, w, b, 1e-5)
    xs = (x.double() + (r.double() if r is not None else 0)).requires_grad_(True)
    wd, bd = w.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(xs, (C,), wd, bd, 1e-5)
    assert E.rel_err(y, ref.detach()) < 1e-5
    dy = torch.randn(rows, C, generator=g)
    ref.backward(dy.double())
    dx, dr, dw, db = E.add_layernorm_backward(x, r, w, dy, mean, rstd)
    tol = 1e-5 if xd == torch.float32 else 1e-2
    assert E.rel_err(dx.double(), xs.grad) < tol
    if r is not None:
        assert E.rel_err(dr.double(), xs.grad) < (1e-5 if rd == torch.float32 else 1e-2)
    else:
        assert dr is None
    assert E.rel_err(dw, wd.grad) < 1e-5
    assert E.rel_err(db, bd.grad) < 1e-5


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_emulated_add_norm3_matches_the_composition(p):
    """layernorm.add_norm3 = norm(x + (r + dropout(r2))) (the MSDA identity
    add and dropout folded into add + LayerNorm) vs the module composition
    through autograd, fp32 residual / identity, bf16 branch.  p > 0: the mask
    is regenerated in the backward; the kept set read off the branch
    gradient (non-zero where kept) drives the composition, and about p of
    the elements are dropped."""
    from emu_product import emulated_product
    from gdino_amd.layernorm import add_norm3
    g = torch.Generator().manual_seed(5)
    rows = 300
    norm = torch.nn.LayerNorm(256)
    with torch.no_grad():
        norm.weight.copy_(torch.randn(256, generator=g))
        norm.bias.copy_(torch.randn(256, generator=g))
    drop = torch.nn.Dropout(p)
    x0 = torch.randn(2, rows // 2, 256, generator=g)
    r0 = torch.randn(2, rows // 2, 256, generator=g)
    r20 = torch.randn(2, rows // 2, 256, generator=g).to(torch.bfloat16)
    dy = torch.randn(2, rows // 2, 256, generator=g)
    x, r, r2 = (t.clone().requires_grad_(True) for t in (x0, r0, r20))
    with emulated_product():
        y = add_norm3(norm, x, r, r2, drop)
        assert y is not None
        y.backward(dy)
    keep = r2.grad != 0 if p > 0 else torch.ones_like(r20, dtype=torch.bool)
    if p > 0:
        assert abs(float((~keep).float().mean()) - p) < 0.01
    xc, rc, r2c = (t.clone().requires_grad_(True) for t in (x0, r0, r20))
    wc, bc = norm.weight.detach().clone().requires_grad_(True), norm.bias.detach().clone().requires_grad_(True)
    branch = torch.where(keep, r2c * (1.0 / (1.0 - p)), torch.zeros((), dtype=torch.bfloat16))
    want = torch.nn.functional.layer_norm(xc + (branch + rc), (256,), wc, bc, norm.eps)
    want.backward(dy)
    assert E.rel_err(y.detach(), want.detach()) < 1e-6
    assert E.rel_err(x.grad, xc.grad) < 1e-5 and E.rel_err(r.grad, rc.grad) < 1e-5
    assert E.rel_err(r2.grad.float(), r2c.grad.float()) < 1e-2
    assert E.rel_err(norm.weight.grad, wc.grad) < 1e-5 and E.rel_err(norm.bias.grad, bc.grad) < 1e-5


@pytest.mark.parametrize("C,bd,dp", [(96, torch.bfloat16, 0.0), (192, torch.float32, 0.2), (384, torch.bfloat16, 0.3),
                                      (768, torch.bfloat16, 0.0)])
def test_emulated_add_scaled_norm_matches_the_composition(C, bd, dp):
    """layernorm.add_scaled_norm = (x + drop_path(branch), norm(...)) vs
    add_drop_path + layer_norm through autograd, the same seeded drop-path
    draw, both outputs consumed (the backward sums their gradients in the
    kernel)."""
    from emu_product import emulated_product
    from gdino_amd.layernorm import add_scaled_norm
    from gdino_amd.misc import add_drop_path
    g = torch.Generator().manual_seed(C)
    norm = torch.nn.LayerNorm(C)
    with torch.no_grad():
        norm.weight.copy_(torch.randn(C, generator=g))
        norm.bias.copy_(torch.randn(C, generator=g))
    x0 = torch.randn(3, 50, C, generator=g)
    b0 = torch.randn(3, 50, C, generator=g).to(bd)
    gs, gy = torch.randn(3, 50, C, generator=g), torch.randn(3, 50, C, generator=g)
    out = {}
    for fused in (True, False):
        x, b = x0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        norm.zero_grad()
        torch.manual_seed(11)
        with emulated_product():
            if fused:
                r = add_scaled_norm(norm, x, b, dp, True)
                assert r is not None
                s, y = r
            else:
                s = add_drop_path(x, b, dp, True)
                y = torch.nn.functional.layer_norm(s, (C,), norm.weight, norm.bias, norm.eps)
            ((s * gs).sum() + (y * gy).sum()).backward()
        out[fused] = (s.detach(), y.detach(), x.grad, b.grad, norm.weight.grad.clone(), norm.bias.grad.clone())
    for a, w in zip(out[True], out[False]):
        assert a.dtype == w.dtype
        assert E.rel_err(a.float(), w.float()) < (1e-2 if a.dtype == torch.bfloat16 else 2e-5)


# ------------------------------------------------ box refinement (boxref.hip)
@pytest.mark.parametrize("dd,transposed_ref,ref_grad", [
    (torch.float32, False, True),
    (torch.bfloat16, True, True),    # the box heads: bf16 MLP output, reference points through a transposed view
    (torch.bfloat16, False, False),  # the decoder's anchor update: detached reference points
])
def test_emulated_box_refine(dd, transposed_ref, ref_grad, monkeypatch):
    """sigmoid(delta + inverse_sigmoid(ref)) forward / backward through the
    product's autograd function vs the composition (GDINO_DISABLE=boxrefine),
    including reference points outside [0, 1], at the clamp edges (0, 1,
    eps, 1 - eps) and NaN."""
    from emu_product import emulated_product
    from gdino_amd.misc import box_refine
    g = torch.Generator().manual_seed(7)
    delta = torch.randn(2, 37, 4, generator=g).to(dd)
    ref = torch.rand(37, 2, 4, generator=g) * 1.2 - 0.1
    ref.view(-1)[:8] = torch.tensor([0.0, 1.0, 1e-3, 1 - 1e-3, 5e-4, 0.9996, -0.0, float("nan")])
    ref = ref.transpose(0, 1) if transposed_ref else ref.transpose(0, 1).contiguous()
    go = torch.randn(2, 37, 4, generator=g)

    def run(disable):
        if disable:
            monkeypatch.setenv("GDINO_DISABLE", "boxrefine")
        else:
            monkeypatch.delenv("GDINO_DISABLE", raising=False)
        d = delta.clone().requires_grad_(True)
        r = ref.detach().clone() if not transposed_ref else ref.detach().transpose(0, 1).clone().transpose(0, 1)
        r.requires_grad_(ref_grad)
        with emulated_product():
            out = box_refine(d, r)
            out.backward(go)
        return out.detach(), d.grad, r.grad

    got, want = run(False), run(True)
    assert got[0].dtype == want[0].dtype == torch.float32
    assert torch.equal(got[0].isnan(), want[0].isnan())
    fin = ~want[0].isnan()
    assert E.rel_err(got[0][fin], want[0][fin]) < 1e-6
    assert got[1].dtype == dd
    gfin = ~want[1].float().isnan()
    assert E.rel_err(got[1].float()[gfin], want[1].float()[gfin]) < (1e-6 if dd == torch.float32 else 2 ** -7)
    if ref_grad:
        assert torch.equal(got[2].isnan(), want[2].isnan())
        rf = ~want[2].isnan()
        assert E.rel_err(got[2][rf], want[2][rf]) < 1e-5
    else:
        assert got[2] is None and want[2] is None


@pytest.mark.parametrize("n,c,bd,sshape,sd,xd", [
    (37, 96, torch.bfloat16, (2, 1, 96), torch.float32, torch.float32),    # layer scale x drop path
    (300, 256, torch.bfloat16, (2, 1, 1), torch.bfloat16, torch.float32),  # drop path only, bf16 mask
    (29, 64, torch.float32, (64,), torch.float32, torch.float32),          # one gamma for all samples
    (50, 128, torch.bfloat16, (1, 1, 128), torch.float32, torch.bfloat16),
    (11, 192, torch.bfloat16, (2, 1, 1), torch.bfloat16, torch.bfloat16),  # bf16 out
])
def test_emulated_add_scaled(n, c, bd, sshape, sd, xd, monkeypatch):
    """csrc/residual.hip (x + branch * s and its backward) through the
    product's autograd function vs the addcmul composition it replaces
    (GDINO_DISABLE=addscaled): forward and d branch within one rounding of
    the output dtype, d x = g, d s (the token reduction) within fp32
    summation-order noise."""
    from emu_product import emulated_product
    from gdino_amd.misc import _AddScaled
    g = torch.Generator().manual_seed(n * c)
    x = torch.randn(2, n, c, generator=g).to(xd)
    br = torch.randn(2, n, c, generator=g).to(bd)
    s = (torch.rand(sshape, generator=g) + 0.5).to(sd)
    go_seed = torch.randn(2, n, c, generator=g)

    def run(disable):
        if disable:
            monkeypatch.setenv("GDINO_DISABLE", "addscaled")
        else:
            monkeypatch.delenv("GDINO_DISABLE", raising=False)
        xx, bb, ss = (t.clone().requires_grad_(True) for t in (x, br, s))
        with emulated_product():
            out = _AddScaled.apply(xx, bb, ss)
            out.backward(go_seed.to(out.dtype))
        return out.detach(), xx.grad, bb.grad, ss.grad

    got, ref = run(False), run(True)
    assert got[0].dtype == ref[0].dtype
    for name, a, b in zip(("out", "dx", "dbranch", "ds"), got, ref):
        assert a.dtype == b.dtype and a.shape == b.shape, name
        a, b = a.double(), b.double()
        tol = 1e-5 if a.dtype == torch.float32 else (2 ** -7 if name in ("out", "dbranch") else 1e-2)
        if name == "ds":
            tol = 1e-4 if s.dtype == torch.float32 else 1e-2
        err = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        assert err <= tol, (name, err)


@pytest.mark.parametrize("local,outliers", [(True, 0.1), (False, 0.0)])
def test_emulated_geometry_shared_kernels_match_per_lane_kernels(local, outliers, monkeypatch):
    """Round 5: the bf16 forward (msda_fwd_gs) and the sorted backward's
    per-sample pass (msda_bwd_samples_gs) compute each sample's geometry on
    one lane of the unit's quad and broadcast it by DPP; their results equal
    the per-lane kernels' (msda_fwd_vec, msda_bwd_samples<.., 2, true>) up to
    the summation rounding of the packed / dot2 arithmetic, including
    locations outside the levels and NaN / inf locations."""
    S = sum(h * w for h, w in MEDIUM)
    value, shapes, lsi, loc, attn, grad_out = _levels_inputs(MEDIUM, 2, S if local else 41, seed=31,
                                                             vdtype=torch.bfloat16, local=local,
                                                             outlier_frac=outliers)
    loc = loc.clone()
    loc.view(-1)[::97] = float("nan")
    loc.view(-1)[5::101] = float("inf")
    res = {}
    for gs in ("0", "1"):
        monkeypatch.setenv("GD_MSDA_FWD_GS", gs)
        monkeypatch.setenv("GD_MSDA_SORTED_GS", gs)
        out = E.msda_forward(value, shapes, lsi, loc, attn)
        gv, gl, ga = E.msda_backward_sorted(value, shapes, lsi, loc, attn, grad_out, host_shapes=MEDIUM)
        res[gs] = (out.float(), gv.float(), gl, ga)
    for a, b, name in zip(res["0"], res["1"], ("out", "grad_value", "grad_loc", "grad_attn")):
        assert torch.isfinite(b).all(), name
        assert E.rel_err(b.double().numpy(), a.double().numpy()) < (1e-2 if name in ("out", "grad_value") else 1e-5), \
            (name, E.rel_err(b.double().numpy(), a.double().numpy()))


@pytest.mark.parametrize("transposed", [False, True])
def test_emulated_query_anchors(transposed, monkeypatch):
    """One decoder layer's anchors (ref_input = ref * valid_ratios and the
    (y, x, w, h) sine embedding of its level-0 slice) from the fused kernel
    (csrc/boxref.hip query_anchor_kernel) vs the composition
    (gen_sineembed_for_position; GDINO_DISABLE=boxrefine): ref_input
    bitwise (the same fp32 products), the embedding to the sin / cos
    implementations' ulps."""
    from emu_product import emulated_product
    from models.GroundingDINO.utils import query_anchors
    g = torch.Generator().manual_seed(3)
    ref = torch.rand(2, 37, 4, generator=g)
    ref = ref.transpose(0, 1) if transposed else ref.transpose(0, 1).contiguous()  # [nq, bs, 4]
    vr = torch.cat([torch.rand(2, 4, 2, generator=g) * 0.5 + 0.5] * 2, -1)          # [bs, L, 4]

    def run(disable):
        if disable:
            monkeypatch.setenv("GDINO_DISABLE", "boxrefine")
        else:
            monkeypatch.delenv("GDINO_DISABLE", raising=False)
        with emulated_product():
            return query_anchors(ref, vr)

    (ri, se), (ri0, se0) = run(False), run(True)
    assert ri.shape == ri0.shape == (37, 2, 4, 4) and se.shape == se0.shape == (37, 2, 512)
    assert torch.equal(ri, ri0)
    assert float((se - se0).abs().max()) < 2e-6


@pytest.mark.parametrize("m,k,n,relu,bias,pad", [
    (300, 256, 256, False, True, 0),     # the encoder's 256 -> 256 (tail tile of 44 rows)
    (257, 96, 288, True, True, 0),       # Swin-T stage 0: K = 96 (half chunk), N = 288 (partial N tile)
    (130, 384, 96, False, False, 8),     # no bias, x rows padded (ldx = K + 8)
    (64, 2048, 136, True, True, 0),      # long K, N = 136 (one full and one 8-wide N tile)
    # the x-resident kernel (K <= 256): K = 192 with padded rows, K = 128
    # with a 40-wide last column block, K = 88 (zero-filled K tail of the
    # 96-wide tile), and a column split over workgroups (few token tiles)
    (200, 192, 576, False, True, 8),
    (77, 128, 40, True, False, 0),
    (150, 88, 64, False, True, 0),
    (40, 256, 1024, True, True, 0),
])
def test_emulated_token_linear_forward(m, k, n, relu, bias, pad):
    """csrc/tlin.hip y = x W^T (+ b) (ReLU), bf16 in / out, fp32 accumulate,
    against the fp64 product rounded once to bf16: every element within one
    bf16 ulp (the accumulation order differs), tails in M, N and K
    zero-filled and masked."""
    from emu_product import emulated_product
    from gdino_amd.wgrad import tlin_forward
    g = torch.Generator().manual_seed(m + k + n)
    xs = torch.randn(m, k + pad, generator=g).to(torch.bfloat16)
    x = xs[:, :k]
    w = (torch.randn(n, k, generator=g) * k ** -0.5).to(torch.bfloat16)
    b = torch.randn(n, generator=g).to(torch.bfloat16) if bias else None
    with emulated_product():
        y = tlin_forward(x, w, b, relu)
    ref = x.double() @ w.double().t() + (b.double() if bias else 0)
    if relu:
        ref = ref.clamp_min(0)
    assert y.shape == (m, n) and y.dtype == torch.bfloat16
    ulp = ref.abs().clamp_min(1e-3) * 2 ** -7
    assert bool(((y.double() - ref).abs() <= ulp).all()), float(((y.double() - ref).abs() / ulp).max())


@pytest.mark.parametrize("m,k,n,pad", [(300, 256, 2048, 0), (130, 64, 136, 8), (100, 192, 264, 8)])
def test_emulated_token_linear_forward_masked(m, k, n, pad):
    """gd_token_linear_forward_masked: the bf16 product where the mask is
    > 0, +0 elsewhere (threshold_backward on the rounded product: negative,
    zero and NaN mask entries all drop the element)."""
    from emu_product import emulated_product
    from gdino_amd.wgrad import masked_dx
    g = torch.Generator().manual_seed(m + n)
    dys = torch.randn(m, k + pad, generator=g).to(torch.bfloat16)
    dy = dys[:, :k]
    w = (torch.randn(k, n, generator=g) * k ** -0.5).to(torch.bfloat16)  # [N_out, K_in] of the Linear
    mask = torch.randn(m, n, generator=g).clamp_min(0).to(torch.bfloat16)
    mask[0, :8] = float("nan")
    mask[1, :8] = -0.0
    with emulated_product():
        y = masked_dx(dy, w, mask)
    ref = dy.double() @ w.double()
    keep = mask.double() > 0
    assert y.shape == (m, n) and y.dtype == torch.bfloat16
    assert bool((y[~keep] == 0).all()) and not bool(torch.signbit(y[~keep]).any())
    ulp = ref.abs().clamp_min(1e-3) * 2 ** -7
    assert bool(((y.double() - ref).abs()[keep] <= ulp[keep]).all())


def test_emulated_relu_linear_pair_folds_the_threshold(monkeypatch):
    """relu TokenLinear -> TokenLinear (the FFN): the second Linear's dX
    kernel applies the ReLU's mask and the first skips its threshold pass;
    every gradient matches the unfused pair (GD_TLIN_MASKED=0) within the
    bf16 rounding of dX."""
    from emu_product import emulated_product
    from gdino_amd import wgrad
    monkeypatch.setattr(wgrad, "TLIN_MASKED_MIN_TOKENS", 64)
    g = torch.Generator().manual_seed(3)
    x0 = torch.randn(2, 96, 64, generator=g)
    w1, b1 = torch.randn(128, 64, generator=g) * 0.125, torch.randn(128, generator=g) * 0.1
    w2, b2 = torch.randn(64, 128, generator=g) * 0.09, torch.randn(64, generator=g) * 0.1
    gy = torch.randn(2, 96, 64, generator=g)

    def run(fold):
        monkeypatch.setattr(wgrad, "TLIN_MASKED", fold)
        x = x0.to(torch.bfloat16).requires_grad_()
        ps = [t.clone().requires_grad_() for t in (w1, b1, w2, b2)]
        with emulated_product():
            h = wgrad.token_linear(x, ps[0].to(torch.bfloat16), ps[1].to(torch.bfloat16), [ps[0]], [ps[1]],
                                   relu=True, fold=True)
            box = h._gd_relu_box
            y = wgrad.token_linear(h, ps[2].to(torch.bfloat16), ps[3].to(torch.bfloat16), [ps[2]], [ps[3]])
            (y.float() * gy).sum().backward()
        return box[0], [x.grad] + [p.grad for p in ps]

    (folded, got), (unfolded, ref) = run(True), run(False)
    assert folded and not unfolded
    for a, b in zip(got, ref):
        assert float((a.float() - b.float()).abs().max()) <= 2e-2 * float(b.float().abs().max())


@pytest.mark.parametrize("second", ["elementwise", "linear"])
def test_emulated_relu_output_with_a_second_consumer(monkeypatch, second):
    """a relu TokenLinear whose output has a second consumer
    besides the next Linear.  Without the caller's single-consumer promise
    (fold=False, the default of castcache.linear_relu) the output is never
    offered for the dX fold, so both consumers' gradients pass the ReLU mask:
    every gradient matches the plain fp32 composition.  A claimed tag is
    removed, so a second Linear consumer can never fold the same ReLU."""
    from emu_product import emulated_product
    from gdino_amd import wgrad
    monkeypatch.setattr(wgrad, "TLIN_MASKED_MIN_TOKENS", 64)
    g = torch.Generator().manual_seed(5)
    x0 = torch.randn(2, 96, 64, generator=g)
    w1, b1 = torch.randn(128, 64, generator=g) * 0.125, torch.randn(128, generator=g) * 0.1
    w2, b2 = torch.randn(64, 128, generator=g) * 0.09, torch.randn(64, generator=g) * 0.1
    w3 = torch.randn(32, 128, generator=g) * 0.09
    gy, gz = torch.randn(2, 96, 64, generator=g), torch.randn(2, 96, 128 if second == "elementwise" else 32,
                                                             generator=g)

    def consumers(h, ps, lin):
        y = lin(h, ps[2], ps[3])
        z = h.float() * 3.0 if second == "elementwise" else lin(h, ps[4], None)
        return (y.float() * gy).sum() + (z.float() * gz).sum()

    def run(masked):
        monkeypatch.setattr(wgrad, "TLIN_MASKED", masked)
        x = x0.to(torch.bfloat16).requires_grad_()
        ps = [t.clone().requires_grad_() for t in (w1, b1, w2, b2, w3)]
        with emulated_product():
            h = wgrad.token_linear(x, ps[0].to(torch.bfloat16), ps[1].to(torch.bfloat16), [ps[0]], [ps[1]],
                                   relu=True)
            assert getattr(h, "_gd_relu_box", None) is None  # not offered without the promise

            def lin(t, w, b):
                return wgrad.token_linear(t, w.to(torch.bfloat16), None if b is None else b.to(torch.bfloat16),
                                          [w], [] if b is None else [b])
            consumers(h, ps, lin).backward()
        return x, ps, [x.grad] + [p.grad for p in ps]

    # the fold enabled (what the second consumer would have broken) vs the
    # unfused threshold path: the same gradients
    x, ps, got = run(True)
    _, _, ref = run(False)
    for a, b in zip(got, ref):
        assert (a is None) == (b is None)
        if a is not None:
            assert float((a.float() - b.float()).abs().max()) <= 1e-6 * float(b.float().abs().max())
    # and both follow the fp64 composition (the ReLU mask taken from the
    # product's bf16 pre-activation, so boundary elements agree)
    xr = x0.to(torch.bfloat16).double().requires_grad_()
    pr = [t.double().requires_grad_() for t in (w1, b1, w2, b2, w3)]
    pre = torch.nn.functional.linear(xr, pr[0], pr[1])
    with torch.no_grad(), emulated_product():
        hp = wgrad.token_linear(x.detach(), ps[0].detach().to(torch.bfloat16), ps[1].detach().to(torch.bfloat16),
                                [ps[0]], [ps[1]], relu=True)
    hr = pre * (hp > 0)
    consumers(hr, pr, lambda t, w, b: torch.nn.functional.linear(t, w, b)).backward()
    for a, b in zip(got, [xr.grad] + [p.grad for p in pr]):
        if a is not None:
            assert float((a.double() - b).abs().max()) <= 3e-2 * float(b.abs().max())

    # a claimed tag is gone: the second Linear consumer cannot fold again
    monkeypatch.setattr(wgrad, "TLIN_MASKED", True)
    with emulated_product():
        h = wgrad.token_linear(x.detach(), ps[0].detach().to(torch.bfloat16), ps[1].detach().to(torch.bfloat16),
                               [ps[0]], [ps[1]], relu=True, fold=True)
        box = h._gd_relu_box
        wgrad.token_linear(h, ps[2].detach().to(torch.bfloat16), ps[3].detach().to(torch.bfloat16), [ps[2]],
                           [ps[3]])
        assert box[0] and getattr(h, "_gd_relu_box", None) is None


@pytest.mark.parametrize("three", [False, True])
def test_emulated_add_norm_two_handles(three):
    """add_norm / add_norm3 with taps=2: two handles on the output, each read
    by its own consumer; the backward kernel sums their gradients (no
    autograd accumulation add) -- same gradients as one output read twice."""
    from emu_product import emulated_product
    from gdino_amd.layernorm import add_norm, add_norm3
    g = torch.Generator().manual_seed(9)
    norm = torch.nn.LayerNorm(256)
    with torch.no_grad():
        norm.weight.copy_(torch.randn(256, generator=g))
        norm.bias.copy_(torch.randn(256, generator=g))
    x0, r0 = torch.randn(3, 40, 256, generator=g), torch.randn(3, 40, 256, generator=g)
    r20 = torch.randn(3, 40, 256, generator=g).to(torch.bfloat16)
    ga, gb = torch.randn(3, 40, 256, generator=g), torch.randn(3, 40, 256, generator=g)
    out = {}
    for taps in (1, 2):
        x, r, r2 = (t.clone().requires_grad_(True) for t in (x0, r0, r20))
        norm.zero_grad()
        with emulated_product():
            if three:
                y = add_norm3(norm, x, r, r2, torch.nn.Identity(), taps=taps)
            else:
                y = add_norm(norm, x, r2, taps=taps)
            ya, yb = (y, y) if taps == 1 else y
            assert ya.shape == yb.shape == x.shape
            ((ya * ga).sum() + (yb.sin() * gb).sum()).backward()
        out[taps] = [t.grad.clone() for t in ((x, r, r2) if three else (x, r2))] + [norm.weight.grad.clone(),
                                                                                     norm.bias.grad.clone()]
    for a, b in zip(out[2], out[1]):
        assert E.rel_err(a.float(), b.float()) < (1e-2 if a.dtype == torch.bfloat16 else 1e-6)


def test_emulated_add_with_twins():
    """gd_add_twin_forward: query = src + pos in fp32 (exact) with the bf16
    twins of query and src written in the same pass (bitwise the casts), the
    twins attached where wgrad.TokenLinear reads them; gradients pass through."""
    from emu_product import emulated_product
    from gdino_amd.misc import add_with_twins
    g = torch.Generator().manual_seed(4)
    a = torch.randn(2, 37, 256, generator=g).requires_grad_()
    b = torch.randn(2, 37, 256, generator=g).requires_grad_()
    with emulated_product(), torch.autocast("cpu", dtype=torch.bfloat16):
        q = add_with_twins(a, b)
    assert torch.equal(q, a + b)
    assert torch.equal(q._gd_bf16[0], (a + b).detach().to(torch.bfloat16)) and q._gd_bf16[1] == q._version
    assert torch.equal(a._gd_bf16[0], a.detach().to(torch.bfloat16))
    gq = torch.randn(2, 37, 256, generator=g)
    q.backward(gq)
    assert torch.equal(a.grad, gq) and torch.equal(b.grad, gq)
