"""Pin the oracle: the C restatement and the torch restatements against the
golden vectors generated from the reference's pure-PyTorch MSDA
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

import oracle
from oracle.msda_torch import msda_gather, msda_grid_sample
from msda_cases import KAT_NAMES, cfg1_inputs, edge_excluded_mask, load_case


@pytest.mark.parametrize("name", KAT_NAMES + ["edge"])
def test_c_oracle_forward_matches_golden(name):
    c = load_case(name)
    out = oracle.msda_forward(c["value"], c["shapes"], c["lsi"], c["loc"], c["attn"])
    np.testing.assert_allclose(out, c["out"], rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("name", KAT_NAMES + ["edge"])
def test_c_oracle_backward_matches_golden(name):
    c = load_case(name)
    gv, gl, ga = oracle.msda_backward(c["value"], c["shapes"], c["lsi"], c["loc"], c["attn"],
                                      c["grad_out"])
    np.testing.assert_allclose(gv, c["grad_value"], rtol=1e-11, atol=1e-13)
    np.testing.assert_allclose(ga, c["grad_attn"], rtol=1e-11, atol=1e-13)
    edge = edge_excluded_mask(c)
    # grid_sample's one-sided derivative on the excluded band edge is the one
    # documented divergence from the CUDA kernel semantics the oracle follows.
    keep = ~np.repeat(edge[..., None], 2, axis=-1)
    np.testing.assert_allclose(gl[keep], c["grad_loc"][keep], rtol=1e-10, atol=1e-12)


def test_edge_case_exercises_band_edges():
    c = load_case("edge")
    assert edge_excluded_mask(c).sum() >= 4


def test_cfg1_oracle_matches_golden_checksums():
    z = load_case("cfg1")
    value, shapes, lsi, loc, attn, grad_out = cfg1_inputs()
    assert abs(float(value.sum()) - float(z["value_sum"])) < 1e-6, "torch CPU RNG changed"
    out = oracle.msda_forward(value, shapes, lsi, loc, attn)
    gv, gl, ga = oracle.msda_backward(value, shapes, lsi, loc, attn, grad_out)
    for name, arr in (("out", out), ("grad_value", gv), ("grad_loc", gl), ("grad_attn", ga)):
        flat = arr.reshape(-1)
        np.testing.assert_allclose(flat[z[f"{name}_idx"]], z[f"{name}_val"], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(flat.sum(), z[f"{name}_sum"], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose((flat * flat).sum(), z[f"{name}_sqsum"], rtol=1e-9)


@pytest.mark.parametrize("name", KAT_NAMES + ["edge"])
def test_torch_restatements_match_golden(name):
    c = load_case(name)
    v, loc, attn = (torch.from_numpy(c[k]) for k in ("value", "loc", "attn"))
    shapes, lsi = torch.from_numpy(c["shapes"]), torch.from_numpy(c["lsi"])
    out_gs = msda_grid_sample(v, shapes, loc, attn)
    out_ga = msda_gather(v, shapes, lsi, loc, attn)
    np.testing.assert_allclose(out_gs.numpy(), c["out"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(out_ga.numpy(), c["out"], rtol=1e-12, atol=1e-14)


def test_gather_restatement_gradcheck():
    c = load_case("kat_grad_d30")
    v = torch.from_numpy(c["value"]).requires_grad_(True)
    loc = torch.from_numpy(c["loc"]).requires_grad_(True)
    attn = torch.from_numpy(c["attn"]).requires_grad_(True)
    shapes, lsi = torch.from_numpy(c["shapes"]), torch.from_numpy(c["lsi"])
    assert torch.autograd.gradcheck(lambda a, b, d: msda_gather(a, shapes, lsi, b, d), (v, loc, attn))
