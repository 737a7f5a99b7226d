"""The decoder's anchor updates with the batched backward
(transformer._BatchedBoxRefine: the layer loop runs bbox_embed + box_refine
without autograd, one node recomputes the shared MLP over all layers in the
backward) against the per-layer autograd path (GDINO_DEFER_BOX_REFINE=0,
reference transformer.py:728-731): same loss and the same gradient for every
parameter, fp32 on the CPU (oracle ops)."""
import torch

from oracle_hooks import oracle_msda, scipy_lsap
from test_stepgraph_protocol import _batch, _model, _no_dropout


def test_batched_anchor_refine_backward_matches_per_layer_autograd():
    import models.GroundingDINO.transformer as tr
    from gdino_amd.stepgraph import TrainStepGraph
    out = {}
    saved = tr.DEFER_BOX_REFINE
    try:
        with oracle_msda(), scipy_lsap():
            for defer in (True, False):
                tr.DEFER_BOX_REFINE = defer
                model, crit, opt = _model(seed=4)
                _no_dropout(model)
                g = TrainStepGraph(model, crit, opt, amp_dtype=None, max_graphs=0, capture_after=10 ** 9)
                inputs, pf = g._prepare(*_batch(21, n_tokens=23))
                model.zero_grad(set_to_none=True)
                loss, _ = g._forward_loss(inputs, pf)
                loss.backward()
                out[defer] = (float(loss), {n: p.grad.clone() for n, p in model.named_parameters()
                                            if p.grad is not None})
    finally:
        tr.DEFER_BOX_REFINE = saved
    (l1, g1), (l0, g0) = out[True], out[False]
    assert abs(l1 - l0) <= 1e-6 * abs(l0)
    assert g1.keys() == g0.keys()
    assert any("bbox_embed" in n for n in g1)
    for n in g0:
        d = float((g1[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-30))
        assert d < 1e-5, (n, d)
