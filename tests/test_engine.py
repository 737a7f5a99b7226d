"""gdino_amd.engine.train_one_epoch -- the reference trainer's epoch loop
(engine_multi.py:353-602) bound to the step graph -- on CPU: an epoch over
odvg-style batches of varying caption length gives the same weights as the
reference loop's eager steps (model -> criterion -> weighted sum ->
zero_grad -> backward -> clip -> step, per batch), and returns the
reference's averaged stats.  The HIP-graph capture is replaced by the
stand-in of tests/test_stepgraph_protocol.py (its replay runs the captured
body eagerly); the GPU side is tests/test_stepgraph_gpu.py."""
import math

import torch

from oracle_hooks import oracle_msda, scipy_lsap
from test_stepgraph_protocol import _batch, _fake_graph_class, _model, _no_dropout


class _Args:
    amp = False
    onecyclelr = False
    debug = False
    graph_image_multiple = 1


def _loader():
    for i, nt in enumerate((14, 27, 40)):
        samples, targets, _, _ = _batch(40 + i, n_tokens=nt)
        yield samples, targets


def test_train_one_epoch_matches_the_reference_loop():
    from gdino_amd.engine import train_one_epoch
    from gdino_amd.stepgraph import TrainStepGraph
    out = {}
    with oracle_msda(), scipy_lsap():
        for mode in ("reference", "engine"):
            model, crit, opt = _model(seed=2)
            _no_dropout(model)
            if mode == "reference":
                # the reference's per-batch eager sequence on the same step body
                g = TrainStepGraph(model, crit, opt, amp_dtype=None, max_graphs=0, capture_after=10 ** 9)
                for samples, targets in _loader():
                    g(samples, targets, [t["caption"] for t in targets], [t["cap_list"] for t in targets])
                stats = None
            else:
                Fake = _fake_graph_class()
                model._gd_step_graph = Fake(model, crit, opt, amp_dtype=None, warmup=1)
                stats = train_one_epoch(model, crit, _loader(), opt, torch.device("cpu"), epoch=0, max_norm=0.1,
                                        args=_Args(), print_freq=2)
            out[mode] = (torch.cat([p.detach().reshape(-1) for p in model.parameters() if p.requires_grad]), stats)
    pr, _ = out["reference"]
    pe, stats = out["engine"]
    assert float((pr - pe).abs().max()) <= 1e-6
    assert math.isfinite(stats["loss"]) and stats["loss"] > 0 and "lr" in stats
    assert stats["step_graph"]["captures"] == 1 and stats["step_graph"]["replays"] == 3  # one 64-token bucket
