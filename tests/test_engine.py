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


def _timeout_rank(rank, world, port, q):
    """One rank of the forced-timeout test: train_one_epoch on the gloo
    group with the device-readiness probe stuck at 'not ready'."""
    import os
    import sys
    from test_stepgraph_protocol import _paths
    _paths()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gdino_amd import engine
        from gdino_amd.train import BucketedGradSync
        model, crit, opt = _model(seed=2)
        _no_dropout(model)
        sync = BucketedGradSync(model.parameters(), bucket_mb=1, first_bucket_mb=0.25)
        Fake = _fake_graph_class()
        # what step_graph_for builds when no group is passed: a gloo group
        grp = engine.make_control_group()
        model._gd_step_graph = Fake(model, crit, opt, amp_dtype=None, warmup=1, grad_sync=sync, control_group=grp)
        backend = dist.get_backend(model._gd_step_graph.agree.group)
        engine._device_ready_fn = lambda device: (lambda: False)  # a device that never finishes

        class Args(_Args):
            sync_timeout = 0.5

        code = None
        with oracle_msda(), scipy_lsap():
            try:
                engine.train_one_epoch(model, crit, [next(_loader())], opt, torch.device("cpu"), epoch=0,
                                       max_norm=0.1, args=Args(), print_freq=1, grad_sync=sync)
            except SystemExit as e:
                code = e.code
        q.put((rank, code, backend))
    finally:
        dist.destroy_process_group()


def test_two_ranks_stuck_device_exits_with_a_message():
    """the engine's loss read-back waits for the
    device with a deadline; a device that never finishes ends every rank
    with exit status 3 instead of a silent hang."""
    import torch.multiprocessing as mp
    from test_stepgraph_protocol import _free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert [r[1] for r in res] == [3, 3], res
    assert all(r[2] == "gloo" for r in res), res


def test_bounded_wait_raises_after_the_deadline():
    import time
    from gdino_amd.engine import DeviceTimeout, bounded_wait
    t0 = time.monotonic()
    try:
        bounded_wait(lambda: False, 0.2, "test")
        raise AssertionError("no timeout")
    except DeviceTimeout as e:
        assert "0 s: test" in str(e) or "test" in str(e)
    assert time.monotonic() - t0 < 5
    bounded_wait(lambda: True, 0.0, "ready")
