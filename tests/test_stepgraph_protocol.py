"""The step graph's host-side protocol on CPU (gdino_amd.stepgraph):

* text padding to a bucket of 64 tokens leaves the losses and gradients
  unchanged (pad tokens are masked everywhere);
* a capture step applies its batch exactly once: the warm-up iterations are
  rolled back (weights, AdamW state, RNG), so the first call equals an eager
  step bit for bit;
* world_size 2 (gloo): ranks with different image sizes capture different
  graphs and still average their gradients exactly like DDP; when rank 1's
  capture fails, EVERY rank drops to the eager step and the gradients still
  equal DDP's.

The HIP-graph capture itself needs a GPU; here ``_record`` is replaced by a
stand-in whose replay runs the same captured body eagerly, so everything
around it -- bucketing, the cache, snapshot / restore, the rank agreement,
the fallback -- is the product code.  The GPU side is
tests/test_stepgraph_gpu.py."""
import os
import socket
import sys
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _paths():
    for p in (HERE, ROOT, os.path.join(ROOT, "open-groundingdino_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)


_paths()


def _fake_graph_class():
    from gdino_amd.stepgraph import TrainStepGraph

    class FakeGraphStep(TrainStepGraph):
        """_record stand-in: the 'graph' replays the captured body eagerly."""
        fail = False

        def _record(self, c, padding_free):
            if self.fail:
                raise RuntimeError("forced capture failure (test)")
            if self.grad_sync is None:
                self.optimizer.zero_grad(set_to_none=True)

            def replay():
                loss, d = self._body(c.inputs, padding_free)
                c.loss_out.copy_(loss)
                for k, v in d.items():
                    c.dict_out[k].copy_(v)
            c.graph = types.SimpleNamespace(replay=replay)
            if self.grad_sync is None:
                c.grads = None

    return FakeGraphStep


def _model(seed=0, queries=50):
    from gdino_amd.config import make_args
    from gdino_amd.train import build_training
    torch.manual_seed(seed)
    args = make_args(device="cpu", num_queries=queries, enc_layers=2, dec_layers=2)
    model, criterion, _, opt = build_training(args, "cpu")
    model.train()
    return model, criterion, opt


def _batch(seed, h=96, w=128, n_tokens=20, n_boxes=3):
    from gdino_amd.train import synthetic_batch
    return synthetic_batch(1, h, w, n_boxes=n_boxes, n_tokens=n_tokens, seed=seed, device="cpu")


def test_text_padding_keeps_losses_and_gradients():
    from oracle_hooks import oracle_msda, scipy_lsap
    from gdino_amd.stepgraph import TrainStepGraph
    model, crit, opt = _model()
    _no_dropout(model)
    b = _batch(5, n_tokens=23)
    res = {}
    with oracle_msda(), scipy_lsap():
        for mult in (1, 64):
            g = TrainStepGraph(model, crit, opt, amp_dtype=None, text_multiple=mult)
            inputs, pf = g._prepare(*b)
            model.zero_grad(set_to_none=True)
            loss, d = g._forward_loss(inputs, pf)
            loss.backward()
            res[mult] = (inputs["input_ids"].shape[1], {k: float(v) for k, v in d.items()},
                         {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})
    (t1, d1, g1), (t64, d64, g64) = res[1], res[64]
    assert t1 == 23 and t64 == 64
    for k in d1:
        assert abs(d1[k] - d64[k]) <= 1e-5 * max(1.0, abs(d1[k])), (k, d1[k], d64[k])
    assert g1.keys() == g64.keys()
    for n in g1:
        s = float(g1[n].abs().max())
        assert float((g1[n] - g64[n]).abs().max()) <= 1e-4 * max(s, 1e-6), n


def test_image_padding_marks_the_added_pixels():
    from gdino_amd.misc import NestedTensor
    from gdino_amd.stepgraph import pad_images
    x = torch.randn(2, 3, 100, 130)
    m = torch.zeros(2, 100, 130, dtype=torch.bool)
    m[1, :, 120:] = True
    xb, mb, pf = pad_images(NestedTensor(x, m), 64)
    assert xb.shape[-2:] == (128, 192) and not pf
    assert torch.equal(xb[..., :100, :130], x) and float(xb[..., 100:, :].abs().sum()) == 0
    assert torch.equal(mb[:, :100, :130], m) and bool(mb[:, 100:].all()) and bool(mb[:, :, 130:].all())
    x2, m2, pf2 = pad_images(NestedTensor(x, m, padding_free=True), 1)
    assert x2 is x and m2 is m and pf2


def test_capture_step_equals_an_eager_step():
    """The first call captures (2 warm-up iterations, rolled back) and
    replays once: weights and AdamW state afterwards are the eager step's
    (same body, same RNG draws), with 0 and 2 warm-ups."""
    from oracle_hooks import oracle_msda, scipy_lsap
    from gdino_amd.stepgraph import TrainStepGraph
    Fake = _fake_graph_class()
    b = _batch(7)
    out = {}
    with oracle_msda(), scipy_lsap():
        for mode in ("eager", "graph", "graph0"):
            model, crit, opt = _model(seed=3)
            if mode == "eager":
                g = TrainStepGraph(model, crit, opt, amp_dtype=None, max_graphs=0, capture_after=10 ** 9)
            else:
                g = Fake(model, crit, opt, amp_dtype=None, warmup=2 if mode == "graph" else 0)
            torch.manual_seed(11)
            loss = float(g(*b))
            st = g.stats()
            params = torch.cat([p.detach().reshape(-1) for p in model.parameters() if p.requires_grad])
            mom = torch.cat([s["exp_avg"].reshape(-1) for s in opt.state.values()])
            steps = {float(s["step"]) for s in opt.state.values()}
            out[mode] = (loss, params, mom, steps, st)
    le, pe, me, se, ste = out["eager"]
    assert ste["eager_steps"] == 1 and se == {1.0}, (ste, se)
    for mode in ("graph", "graph0"):
        lg, pg, mg, sg, stg = out[mode]
        assert stg["captures"] == 1 and stg["replays"] == 1 and sg == {1.0}, (mode, stg, sg)
        _close(le, pe, me, lg, pg, mg)


def _close(le, pe, me, lg, pg, mg):
    # the CPU kernels' own run-to-run noise (parallel index_add / grid_sample
    # backward) is ~1e-9 here; a warm-up left un-rolled-back (a second AdamW
    # step, other dropout draws) moves the weights by ~1e-5
    assert abs(le - lg) <= 1e-6 * abs(le)
    assert float((pe - pg).abs().max()) <= 1e-6
    assert float((me - mg).abs().max()) <= 1e-6 * max(1e-3, float(me.abs().max()))


def test_graph_cache_buckets_and_evicts():
    """Batches of many caption lengths share the 64-token buckets; a full
    cache captures a new shape only once it was seen capture_after times
    (eager until then), evicting the least recently used graph."""
    from oracle_hooks import oracle_msda, scipy_lsap
    Fake = _fake_graph_class()
    model, crit, opt = _model(seed=1, queries=30)
    for grp in opt.param_groups:
        grp["lr"] = 0.0
    g = Fake(model, crit, opt, amp_dtype=None, warmup=1, max_graphs=2, capture_after=2)
    with oracle_msda(), scipy_lsap():
        for i, nt in enumerate((12, 30, 45, 60)):        # T bucket 64, one image size
            g(*_batch(20 + i, n_tokens=nt))
        assert g.captures == 1 and g.replays == 4
        g(*_batch(30, h=128, n_tokens=20))                # second shape: cache not full -> capture
        assert g.captures == 2
        g(*_batch(31, h=160, n_tokens=20))                # third shape, first sighting: eager
        assert g.captures == 2 and g.eager_steps == 1
        g(*_batch(32, h=160, n_tokens=70))                # T bucket 128: another shape, eager
        g(*_batch(33, h=160, n_tokens=25))                # seen twice -> capture, evicts the LRU graph
        assert g.captures == 3 and g.evictions == 1 and len(g.graphs) == 2
    assert g.mode == "graph"


# ----------------------------------------------------------- two gloo ranks
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _no_dropout(model):
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
        if hasattr(m, "drop_prob"):
            m.drop_prob = 0.0


def _rank_worker(rank, world, port, fail_rank, q):
    _paths()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle_hooks import oracle_msda, scipy_lsap
        from gdino_amd.train import BucketedGradSync
        Fake = _fake_graph_class()
        # different image sizes per rank: different graph signatures
        batches = [_batch(100 + 10 * rank + s, h=96 + 16 * rank) for s in range(2)]
        grads, modes = {}, None
        for mode in ("ddp", "graph"):
            model, crit, opt = _model(seed=0)
            _no_dropout(model)
            opt = torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=0.0)
            with oracle_msda(), scipy_lsap():
                if mode == "ddp":
                    from gdino_amd.stepgraph import TrainStepGraph
                    # DDP over the same step body (the eager TrainStepGraph step)
                    net = torch.nn.parallel.DistributedDataParallel(model)
                    g = TrainStepGraph(model, crit, opt, amp_dtype=None, clip_max_norm=0.0, max_graphs=0,
                                       capture_after=10 ** 9)
                    for b in batches:
                        inputs, pf = g._prepare(*b)
                        opt.zero_grad(set_to_none=True)
                        _ddp_loss(g, net, inputs, pf).backward()
                else:
                    sync = BucketedGradSync(model.parameters(), bucket_mb=1, first_bucket_mb=0.25)
                    g = Fake(model, crit, opt, amp_dtype=None, clip_max_norm=0.0, grad_sync=sync, warmup=1)
                    g.fail = rank == fail_rank
                    for b in batches:
                        g(*b)
                    modes = g.agree.gather(g.mode)
            grads[mode] = torch.cat([p.grad.reshape(-1) for p in model.parameters() if p.grad is not None])
        q.put((rank, float((grads["ddp"] - grads["graph"]).abs().max()), float(grads["ddp"].abs().max()),
               modes))
    finally:
        dist.destroy_process_group()


def _ddp_loss(g, net, inputs, pf):
    """the step body's forward + loss, with forward_core reached through the
    DDP wrapper (so DDP's reducer sees the backward)"""
    from gdino_amd.train import weighted_loss
    model = net.module
    model.forward = model.forward_core  # instance attribute: DDP calls module(*inputs)
    try:
        core = net(inputs["images"], inputs["mask"], inputs["input_ids"], inputs["token_type_ids"],
                   inputs["text_token_mask"], inputs["self_masks"], inputs["position_ids"])
        outputs = model.assemble_outputs(core)
        prep = {n: inputs[n] for n in ("tgt_boxes", "maps", "valid", "sizes", "num_boxes")}
        loss_dict, _ = g.criterion.loss_prepared(outputs, prep)
        return weighted_loss(loss_dict, g.criterion.weight_dict)
    finally:
        del model.forward


@pytest.mark.parametrize("fail_rank", [None, 1])
def test_two_ranks_graph_protocol_matches_ddp(fail_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, fail_rank, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=900)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted(q.get(timeout=5) for _ in range(2))
    for rank, diff, scale, modes in res:
        assert diff <= 1e-5 * max(scale, 1.0), res
        assert modes == (["graph", "graph"] if fail_rank is None else ["eager", "eager"]), res
