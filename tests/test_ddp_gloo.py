"""Data-parallel path on CPU: world_size-2 gloo, the full model wrapped in
DDP exactly as bench.py / the reference main.py do (main.py:258-261), each
rank a different synthetic batch, three bf16-autocast train steps.  Checks that the gradient all-reduce makes
every rank's gradients and post-step parameters identical, and that the
criterion's num_boxes all-reduce (groundingdino.py:574-576) runs."""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "open-groundingdino_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle_hooks import oracle_msda
        from gdino_amd.config import make_args
        from gdino_amd.train import build_training, synthetic_batch, train_step
        torch.manual_seed(0)  # identical init on every rank (DDP also broadcasts)
        args = make_args(device="cpu", num_queries=50, enc_layers=2, dec_layers=2)
        model, criterion, _, opt = build_training(args, "cpu")
        ddp = torch.nn.parallel.DistributedDataParallel(model, static_graph=True)
        samples, targets, caps, cats = synthetic_batch(1, 96, 128, n_boxes=2, n_tokens=20, seed=100 + rank,
                                                       device="cpu")
        with oracle_msda():
            # bf16 autocast as in bench.py: exercises the cast cache, the fused
            # projections and the packed in-projection under DDP; three steps
            # so static_graph's recorded plan and the per-step cache refresh
            # (optimizer updates bump parameter versions) are both used
            for _ in range(3):
                loss = train_step(ddp, criterion, opt, samples, targets, caps, cats, amp_dtype=torch.bfloat16)
        grads = torch.cat([p.grad.reshape(-1) for p in model.parameters() if p.grad is not None])
        params = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        ref_g, ref_p = grads.clone(), params.clone()
        dist.broadcast(ref_g, 0)
        dist.broadcast(ref_p, 0)
        q.put((rank, float(loss), bool(torch.allclose(grads, ref_g)), bool(torch.equal(params, ref_p)),
               float(grads.abs().sum())))
    finally:
        dist.destroy_process_group()


def test_ddp_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs)
    (r0, l0, g0, p0, s0), (r1, l1, g1, p1, s1) = res
    assert g0 and g1, "gradients differ across ranks after DDP all-reduce"
    assert p0 and p1, "parameters differ across ranks after the optimizer step"
    assert l0 != l1, "ranks should have seen different batches"
    assert s0 > 0


def _worker_grad_allreduce(rank, world, port, q):
    """GradAllReduce (post-backward) and BucketedGradSync (overlapped with
    the backward: per-bucket all-reduces issued from post-accumulate hooks,
    gradients as views of the bucket buffers -- the multi-GPU HIP-graph
    step's gradient averaging) against DDP on the same model, batches and
    seeds: identical gradients (DDP also averages over ranks), small buckets
    so the bucket boundaries are exercised.  Two steps each (lr 0): the
    first backward records the bucket order, the second runs overlapped."""
    sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "open-groundingdino_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle_hooks import oracle_msda
        from gdino_amd.config import make_args
        from gdino_amd.train import BucketedGradSync, GradAllReduce, build_training, synthetic_batch, train_step
        args = make_args(device="cpu", num_queries=50, enc_layers=2, dec_layers=2)
        samples, targets, caps, cats = synthetic_batch(1, 96, 128, n_boxes=2, n_tokens=20, seed=200 + rank,
                                                       device="cpu")
        grads = {}
        nb = 0
        for mode in ("ddp", "manual", "bucketed"):
            torch.manual_seed(0)
            model, criterion, _, opt = build_training(args, "cpu")
            for m in model.modules():  # the same function in both runs
                if isinstance(m, torch.nn.Dropout):
                    m.p = 0.0
                if hasattr(m, "drop_prob"):
                    m.drop_prob = 0.0
            opt = torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=0.0)
            if mode == "ddp":
                net, sync = torch.nn.parallel.DistributedDataParallel(model), None
            elif mode == "manual":
                net, sync = model, GradAllReduce(model.parameters(), bucket_mb=1)
            else:
                net, sync = model, BucketedGradSync(model.parameters(), bucket_mb=1, first_bucket_mb=0.25)
            with oracle_msda():
                for _ in range(2):
                    train_step(net, criterion, opt, samples, targets, caps, cats, amp_dtype=None,
                               clip_max_norm=0.0, grad_sync=sync)
            grads[mode] = torch.cat([p.grad.reshape(-1) for p in model.parameters() if p.grad is not None])
            if mode == "bucketed":
                nb = len(sync.buckets)
                # every gradient lives in a bucket buffer (no flatten copies)
                assert all(any(p.grad.data_ptr() >= b["flat"].data_ptr() and
                               p.grad.data_ptr() < b["flat"].data_ptr() + b["flat"].numel() * 4
                               for b in sync.buckets) for p in model.parameters() if p.grad is not None)
        q.put((rank, max(float((grads["ddp"] - grads[m]).abs().max()) for m in ("manual", "bucketed")),
               float(grads["ddp"].abs().max()), nb))
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_matches_ddp_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_grad_allreduce, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs)
    for _, diff, scale, nb in res:
        assert diff <= 1e-6 * max(scale, 1.0), res
        assert nb > 3, res  # several buckets: boundaries exercised
