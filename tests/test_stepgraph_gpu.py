"""The whole train step as one HIP graph (gdino_amd.stepgraph.TrainStepGraph)
against the eager train step (train.train_step) on the GPU: same model,
weights and batches; after the same number of optimizer steps the losses
and parameters agree (the only differences are float-atomic summation
orders of the decoder MSDA backward and index_add, ~1e-7 relative).  Also:
a second batch with other target counts replays the same graph (padded
target slots), the LR scheduler acts on replays (lr is a device tensor),
and the gradient all-reduce is captured (1-rank RCCL group)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(seed=0):
    from gdino_amd.config import make_args
    from gdino_amd.train import build_training
    torch.manual_seed(seed)
    args = make_args(device=DEV, enc_layers=2, dec_layers=2, num_queries=300)
    model, criterion, _, opt = build_training(args, torch.device(DEV))
    for m in model.modules():  # the same function in both runs (dropout draws differ)
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
        if hasattr(m, "drop_prob"):
            m.drop_prob = 0.0
    model.train()
    return model, criterion, opt


def _batch(seed, n_boxes):
    from gdino_amd.train import synthetic_batch
    return synthetic_batch(2, 320, 384, n_boxes=n_boxes, n_tokens=40, seed=seed, device=DEV)


def _params(model):
    return torch.cat([p.detach().reshape(-1).float() for p in model.parameters() if p.requires_grad])


def _run(grad_sync_factory=None):
    from gdino_amd.stepgraph import TrainStepGraph
    from gdino_amd.train import train_step
    b1, b2 = _batch(11, 5), _batch(12, 3)
    losses = {}
    finals = {}
    for mode in ("eager", "graph"):
        model, crit, opt = _model()
        sync = grad_sync_factory(model) if grad_sync_factory else None
        sched = torch.optim.lr_scheduler.StepLR(opt, 1, gamma=0.5)
        ls = []
        if mode == "eager":
            for _ in range(3):  # = the graph's 2 warm-up steps + its first replay
                ls.append(float(train_step(model, crit, opt, *b1, grad_sync=sync)))
            sched.step()
            ls.append(float(train_step(model, crit, opt, *b2, grad_sync=sync)))
        else:
            g = TrainStepGraph(model, crit, opt, grad_sync=sync, warmup=2)
            ls.append(float(g(*b1)))
            sched.step()  # fills the device lr tensors: acts on the replay
            ls.append(float(g(*b2)))
            assert g.captures == 1, "5 and 3 targets pad to the same 8-slot graph"
        torch.cuda.synchronize()
        losses[mode] = ls
        finals[mode] = _params(model)
    return losses, finals


def _check(losses, finals):
    le, lg = losses["eager"], losses["graph"]
    assert abs(le[2] - lg[0]) <= 1e-4 * abs(le[2]), (le, lg)
    assert abs(le[3] - lg[1]) <= 1e-4 * abs(le[3]), (le, lg)
    d = (finals["eager"] - finals["graph"]).abs().max()
    moved = (finals["eager"] - _params(_model()[0])).abs().max()
    assert moved > 0
    assert float(d) <= 1e-3 * float(moved), (float(d), float(moved))


def test_step_graph_matches_eager_steps():
    _check(*_run())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_step_graph_captures_the_bucketed_allreduce():
    """BucketedGradSync inside the captured step on a 1-rank RCCL group: the
    per-bucket all-reduces are graph nodes (a 1-rank sum is the identity, so
    the result must equal the eager steps)."""
    import torch.distributed as dist
    from gdino_amd.train import BucketedGradSync
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV, 0))
    try:
        losses, finals = _run(lambda m: BucketedGradSync(m.parameters(), bucket_mb=4, first_bucket_mb=1))
    finally:
        dist.destroy_process_group()
    _check(losses, finals)
