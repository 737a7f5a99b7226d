"""The reference trainer's epoch loop on the fast path.

``train_one_epoch`` has the signature of the reference's
engine_multi.py:353-356 (and engine.py's upstream form) so that main.py's
call site (main.py:410) can bind it unchanged:

    from gdino_amd.engine import train_one_epoch      # instead of engine_multi's

Per batch the reference runs model(...), criterion(...), the weighted sum,
optimizer.zero_grad(), losses.backward(), clip_grad_norm_(max_norm) and
optimizer.step() as separate eager calls (engine_multi.py:499-564): 16.8
images/s on this model, a launch-bound step.  Here the same step -- same
losses, same update -- runs through gdino_amd.stepgraph.TrainStepGraph:
one HIP-graph replay per batch, with the batch's shapes bucketed (text to
64-token multiples, targets to 8 slots, the image canvas to
``args.graph_image_multiple`` pixels, default 32) and a bounded cache of
graphs; rare shapes take the identical eager step.

What changes relative to the reference loop, and why:
  * the loss is read back every ``print_freq`` steps, not every step (a
    per-step ``.item()`` waits for the whole step and stalls the queue);
    a non-finite loss still stops training (at that check, as the
    reference's sys.exit(1));
  * bf16 autocast (``args.amp``) needs no GradScaler;
  * the PAVE crop tiling of engine_multi.py:378-497 is product-specific and
    out of scope: batches are (samples, targets) or (samples, targets,
    prepared_text) from gdino_amd.data.ODVGCollator; a 3-tuple whose middle
    element is a tensor is taken as the reference's (samples, ori_samples,
    targets) and ori_samples is ignored.
  * Data parallel: pass the UNWRAPPED model and a train.BucketedGradSync
    (``grad_sync=``) -- DDP's reducer cannot follow graph replays; the
    bucketed sync does the same bucketed, backward-overlapped all-reduce
    inside the graph.  A DDP-wrapped model is accepted and runs the eager
    reference step through DDP.
"""
from __future__ import annotations

import math
import sys
import time

import torch

from .stepgraph import TrainStepGraph
from .train import train_step


def _split(batch):
    if len(batch) == 2:
        return batch[0], batch[1], None
    if len(batch) == 3 and torch.is_tensor(batch[1]):  # reference (samples, ori_samples, targets)
        return batch[0], batch[2], None
    return batch[0], batch[1], batch[2]


def _to_device(samples, targets, device):
    samples = samples.to(device, non_blocking=True)
    out = []
    for t in targets:
        d = {k: (v.to(device, non_blocking=True) if torch.is_tensor(v) else v) for k, v in t.items()}
        out.append(d)
    return samples, out


def step_graph_for(model, criterion, optimizer, max_norm, args=None, grad_sync=None, control_group=None):
    """The TrainStepGraph cached on the model for this optimizer."""
    g = getattr(model, "_gd_step_graph", None)
    if g is None or g.optimizer is not optimizer or g.criterion is not criterion:
        amp = torch.bfloat16 if getattr(args, "amp", True) else None
        g = TrainStepGraph(model, criterion, optimizer, clip_max_norm=max_norm, amp_dtype=amp,
                           grad_sync=grad_sync, control_group=control_group,
                           image_multiple=int(getattr(args, "graph_image_multiple", 32)),
                           max_graphs=int(getattr(args, "graph_cache", 4)))
        model._gd_step_graph = g
    return g


def train_one_epoch(model: torch.nn.Module, criterion: torch.nn.Module, data_loader, optimizer: torch.optim.Optimizer,
                    device: torch.device, epoch: int, max_norm: float = 0, wo_class_error=False, lr_scheduler=None,
                    args=None, logger=None, grad_sync=None, control_group=None, print_freq: int = 10):
    """Reference engine_multi.py:353-602 (train_one_epoch) on the graph
    step.  -> the epoch's averaged stats (loss, the weighted loss terms,
    lr), like the reference's ``resstat``."""
    model.train()
    criterion.train()
    ddp = isinstance(model, torch.nn.parallel.DistributedDataParallel)
    g = None if ddp else step_graph_for(model, criterion, optimizer, max_norm, args, grad_sync, control_group)
    sums, n, pending, t0 = {}, 0, [], time.time()
    header = f"Epoch: [{epoch}]"
    out = sys.stdout if logger is None else None

    def flush(i):
        nonlocal pending
        for loss, terms in pending:
            v = float(loss)
            if not math.isfinite(v):
                print(f"Loss is {v}, stopping training", file=sys.stderr)
                print({k: float(x) for k, x in terms.items()} if terms else {}, file=sys.stderr)
                sys.exit(1)
            sums["loss"] = sums.get("loss", 0.0) + v
            for k, x in (terms or {}).items():
                if k in criterion.weight_dict:
                    sums[k] = sums.get(k, 0.0) + float(x) * criterion.weight_dict[k]
        pending = []
        msg = (f"{header} [{i}] loss: {sums.get('loss', 0.0) / max(n, 1):.4f} "
               f"lr: {float(optimizer.param_groups[0]['lr']):.6f} ({(time.time() - t0) / max(n, 1):.3f} s/it)")
        if logger is not None:
            logger.info(msg)
        elif out is not None:
            print(msg, file=out, flush=True)

    for i, batch in enumerate(data_loader):
        samples, targets, prepared = _split(batch)
        captions = [t["caption"] for t in targets]
        cap_list = [t["cap_list"] for t in targets]
        samples, targets = _to_device(samples, targets, device)
        if g is None:
            amp = torch.bfloat16 if getattr(args, "amp", True) else None
            loss = train_step(model, criterion, optimizer, samples, targets, captions, cap_list,
                              clip_max_norm=max_norm, amp_dtype=amp)
            terms = None
        else:
            loss = g(samples, targets, captions, cap_list, prepared_text=prepared)
            terms = g.loss_dict()
            terms = {k: v.clone() for k, v in terms.items()} if terms is not None else None
        pending.append((loss.clone(), terms))
        n += 1
        if args is not None and getattr(args, "onecyclelr", False) and lr_scheduler is not None:
            lr_scheduler.step()
        if (i + 1) % print_freq == 0:
            flush(i + 1)
        if args is not None and getattr(args, "debug", False) and (i + 1) % 15 == 0:
            break
    flush(n)
    if getattr(criterion, "loss_weight_decay", False):
        criterion.loss_weight_decay(epoch=epoch)
    if getattr(criterion, "tuning_matching", False):
        criterion.tuning_matching(epoch)
    stats = {k: v / max(n, 1) for k, v in sums.items()}
    stats["lr"] = float(optimizer.param_groups[0]["lr"])
    if g is not None:
        stats["step_graph"] = g.stats()
    return stats
