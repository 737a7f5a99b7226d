"""Checkpoint save / resume / partial load, as the reference's main.py does.

    save_checkpoint(path, model, optimizer, lr_scheduler, epoch, args)
        main.py:414-434: {'model', 'optimizer', 'lr_scheduler', 'epoch',
        'args'} of the unwrapped model (DDP's .module), written by rank 0 only
        (util/misc.py save_on_master).
    resume_path(output_dir, resume)
        main.py:347-348: output_dir/checkpoint.pth, when present, wins over
        --resume (auto-resume after a preemption).
    resume(path, model, optimizer, lr_scheduler, eval_only=False) -> start_epoch
        main.py:349-362: non-strict model load of the DDP-prefix-stripped state
        dict; optimizer, scheduler and epoch only when all three are present
        and not evaluating.
    load_pretrained(path, model, finetune_ignore) -> (load_result, ignored)
        main.py:364-381: --pretrain_model_path: non-strict load of
        checkpoint['model'] minus every key containing one of the
        finetune_ignore keywords (e.g. ['label_enc.weight', 'bert',
        'class_embed'] when finetuning on new labels).

Differences, both deliberate:
  * loading never unpickles code: torch.load(weights_only=True), with
    argparse.Namespace allow-listed because the reference pickles its args
    Namespace into every checkpoint (main.py:430), so reference checkpoints
    still load;
  * ``args`` is saved as a plain dict (our own checkpoints need no allow-list).
"""
from __future__ import annotations

import argparse
import os
from typing import Iterable, Optional, Sequence, Tuple

import torch

from .misc import clean_state_dict


def _unwrap(model: torch.nn.Module) -> torch.nn.Module:
    return model.module if hasattr(model, "module") else model


def _is_main() -> bool:
    import torch.distributed as dist
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


def load_checkpoint(path: str, map_location="cpu") -> dict:
    """torch.load without executing anything from the file (weights_only),
    accepting the argparse.Namespace the reference stores under 'args'.
    The reference's ``https`` branch (main.py:351-353, load_state_dict_from_url)
    is rejected explicitly: there is no egress on the training hosts, and a
    silent local-path fallback would hide a misconfigured --resume."""
    if str(path).startswith(("http://", "https://")):
        raise ValueError(f"resume from a URL is not supported (no network): {path}; download it and pass the path")
    with torch.serialization.safe_globals([argparse.Namespace]):
        return torch.load(path, map_location=map_location, weights_only=True)


def save_checkpoint(path: str, model, optimizer=None, lr_scheduler=None, epoch: Optional[int] = None,
                    args=None) -> None:
    """main.py:414-434 (rank 0 only: util/misc.py save_on_master)."""
    if not _is_main():
        return
    weights = {"model": _unwrap(model).state_dict()}
    if optimizer is not None:
        weights["optimizer"] = optimizer.state_dict()
    if lr_scheduler is not None:
        weights["lr_scheduler"] = lr_scheduler.state_dict()
    if epoch is not None:
        weights["epoch"] = int(epoch)
    if args is not None:
        weights["args"] = dict(vars(args)) if isinstance(args, argparse.Namespace) else dict(args)
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(weights, tmp)
    os.replace(tmp, path)  # a preempted save never leaves a truncated checkpoint.pth


def resume_path(output_dir: Optional[str], resume: Optional[str] = None) -> Optional[str]:
    """main.py:347-348: output_dir/checkpoint.pth overrides --resume."""
    if output_dir:
        p = os.path.join(output_dir, "checkpoint.pth")
        if os.path.exists(p):
            return p
    return resume or None


def resume(path: str, model, optimizer=None, lr_scheduler=None, eval_only: bool = False) -> int:
    """main.py:349-362 -> the epoch to start from (0 when the checkpoint has
    no training state)."""
    ck = load_checkpoint(path)
    _unwrap(model).load_state_dict(clean_state_dict(ck["model"]), strict=False)
    if (not eval_only and optimizer is not None and lr_scheduler is not None
            and all(k in ck for k in ("optimizer", "lr_scheduler", "epoch"))):
        optimizer.load_state_dict(ck["optimizer"])
        lr_scheduler.load_state_dict(ck["lr_scheduler"])
        return int(ck["epoch"]) + 1
    return 0


def filter_ignored(state_dict: dict, ignore: Optional[Iterable[str]]) -> Tuple[dict, list]:
    """main.py:368-378 check_keep: drop every key containing an ignore keyword."""
    words = list(ignore or [])
    kept, dropped = {}, []
    for k, v in state_dict.items():
        if any(w in k for w in words):
            dropped.append(k)
        else:
            kept[k] = v
    return kept, dropped


def load_pretrained(path: str, model, finetune_ignore: Optional[Sequence[str]] = None):
    """main.py:364-381 (--pretrain_model_path + finetune_ignore)."""
    ck = load_checkpoint(path)
    sd = ck["model"] if "model" in ck else ck
    kept, dropped = filter_ignored(clean_state_dict(sd), finetune_ignore)
    return _unwrap(model).load_state_dict(kept, strict=False), dropped
