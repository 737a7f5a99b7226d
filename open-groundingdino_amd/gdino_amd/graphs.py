"""HIP-graph capture of the Grounding DINO forward and backward.

The eager train step issues ~10k kernels per step (thousands of small
elementwise ops around the GEMMs, MSDA and attention kernels); at ~5-10 us
of host work per launch the GPU idles ~40 % of the step.  On MI355X the
launch path is the bottleneck, so the tensor-only body of the model
(``GroundingDINO.forward_core``: BERT, Swin, input projections, encoder with
fusion + text enhancer, two-stage selection, decoder, heads) is captured once
into one HIP graph for the forward and one for the backward
(torch.cuda.make_graphed_callables over ROCm's hipGraph) and replayed every
step.  Tokenization, the criterion (its Hungarian matching needs the
host) and the optimizer stay eager around the replays.

Requirements the model meets for capture: static shapes for a fixed batch
geometry, no host synchronisation inside forward_core, every device constant
(Swin shift masks, level shapes) created before capture (the warm-up
iterations do it), and the HIP kernels launched on the current stream.
"""
from __future__ import annotations

import os
from typing import Sequence

import torch
from torch import nn


class _Core(nn.Module):
    """nn.Module view of model.forward_core so that make_graphed_callables
    treats the model's parameters as graph inputs (their grads come out of
    the backward graph)."""

    def __init__(self, model):
        super().__init__()
        self.model = model
        self._none_mask = None

    def forward(self, *args):
        outs = self.model.forward_core(*args)
        self._none_mask = tuple(o is None for o in outs)
        return tuple(o for o in outs if o is not None)


def capture(model, sample_inputs: Sequence[torch.Tensor], amp_dtype=torch.bfloat16, warmup: int = 3):
    """Capture model.forward_core(*sample_inputs) (train mode).  Afterwards
    model.forward routes through the graphed callable; inputs are copied into
    the graph's static input buffers on every call, so any batch with the
    same shapes can be fed."""
    core = _Core(model)
    with torch.autocast(device_type="cuda", dtype=amp_dtype, enabled=amp_dtype is not None,
                        cache_enabled=False):
        graphed = torch.cuda.make_graphed_callables(core, tuple(sample_inputs), num_warmup_iters=warmup)
    none_mask = core._none_mask

    debug = os.environ.get("GDINO_GRAPH_DEBUG") == "1"

    def call(*args):
        if debug:
            torch.cuda.synchronize()
            print("graphs: pre-replay sync ok", flush=True)
        res = graphed(*args)
        if debug:
            torch.cuda.synchronize()
            print("graphs: replay sync ok", flush=True)
        outs = iter(res)
        return tuple(None if is_none else next(outs) for is_none in none_mask)

    model._graphed_core = call
    return call


def release(model) -> None:
    model._graphed_core = None
