"""The whole Grounding DINO train step as ONE HIP graph.

Round 3 captured forward_core and its backward (gdino_amd.graphs) and ran the
criterion and the optimizer eagerly between the replays.  The criterion's
Hungarian matching needed the host (one device->host copy, a host wait for
the forward, scipy, then the post-matching loss launches), so every step
serialised there, and the eager launches between the replays left the
device idle about 13 ms per step.  With the matching on the device
(gdino_amd.lsap, scipy's algorithm) nothing in the step needs the host, so
the step is captured whole and replayed with one launch:

    forward_core -> SetCriterion.loss_prepared (cost matrices, device LSA,
    token focal / L1 / GIoU) -> weighted sum -> backward (+ the bucketed
    RCCL gradient all-reduce overlapped with it, train.BucketedGradSync, for
    N > 1) -> clip_grad_norm_ -> fused AdamW (capturable, lr as a device
    tensor so the LR scheduler still acts on replays).

The host side per step is the text tokenisation and the target packing
(SetCriterion.prepare_targets: positive maps, padded targets), both copied
asynchronously into the graph's static input buffers.  A graph is captured
per batch signature (image size, text length, padded target count); the
target count is padded to a multiple of ``kmax_multiple`` so batches with
different numbers of boxes share a graph (the padded pair slots are masked
exactly in loss_prepared).

Reference: the step engine_multi.py:499-564 / main.py:254-292 run eagerly.
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

import torch

from . import _lib, castcache
from .misc import no_padding
from .train import BucketedGradSync, weighted_loss

_VERBOSE = os.environ.get("GDINO_STEPGRAPH_VERBOSE") == "1"


def _log(msg):
    if _VERBOSE:
        print(f"[stepgraph {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


# Process-group settings for collectives inside a captured graph, to be in
# the environment before init_process_group (bench.setup_dist sets them when
# the step graph runs with N > 1):
#  * no CUDA-event cache: ProcessGroupNCCL recycles its work events, and its
#    watchdog thread querying an event whose last record was made inside a
#    capture fails with hipErrorCapturedEvent and terminates the process
#    (seen on a 1-rank RCCL group, tests/test_stepgraph_gpu.py);
#  * no async error handling (the watchdog's abort path), as PyTorch's CUDA
#    graph notes prescribe for captured collectives.
RCCL_CAPTURE_ENV = {"TORCH_NCCL_CUDA_EVENT_CACHE": "0", "TORCH_NCCL_ASYNC_ERROR_HANDLING": "0"}


def _static_like(t: torch.Tensor) -> torch.Tensor:
    return torch.empty_like(t, memory_format=torch.contiguous_format)


_lib.register("gd_graph_memsets_to_kernels", [ctypes.c_void_p])


def memsets_to_kernels(graph: "torch.cuda.CUDAGraph") -> int:
    """Replace every memset node of a captured (keep_graph=True, not yet
    instantiated) graph by a fill-kernel node (csrc/graph.hip): on ROCm 7.0
    a replay's memset nodes stop taking effect once eager device-to-device
    copies ran between replays (tools/graph_node_order_probe.py), and
    PyTorch's multi-block reductions zero their semaphores with one -- the
    train-step graph then returned wrong bias gradients after a host-side
    gradient copy (tools/stepgraph_diag.py --flows).  -> nodes replaced."""
    fn = _lib.lib().gd_graph_memsets_to_kernels
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p]
    n = int(fn(ctypes.c_void_p(graph.raw_cuda_graph())))
    if n < 0:
        raise RuntimeError("gd_graph_memsets_to_kernels: a memset node of the captured graph is not expressible "
                           "as a fill kernel")
    return n


class _Captured:
    def __init__(self):
        # kept un-instantiated after capture: its memset nodes are rewritten
        # (memsets_to_kernels) before the first replay
        self.graph = torch.cuda.CUDAGraph(keep_graph=True)
        self.memsets_replaced = 0
        self.inputs = {}
        self.loss = None
        self.loss_dict = None

    def load(self, inputs):
        for k, v in inputs.items():
            self.inputs[k].copy_(v, non_blocking=True)


class TrainStepGraph:
    """Callable like train.train_step(samples, targets, captions, cat_lists)
    -> loss tensor, replaying a captured whole-step graph.

    ``warmup`` eager iterations (full optimizer steps, on a side stream)
    precede each capture: they initialise the library handles, the weight
    shadows / cast caches, the criterion's index caches and, for N > 1, the
    gradient buckets."""

    def __init__(self, model, criterion, optimizer, clip_max_norm: float = 0.1, amp_dtype=torch.bfloat16,
                 grad_sync: BucketedGradSync | None = None, warmup: int = 2, kmax_multiple: int = 8):
        self.model, self.criterion, self.optimizer = model, criterion, optimizer
        self.clip_max_norm, self.amp_dtype = clip_max_norm, amp_dtype
        self.grad_sync, self.warmup, self.kmax_multiple = grad_sync, warmup, kmax_multiple
        self.graphs = {}
        self.captures = 0
        # After each replay the host waits for the whole device
        # (hipDeviceSynchronize) before it enqueues the next step's input
        # copies: with the next step's copies and replay enqueued behind a
        # running replay -- unbounded, or bounded by an event recorded after
        # the launch -- the box faulted (illegal address) within the first
        # replays; with a device-wide sync after every replay it ran clean
        # (DESIGN §7).  The host's preparation of a step (~2 ms) is then not
        # hidden.  GDINO_STEPGRAPH_SYNC=event: the event-bounded variant.
        self.sync_mode = os.environ.get("GDINO_STEPGRAPH_SYNC", "device")
        self.max_inflight = 1
        self._inflight = []
        device = next(model.parameters()).device
        for g in optimizer.param_groups:  # capturable fused AdamW; lr a device tensor the scheduler fills
            g["capturable"] = True
            if not torch.is_tensor(g["lr"]):
                g["lr"] = torch.tensor(float(g["lr"]), dtype=torch.float32, device=device)

    # ------------------------------------------------------------ inputs
    def _prepare(self, samples, targets, captions, cat_lists):
        model = self.model
        device = samples.tensors.device
        text, token = model.prepare_text(captions, device)
        k = max(max((len(t["labels"]) for t in targets), default=0), 1)
        k = -(-k // self.kmax_multiple) * self.kmax_multiple
        prep = self.criterion.prepare_targets(targets, cat_lists, captions, token, device, kmax=k)
        inputs = {"images": samples.tensors, "mask": samples.mask}
        for n in ("input_ids", "token_type_ids", "text_token_mask", "self_masks", "position_ids"):
            inputs[n] = text[n]
        for n in ("tgt_boxes", "maps", "valid", "sizes", "num_boxes"):
            inputs[n] = prep[n]
        return inputs

    @staticmethod
    def _signature(inputs):
        return tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(inputs.items()))

    # -------------------------------------------------------------- step
    def _body(self, inp, padding_free=False):
        """forward + loss + backward + all-reduce + clip + optimizer step;
        only device work, no host synchronisation.  ``padding_free``: the
        batch's image mask is all False (part of the graph's signature)."""
        model, crit = self.model, self.criterion
        dev_type = inp["images"].device.type
        with torch.autocast(device_type=dev_type, dtype=self.amp_dtype, enabled=self.amp_dtype is not None), \
                no_padding(padding_free):
            core = model.forward_core(inp["images"], inp["mask"], inp["input_ids"], inp["token_type_ids"],
                                      inp["text_token_mask"], inp["self_masks"], inp["position_ids"])
            outputs = model.assemble_outputs(core)
            prep = {n: inp[n] for n in ("tgt_boxes", "maps", "valid", "sizes", "num_boxes")}
            loss_dict, _ = crit.loss_prepared(outputs, prep)
            loss = weighted_loss(loss_dict, crit.weight_dict)
        if self.grad_sync is not None:
            self.grad_sync.zero_grad()
        loss.backward()
        if self.grad_sync is not None:
            self.grad_sync.after_backward()
        if self.clip_max_norm > 0:
            torch.nn.utils.clip_grad_norm_(model.parameters(), self.clip_max_norm, foreach=True)
        self.optimizer.step()
        return loss.detach(), {k: v.detach() for k, v in loss_dict.items()}

    def _capture(self, key, inputs, padding_free=False):
        c = _Captured()
        for k, v in inputs.items():
            c.inputs[k] = _static_like(v)
        c.load(inputs)
        # warm-up and capture on ONE side stream: the autograd engine runs a
        # parameter's AccumulateGrad on the stream the node was created on
        # (its first forward use); an AccumulateGrad node created on another
        # stream and kept alive (e.g. by a cached weight cast's grad_fn) makes
        # the captured backward synchronise with that stream, which HIP
        # refuses during capture (hipErrorStreamCaptureUnsupported)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        castcache.drop_autograd_refs()
        with torch.cuda.stream(side):
            for i in range(self.warmup):
                if self.grad_sync is None:
                    self.optimizer.zero_grad(set_to_none=True)
                self._body(c.inputs, padding_free)
                if _VERBOSE:
                    side.synchronize()
                    _log(f"warm-up step {i} done")
        castcache.drop_autograd_refs()
        side.synchronize()
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            # ProcessGroupNCCL's watchdog thread polls the warm-up's
            # collectives (about every 100 ms) by querying their end events,
            # recorded on the communication stream; once the capture forks
            # that stream, HIP refuses the query (hipErrorCapturedEvent) and
            # the watchdog terminates the process.  Let it retire them first.
            import time
            torch.cuda.synchronize()
            time.sleep(1.0)
        if self.grad_sync is None:
            # the captured backward allocates the gradients from the graph's
            # pool; every replay rewrites them in place
            self.optimizer.zero_grad(set_to_none=True)
        # (a private memory pool per graph: a shared one would let a later
        # capture reuse memory an earlier graph's replays still write)
        _log("capture begins")
        with torch.cuda.graph(c.graph, stream=side):
            c.loss, c.loss_dict = self._body(c.inputs, padding_free)
        torch.cuda.current_stream().wait_stream(side)
        c.memsets_replaced = memsets_to_kernels(c.graph)
        c.graph.instantiate()
        _log(f"memset nodes replaced by fill kernels: {c.memsets_replaced}")
        _log(f"captured ({c.graph.__class__.__name__})")
        self.graphs[key] = c
        self.captures += 1
        return c

    def __call__(self, samples, targets, captions, cat_lists):
        # the previous replay finishes before this step enqueues anything
        # (its input copies included): see max_inflight
        while len(self._inflight) >= self.max_inflight:
            self._inflight.pop(0).synchronize()
        inputs = self._prepare(samples, targets, captions, cat_lists)
        pf = bool(getattr(samples, "padding_free", False))
        key = self._signature(inputs) + (("padding_free", pf),)
        c = self.graphs.get(key)
        if c is None:
            c = self._capture(key, inputs, pf)
        else:
            c.load(inputs)
        c.graph.replay()
        if self.sync_mode == "device":
            torch.cuda.synchronize()
        else:
            ev = torch.cuda.Event()
            ev.record()
            self._inflight.append(ev)
        castcache._on_optimizer_step()  # the replay stepped the optimizer: cast copies are stale
        if _VERBOSE:
            torch.cuda.synchronize()
            _log(f"replay done, loss {float(c.loss):.4f}")
        return c.loss

    def release(self):
        for ev in self._inflight:
            ev.synchronize()
        self._inflight.clear()
        self.graphs.clear()
