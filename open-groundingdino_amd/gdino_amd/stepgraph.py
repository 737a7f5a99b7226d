"""The whole Grounding DINO train step as ONE HIP graph, for real batches.

With the Hungarian matching on the device (gdino_amd.lsap, scipy's
algorithm) nothing in the step needs the host, so the step is captured whole
and replayed with one launch:

    forward_core -> SetCriterion.loss_prepared (cost matrices, device LSA,
    token focal / L1 / GIoU) -> weighted sum -> backward (+ the bucketed
    RCCL gradient all-reduce overlapped with it, train.BucketedGradSync, for
    N > 1) -> clip_grad_norm_ -> fused AdamW (capturable, lr as a device
    tensor so the LR scheduler still acts on replays).

The host side per step is the text tokenisation and the target packing
(SetCriterion.prepare_targets: positive maps, padded targets), both copied
asynchronously into the graph's static input buffers.

Real batches (odvg: captions of every length, multi-scale images, any
number of boxes) vary in shape, and a graph replays one shape.  So:

  * shapes are bucketed: the text is padded to a multiple of
    ``text_multiple`` tokens (pad tokens are masked everywhere -- BERT's
    phrase masks, BiAttention, the contrastive head -- so the real tokens'
    results do not change), the target count to a multiple of
    ``kmax_multiple`` (padded pair slots are masked exactly in
    loss_prepared) and, when ``image_multiple`` > 1, the image canvas to a
    multiple of it (the padding mask covers the added pixels, as the
    reference's NestedTensor batching does for its batch maximum);
  * graphs live in a bounded LRU cache (``max_graphs``) and share ONE memory
    pool, so memory does not grow with the number of shapes seen; a shape
    that would evict a graph is captured only once it has been seen
    ``capture_after`` times, and runs the same step eagerly until then;
  * each capture is preceded by ``warmup`` eager iterations (library
    handles, weight shadows, the criterion's caches) whose effect on the
    weights, the optimizer state and the RNG is rolled back, so a batch is
    applied exactly once whether it captured a graph or not; the warm-ups
    issue no collective (misc.local_only), so a capture on one rank never
    adds collectives the other ranks do not issue (the captured collectives
    only run at replay);
  * N > 1: the ranks agree, on the host, whether anyone captures this step
    and whether every capture succeeded; if one failed, EVERY rank drops
    its graphs and runs the eager step from then on (same collectives,
    same order: BucketedGradSync launches buckets in index order in both
    modes).  ``control_group`` (a gloo group) carries these agreements
    without a device synchronisation; its timeout bounds every wait.

Reference: the step engine_multi.py:499-564 / main.py:254-292 run eagerly;
gdino_amd.engine.train_one_epoch is the drop-in that runs it through here.
"""
from __future__ import annotations

import collections
import contextlib
import ctypes
import os
import sys
import time

import torch
import torch.distributed as dist

from . import _lib, castcache
from .misc import bump_mask_epoch, local_only, no_padding
from .train import BucketedGradSync, weighted_loss

_VERBOSE = os.environ.get("GDINO_STEPGRAPH_VERBOSE") == "1"
# A/B knobs: the capture's error mode and the cache's shared memory pool
_CAPTURE_MODE = os.environ.get("GDINO_CAPTURE_MODE", "thread_local")
_SHARED_POOL = os.environ.get("GDINO_GRAPH_POOL", "shared") == "shared"


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
_lib.register("gd_stream_abort_capture", [ctypes.c_void_p])


def memsets_to_kernels(graph: "torch.cuda.CUDAGraph") -> int:
    """Replace every memset node of a captured (keep_graph=True, not yet
    instantiated) graph by a fill-kernel node (csrc/graph.hip): on ROCm 7.0
    a replay's memset nodes stop taking effect once eager device-to-device
    copies ran between replays, and PyTorch's multi-block
    reductions zero their semaphores with one.  The library validates every
    node before it edits any.  -> nodes replaced."""
    fn = _lib.lib().gd_graph_memsets_to_kernels
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p]
    n = int(fn(ctypes.c_void_p(graph.raw_cuda_graph())))
    if n < 0:
        raise RuntimeError("gd_graph_memsets_to_kernels: a memset node of the captured graph is not expressible "
                           "as a fill kernel (the graph was left unchanged)")
    return n


# ----------------------------------------------------------- rank agreement
def make_control_group(timeout_s: float = 600.0):
    """A gloo group over the default group's ranks for the step graph's host
    agreements (collective: every rank calls it).  None when not
    distributed."""
    import datetime
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return None
    return dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))


class Agreement:
    """Host-side agreement among the ranks of a data-parallel job: any /
    all of a per-rank flag, and a gather of small objects.  With one rank
    (or no process group) the rank's own value."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank() if self.world > 1 else 0

    def _dev(self):
        be = dist.get_backend(self.group)
        return torch.device("cuda", torch.cuda.current_device()) if be == "nccl" else torch.device("cpu")

    def _reduce(self, flag: bool, op) -> bool:
        if self.world == 1:
            return bool(flag)
        t = torch.tensor([int(bool(flag))], dtype=torch.int32, device=self._dev())
        dist.all_reduce(t, op=op, group=self.group)
        return bool(int(t.item()))

    def any(self, flag: bool) -> bool:
        return self._reduce(flag, dist.ReduceOp.MAX)

    def all(self, flag: bool) -> bool:
        return self._reduce(flag, dist.ReduceOp.MIN)

    def gather(self, obj) -> list:
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.group)
        return out


# ------------------------------------------------------------- the graphs
class _Captured:
    def __init__(self):
        self.graph = None          # torch.cuda.CUDAGraph (or a test's stand-in with .replay())
        self.memsets_replaced = 0
        self.inputs = {}           # static input buffers (outside the graph pool)
        self.loss_out = None       # outputs copied here inside the graph (outside the pool: a
        self.dict_out = None       # later graph of the shared pool may reuse the body's memory)
        self.grads = None          # grad_sync None: the gradients the capture allocated
        self.fresh = False         # inputs already loaded (the capture loaded them)

    def load(self, inputs):
        for k, v in inputs.items():
            self.inputs[k].copy_(v, non_blocking=True)


def pad_images(samples, multiple: int):
    """(images, mask, padding_free) with the canvas padded to a multiple of
    ``multiple`` pixels on each side; the added pixels are padding (mask
    True), as NestedTensor batching pads to the batch maximum
    (reference util/misc.py:285-397)."""
    x, m = samples.tensors, samples.mask
    pf = bool(getattr(samples, "padding_free", False))
    if multiple <= 1:
        return x, m, pf
    H, W = x.shape[-2:]
    Hb, Wb = -(-H // multiple) * multiple, -(-W // multiple) * multiple
    if (Hb, Wb) == (H, W):
        return x, m, pf
    xb = x.new_zeros(x.shape[:-2] + (Hb, Wb))
    xb[..., :H, :W] = x
    mb = torch.ones(x.shape[0], Hb, Wb, dtype=torch.bool, device=x.device)
    mb[:, :H, :W] = m if m is not None else False
    return xb, mb, False


class TrainStepGraph:
    """Callable like train.train_step(samples, targets, captions, cat_lists)
    -> loss tensor (the weighted total; not synchronised).  See the module
    docstring for the bucketing, the graph cache and the rank protocol.

    ``mode``: "graph", or "eager" once a capture failed on any rank.
    ``stats()``: captures / replays / eager steps / evictions."""

    def __init__(self, model, criterion, optimizer, clip_max_norm: float = 0.1, amp_dtype=torch.bfloat16,
                 grad_sync: BucketedGradSync | None = None, warmup: int = 2, kmax_multiple: int = 8,
                 text_multiple: int = 64, image_multiple: int = 1, max_graphs: int = 4, capture_after: int = 2,
                 control_group=None, sync_mode: str | None = None):
        self.model, self.criterion, self.optimizer = model, criterion, optimizer
        self.clip_max_norm, self.amp_dtype = clip_max_norm, amp_dtype
        self.grad_sync, self.warmup, self.kmax_multiple = grad_sync, warmup, kmax_multiple
        self.text_multiple, self.image_multiple = text_multiple, image_multiple
        self.max_graphs, self.capture_after = max_graphs, capture_after
        self.graphs = collections.OrderedDict()   # key -> _Captured, least recently used first
        self.seen = collections.Counter()
        self.captures = self.replays = self.eager_steps = self.evictions = 0
        self.mode = "graph"
        self.fallback_reason = None
        self.last_terms = None
        self.agree = Agreement(control_group)
        self.device = next(model.parameters()).device
        self.on_gpu = self.device.type == "cuda"
        self.pool = None    # one graph memory pool shared by every graph of the cache
        self.side = None    # the stream of the plan, the warm-ups and the captures
        self._grads_of = None
        # After each replay the host records an event and, before the next
        # step's replay, waits for it (one step in flight: the host's
        # preparation of step i+1 -- tokenisation, target packing -- overlaps
        # replay i).  GDINO_STEPGRAPH_SYNC=device: a device-wide
        # synchronisation after every replay instead (round 4's default,
        # kept for A/B).
        self.sync_mode = sync_mode or os.environ.get("GDINO_STEPGRAPH_SYNC", "event")
        self.max_inflight = 1
        self._inflight = []
        if self.on_gpu:
            for g in getattr(optimizer, "param_groups", []):  # capturable fused AdamW; lr a device tensor
                g["capturable"] = True
                if not torch.is_tensor(g["lr"]):
                    g["lr"] = torch.tensor(float(g["lr"]), dtype=torch.float32, device=self.device)

    def stats(self):
        return {"mode": self.mode, "captures": self.captures, "replays": self.replays,
                "eager_steps": self.eager_steps, "evictions": self.evictions, "graphs": len(self.graphs),
                "fallback_reason": self.fallback_reason}

    # ------------------------------------------------------------ inputs
    def _prepare(self, samples, targets, captions, cat_lists, prepared_text=None):
        """-> (static-shape input dict on the device, padding_free).
        ``prepared_text``: prepare_text_host's result made in a DataLoader
        worker (gdino_amd.data.ODVGCollator), else tokenised here."""
        model = self.model
        images, mask, pf = pad_images(samples, self.image_multiple)
        device = images.device
        text, token = model.prepare_text(captions, device, prepared=prepared_text, pad_multiple=self.text_multiple)
        k = max(max((len(t["labels"]) for t in targets), default=0), 1)
        k = -(-k // self.kmax_multiple) * self.kmax_multiple
        prep = self.criterion.prepare_targets(targets, cat_lists, captions, token, device, kmax=k)
        inputs = {"images": images, "mask": mask}
        for n in ("input_ids", "token_type_ids", "text_token_mask", "self_masks", "position_ids"):
            inputs[n] = text[n]
        for n in ("tgt_boxes", "maps", "valid", "sizes", "num_boxes"):
            inputs[n] = prep[n]
        return inputs, pf

    @staticmethod
    def _signature(inputs):
        return tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(inputs.items()))

    # -------------------------------------------------------------- step
    def _forward_loss(self, inp, padding_free=False):
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
        return loss, loss_dict

    def _body(self, inp, padding_free=False):
        """forward + loss + backward + all-reduce + clip + optimizer step;
        only device work, no host synchronisation (the captured region)."""
        loss, loss_dict = self._forward_loss(inp, padding_free)
        if self.grad_sync is not None:
            self.grad_sync.zero_grad()
        loss.backward()
        if self.grad_sync is not None:
            self.grad_sync.after_backward()
        if self.clip_max_norm > 0:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.clip_max_norm, foreach=True)
        self.optimizer.step()
        return loss.detach(), {k: v.detach() for k, v in loss_dict.items()}

    def _stream_ctx(self):
        if not self.on_gpu:
            return contextlib.nullcontext()
        if self.side is None:
            self.side = torch.cuda.Stream()
        self.side.wait_stream(torch.cuda.current_stream())
        return torch.cuda.stream(self.side)

    def _side_done(self):
        if self.on_gpu:
            torch.cuda.current_stream().wait_stream(self.side)
            self.side.synchronize()

    def _plan(self, inp, pf):
        """N > 1, first step: the gradient buckets from one recording
        backward (no optimizer step, no collective) and rank 0's order
        (BucketedGradSync.plan; every rank gets here exactly once)."""
        def record():
            castcache.drop_autograd_refs()
            with self._stream_ctx(), local_only():
                loss, _ = self._forward_loss(inp, pf)
                loss.backward()
            castcache.drop_autograd_refs()
            self._side_done()
        try:
            self.grad_sync.plan(record)
        except Exception as e:  # the buckets exist (rank 0's order); the step runs eagerly below
            _log(f"bucket recording failed: {e!r}")

    # ---------------------------------------------- snapshot around warm-ups
    def _snapshot(self):
        params = [p for p in self.model.parameters() if p.requires_grad]
        bufs = [b for b in self.model.buffers() if b.is_floating_point() or b.dtype in (torch.int64, torch.int32)]
        with torch.no_grad():
            sp = [p.detach().clone() for p in params]
            sb = [b.detach().clone() for b in bufs]
        st = {}
        for p, s in getattr(self.optimizer, "state", {}).items():
            st[id(p)] = {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in s.items()}
        rng = (torch.get_rng_state(), torch.cuda.get_rng_state(self.device) if self.on_gpu else None)
        return params, sp, bufs, sb, st, rng

    def _restore(self, snap):
        """Roll the warm-ups back in place (tensor identities are kept: graphs
        captured earlier read these addresses).  Optimizer state that the
        warm-ups created is reset to AdamW's initial values (zeros, step 0)."""
        params, sp, bufs, sb, st, rng = snap
        with torch.no_grad():
            if params:
                torch._foreach_copy_(params, sp)
            for b, v in zip(bufs, sb):
                # only the buffers the warm-ups changed: a copy bumps the
                # version counter, and caches keyed on it (e.g. the window
                # attention's relative-index check, a host sync) would then
                # be re-evaluated inside the capture
                if not torch.equal(b, v):
                    b.copy_(v)
            for p, s in getattr(self.optimizer, "state", {}).items():
                old = st.get(id(p))
                for k, v in s.items():
                    if torch.is_tensor(v):
                        if old is not None and k in old:
                            v.copy_(old[k])
                        else:
                            v.zero_()
                    elif old is not None and k in old:
                        s[k] = old[k]
                    elif k == "step":
                        s[k] = 0
        torch.set_rng_state(rng[0])
        if rng[1] is not None:
            torch.cuda.set_rng_state(rng[1], self.device)
        castcache._on_optimizer_step()  # the weight shadows no longer match the weights

    # ------------------------------------------------------------ capture
    def _capture(self, key, inputs, padding_free=False):
        while len(self.graphs) >= self.max_graphs:
            old_key, old = self.graphs.popitem(last=False)
            self._free(old)
            self.evictions += 1
            _log(f"evicted graph {old_key[:2]}")
        c = _Captured()
        for k, v in inputs.items():
            c.inputs[k] = _static_like(v)
        c.load(inputs)
        snap = self._snapshot()
        last = None
        try:
            # warm-up and capture on ONE side stream: the autograd engine runs
            # a parameter's AccumulateGrad on the stream the node was created on
            # (its first forward use); an AccumulateGrad node created on another
            # stream and kept alive (e.g. by a cached weight cast's grad_fn)
            # makes the captured backward synchronise with that stream, which
            # HIP refuses during capture (hipErrorStreamCaptureUnsupported)
            castcache.drop_autograd_refs()
            with self._stream_ctx(), local_only():
                for i in range(self.warmup):
                    if self.grad_sync is None:
                        self.optimizer.zero_grad(set_to_none=True)
                    last = self._body(c.inputs, padding_free)
                    _log(f"warm-up step {i} done")
                if last is None:  # no warm-up: one forward for the output shapes
                    with torch.no_grad():
                        last = self._forward_loss(c.inputs, padding_free)
            castcache.drop_autograd_refs()
            self._side_done()
        finally:
            self._restore(snap)
        loss, loss_dict = last
        c.loss_out = torch.empty_like(loss)
        c.dict_out = {k: torch.empty_like(v) for k, v in loss_dict.items()}
        del last, loss, loss_dict
        self._record(c, padding_free)
        c.fresh = True
        self.graphs[key] = c
        self.captures += 1
        return c

    def _record(self, c, padding_free):
        """Capture the body into c.graph (GPU).  The graph shares self.pool
        with every other graph of the cache; nothing that must survive
        between steps lives in the pool (static inputs, outputs, optimizer
        state and, with grad_sync, the gradient buckets are allocated
        outside it; without grad_sync each graph keeps the gradients its
        capture allocated, re-attached after its replays)."""
        if self.grad_sync is None:
            # the captured backward allocates the gradients from the graph's
            # pool; every replay rewrites them in place
            self.optimizer.zero_grad(set_to_none=True)
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        c.graph = g = torch.cuda.CUDAGraph(keep_graph=True)
        side = self._stream_ctx_stream()
        torch.cuda.synchronize()
        self._retire_collectives()
        bump_mask_epoch()  # no derived mask computed outside this capture is reused inside it
        _log("capture begins")
        # capture_begin / capture_end by hand instead of torch.cuda.graph:
        # when the body fails part-way, its __exit__ raises from capture_end
        # before it restores the current stream, and every later "eager"
        # launch would go to the invalidated capture stream.  Here the
        # stream context always unwinds, the invalidated capture is ended
        # (gd_stream_abort_capture) and the side stream is replaced.
        # thread_local: calls other threads make meanwhile (ProcessGroupNCCL's
        # watchdog polling the events of earlier eager collectives) do not
        # invalidate the capture
        with torch.cuda.stream(side):
            g.capture_begin(pool=self.pool if _SHARED_POOL else None, capture_error_mode=_CAPTURE_MODE)
            try:
                loss, loss_dict = self._body(c.inputs, padding_free)
                c.loss_out.copy_(loss)
                for k, v in loss_dict.items():
                    c.dict_out[k].copy_(v)
            except BaseException:
                self._abandon_capture(g, side)
                raise
            try:
                g.capture_end()
            except BaseException:
                self._abandon_capture(g, side)
                raise
        torch.cuda.current_stream().wait_stream(self.side)
        bump_mask_epoch()  # nor one of the capture's (graph-pool) masks outside it
        if self.grad_sync is None:
            c.grads = [p.grad for p in self.model.parameters() if p.requires_grad]
            self._grads_of = c
        c.memsets_replaced = memsets_to_kernels(c.graph)
        c.graph.instantiate()
        _log(f"captured; memset nodes replaced by fill kernels: {c.memsets_replaced}")

    def _retire_collectives(self):
        """Wait until ProcessGroupNCCL's watchdog has retired every eager
        collective: once the capture joins the communicator's stream, HIP
        refuses queries of events last recorded on that stream
        (hipErrorCapturedEvent), and the watchdog would abort the process
        polling an earlier work's end event."""
        if not (dist.is_available() and dist.is_initialized()):
            return
        groups = [dist.group.WORLD]
        gs = getattr(self.grad_sync, "group", None)
        if gs is not None and gs is not dist.group.WORLD:
            groups.append(gs)
        for grp in groups:
            if dist.get_backend(grp) != "nccl":
                continue
            grp._wait_for_pending_works()

    def _abandon_capture(self, g, side):
        """After a failed capture: end the stream's (invalidated) capture,
        release the allocator's capture routing, drop the stream."""
        try:
            g.capture_end()
        except BaseException:  # noqa: BLE001 -- the capture is already invalid
            pass
        try:
            fn = _lib.lib().gd_stream_abort_capture
            fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p]
            fn(ctypes.c_void_p(side.cuda_stream))
        except Exception:  # noqa: BLE001
            pass
        try:
            torch._C._cuda_endAllocateToPool(self.device.index if self.device.index is not None else
                                             torch.cuda.current_device(), g.pool())
        except Exception:  # noqa: BLE001 -- already ended by capture_end
            pass
        self.side = None

    def _stream_ctx_stream(self):
        if self.side is None:
            self.side = torch.cuda.Stream()
        self.side.wait_stream(torch.cuda.current_stream())
        return self.side

    def _free(self, c):
        self._drain()
        if c.graph is not None and hasattr(c.graph, "reset"):
            c.graph.reset()
        if self._grads_of is c:
            self._grads_of = None
        c.graph = None
        c.grads = None

    # ------------------------------------------------------------- eager
    def _eager(self, inputs, padding_free):
        if self.grad_sync is None:
            self.optimizer.zero_grad(set_to_none=True)
            self._grads_of = None
        loss, terms = self._body(inputs, padding_free)
        self.eager_steps += 1
        self.last_terms = terms
        return loss

    def _to_eager(self, reason):
        """Every rank: drop the graphs, run the eager step from now on."""
        self.fallback_reason = repr(reason)[:300] if reason is not None else "capture failed on another rank"
        print(f"warning: step graph disabled on rank {self.agree.rank}: {self.fallback_reason}",
              file=sys.stderr, flush=True)
        self.release()
        # the capture recorded (never ran) the shadow refresh while marking
        # the shadows current: they still hold a warm-up's weights
        castcache.clear()
        self.mode = "eager"

    # ------------------------------------------------------------- queue
    def _drain(self):
        for ev in self._inflight:
            ev.synchronize()
        self._inflight.clear()

    def _after_replay(self):
        if not self.on_gpu:
            return
        if self.sync_mode == "device":
            torch.cuda.synchronize()
        else:
            ev = torch.cuda.Event()
            ev.record()
            self._inflight.append(ev)

    # -------------------------------------------------------------- call
    def __call__(self, samples, targets, captions, cat_lists, prepared_text=None):
        inputs, pf = self._prepare(samples, targets, captions, cat_lists, prepared_text)
        # at most max_inflight replays queued: this step's host preparation
        # above overlapped the previous replay
        while len(self._inflight) >= self.max_inflight:
            self._inflight.pop(0).synchronize()
        if self.grad_sync is not None and self.grad_sync.buckets is None:
            self._plan(inputs, pf)
        key = self._signature(inputs) + (("padding_free", pf),)
        c, need = None, False
        if self.mode == "graph":
            self.seen[key] += 1
            c = self.graphs.get(key)
            if c is not None:
                self.graphs.move_to_end(key)
            else:
                need = len(self.graphs) < self.max_graphs or self.seen[key] >= self.capture_after
        if self.mode == "graph" and self.agree.any(need):
            ok, err = True, None
            if need:
                try:
                    c = self._capture(key, inputs, pf)
                except Exception as e:  # noqa: BLE001 -- any capture failure: every rank goes eager
                    import traceback
                    ok, err, c = False, repr(e), None
                    print(f"[stepgraph] capture failed on rank {self.agree.rank}:\n{traceback.format_exc()}",
                          file=sys.stderr, flush=True)
                if not ok:
                    # the aborted body's frames (held by the traceback) keep
                    # context managers open -- e.g. a non-reentrant
                    # checkpoint's saved-tensor hooks live in a suspended
                    # generator until it is collected, and would capture the
                    # next forward's tensors; drop them before the eager step
                    import gc
                    gc.collect()
                    if self.on_gpu:
                        torch.cuda.synchronize()
            if not self.agree.all(ok):
                self._to_eager(err)
                c = None
        if c is None:
            loss = self._eager(inputs, pf)
        else:
            if not c.fresh:
                c.load(inputs)
            c.fresh = False
            c.graph.replay()
            self.replays += 1
            if self.grad_sync is None and self._grads_of is not c and c.grads is not None:
                for p, g in zip((p for p in self.model.parameters() if p.requires_grad), c.grads):
                    p.grad = g
                self._grads_of = c
            loss = c.loss_out
            self.last_terms = c.dict_out
            castcache._on_optimizer_step()  # the replay stepped the optimizer: cast copies are stale
        self._after_replay()
        if _VERBOSE and self.on_gpu:
            torch.cuda.synchronize()
            _log(f"step done ({'replay' if c is not None else 'eager'}), loss {float(loss):.4f}")
        return loss

    def loss_dict(self):
        """The last step's loss terms (device tensors; a replayed graph's are
        rewritten by its next replay), or None before the first step."""
        return self.last_terms

    def release(self):
        self._drain()
        for c in list(self.graphs.values()):
            self._free(c)
        self.graphs.clear()
