"""Training-step plumbing around the drop-in model: synthetic odvg batches,
optimizer parameter groups, freezing, and one train step.

Restates what the reference's main.py / engine_multi.py do around
``model`` and ``criterion`` (main.py:254-292, engine_multi.py:499-564)
without the PAVE crop tiling (product-specific, out of scope):
  * freezing: names containing 'attn' stay trainable, then any name
    containing a freeze keyword is frozen (main.py:269-281; 'bert' by cfg);
  * AdamW over util/get_param_dicts.py 'ddetr_in_mmdet' groups (:34-53);
  * autocast (bf16 here; the reference's --amp is fp16) -> model ->
    criterion -> weighted sum -> backward -> clip_grad_norm_(0.1) -> step.
"""
from __future__ import annotations

import functools
import random
from typing import List, Tuple

import torch

from .misc import NestedTensor, collectives_enabled


# ------------------------------------------------------------------ batches
def _phrase_words(rng: random.Random, n_words: int, used: set) -> str:
    while True:
        words = [f"w{rng.randrange(10000, 99999)}" for _ in range(n_words)]
        p = " ".join(words)
        if p not in used:
            used.add(p)
            return p


def synthetic_caption(rng: random.Random, n_tokens: int = 256) -> List[str]:
    """Phrases whose caption ' . '.join(phrases) + ' .' tokenizes to exactly
    n_tokens ([CLS] + words and '.' separators + [SEP]) with the offline
    tokenizer (one token per word); phrase lengths 1-8 words."""
    budget = n_tokens - 2  # CLS, SEP
    phrases, used = [], set()
    while budget > 0:
        n = min(rng.randint(1, 8), budget - 1)
        if n <= 0:
            break
        phrases.append(_phrase_words(rng, n, used))
        budget -= n + 1  # words + '.'
    if budget > 0:  # one token left over: lengthen the last phrase
        phrases[-1] = phrases[-1] + f" w{rng.randrange(10000, 99999)}"
    return phrases


def synthetic_grounding(rng: random.Random, n_boxes: int, n_phrases: int = 6) -> Tuple[List[str], List[int]]:
    """VG-style regions (datasets/odvg.py:236-252): free-text phrases of 2-6
    words, several boxes sharing a phrase; the caption is the unique phrases
    (first-occurrence order) and a box's label indexes its phrase.
    -> (unique phrases, label per box)."""
    used: set = set()
    n_uniq = max(1, min(n_phrases, (n_boxes + 1) // 2))  # boxes share phrases
    pool = [_phrase_words(rng, rng.randint(2, 6), used) for _ in range(n_uniq)]
    phrases = [pool[i % len(pool)] for i in range(n_boxes)]  # every phrase used, some repeated
    rng.shuffle(phrases)
    uniq = list(dict.fromkeys(phrases))
    index = {p: i for i, p in enumerate(uniq)}
    return uniq, [index[p] for p in phrases]


def synthetic_batch(bs: int, height: int, width: int, n_boxes: int = 8, n_tokens: int = 256, seed: int = 0,
                    device="cuda", dtype=torch.float32, vg_images: int = 0) -> Tuple[NestedTensor, list, list, list]:
    """-> (samples, targets, captions, cat_lists) shaped like an odvg batch
    (datasets/odvg.py:254-260): boxes cxcywh normalised (centres U[0.2,0.8],
    sizes U[0.05,0.3]), labels index the image's phrase list.  The first
    bs - vg_images images are OD-style (category-name captions of n_tokens
    tokens); the last vg_images are VG-style grounding samples
    (synthetic_grounding: a short caption of unique free-text phrases, boxes
    sharing phrases) -- BASELINE config 5's mixed OD+VG batch."""
    rng = random.Random(seed)
    g = torch.Generator().manual_seed(seed)
    imgs = torch.randn(bs, 3, height, width, generator=g).to(device, dtype)
    mask = torch.zeros(bs, height, width, dtype=torch.bool, device=device)
    targets, captions, cat_lists = [], [], []
    for i in range(bs):
        if i >= bs - vg_images:
            cats, vg_labels = synthetic_grounding(rng, n_boxes)
            labels = torch.as_tensor(vg_labels, dtype=torch.int64)
        else:
            cats = synthetic_caption(rng, n_tokens)
            labels = torch.randint(0, len(cats), (n_boxes,), generator=g)
        caption = " . ".join(cats) + " ."
        ctr = torch.rand(n_boxes, 2, generator=g) * 0.6 + 0.2
        wh = torch.rand(n_boxes, 2, generator=g) * 0.25 + 0.05
        boxes = torch.cat([ctr, wh], -1)
        targets.append({"boxes": boxes.to(device), "labels": labels.to(device), "caption": caption,
                        "cap_list": cats, "size": torch.tensor([height, width], device=device),
                        "orig_size": torch.tensor([height, width], device=device)})
        captions.append(caption)
        cat_lists.append(cats)
    return NestedTensor(imgs, mask, padding_free=True), targets, captions, cat_lists


# --------------------------------------------------------------- optimizer
def _match(name, keywords):
    return any(k in name for k in keywords)


def apply_freeze(args, model) -> None:
    if getattr(args, "freeze_keywords", None) is None:
        return
    for name, p in model.named_parameters():
        if "attn" in name:
            p.requires_grad_(True)
        elif _match(name, args.freeze_keywords):
            p.requires_grad_(False)


def get_param_dict(args, model):
    """util/get_param_dicts.py:15-85 ('default' and 'ddetr_in_mmdet')."""
    kind = getattr(args, "param_dict_type", "default")
    named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
    if kind == "default":
        return [{"params": [p for n, p in named if "backbone" not in n]},
                {"params": [p for n, p in named if "backbone" in n], "lr": args.lr_backbone}]
    if kind == "ddetr_in_mmdet":
        bb, lp = args.lr_backbone_names, args.lr_linear_proj_names
        return [
            {"params": [p for n, p in named if not _match(n, bb) and not _match(n, lp)], "lr": args.lr},
            {"params": [p for n, p in named if _match(n, bb)], "lr": args.lr_backbone},
            {"params": [p for n, p in named if _match(n, lp)], "lr": args.lr_linear_proj_mult},
        ]
    raise ValueError(f"param_dict_type {kind} not supported")


def build_optimizer(args, model):
    groups = [g for g in get_param_dict(args, model) if g["params"]]
    # fused AdamW: one multi-tensor launch chain instead of per-parameter ops
    return torch.optim.AdamW(groups, lr=args.lr, weight_decay=args.weight_decay,
                             fused=next(model.parameters()).is_cuda)


# -------------------------------------------------------------------- step
_LOSS_WEIGHTS = {}


def weighted_loss(loss_dict, weight_dict):
    """sum(loss_dict[k] * weight_dict[k] for k in loss_dict if k in
    weight_dict) (reference engine.py's total loss) as one stack, one
    multiply by a cached on-device weight vector and one sum: 3 launches
    instead of a multiply and an add per term (about 45 terms with the 5 aux
    heads and the encoder head).  Each term's gradient is its weight exactly,
    as in the per-term sum; only the rounding of the reported total differs."""
    keys = [k for k in loss_dict if k in weight_dict]
    if not keys or any(loss_dict[k].dim() for k in keys):
        return sum(loss_dict[k] * weight_dict[k] for k in keys)
    dt = functools.reduce(torch.promote_types, (loss_dict[k].dtype for k in keys), torch.float32)
    vals = [loss_dict[k].to(dt) for k in keys]
    dev = vals[0].device
    ck = (tuple(keys), tuple(float(weight_dict[k]) for k in keys), dev, dt)
    w = _LOSS_WEIGHTS.get(ck)
    if w is None:
        if len(_LOSS_WEIGHTS) > 16:
            _LOSS_WEIGHTS.clear()
        w = _LOSS_WEIGHTS[ck] = torch.tensor(ck[1], dtype=dt).to(dev)
    return (torch.stack(vals) * w).sum()


class GradAllReduce:
    """Data-parallel gradient averaging after the backward pass, for the
    HIP-graph train step (DDP's per-bucket hooks cannot fire inside a graph
    replay): the gradients are all-reduced in buckets of ``bucket_mb``
    (fewer, larger RCCL ring all-reduces over xGMI), then divided by the
    world size -- DDP's result (reference main.py:258-261), without the
    overlap with the backward.  Parameters without a gradient are skipped
    (every rank runs the same graph, so the pattern agrees)."""

    def __init__(self, params, bucket_mb: int = 64, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.params = [p for p in params if p.requires_grad]
        self.bucket_bytes = bucket_mb << 20

    def __call__(self):
        from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
        world = self.dist.get_world_size(self.group)
        grads = [p.grad for p in self.params if p.grad is not None]
        bucket, size = [], 0
        for g in grads + [None]:
            if g is not None and (not bucket or (size + g.numel() * g.element_size() <= self.bucket_bytes
                                                 and g.dtype == bucket[0].dtype)):
                bucket.append(g)
                size += g.numel() * g.element_size()
                continue
            if bucket:
                flat = _flatten_dense_tensors(bucket)
                self.dist.all_reduce(flat, group=self.group)
                flat.div_(world)
                torch._foreach_copy_(bucket, _unflatten_dense_tensors(flat, bucket))
            bucket, size = ([g], g.numel() * g.element_size()) if g is not None else ([], 0)


class BucketedGradSync:
    """Data-parallel gradient averaging overlapped with the backward pass --
    DDP's reducer (reference main.py:258-261) restated so that it also runs
    INSIDE a captured HIP graph (gdino_amd.stepgraph), where DDP's own
    bookkeeping cannot follow replays.

    * The bucket plan follows the order in which the backward finishes
      gradients, recorded by one backward pass (DDP rebuilds its buckets
      after the first iteration the same way).  Rank 0's recorded order is
      broadcast and every rank builds the same buckets from it (DDP syncs
      its rebuilt bucket indices with rank 0 too), so the ranks' bucket
      sizes and order agree even where their batches take different paths.
      A bucket holds up to ``bucket_mb`` of gradients, the first one
      ``first_bucket_mb`` so the first collective starts early.
    * Each bucketed parameter's ``.grad`` is a view into its bucket's flat
      buffer (DDP's gradient_as_bucket_view): the backward accumulates
      straight into the buffer, and there is no flatten / unflatten copy.
    * A post-accumulate-grad hook counts a bucket's ready gradients.  Buckets
      are launched strictly in index order (a cursor, as DDP's reducer):
      when bucket i fills, it and every following bucket that is full are
      divided by the world size and all-reduced asynchronously (the process
      group's communication stream) while the backward goes on.  Every rank
      therefore issues the same collectives in the same order, whatever
      order its gradients arrive in.  A callback at the end of the backward
      launches what is left (in order) and waits for every bucket (the
      current stream waits on the communication stream: no host block).
    * ``zero_grad()`` replaces optimizer.zero_grad(set_to_none=True), which
      would drop the views.
    * Under ``misc.local_only()`` (the step graph's rolled-back warm-up
      iterations) nothing is reduced.
    ``control_group`` (optional, e.g. a gloo group): where rank 0's order is
    broadcast; default the gradient group.  Same averaged gradients as DDP
    (tests/test_ddp_gloo.py).  Parameters that receive no gradient in rank
    0's recording backward keep ``.grad = None``."""

    def __init__(self, params, bucket_mb: float = 25, first_bucket_mb: float = 1, group=None, control_group=None):
        import torch.distributed as dist
        self.dist, self.group, self.control_group = dist, group, control_group
        self.world = dist.get_world_size(group)
        self.params = [p for p in params if p.requires_grad]
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.first_bytes = int(first_bucket_mb * (1 << 20))
        self.order = []          # grad-ready order seen by the recording backward
        self.buckets = None      # [{"flat", "params", "pending", "work", "ready"}]
        self.bucket_of = {}
        self._queued = False
        self._next = 0           # launch cursor: the first bucket not yet launched
        self._handles = [p.register_post_accumulate_grad_hook(self._ready) for p in self.params]

    @staticmethod
    def _local():
        return not collectives_enabled()

    # ---------------------------------------------------------------- hooks
    def _ready(self, p):
        if self.buckets is None:
            self.order.append(p)
            return
        if self._local():
            return
        if not self._queued:
            self._queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        b = self.bucket_of.get(id(p))
        if b is None:
            return
        b["pending"] -= 1
        if b["pending"] == 0:
            b["ready"] = True
            self._launch_ready()

    def _launch_ready(self):
        while self._next < len(self.buckets) and self.buckets[self._next]["ready"]:
            self._launch(self.buckets[self._next])
            self._next += 1

    def _launch(self, b):
        b["flat"].div_(self.world)
        b["work"] = self.dist.all_reduce(b["flat"], group=self.group, async_op=True)

    def _finalize(self):
        for b in self.buckets:  # buckets with a parameter that got no gradient this pass
            b["ready"] = True
        self._launch_ready()
        for b in self.buckets:
            b["work"].wait()
            b["work"] = None
            b["pending"] = len(b["params"])
            b["ready"] = False
        self._next = 0
        self._queued = False

    # ------------------------------------------------------------ lifecycle
    def _agreed_order(self):
        """Rank 0's recorded order (parameter indices), broadcast to every
        rank; a rank without a recording contributes nothing."""
        seen, mine = set(), []
        for p in self.order:
            if id(p) not in seen and p.grad is not None:
                seen.add(id(p))
                mine.append(self.index[id(p)])
        self.order = []
        if self.world == 1:
            return mine
        box = [mine]
        self.dist.broadcast_object_list(box, src=self.dist.get_global_rank(self.group, 0)
                                        if self.group is not None else 0, group=self.control_group or self.group)
        return list(box[0])

    def _build(self, order):
        """Buckets over ``order`` (indices into self.params); existing grads
        move into the flat buffers, missing ones start at zero."""
        self.buckets, cur, size = [], [], 0
        for i in order:
            p = self.params[i]
            nbytes = p.numel() * 4
            cap = self.first_bytes if not self.buckets else self.bucket_bytes
            if cur and (size + nbytes > cap or p.dtype != cur[0].dtype):
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(cur)
        built = []
        for ps in self.buckets:
            flat = torch.zeros(sum(p.numel() for p in ps), dtype=ps[0].dtype, device=ps[0].device)
            off = 0
            for p in ps:
                view = flat[off:off + p.numel()].view_as(p)
                if p.grad is not None:
                    view.copy_(p.grad)
                p.grad = view
                off += p.numel()
            b = {"flat": flat, "params": ps, "pending": len(ps), "work": None, "ready": False}
            built.append(b)
            for p in ps:
                self.bucket_of[id(p)] = b
        self.buckets = built
        self._next = 0

    def plan(self, run_backward):
        """Build the buckets from one recording backward ``run_backward()``
        (forward + backward, no optimizer step; run under local_only by the
        caller).  Every rank calls this exactly once, also when its
        recording fails (it then takes rank 0's order)."""
        if self.buckets is not None:
            return
        try:
            run_backward()
        except Exception:
            self.order = []
            raise
        finally:
            order = self._agreed_order()
            self._build(order)

    def after_backward(self):
        """Call after every backward (train_step does): the first, recording
        pass builds the buckets from rank 0's order and all-reduces them in
        one go; later passes were already reduced by the hooks."""
        if self.buckets is not None:
            return
        self._build(self._agreed_order())
        if self._local():
            return
        for b in self.buckets:
            b["ready"] = True
        self._launch_ready()
        for b in self.buckets:
            b["work"].wait()
            b["work"] = None
            b["ready"] = False
        self._next = 0

    def zero_grad(self):
        if self.buckets is None:
            for p in self.params:
                p.grad = None
        else:
            for b in self.buckets:
                b["flat"].zero_()

    def bucket_sizes_mb(self):
        return [b["flat"].numel() * b["flat"].element_size() / 2 ** 20 for b in (self.buckets or [])]

    def remove(self):
        for h in self._handles:
            h.remove()


def train_step(model, criterion, optimizer, samples, targets, captions, cat_lists, clip_max_norm=0.1,
               amp_dtype=torch.bfloat16, grad_sync=None):
    """One optimisation step; returns the weighted loss tensor (not synced).
    ``grad_sync``: a BucketedGradSync (all-reduce overlapped with the
    backward; its after_backward() is called) or a plain callable run
    between backward and clipping (GradAllReduce)."""
    dev_type = samples.tensors.device.type
    with torch.autocast(device_type=dev_type, dtype=amp_dtype, enabled=amp_dtype is not None):
        outputs = model(samples, captions=captions)
        loss_dict = criterion(outputs, targets, cat_lists, captions)
        loss = weighted_loss(loss_dict, criterion.weight_dict)
    if isinstance(grad_sync, BucketedGradSync):
        grad_sync.zero_grad()
    else:
        optimizer.zero_grad(set_to_none=True)
    loss.backward()
    if isinstance(grad_sync, BucketedGradSync):
        grad_sync.after_backward()
    elif grad_sync is not None:
        grad_sync()
    if clip_max_norm > 0:
        torch.nn.utils.clip_grad_norm_(model.parameters(), clip_max_norm, foreach=True)
    optimizer.step()
    return loss.detach()


def forward_step(model, samples, captions, amp_dtype=torch.bfloat16):
    """BASELINE config 2: one inference forward (eval mode, no autograd) of
    model(samples, captions=...) under bf16 autocast; returns the output dict."""
    dev_type = samples.tensors.device.type
    with torch.no_grad(), torch.autocast(device_type=dev_type, dtype=amp_dtype, enabled=amp_dtype is not None):
        return model(samples, captions=captions)


def set_activation_checkpointing(model, enabled: bool) -> int:
    """Switch the reference's activation checkpointing (cfg use_checkpoint:
    Swin blocks and fusion layers; use_transformer_ckpt: the deformable
    encoder layers) on or off at run time.  It trades recompute for
    activation memory: the backward re-runs each checkpointed forward.  The
    losses and gradients are the same either way (the recompute replays the
    RNG state; tests/test_model_cpu.py), so on a 288 GB MI355X, where the
    bs=2 800x1333 step's activations fit many times over, the step can skip
    the recompute.  Returns the number of modules switched."""
    n = 0
    for m in model.modules():
        for attr in ("use_checkpoint", "use_transformer_ckpt"):
            if isinstance(getattr(m, attr, None), bool):
                setattr(m, attr, bool(enabled))
                n += 1
    return n


def activation_checkpointing(model) -> bool:
    return any(getattr(m, a, False) is True for m in model.modules()
               for a in ("use_checkpoint", "use_transformer_ckpt"))


def build_training(args, device):
    from models.GroundingDINO import build_groundingdino
    model, criterion, post = build_groundingdino(args)
    model.to(device)
    apply_freeze(args, model)
    optimizer = build_optimizer(args, model)
    return model, criterion, post, optimizer


def small_train_step(device, height=256, width=320, seed=0, stochastic=True) -> float:
    """smoke(): one tiny train step of the full Swin-T + BERT-base model.
    stochastic=False zeroes every dropout / drop-path rate, so the loss
    depends on the weights, the batch and the kernels' rounding only, not on
    the order the step draws random numbers in (smoke pins it)."""
    from .config import make_args
    torch.manual_seed(seed)
    args = make_args(device=str(device))
    model, criterion, _, opt = build_training(args, device)
    model.train()
    if not stochastic:
        for m in model.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
            if hasattr(m, "drop_prob"):
                m.drop_prob = 0.0
    samples, targets, captions, cats = synthetic_batch(1, height, width, n_boxes=3, n_tokens=24, seed=seed,
                                                       device=device)
    loss = train_step(model, criterion, opt, samples, targets, captions, cats)
    return float(loss)
