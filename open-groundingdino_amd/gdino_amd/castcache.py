"""Per-parameter autocast weight cache.

Under bf16 autocast every Linear casts its fp32 weight and bias to bf16 on
each call. autocast's own cache lives only inside one autocast region, so the
checkpoint recompute in the backward pass (Swin blocks and encoder layers,
use_checkpoint / use_transformer_ckpt) casts them again. The frozen BERT's
weights are also re-cast every step, and a slice of a parameter (the q/k/v
rows of MultiheadAttention.in_proj_weight) is never cached at all. In total
that is several hundred cast launches per step on a launch-bound step.

``cached_cast(p, dtype)`` returns a bf16 copy of parameter ``p`` that stays
valid while ``p._version`` is unchanged and, for a trainable parameter, no
optimizer step has run since the copy was made:

* The fused AdamW kernel (``torch.optim.AdamW(fused=True)``, the bench's and
  build_optimizer's optimizer) updates the parameters in place WITHOUT
  bumping their version counters (the foreach path does bump them).  A
  version check alone therefore served the step-1 weights forever: the
  forward never saw an update (round-2 bug, found by comparing the eager
  loss trajectory with the HIP-graph one, which bypasses this cache; pinned
  by test_cast_cache_follows_fused_adamw_updates).  A global
  optimizer-step post hook (every torch.optim.Optimizer) bumps a generation
  counter, and copies of trainable parameters are valid for one generation.
* Frozen weights (requires_grad False, e.g. the BERT) are cast once.

The copy is produced by the same ``p.to(dtype)`` autocast would run, so the
numerics are bit-identical. When grad mode is on the copy is created with its
cast node, so gradients reach the fp32 parameter through one ToCopyBackward
per step.

The cache is bypassed while a HIP graph is being captured: a graph must
contain the cast, or its replays would read a stale copy after the optimizer
step.

Step shadows (``refresh_shadows``, GDINO_CAST_SHADOWS=0 to disable): at the
start of every training forward (GroundingDINO.forward_core, so also inside
the captured forward graph) ONE multi-tensor copy kernel casts every
trainable fp32 parameter into a persistent bf16 shadow, and cached_cast hands
out the shadow (through _ShadowCast, whose backward is ToCopyBackward's
grad.to(fp32)) while it is current: same generation, same parameter version.
A captured step thus carries one cast launch instead of one per Linear call
(several hundred graph nodes, the checkpoint recomputes included).  Frozen
parameters (the BERT) keep their one eager cast, also under capture (a
frozen weight loaded after capture needs a re-capture, as any graph input
whose storage is replaced does).
"""
from __future__ import annotations

import os
import weakref

import torch
import torch.nn.functional as F
from torch import nn
from torch.optim.optimizer import register_optimizer_step_post_hook

ENABLED = os.environ.get("GDINO_CAST_CACHE", "1") != "0"
# one GEMM for Linears that read the same input (linear_shared_input)
FUSE_SHARED_INPUT = os.environ.get("GDINO_FUSE_PROJ", "1") != "0"
# tests: fuse also without autocast (native dtype), to pin the fused path
# against the fp64 reference goldens
FUSE_WITHOUT_AUTOCAST = False
_cache: dict = {}
_generation = 0


def _on_optimizer_step(*_args, **_kwargs) -> None:
    """Invalidate the copies of trainable parameters after any optimizer step."""
    global _generation
    _generation += 1


register_optimizer_step_post_hook(_on_optimizer_step)


def _gen(trainable: bool) -> int:
    return _generation if trainable else -1


def autocast_dtype(x: torch.Tensor):
    """The autocast lower-precision dtype active for x's device, or None
    (also None when the cache is disabled: callers then fall back to
    autocast's own casting)."""
    if not ENABLED:
        return None
    dev = x.device.type
    if dev not in ("cuda", "cpu") or not torch.is_autocast_enabled(dev):
        return None
    return torch.get_autocast_dtype(dev)


def _capturing(p: torch.Tensor) -> bool:
    return p.is_cuda and torch.cuda.is_current_stream_capturing()


SHADOWS = os.environ.get("GDINO_CAST_SHADOWS", "1") != "0"
_shadow: dict = {}       # id(p) -> [weakref(p), bf16 shadow, p._version at the refresh, group key or None]
_shadow_state = None     # (generation, dtype) of the last refresh
# parameter groups the fused projections concatenate (_cached_cat): their
# shadows are laid out back to back in one buffer, so the concatenation is
# that buffer -- a view, no cat kernel per call (GDINO_GROUP_SHADOWS=0: off)
GROUP_SHADOWS = os.environ.get("GDINO_GROUP_SHADOWS", "1") != "0"
_groups: dict = {}       # key (tuple of ids) -> tuple of weakrefs, registered by _cached_cat
_group_buf: dict = {}    # key -> the group's shadow buffer
_groups_pending = False  # a group registered since the last layout


class _ShadowCast(torch.autograd.Function):
    """p -> its refreshed low-precision shadow; backward = ToCopyBackward."""

    @staticmethod
    def forward(ctx, p, shadow):
        ctx.dtype = p.dtype
        return shadow.detach()

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.dtype), None


def _shadow_params(model: nn.Module):
    """The trainable fp32 parameters, rebuilt whenever the parameter set or
    a requires_grad flag changes (a later freeze / unfreeze, a
    load_state_dict(assign=True), a re-wrap): a stale list would keep casting
    frozen weights, or silently leave new ones on one cast per use."""
    params = list(model.parameters())
    sig = tuple((id(q), q.requires_grad, q.dtype) for q in params)
    cached = getattr(model, "_gd_shadow_params", None)
    if cached is None or cached[0] != sig:
        seen, ps = set(), []
        for q in params:
            if q.requires_grad and q.dtype == torch.float32 and id(q) not in seen:
                seen.add(id(q))
                ps.append(q)
        cached = (sig, ps)
        model._gd_shadow_params = cached
    return cached[1]


def refresh_shadows(model: nn.Module, x: torch.Tensor) -> None:
    """Cast every trainable fp32 parameter of ``model`` into its persistent
    shadow in one multi-tensor copy, when a training forward under bf16
    autocast is about to run (x: any input on the model's device)."""
    global _shadow_state, _groups_pending
    dt = autocast_dtype(x) if SHADOWS else None
    if dt is None or not torch.is_grad_enabled() or not model.training:
        return
    ps = _shadow_params(model)
    if not ps or any(q.device != x.device for q in ps):
        return
    if _shadow_state == (_generation, dt) and not _capturing(x) and not _groups_pending and all(
            _current_shadow(q, dt) is not None for q in ps):
        return  # already this step's weights (a second forward before the optimizer step)
    if GROUP_SHADOWS:
        _layout_groups(ps, dt)
    _groups_pending = False
    dsts, srcs = [], []
    for q in ps:
        e = _shadow.get(id(q))
        if e is None or e[0]() is not q or e[1].shape != q.shape or e[1].dtype != dt:
            e = [weakref.ref(q), torch.empty(q.shape, dtype=dt, device=q.device), None, None]
            _shadow[id(q)] = e
        e[2] = q._version
        dsts.append(e[1])
        srcs.append(q.detach())
    with torch.no_grad():
        torch._foreach_copy_(dsts, srcs)
    _shadow_state = (_generation, dt)


def _layout_groups(ps, dt) -> None:
    """Give every registered group whose members are all trainable shadowed
    parameters one shadow buffer, the members' shadows being consecutive
    slices of it along dim 0 (what torch.cat(dim=0) of them would produce).
    A parameter takes part in one group at most; done once per group."""
    live = {id(q) for q in ps}
    taken = set()
    for key, refs in list(_groups.items()):
        members = [r() for r in refs]
        if any(m is None for m in members):
            del _groups[key]
            _group_buf.pop(key, None)
            continue
        if not all(id(m) in live for m in members) or any(id(m) in taken for m in members):
            continue
        taken.update(id(m) for m in members)
        buf = _group_buf.get(key)
        tail = members[0].shape[1:]
        if buf is not None and buf.dtype == dt and all(
                (_shadow.get(id(m)) or [None] * 4)[3] == key for m in members):
            continue  # laid out already
        if any(m.shape[1:] != tail or m.device != members[0].device for m in members):
            continue
        buf = torch.empty((sum(m.shape[0] for m in members),) + tuple(tail), dtype=dt, device=members[0].device)
        _group_buf[key] = buf
        off = 0
        for m in members:
            n = m.shape[0]
            _shadow[id(m)] = [weakref.ref(m), buf[off:off + n], None, key]
            off += n


class _GroupShadow(torch.autograd.Function):
    """(p_1, ..., p_k) -> their group's shadow buffer (= the bf16 cat of the
    parameters along dim 0); backward: split + ToCopyBackward per member."""

    @staticmethod
    def forward(ctx, buf, *ps):
        ctx.rows = [p.shape[0] for p in ps]
        ctx.dtypes = [p.dtype for p in ps]
        return buf.detach()

    @staticmethod
    def backward(ctx, g):
        return (None,) + tuple(x.to(d) for x, d in zip(g.split(ctx.rows, 0), ctx.dtypes))


def _current_shadow(p: torch.Tensor, dtype: torch.dtype):
    if _shadow_state != (_generation, dtype):
        return None
    e = _shadow.get(id(p))
    if e is None or e[0]() is not p or e[2] != p._version:
        return None
    return e[1]


def _from_shadow(p, s, grad):
    return _ShadowCast.apply(p, s) if grad else s


def cached_cast(p: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Callers only use this when ENABLED (otherwise they hand the fp32
    parameter to autocast, whose own per-region cache then applies)."""
    if p.dtype == dtype:
        return p
    grad = torch.is_grad_enabled() and p.requires_grad
    key = id(p)
    ver = (p._version, _gen(p.requires_grad))
    sh = _current_shadow(p, dtype) if p.requires_grad else None
    if _capturing(p):
        if sh is not None:
            return _from_shadow(p, sh, grad)
        ent = _cache.get(key)
        if not p.requires_grad and ent is not None and ent[0]() is p and ent[1] == ver and ent[2] == dtype \
                and ent[3] == grad:
            return ent[4]  # frozen: the eager copy made before capture
        return p.to(dtype)
    ent = _cache.get(key)
    if ent is not None and ent[0]() is p and ent[1] == ver and ent[2] == dtype and ent[3] == grad:
        return ent[4]
    t = _from_shadow(p, sh, grad) if sh is not None else p.to(dtype)
    _cache[key] = (weakref.ref(p), ver, dtype, grad, t)
    if len(_cache) > 8192:  # drop entries of freed parameters
        for k in [k for k, v in _cache.items() if v[0]() is None]:
            del _cache[k]
    return t


def drop_autograd_refs() -> None:
    """Forget the cached casts that carry a grad_fn: each keeps its
    parameter's AccumulateGrad node (and the stream it was created on) alive
    across steps.  The step-graph capture drops them so that every node of
    the captured backward is (re)created on the capture stream."""
    for k in [k for k, v in _cache.items() if v[3]]:
        del _cache[k]


def clear() -> None:
    global _shadow_state
    _cache.clear()
    _shadow.clear()
    _groups.clear()
    _group_buf.clear()
    _shadow_state = None


def _token_linear_ok(x, params, out_features, dt):
    """Route to gdino_amd.wgrad.token_linear: the GPU, bf16 autocast,
    trainable fp32 parameters.  -> "splitk" (split-K weight-gradient kernel,
    a qualifying token-heavy shape), "lib" (library GEMM with fp32 output) or
    None (autocast's own path)."""
    # (also inside a HIP-graph capture: the split-K kernel and the fp32-output
    # library GEMM are capturable; without them a captured backward ran the
    # bf16 library GEMMs + a cast kernel per weight, +25 ms per step)
    if dt != torch.bfloat16 or not torch.is_grad_enabled():
        return None
    if any(p.dtype != torch.float32 or not p.requires_grad for p in params):
        return None
    from . import wgrad
    if wgrad.eligible(x, out_features, dt):
        return "splitk"
    return "lib" if wgrad.lib_eligible(x, dt) else None


def linear2d(x: torch.Tensor, w: torch.Tensor, b=None) -> torch.Tensor:
    """F.linear(x, w, b) as ONE 2-D GEMM over the flattened tokens: F.linear
    on a 3-D input that cannot be viewed 2-D (a [L, B, C] transpose)
    dispatches a bmm against the weight expanded to [L, C_out, C_in]; here
    such an input is copied contiguous first (reshape)."""
    if x.dim() <= 2 or x.is_contiguous():
        return F.linear(x, w, b)
    x2 = x.reshape(-1, x.shape[-1])
    return F.linear(x2, w, b).view(*x.shape[:-1], w.shape[0])


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None) -> torch.Tensor:
    """F.linear with cached weight / bias casts under autocast."""
    dt = autocast_dtype(x) if ENABLED else None
    if dt is not None and weight.is_floating_point():
        wc = cached_cast(weight, dt)
        bc = None if bias is None else cached_cast(bias, dt)
        params = [weight] + ([bias] if bias is not None else [])
        route = _token_linear_ok(x, params, weight.shape[0], dt)
        if route is not None:
            from . import wgrad
            return wgrad.token_linear(x, wc, bc, [weight], [] if bias is None else [bias], route == "lib")
        return linear2d(x, wc, bc)
    return linear2d(x, weight, bias)


# GDINO_FUSED_RELU=0: the activation as its own kernel (A/B)
FUSED_RELU = os.environ.get("GDINO_FUSED_RELU", "1") != "0"


def linear_relu(x: torch.Tensor, layer: nn.Linear, fold_into_consumer: bool = False) -> torch.Tensor:
    """F.relu(layer(x)): on the token-linear route (GPU, bf16 autocast,
    trainable fp32 parameters) the ReLU runs in the GEMM's epilogue and its
    backward masks by the saved output; elsewhere the plain composition.

    ``fold_into_consumer``: the CALLER guarantees that the result has exactly
    one consumer, the next Linear (``ffn`` / utils.MLP own both layers);
    that Linear may then fold this ReLU's backward into its dX kernel.
    Without the promise the output is never offered for the fold, so a
    second consumer always receives a correctly masked gradient (ADVICE
    round 5)."""
    weight, bias = layer.weight, layer.bias
    dt = autocast_dtype(x) if ENABLED else None
    if FUSED_RELU and dt is not None and bias is not None and weight.is_floating_point():
        params = [weight, bias]
        route = _token_linear_ok(x, params, weight.shape[0], dt)
        if route is not None:
            from . import wgrad
            return wgrad.token_linear(x, cached_cast(weight, dt), cached_cast(bias, dt), [weight], [bias],
                                      route == "lib", relu=True, fold=fold_into_consumer)
    return F.relu(layer(x))


def ffn(x: torch.Tensor, linear1: nn.Linear, linear2: nn.Module, dropout=None) -> torch.Tensor:
    """linear2(dropout(relu(linear1(x)))) -- the FFN sublayer that owns both
    Linears, so the ReLU output's only consumer is linear2 (through an
    identity dropout) and its backward may be folded into linear2's dX."""
    h = linear_relu(x, linear1, fold_into_consumer=True)
    if dropout is not None:
        h = dropout(h)
    return linear2(h)


class CachedCastLinear(nn.Linear):
    """nn.Linear using cached_cast under autocast (same parameters)."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)


def install(model: nn.Module) -> int:
    """Switch every plain nn.Linear of ``model`` to CachedCastLinear (class
    swap: parameters, state dict and hooks are untouched).  Returns the count."""
    n = 0
    for m in model.modules():
        if type(m) is nn.Linear:
            m.__class__ = CachedCastLinear
            n += 1
    return n


def _cached_cat(params, dtype):
    """bf16 concatenation (dim 0) of several parameters, cached like
    cached_cast; gradients reach each parameter through the cat's split."""
    ps = tuple(params)
    gkey = tuple(id(p) for p in ps)
    if GROUP_SHADOWS and gkey not in _groups and all(p.requires_grad for p in ps):
        global _groups_pending
        _groups[gkey] = tuple(weakref.ref(p) for p in ps)  # laid out by the next refresh_shadows
        _groups_pending = True
    shs = [_current_shadow(p, dtype) if p.requires_grad else None for p in ps]
    grad = torch.is_grad_enabled() and any(p.requires_grad for p in ps)
    if all(sh is not None for sh in shs) and all(_shadow[id(p)][3] == gkey for p in ps):
        buf = _group_buf[gkey]
        return _GroupShadow.apply(buf, *ps) if grad else buf  # the cat, as a buffer: no kernel
    if all(sh is not None for sh in shs):
        def make():  # one bf16 cat of the step's shadows (no fp32 cat + cast)
            return torch.cat([_from_shadow(p, sh, torch.is_grad_enabled()) for p, sh in zip(ps, shs)])
    else:
        def make():
            return torch.cat(ps).to(dtype)  # = cat of the casts, one cast kernel (and one in backward)
    key = ("cat",) + tuple(id(p) for p in ps)
    vers = tuple(p._version for p in ps) + (_gen(any(p.requires_grad for p in ps)),)
    ent = _cache.get(key)
    hit = (ent is not None and all(r() is p for r, p in zip(ent[0], ps)) and ent[1] == vers and ent[2] == dtype
           and ent[3] == grad)
    if _capturing(ps[0]):
        # frozen parameters: the eager copy made before the capture (constant
        # across replays); trainable ones are re-concatenated inside the graph
        return ent[4] if hit and not any(p.requires_grad for p in ps) else make()
    if hit:
        return ent[4]
    t = make()
    _cache[key] = (tuple(weakref.ref(p) for p in ps), vers, dtype, grad, t)
    return t


def linear_shared_input_joint(x: torch.Tensor, layers):
    """The one-GEMM output of ``linear_shared_input`` left unsplit ([..., sum
    of out_features], the layers' outputs side by side), or None when the
    fused route does not apply.  A consumer that reads the column blocks in
    place (biattn.BiAttnTokens) then hands back ONE gradient tensor: no
    split backward's concatenation of the blocks' gradients."""
    dt = autocast_dtype(x)
    if dt is None or not FUSE_SHARED_INPUT or any(m.bias is None for m in layers):
        return None
    w = _cached_cat([m.weight for m in layers], dt)
    b = _cached_cat([m.bias for m in layers], dt)
    params = [m.weight for m in layers] + [m.bias for m in layers]
    route = _token_linear_ok(x, params, w.shape[0], dt)
    if route is None:
        return None
    from . import wgrad
    return wgrad.token_linear(x, w, b, [m.weight for m in layers], [m.bias for m in layers], route == "lib")


def linear_shared_input(x: torch.Tensor, layers):
    """[layer(x) for layer in layers] for nn.Linear layers reading the same
    input.  Under autocast with the cache on, one GEMM against the cached
    concatenated bf16 weight (x is cast once); otherwise the plain per-layer
    calls.  Parameters are untouched (state dict unchanged)."""
    dt = autocast_dtype(x)
    if dt is None and FUSE_WITHOUT_AUTOCAST:
        dt = x.dtype
    if dt is None or not FUSE_SHARED_INPUT or any(m.bias is None for m in layers):
        return [m(x) for m in layers]
    w = _cached_cat([m.weight for m in layers], dt)
    b = _cached_cat([m.bias for m in layers], dt)
    from .misc import split_last
    params = [m.weight for m in layers] + [m.bias for m in layers]
    route = _token_linear_ok(x, params, w.shape[0], dt)
    if route is not None:
        from . import wgrad
        y = wgrad.token_linear(x, w, b, [m.weight for m in layers], [m.bias for m in layers], route == "lib")
    else:
        y = linear2d(x, w, b)
    return list(split_last(y, [m.out_features for m in layers]))
