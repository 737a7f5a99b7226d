"""Small host-side utilities the model needs (the reference pulls them from
groundingdino/util/misc.py and timm): NestedTensor, padding of image lists,
inverse_sigmoid, distributed helpers, DropPath, trunc_normal_."""
from __future__ import annotations

import contextlib
import contextvars
import ctypes
from typing import Optional

import torch
import torch.distributed as dist
from torch import Tensor, nn

from . import _lib


_CONSTS = {}


def device_const(key, make, device) -> Tensor:
    """A small constant tensor built on the host once per (key, device) and
    kept resident (no host->device copy inside a captured HIP graph)."""
    k = (key, str(device))
    t = _CONSTS.get(k)
    if t is None:
        t = make().to(device)
        _CONSTS[k] = t
    return t


# per-tensor derived-mask caches (inverted, mha.merge_masks) are keyed on
# this epoch too: the step graph bumps it around every capture, so a capture
# records its own mask kernels instead of baking in a warm-up's result (the
# static inputs are refilled in place on every replay)
_MASK_EPOCH = [0]


def bump_mask_epoch() -> None:
    _MASK_EPOCH[0] += 1


def mask_cache_key(*ts) -> tuple:
    return tuple(t._version for t in ts) + (_MASK_EPOCH[0],)


def inverted(mask: Tensor) -> Tensor:
    """~mask, computed once per mask object, version and cache epoch: the
    layers of one step invert the same text / padding masks again and again
    (one kernel each)."""
    key = mask_cache_key(mask)
    c = getattr(mask, "_gd_inv", None)
    if c is not None and c[0] == key:
        return c[1]
    r = ~mask
    mask._gd_inv = (key, r)
    return r


def topk_indices(x: Tensor, k: int) -> Tensor:
    """torch.topk(x, k, dim=1)[1] (two-stage proposal selection,
    reference transformer.py:292-296), safe inside a captured HIP graph.

    For slices of >= 20 000 elements PyTorch's topk switches to its
    multi-block radix select, whose captured replay does not follow new
    input data (a round-3 capture probe, profiles/r03_graph_topk_probe.log:
    the replay on new scores returns a different index set than eager).
    S = 22 223 encoder tokens at 800x1333 is above that switch, 6 800 at
    512x640 is below it: the size dependence of the round-2 graph fault.
    Under capture the selection is a stable descending sort and a slice:
    the same indices in the same order for distinct values (ties: lowest
    index first; topk leaves tie order unspecified)."""
    if x.is_cuda and torch.cuda.is_current_stream_capturing():
        return torch.sort(x, dim=1, descending=True, stable=True)[1][:, :k]
    return torch.topk(x, k, dim=1)[1]


_PADDING_FREE = contextvars.ContextVar("gd_padding_free", default=False)


@contextlib.contextmanager
def no_padding(flag: bool = True):
    """Within: the batch's padding mask is known on the host to be all False
    (every image fills the padded canvas), so masking by it is the identity
    and the deformable attention skips its value masked_fill (forward and
    backward: three passes over a [B, S, 256] tensor per MSDA layer)."""
    tok = _PADDING_FREE.set(bool(flag))
    try:
        yield
    finally:
        _PADDING_FREE.reset(tok)


def padding_free() -> bool:
    return _PADDING_FREE.get()


class NestedTensor:
    """Batched images + padding mask (True on padded pixels).
    Contract of groundingdino/util/misc.py:399-480; the model also accepts any
    object with ``.tensors`` and ``.mask`` (e.g. the reference's own class).
    ``padding_free``: the host knows the mask is all False (no image was
    padded), which lets the model skip masking by it."""

    def __init__(self, tensors: Tensor, mask: Optional[Tensor], padding_free: bool = False):
        self.tensors = tensors
        self.mask = mask
        self.padding_free = bool(padding_free)

    def to(self, device, non_blocking=False):
        m = None if self.mask is None else self.mask.to(device, non_blocking=non_blocking)
        return NestedTensor(self.tensors.to(device, non_blocking=non_blocking), m, self.padding_free)

    def decompose(self):
        return self.tensors, self.mask

    def pin_memory(self):
        """DataLoader(pin_memory=True) hook: page-locked host tensors, so the
        host->device copy of the batch is asynchronous."""
        return NestedTensor(self.tensors.pin_memory(), None if self.mask is None else self.mask.pin_memory(),
                            self.padding_free)

    @property
    def device(self):
        return self.tensors.device

    @property
    def shape(self):
        return {"tensors.shape": self.tensors.shape, "mask.shape": self.mask.shape}

    def __repr__(self):
        return f"NestedTensor(tensors={tuple(self.tensors.shape)}, mask={None if self.mask is None else tuple(self.mask.shape)})"


class _SplitLast(torch.autograd.Function):
    """x.split(sizes, -1) whose backward is ONE cat of the pieces' gradients
    (autograd's split backward builds a zero-filled full-size gradient per
    piece, copies it in and sums them: 3 kernels per piece)."""

    @staticmethod
    def forward(ctx, x, sizes):
        ctx.sizes = sizes
        ctx.meta = (x.shape[:-1], x.dtype, x.device)
        return tuple(x.split(sizes, -1))

    @staticmethod
    def backward(ctx, *grads):
        lead, dt, dev = ctx.meta
        gs = [g if g is not None else torch.zeros(*lead, n, dtype=dt, device=dev) for g, n in zip(grads, ctx.sizes)]
        return torch.cat(gs, -1), None


def split_last(x: Tensor, sizes) -> tuple:
    """x.split(sizes, dim=-1) with a single-cat backward (same values and
    gradients)."""
    sizes = [int(n) for n in sizes]
    if not (torch.is_grad_enabled() and x.requires_grad):
        return tuple(x.split(sizes, -1))
    return _SplitLast.apply(x, sizes)


def nested_tensor_from_tensor_list(tensor_list) -> NestedTensor:
    """Zero-pad [C,H,W] images to the batch max size; mask marks the padding
    (groundingdino/util/misc.py:483-506)."""
    if isinstance(tensor_list, Tensor) and tensor_list.dim() == 4:
        b, _, h, w = tensor_list.shape
        return NestedTensor(tensor_list, torch.zeros((b, h, w), dtype=torch.bool, device=tensor_list.device), True)
    if tensor_list[0].ndim != 3:
        raise ValueError("not supported")
    c = max(t.shape[0] for t in tensor_list)
    h = max(t.shape[1] for t in tensor_list)
    w = max(t.shape[2] for t in tensor_list)
    first = tensor_list[0]
    batch = first.new_zeros((len(tensor_list), c, h, w))
    mask = torch.ones((len(tensor_list), h, w), dtype=torch.bool, device=first.device)
    for i, img in enumerate(tensor_list):
        batch[i, : img.shape[0], : img.shape[1], : img.shape[2]].copy_(img)
        mask[i, : img.shape[1], : img.shape[2]] = False
    return NestedTensor(batch, mask, all(tuple(t.shape[1:]) == (h, w) for t in tensor_list))


def inverse_sigmoid(x: Tensor, eps: float = 1e-3) -> Tensor:
    """logit with clamping (reference util/misc.py:614-618)."""
    x = x.clamp(min=0, max=1)
    return torch.log(x.clamp(min=eps) / (1 - x).clamp(min=eps))


class _BoxRefine(torch.autograd.Function):
    """sigmoid(delta + inverse_sigmoid(ref)) in one kernel each way
    (csrc/boxref.hip): the composition is ~20 launches per call on
    [2, 900, 4] tensors, 12 calls per train step."""

    @staticmethod
    def forward(ctx, delta, ref, eps):
        shape, ds = _geo3(delta)
        _, rs = _geo3(ref)
        out = torch.empty(delta.shape, dtype=torch.float32, device=delta.device)
        _lib.call("gd_box_refine_forward", _lib.dtype_code(delta), delta.data_ptr(), *ds, ref.data_ptr(), *rs,
                  *shape, float(eps), out.data_ptr(), _lib.stream_of(delta),
                  nbytes=out.numel() * (delta.element_size() + 8))
        ctx.save_for_backward(out, ref)
        ctx.meta = (eps, delta.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        out, ref = ctx.saved_tensors
        eps, ddtype = ctx.meta
        g = g.float().contiguous()
        gd = torch.empty(out.shape, dtype=ddtype, device=g.device) if ctx.needs_input_grad[0] else None
        gr = torch.empty(out.shape, dtype=torch.float32, device=g.device) if ctx.needs_input_grad[1] else None
        if gd is not None or gr is not None:
            shape, rs = _geo3(ref)
            _lib.call("gd_box_refine_backward", _lib.dtype_code(gd if gd is not None else out), g.data_ptr(),
                      out.data_ptr(), ref.data_ptr(), *rs, *shape, float(eps), _lib.ptr(gd), _lib.ptr(gr),
                      _lib.stream_of(g), nbytes=out.numel() * 16)
        return gd, gr, None


def _geo3(t):
    """(shape, strides) of a 2-D / 3-D tensor as 3-D"""
    if t.dim() == 2:
        return (1,) + tuple(t.shape), (0,) + tuple(t.stride())
    return tuple(t.shape), tuple(t.stride())


def box_refine(delta: Tensor, ref: Tensor, eps: float = 1e-3) -> Tensor:
    """sigmoid(delta + inverse_sigmoid(ref, eps)): the decoder's anchor update
    (reference transformer.py:728-731) and the per-layer box heads (reference
    groundingdino.py:325-327).  One HIP kernel forward and one backward
    (csrc/boxref.hip) on the device; the composition elsewhere
    (GDINO_DISABLE=boxrefine, CPU)."""
    if (_lib.enabled("boxrefine") and _lib.on_device(delta) and _lib.on_device(ref) and delta.shape == ref.shape
            and delta.dim() in (2, 3) and delta.numel() > 0 and delta.dtype in (torch.float32, torch.bfloat16)
            and ref.dtype == torch.float32):
        return _BoxRefine.apply(delta, ref, eps)
    return (delta + inverse_sigmoid(ref, eps)).sigmoid()


def is_dist_avail_and_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


_LOCAL_ONLY = contextvars.ContextVar("gdino_local_only", default=False)


@contextlib.contextmanager
def local_only(flag: bool = True):
    """Within: the train step issues no collective (the criterion's num_boxes
    all-reduce is skipped, BucketedGradSync reduces nothing).  The step
    graph's warm-up iterations run this way -- their effects on the weights
    and the optimizer are rolled back afterwards -- so that a capture on one
    rank never adds collectives the other ranks do not issue."""
    tok = _LOCAL_ONLY.set(bool(flag))
    try:
        yield
    finally:
        _LOCAL_ONLY.reset(tok)


def collectives_enabled() -> bool:
    return is_dist_avail_and_initialized() and not _LOCAL_ONLY.get()


def get_world_size() -> int:
    return dist.get_world_size() if is_dist_avail_and_initialized() else 1


def get_rank() -> int:
    return dist.get_rank() if is_dist_avail_and_initialized() else 0


def drop_path(x: Tensor, drop_prob: float = 0.0, training: bool = False) -> Tensor:
    """Stochastic depth per sample (timm semantics: scale kept paths by 1/keep)."""
    if drop_prob == 0.0 or not training:
        return x
    keep = 1.0 - drop_prob
    shape = (x.shape[0],) + (1,) * (x.ndim - 1)
    mask = x.new_empty(shape).bernoulli_(keep)
    return x * mask.div_(keep)


def add_drop_path(x: Tensor, branch: Tensor, drop_prob: float = 0.0, training: bool = False,
                  gamma: Optional[Tensor] = None) -> Tensor:
    """x + drop_path(branch) (times a layer-scale ``gamma`` when given) as ONE
    elementwise kernel: x + branch * s with s = gamma * mask / keep broadcast
    per sample ([B, 1, C] or [B, 1, 1]) -- the residual endings of the Swin
    blocks (swin_transformer.py:295-296) and of the BiAttention block
    (fuse_modules.py:285-286), which the composition runs as two or three
    passes (scale, mask multiply, add).  The per-sample mask is drawn exactly
    as ``drop_path`` draws it (same generator call, same shape).  The add
    runs outside autocast, whose type promotion would insert a cast kernel for
    a bf16 branch; the kernel reads it in place and adds in fp32."""
    s = gamma
    if drop_prob > 0.0 and training:
        keep = 1.0 - drop_prob
        # in the dtype the composition's drop_path sees (gamma * branch, or
        # the branch itself), so the mask and its 1 / keep rounding match
        mdt = branch.dtype if gamma is None else torch.result_type(gamma, branch)
        mask = torch.empty((branch.shape[0],) + (1,) * (branch.ndim - 1), dtype=mdt,
                           device=branch.device).bernoulli_(keep).div_(keep)
        s = mask if s is None else s * mask
    if s is None:
        if x.dtype == torch.float32 and branch.dtype == torch.bfloat16 and x.shape == branch.shape:
            # a fp32 residual plus a bf16 branch, unscaled (the Swin blocks
            # whose drop-path rate is 0): the same kernel with a unit scale
            # reads the branch in place (PyTorch's mixed-dtype add kernel ran
            # at ~1.4 TB/s, 90 us on Swin-T stage 0)
            one = device_const(("unit_scale",), lambda: torch.ones(1, dtype=torch.float32), x.device)
            if _scale_layout(x, one) is not None:
                return _AddScaled.apply(x, branch, one)
        return x + branch
    return _AddScaled.apply(x, branch, s)


_p, _i, _i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
_lib.register("gd_box_refine_forward", [_i, _p, _i64, _i64, _i64, _p, _i64, _i64, _i64, _i64, _i64, _i64,
                                        ctypes.c_float, _p, _p])
_lib.register("gd_box_refine_backward", [_i, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64, ctypes.c_float, _p,
                                         _p, _p])
# the decoder's per-layer anchors (models/GroundingDINO/utils.query_anchors)
_lib.register("gd_query_anchor_forward", [_p] + [_i64] * 5 + [_p, _i] + [_p] * 4)
_lib.register("gd_add_scaled_forward", [_i, _p, _i, _p, _p, _i64, _i, _i64, _i64, _i, _i, _p, _p])
_lib.register("gd_add_scaled_backward", [_i, _p, _i, _p, _p, _i64, _i, _i64, _i64, _i, _p, _p, _p, _p])


_lib.register("gd_add_twin_forward", [_p, _p, _i64, _p, _p, _p, _p])


class _AddTwins(torch.autograd.Function):
    """out = a + b (fp32); the same kernel writes the bf16 copies of out and
    of a into the given buffers (out16, a16: no gradient)."""

    @staticmethod
    def forward(ctx, a, b, out16, a16):
        out = torch.empty_like(a)
        _lib.call("gd_add_twin_forward", a.data_ptr(), b.data_ptr(), a.numel(), out.data_ptr(), out16.data_ptr(),
                  _lib.ptr(a16), _lib.stream_of(a), nbytes=a.numel() * (12 + (2 if a16 is None else 4)))
        return out

    @staticmethod
    def backward(ctx, g):
        return g, g, None, None


def add_with_twins(a: Tensor, b: Tensor) -> Tensor:
    """a + b, plus bf16 twins of the sum and of ``a`` written in the same
    pass when both feed bf16-autocast Linears (the deformable encoder layer's
    query = src + pos, reference transformer.py:780-781: the query feeds the
    sampling-offset / attention-weight projections, src the value projection,
    ms_deform_attn.py:290-297) -- one kernel instead of the add and two cast
    kernels.  Elsewhere the plain add."""
    if not (_lib.enabled("addscaled") and _lib.on_device(a) and torch.is_autocast_enabled(a.device.type)
            and torch.get_autocast_dtype(a.device.type) == torch.bfloat16 and a.dtype == b.dtype == torch.float32
            and a.shape == b.shape and a.numel() % 4 == 0 and _aligned(a, b)):
        return a + b
    tw = getattr(a, "_gd_bf16", None)
    have_a = tw is not None and tw[1] == a._version and tw[0].dtype == torch.bfloat16 and tw[0].shape == a.shape
    out16 = torch.empty(a.shape, dtype=torch.bfloat16, device=a.device)
    a16 = None if have_a else torch.empty(a.shape, dtype=torch.bfloat16, device=a.device)
    out = _AddTwins.apply(a, b, out16, a16)
    out._gd_bf16 = (out16, out._version)
    if a16 is not None:
        a._gd_bf16 = (a16, a._version)
    return out


def _scale_layout(x, s):
    """(s as fp32 [Bs, 1, Cs], batch stride, channel stride) when the HIP
    kernel (csrc/residual.hip) takes x [B, N, C] and this broadcast of s,
    else None (the composition runs)."""
    if not (_lib.enabled("addscaled") and _lib.on_device(x) and x.dim() == 3 and s.dim() <= 3):
        return None
    b, _, c = x.shape
    s3 = s.reshape((1,) * (3 - s.dim()) + tuple(s.shape))
    if c % 4 or c > 1024 or s3.shape[1] != 1 or s3.shape[0] not in (1, b) or s3.shape[2] not in (1, c):
        return None
    s32 = s3.detach().float().contiguous()
    return s32, (s3.shape[2] if s3.shape[0] == b and b > 1 else 0), (1 if s3.shape[2] == c and c > 1 else 0)


def _aligned(*ts):
    return all(t.dtype in (torch.float32, torch.bfloat16) and t.data_ptr() % 16 == 0 and t.is_contiguous()
               for t in ts)


class _AddScaled(torch.autograd.Function):
    """x + branch * s, s broadcast per sample over the tokens ([B, 1, C] or
    [B, 1, 1], or one scale for all samples; fp32 or branch's dtype).

    On the GPU: one streaming kernel forward and one backward + a fixed-order
    partial merge (csrc/residual.hip: d branch = g * s in branch's dtype and
    d s = sum over the tokens of g * branch in the same pass over g).  The
    composition (CPU, GDINO_DISABLE=addscaled): an addcmul forward (outside
    autocast, whose promotion would add a cast kernel for a bf16 branch); a
    mul into a branch-dtype tensor and a ones-vector GEMM over the g * branch
    product backward (PyTorch's sum over dim 1 of a [2, 22223, 256] tensor ran
    at ~0.35 TB/s)."""

    @staticmethod
    def forward(ctx, x, branch, s):
        # the branch is only needed for d s (a layer-scale gamma); a drop-path
        # mask needs no gradient, and keeping the branch alive until backward
        # would hold one activation per residual for nothing
        ctx.save_for_backward(branch if ctx.needs_input_grad[2] else None, s)
        ctx.branch_meta = (branch.shape, branch.dtype)
        lay = _scale_layout(x, s) if x.shape == branch.shape else None
        out_dtype = torch.promote_types(torch.promote_types(x.dtype, branch.dtype), s.dtype)
        if lay is not None:
            xc, bc = x.contiguous(), branch.contiguous()
            out = torch.empty(x.shape, dtype=out_dtype, device=x.device)
            if _aligned(xc, bc, out):
                s32, sbs, scs = lay
                bsz, n, c = x.shape
                _lib.call("gd_add_scaled_forward", _lib.dtype_code(xc), xc.data_ptr(), _lib.dtype_code(bc),
                          bc.data_ptr(), s32.data_ptr(), sbs, scs, bsz, n, c, _lib.dtype_code(out),
                          out.data_ptr(), _lib.stream_of(x),
                          nbytes=x.numel() * (xc.element_size() + bc.element_size() + out.element_size()))
                ctx.kernel = True
                ctx.lay = lay  # the backward reuses the fp32 scale (no second cast kernel)
                return out
        ctx.kernel = False
        with torch.autocast(device_type=x.device.type, enabled=False):
            return torch.addcmul(x, branch, s)

    @staticmethod
    def backward(ctx, g):
        branch, s = ctx.saved_tensors
        if ctx.kernel:
            return _AddScaled._backward_kernel(ctx, g, branch, s)
        gb = gs = None
        if ctx.needs_input_grad[1]:
            shape, dtype = ctx.branch_meta
            gb = torch.empty(shape, dtype=dtype, device=g.device)
            torch.mul(g, s, out=gb)
        if ctx.needs_input_grad[2]:
            c = g.shape[-1]
            cs = c if s.shape[-1] == c else 1
            prod = torch.mul(g, branch)
            if s.dim() < g.dim() or s.shape[0] == 1:  # one scale for every sample ([C] or [1, 1, C])
                p2 = prod.reshape(-1, c)
                gs = (p2.new_ones(1, p2.shape[0]) @ p2).reshape(-1)
                gs = gs if cs == c else gs.sum(-1, keepdim=True)
            else:  # per sample: [B, 1, C] / [B, 1, 1]
                b = g.shape[0]
                p3 = prod.reshape(b, -1, c)
                gs = torch.bmm(p3.new_ones(b, 1, p3.shape[1]), p3)  # [b, 1, c]
                gs = gs if cs == c else gs.sum(-1, keepdim=True)
            gs = gs.reshape(s.shape).to(s.dtype)
        return g if ctx.needs_input_grad[0] else None, gb, gs

    @staticmethod
    def _backward_kernel(ctx, g, branch, s):
        shape, dtype = ctx.branch_meta
        bsz, n, c = shape
        s32, sbs, scs = ctx.lay
        g = g.contiguous()
        if g.dtype not in (torch.float32, torch.bfloat16):
            g = g.float()
        want_b, want_s = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        gb = torch.empty(shape, dtype=dtype, device=g.device) if want_b else None
        gs_bc = ws = None
        if want_s:
            gs_bc = torch.empty(bsz, c, dtype=torch.float32, device=g.device)
            fn = _lib.lib().gd_add_scaled_workspace_bytes
            fn.restype, fn.argtypes = ctypes.c_size_t, [_i64, _i64, _i]
            ws = torch.empty((int(fn(bsz, n, c)) + 3) // 4, dtype=torch.float32, device=g.device)
            branch = branch.contiguous()
        if (want_b or want_s) and _aligned(*[t for t in (g, gb, branch if want_s else None) if t is not None]):
            _lib.call("gd_add_scaled_backward", _lib.dtype_code(g), g.data_ptr(), _lib.dtype_code(branch)
                      if want_s else _lib.dtype_code(gb), _lib.ptr(branch if want_s else None), s32.data_ptr(),
                      sbs, scs, bsz, n, c, _lib.ptr(gb), _lib.ptr(gs_bc), _lib.ptr(ws), _lib.stream_of(g),
                      nbytes=g.numel() * (g.element_size() + (2 * gb.element_size() if want_b else 0)
                                          + (branch.element_size() if want_s else 0)))
        elif want_b or want_s:  # unaligned views: the composition
            if want_b:
                torch.mul(g, s, out=gb)
            if want_s:
                gs_bc = torch.mul(g, branch).float().sum(1)
        gs = None
        if want_s:
            s3 = s.reshape((1,) * (3 - s.dim()) + tuple(s.shape))
            if s3.shape[2] == 1:
                gs_bc = gs_bc.sum(-1, keepdim=True)
            if s3.shape[0] == 1:
                gs_bc = gs_bc.sum(0, keepdim=True)
            gs = gs_bc.reshape(s.shape).to(s.dtype)
        return g if ctx.needs_input_grad[0] else None, gb, gs


class DropPath(nn.Module):
    def __init__(self, drop_prob: float = 0.0):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        return drop_path(x, self.drop_prob, self.training)

    def extra_repr(self):
        return f"drop_prob={self.drop_prob}"


def trunc_normal_(tensor: Tensor, mean=0.0, std=1.0, a=-2.0, b=2.0) -> Tensor:
    with torch.no_grad():
        return nn.init.trunc_normal_(tensor, mean=mean, std=std, a=a, b=b)


def to_2tuple(x):
    return tuple(x) if isinstance(x, (tuple, list)) else (x, x)


def clean_state_dict(state_dict):
    """Strip DDP's ``module.`` prefix (util/misc.py:620-626)."""
    return {(k[7:] if k.startswith("module.") else k): v for k, v in state_dict.items()}


def accuracy(output, target, topk=(1,)):
    if target.numel() == 0:
        return [torch.zeros([], device=output.device)]
    maxk = max(topk)
    _, pred = output.topk(maxk, 1, True, True)
    correct = pred.t().eq(target.view(1, -1).expand_as(pred.t()))
    return [correct[:k].reshape(-1).float().sum(0).mul_(100.0 / target.size(0)) for k in topk]


def sigmoid_focal_loss(inputs, targets, num_boxes, alpha: float = 0.25, gamma: float = 2,
                       no_reduction=False):
    """RetinaNet focal loss (reference utils.py:152-181)."""
    prob = inputs.sigmoid()
    ce = nn.functional.binary_cross_entropy_with_logits(inputs, targets, reduction="none")
    p_t = prob * targets + (1 - prob) * (1 - targets)
    loss = ce * ((1 - p_t) ** gamma)
    if alpha >= 0:
        loss = (alpha * targets + (1 - alpha) * (1 - targets)) * loss
    if no_reduction:
        return loss
    return loss.mean(1).sum() / num_boxes


__all__ = [n for n in dir() if not n.startswith("_") and n not in ("math", "List", "Optional")]
