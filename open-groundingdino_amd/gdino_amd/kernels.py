"""Dispatch points of the fused attention-family ops on the hot path.

Every model module calls the ops below instead of composing them from torch
primitives, so that the implementation behind each op is one swap:

  window_attention   Swin W-MSA / SW-MSA core   swin_transformer.py:134-174
  window_attention_packed  the same on the packed qkv Linear output with the
                     bias table + index (what WindowAttention.forward calls)
  window_attention_image  the same on the unpartitioned image's qkv, with the
                     Swin block's pad / roll / partition / reverse / crop
                     (swin_transformer.py:250-290) fused in
  attention          masked attention (BERT self-attn, text enhancer, decoder
                     self-attn and text cross-attn): gdino_amd/attn.py
  bi_attention       BiMultiHeadAttention core   fuse_modules.py:162-246
  contrastive_logits ContrastiveEmbed            utils.py:242-273
  contrastive_rowmax its max over tokens, the two-stage proposal score
                     (transformer.py:292-296), without the [B, S, 256] logits

``IMPL[name]`` selects the implementation; ``"hip"`` entries are the
hand-written gfx950 kernels of csrc/ (registered by their modules when the
library provides them), ``"torch"`` entries compose ROCm library kernels
(hipBLASLt GEMMs, PyTorch's flash/mem-efficient SDPA) and are what an op uses
until its HIP kernel lands.  Tests may install oracle implementations through
``override`` — the product never imports the oracle.
"""
from __future__ import annotations

import contextlib
from typing import Callable, Dict, Optional

import torch
import torch.nn.functional as F

_REGISTRY: Dict[str, Dict[str, Callable]] = {}
IMPL: Dict[str, str] = {}


def register(op: str, impl: str, fn: Callable, default: bool = False) -> None:
    _REGISTRY.setdefault(op, {})[impl] = fn
    if default or op not in IMPL:
        IMPL[op] = impl


def get(op: str) -> Callable:
    return _REGISTRY[op][IMPL[op]]


@contextlib.contextmanager
def override(op: str, fn: Callable):
    """Temporarily route ``op`` to ``fn`` (tests)."""
    register(op, "_override", fn)
    prev = IMPL[op]
    IMPL[op] = "_override"
    try:
        yield
    finally:
        IMPL[op] = prev


# ---------------------------------------------------------------------------
# torch-composed implementations (ROCm library kernels)
# ---------------------------------------------------------------------------
def _window_attention_torch(q, k, v, bias, mask, scale):
    """q, k, v: [B_, nH, N, hd]; bias: [nH, N, N]; mask: [nW, N, N] or None
    (0 / -100 entries, windows of one image consecutive).  -> [B_, nH, N, hd]"""
    attn = (q * scale) @ k.transpose(-2, -1)
    attn = attn + bias.unsqueeze(0).to(attn.dtype)
    if mask is not None:
        nw = mask.shape[0]
        b_, nh, n, _ = attn.shape
        attn = attn.view(b_ // nw, nw, nh, n, n) + mask.to(attn.dtype)[None, :, None]
        attn = attn.view(b_, nh, n, n)
    attn = attn.softmax(-1)
    return attn @ v


def _attention_torch(q, k, v, attn_mask: Optional[torch.Tensor] = None, scale: Optional[float] = None,
                     dropout_p: float = 0.0):
    """q: [B, H, Lq, hd], k/v: [B, H, Lk, hd]; attn_mask additive float
    broadcastable to [B, H, Lq, Lk] or bool (True = attend)."""
    return F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask, dropout_p=dropout_p, scale=scale)


def _contrastive_torch(x, text, text_token_mask, max_text_len):
    """x [B, Q, C] . text [B, T, C]^T, -inf on padded tokens, right-padded with
    -inf to max_text_len -> [B, Q, max_text_len] (fp32 like the reference's
    torch.full default dtype)."""
    res = x @ text.transpose(-1, -2)
    out = torch.full((*res.shape[:-1], max_text_len), float("-inf"), device=res.device, dtype=torch.float32)
    t = res.shape[-1]
    out[..., :t] = res.float().masked_fill(~text_token_mask[:, None, :], float("-inf"))
    return out


def _bi_attention_torch(q, k, v_v, v_l, pad_v=None, pad_l=None, dropout_p=0.0):
    """BiMultiHeadAttention core as two fused softmax attentions over ONE
    score matrix s = q.k^T ([B*H, S, T] never materialised):

      out_v = softmax_T(s + mask_l) . v_l        [B*H, S, hd]
      out_l = softmax_S(s^T + mask_v) . v_v      [B*H, T, hd]

    q: [B, H, S, hd] (already scaled), k/v_l: [B, H, T, hd], v_v: [B, H, S, hd];
    pad_v [B, S] / pad_l [B, T] True = padding.

    The reference (fuse_modules.py:174-217) subtracts the global max, then
    the per-token column max, and clamps to +-5e4 before each softmax.
    Softmax is shift-invariant, so the subtractions change nothing and the
    clamps only act where scores spread by more than 5e4 -- the reference's
    own fp16 guard; with fp32 softmax statistics that case does not arise.
    """
    keep_l = None if pad_l is None else ~pad_l[:, None, None, :]
    keep_v = None if pad_v is None else ~pad_v[:, None, None, :]
    out_v = F.scaled_dot_product_attention(q, k, v_l, attn_mask=keep_l, dropout_p=dropout_p, scale=1.0)
    out_l = F.scaled_dot_product_attention(k, q, v_v, attn_mask=keep_v, dropout_p=dropout_p, scale=1.0)
    return out_v, out_l


register("bi_attention", "torch", _bi_attention_torch)
register("window_attention", "torch", _window_attention_torch)
register("attention", "torch", _attention_torch)
register("contrastive_logits", "torch", _contrastive_torch)


def window_attention(q, k, v, bias, mask, scale):
    return get("window_attention")(q, k, v, bias, mask, scale)


def window_attention_packed(qkv, table, rel_index, mask, scale):
    """qkv [B_, N, 3, nH, hd], table [(2Wh-1)(2Ww-1), nH], rel_index [N*N],
    mask [nW, N, N] or None -> [B_, N, nH*hd] (gdino_amd/wattn.py)."""
    return get("window_attention_packed")(qkv, table, rel_index, mask, scale)


def window_attention_image(qkv, qkv_bias, table, rel_index, mask, hw, ws, shift, scale):
    """qkv [B, H*W, 3C] (the qkv Linear of the normed tokens), qkv_bias [3C]
    or None, mask [nW, N, N] (used when shift > 0) -> [B, H*W, C]
    (gdino_amd/wattn.py)."""
    return get("window_attention_image")(qkv, qkv_bias, table, rel_index, mask, hw, ws, shift, scale)


def attention(q, k, v, attn_mask=None, scale=None, dropout_p=0.0):
    return get("attention")(q, k, v, attn_mask, scale, dropout_p)


def bi_attention(*args, **kw):
    return get("bi_attention")(*args, **kw)


def contrastive_logits(x, text, text_token_mask, max_text_len):
    return get("contrastive_logits")(x, text, text_token_mask, max_text_len)


def contrastive_rowmax(x, text, text_token_mask):
    """max_t contrastive_logits(x, text, mask)[..., t] -> [B, Q] fp32, no grad."""
    return get("contrastive_rowmax")(x, text, text_token_mask)


# HIP implementations register themselves as the defaults for CUDA tensors.
from . import biattn  # noqa: E402,F401
from . import wattn  # noqa: E402,F401
from . import attn  # noqa: E402,F401
from . import contrastive  # noqa: E402,F401
from . import msda_prologue  # noqa: E402,F401
from . import wgrad  # noqa: E402,F401
from . import layernorm  # noqa: E402,F401
from . import lsap  # noqa: E402,F401  (the device Hungarian matching)
