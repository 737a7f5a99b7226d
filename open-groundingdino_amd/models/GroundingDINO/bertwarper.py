"""BERT text encoder wrapper and sub-sentence masks.

``BertModelWarper`` keeps the reference's structure and state-dict names
(models/GroundingDINO/bertwarper.py:17-166: ``bert.embeddings.*``,
``bert.encoder.layer.N.*``, ``bert.pooler.*`` of a HF BertModel) and its
call contract (``input_ids``, 3-D ``attention_mask`` [B, T, T] block-diagonal
per phrase, ``position_ids`` restarting per phrase).  Self-attention runs
through ``gdino_amd.kernels.attention`` via transformers' attention-interface
registry (``config._attn_implementation = "gdino_amd"``).  The reference body
calls ``get_head_mask`` / a 3-argument ``get_extended_attention_mask``, both
gone from transformers 5.x; the 3-D mask is handed to the
attention op as a boolean keep-mask, equivalent to the reference's additive
``(1 - m) * finfo.min`` because no row of the block-diagonal mask is empty.

``generate_masks_with_special_tokens[_and_transfer_map]`` produce the same
masks as bertwarper.py:176-273 but on the host from the CPU token ids with
numpy (no per-special-token device indexing / host syncs), then move once.
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch
from torch import nn

from gdino_amd import kernels

_IMPL_NAME = "gdino_amd"


def _hf_attention(module, query, key, value, attention_mask, scaling=None, dropout=0.0, **kwargs):
    """transformers attention interface -> kernels.attention.
    q/k/v [B, H, T, hd]; returns ([B, T, H, hd], None)."""
    mask = attention_mask
    if mask is not None and mask.dtype != torch.bool and mask.dtype != query.dtype:
        mask = mask.to(query.dtype)
    out = kernels.attention(query, key, value, mask, scaling, dropout)
    return out.transpose(1, 2).contiguous(), None


def _register_interface():
    from transformers import AttentionInterface
    AttentionInterface.register(_IMPL_NAME, _hf_attention)


class BertModelWarper(nn.Module):
    def __init__(self, bert_model):
        super().__init__()
        _register_interface()
        self.config = bert_model.config
        self.config._attn_implementation = _IMPL_NAME
        self.embeddings = bert_model.embeddings
        self.encoder = bert_model.encoder
        self.pooler = bert_model.pooler

    def forward(self, input_ids=None, attention_mask=None, token_type_ids=None, position_ids=None,
                head_mask=None, inputs_embeds=None, return_dict=True, **kwargs):
        if (input_ids is None) == (inputs_embeds is None):
            raise ValueError("You have to specify exactly one of input_ids or inputs_embeds")
        ref = input_ids if input_ids is not None else inputs_embeds[..., 0]
        b, t = ref.shape[:2]
        device = ref.device
        if attention_mask is None:
            attention_mask = torch.ones((b, t), dtype=torch.bool, device=device)
        if token_type_ids is None:
            token_type_ids = torch.zeros((b, t), dtype=torch.long, device=device)
        keep = attention_mask.bool()
        if keep.dim() == 2:  # padding mask -> [B, 1, 1, T]
            keep = keep[:, None, None, :]
        elif keep.dim() == 3:  # [B, T, T] -> [B, 1, T, T]
            keep = keep[:, None]
        hidden = self.embeddings(input_ids=input_ids, position_ids=position_ids,
                                 token_type_ids=token_type_ids, inputs_embeds=inputs_embeds)
        if self._fast_ok(hidden, head_mask):
            seq = self._encode_frozen(hidden, keep)
        else:
            enc = self.encoder(hidden, attention_mask=keep)
            seq = enc[0] if isinstance(enc, (tuple, list)) else enc.last_hidden_state
        pooled = self.pooler(seq) if self.pooler is not None else None
        return {"last_hidden_state": seq, "pooler_output": pooled}

    # GDINO_BERT_FAST=0: the transformers layer stack (A/B)
    FAST = True

    def _fast_ok(self, hidden, head_mask) -> bool:
        """The frozen-encoder path: every encoder parameter frozen (cfg
        freeze_keywords ['bert'], train.apply_freeze) and nothing upstream
        needing a gradient, or no autograd; bf16
        autocast on the HIP device, the stock post-norm GELU BERT layout."""
        import os
        from gdino_amd import _lib, castcache
        from gdino_amd.layernorm import WIDTHS
        cfg = self.config
        return (self.FAST and os.environ.get("GDINO_BERT_FAST", "1") != "0" and head_mask is None
                and _lib.on_device(hidden) and castcache.autocast_dtype(hidden) == torch.bfloat16
                and cfg.hidden_act == "gelu" and not getattr(cfg, "is_decoder", False)
                and cfg.hidden_size in WIDTHS and cfg.hidden_size % cfg.num_attention_heads == 0
                and (cfg.hidden_size // cfg.num_attention_heads) in (32, 64)
                and (not torch.is_grad_enabled() or not any(p.requires_grad for p in self.encoder.parameters()))
                # trainable embeddings (a partial freeze) need the module
                # stack: the frozen path runs under no_grad
                and not (torch.is_grad_enabled() and hidden.requires_grad))

    def _encode_frozen(self, hidden, keep):
        """The 12 BertLayers (transformers modeling_bert BertLayer: self
        attention, BertSelfOutput, BertIntermediate, BertOutput) on the
        product's kernels, with nothing to differentiate: Q, K and V as ONE
        GEMM against the cached concatenated bf16 weight, the masked-attention
        kernel reading q / k / v in place from it (attention dropout in the
        kernel), and each ``LayerNorm(dropout(dense(x)) + residual)`` as the
        add + LayerNorm kernel, whose bf16 twin feeds the next GEMM (no cast
        kernels).  The same arithmetic as the module stack under bf16
        autocast (bf16 GEMMs, fp32 residual stream and LayerNorm, bf16 GELU)
        up to the summation order of the fused Q/K/V product."""
        import torch.nn.functional as F

        from gdino_amd import castcache
        from gdino_amd.layernorm import add_norm
        cfg = self.config
        dt = torch.bfloat16
        b, t, c = hidden.shape
        nh = cfg.num_attention_heads
        hd = c // nh

        # the Dropout modules' own rates and modes (callers may zero them), as
        # the module stack reads them
        def drop(x, m):
            return F.dropout(x, m.p, m.training)

        def lin(x, layer):
            return F.linear(x, castcache.cached_cast(layer.weight, dt), castcache.cached_cast(layer.bias, dt))

        def as16(h):
            tw = getattr(h, "_gd_bf16", None)
            if tw is not None and tw[1] == h._version and tw[0].shape == h.shape:
                return tw[0]
            return h.to(dt)

        with torch.no_grad():
            h = hidden
            for layer in self.encoder.layer:
                sa = layer.attention.self
                wqkv = castcache._cached_cat([sa.query.weight, sa.key.weight, sa.value.weight], dt)
                bqkv = castcache._cached_cat([sa.query.bias, sa.key.bias, sa.value.bias], dt)
                qkv = F.linear(as16(h), wqkv, bqkv)                       # [B, T, 3C]
                q, k, v = (qkv[..., i * c:(i + 1) * c].view(b, t, nh, hd).transpose(1, 2) for i in range(3))
                # [B, H, T, hd] over [B, T, H, hd] storage
                ctx = kernels.attention(q, k, v, keep, hd ** -0.5, sa.dropout.p if sa.dropout.training else 0.0)
                ctx = ctx.transpose(1, 2).reshape(b, t, c)
                so = layer.attention.output
                h = add_norm(so.LayerNorm, h, drop(lin(ctx, so.dense), so.dropout))
                inter = F.gelu(lin(as16(h), layer.intermediate.dense))
                out = layer.output
                h = add_norm(out.LayerNorm, h, drop(lin(inter, out.dense), out.dropout))
        return h


class TextEncoderShell(nn.Module):
    def __init__(self, text_encoder):
        super().__init__()
        self.text_encoder = text_encoder
        self.config = self.text_encoder.config

    def forward(self, **kw):
        return self.text_encoder(**kw)


def _phrase_blocks(ids: np.ndarray, special_ids) -> tuple:
    """Host computation of the reference's phrase blocks.

    For every special token at column c (not the first / last column) the
    block (prev, c] — prev = the previous special column of that row — gets
    full attention and position ids 0..len-1; columns 0 and T-1 only see
    themselves (bertwarper.py:240-262)."""
    b, t = ids.shape
    special = np.isin(ids, np.asarray(list(special_ids), dtype=ids.dtype))
    mask = np.zeros((b, t, t), dtype=bool)
    idx = np.arange(t)
    mask[:, idx, idx] = True
    pos = np.zeros((b, t), dtype=np.int64)
    cate = [[] for _ in range(b)]
    for r in range(b):
        prev = 0
        for c in np.flatnonzero(special[r]):
            if c == 0 or c == t - 1:
                pos[r, c] = 0
            else:
                mask[r, prev + 1:c + 1, prev + 1:c + 1] = True
                pos[r, prev + 1:c + 1] = np.arange(c - prev)
                m = np.zeros(t, dtype=bool)
                m[prev + 1:c] = True
                cate[r].append(m)
            prev = c
    return mask, pos, cate


def generate_masks_with_special_tokens(tokenized, special_tokens_list, tokenizer):
    ids = tokenized["input_ids"]
    mask, pos, _ = _phrase_blocks(ids.cpu().numpy(), special_tokens_list)
    return (torch.from_numpy(mask).to(ids.device),
            torch.from_numpy(pos).to(ids.device))


def generate_masks_with_special_tokens_and_transfer_map(tokenized, special_tokens_list, tokenizer):
    ids = tokenized["input_ids"]
    mask, pos, cate = _phrase_blocks(ids.cpu().numpy(), special_tokens_list)
    dev = ids.device
    cate_t: List[torch.Tensor] = [
        torch.from_numpy(np.stack(c)).to(dev) if c else torch.zeros((0, ids.shape[1]), dtype=torch.bool, device=dev)
        for c in cate]
    return (torch.from_numpy(mask).to(dev),
            torch.from_numpy(pos).to(dev), cate_t)
