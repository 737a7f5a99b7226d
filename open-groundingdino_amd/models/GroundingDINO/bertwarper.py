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
        enc = self.encoder(hidden, attention_mask=keep)
        seq = enc[0] if isinstance(enc, (tuple, list)) else enc.last_hidden_state
        pooled = self.pooler(seq) if self.pooler is not None else None
        return {"last_hidden_state": seq, "pooler_output": pooled}


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
