"""Text-enhancer encoder layer (reference transformer_vanilla.py:72-123):
post-norm self-attention over the text tokens with the phrase mask, then FFN.
Attention runs through gdino_amd.mha (nn.MultiheadAttention layout)."""
from typing import Optional

import torch
from torch import Tensor, nn

from gdino_amd.layernorm import add_norm
from gdino_amd.mha import MultiheadAttention

from .utils import _get_activation_fn, _get_clones, ffn


class TransformerEncoderLayer(nn.Module):
    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation="relu",
                 normalize_before=False):
        super().__init__()
        self.self_attn = MultiheadAttention(d_model, nhead, dropout=dropout)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.dropout = nn.Dropout(dropout)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.dropout1 = nn.Dropout(dropout)
        self.dropout2 = nn.Dropout(dropout)
        self.activation = _get_activation_fn(activation)
        self.normalize_before = normalize_before
        self.nhead = nhead

    def forward(self, src, src_mask: Optional[Tensor] = None, src_key_padding_mask: Optional[Tensor] = None,
                pos: Optional[Tensor] = None):
        # src [T, B, C] sequence-first.  A per-sample [B, T, T] mask is tiled
        # head-major with .repeat (reference :106-108) and then read by the
        # attention in batch-major (b*H + h) order, exactly as the reference's
        # nn.MultiheadAttention call does; with B > 1 the heads therefore see
        # interleaved samples' masks.  Kept bit-for-bit (parity); the padding
        # mask is not passed, also as in the reference (:113-115).
        if src_mask is not None and src_mask.dim() == 3 and src_mask.shape[0] == src.shape[1]:
            src_mask = src_mask.repeat(self.nhead, 1, 1)
        qk = src if pos is None else src + pos
        attn = self.self_attn(qk, qk, value=src, attn_mask=src_mask)[0]
        src = add_norm(self.norm1, src, self.dropout1(attn))
        y = ffn(self.linear1, self.activation, self.dropout, self.linear2, src)
        return add_norm(self.norm2, src, self.dropout2(y))


class TextTransformer(nn.Module):
    def __init__(self, num_layers, d_model=256, nheads=8, dim_feedforward=2048, dropout=0.1):
        super().__init__()
        self.num_layers = num_layers
        self.d_model = d_model
        self.nheads = nheads
        self.dim_feedforward = dim_feedforward
        self.norm = None
        layer = TransformerEncoderLayer(d_model=d_model, nhead=nheads, dim_feedforward=dim_feedforward,
                                        dropout=dropout)
        self.layers = _get_clones(layer, num_layers)

    def forward(self, memory_text: torch.Tensor, text_attention_mask: torch.Tensor):
        out = memory_text.transpose(0, 1)
        for layer in self.layers:
            out = layer(out, src_key_padding_mask=text_attention_mask)
        if self.norm is not None:
            out = self.norm(out)
        return out.transpose(0, 1)
