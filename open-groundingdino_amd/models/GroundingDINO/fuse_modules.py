"""Image <-> text feature fusion (reference fuse_modules.py:99-295).

``BiMultiHeadAttention`` keeps the reference's projections and parameter
names; its core (one score matrix, softmax over text tokens for the image
side and over image tokens for the text side) runs through
``gdino_amd.kernels.bi_attention`` — without materialising the
[B*H, S, T] score matrix the reference builds twice (182 MB fp32 each at
800x1333, bs=2; SURVEY §7 hard part 4).  ``BiAttentionBlock`` adds the
pre-LayerNorms, layer-scale gammas (init 1e-4) and DropPath as the reference.
"""
import torch
import torch.nn as nn

from gdino_amd import biattn, kernels
from gdino_amd import castcache
from gdino_amd.layernorm import layer_norm
from gdino_amd.misc import DropPath, add_drop_path


class BiMultiHeadAttention(nn.Module):
    def __init__(self, v_dim, l_dim, embed_dim, num_heads, dropout=0.1, cfg=None):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        self.v_dim = v_dim
        self.l_dim = l_dim
        assert self.head_dim * num_heads == embed_dim, (
            f"embed_dim must be divisible by num_heads (got `embed_dim`: {embed_dim} and `num_heads`: {num_heads}).")
        self.scale = self.head_dim ** (-0.5)
        self.dropout = dropout
        self.v_proj = nn.Linear(v_dim, embed_dim)
        self.l_proj = nn.Linear(l_dim, embed_dim)
        self.values_v_proj = nn.Linear(v_dim, embed_dim)
        self.values_l_proj = nn.Linear(l_dim, embed_dim)
        self.out_v_proj = nn.Linear(embed_dim, v_dim)
        self.out_l_proj = nn.Linear(embed_dim, l_dim)
        self.stable_softmax_2d = True
        self.clamp_min_for_underflow = True
        self.clamp_max_for_overflow = True
        self._reset_parameters()

    def _reset_parameters(self):
        for lin in (self.v_proj, self.l_proj, self.values_v_proj, self.values_l_proj, self.out_v_proj,
                    self.out_l_proj):
            nn.init.xavier_uniform_(lin.weight)
            lin.bias.data.fill_(0)

    def _heads(self, x):
        b, n, _ = x.shape
        return x.view(b, n, self.num_heads, self.head_dim).transpose(1, 2)

    def forward(self, v, l, attention_mask_v=None, attention_mask_l=None):
        """v [B, S, v_dim], l [B, T, l_dim]; masks True = padding."""
        b, s, _ = v.shape
        t = l.shape[1]
        # projections sharing an input run as one GEMM on the training path
        p = self.dropout if self.training else 0.0
        if p == 0.0:
            # token-major core (gdino_amd/biattn.py) on the joint projection
            # outputs: no head-split copies, no split / concatenation
            qvv = castcache.linear_shared_input_joint(v, (self.v_proj, self.values_v_proj))
            klv = castcache.linear_shared_input_joint(l, (self.l_proj, self.values_l_proj))
            if biattn.tokens_ok(qvv, klv, self.num_heads):
                out_v, out_l = biattn.bi_attention_tokens(qvv, klv, attention_mask_v, attention_mask_l,
                                                          self.num_heads, self.scale)
                return self.out_v_proj(out_v), self.out_l_proj(out_l)
            if qvv is not None and klv is not None:
                from gdino_amd.misc import split_last
                qv, vv = split_last(qvv, [self.embed_dim, self.embed_dim])
                kl, vl = split_last(klv, [self.embed_dim, self.embed_dim])
            else:
                qv, vv = castcache.linear_shared_input(v, (self.v_proj, self.values_v_proj))
                kl, vl = castcache.linear_shared_input(l, (self.l_proj, self.values_l_proj))
        else:
            qv, vv = castcache.linear_shared_input(v, (self.v_proj, self.values_v_proj))
            kl, vl = castcache.linear_shared_input(l, (self.l_proj, self.values_l_proj))
        q = self._heads(qv * self.scale)
        k, vv, vl = self._heads(kl), self._heads(vv), self._heads(vl)
        out_v, out_l = kernels.bi_attention(q, k, vv, vl, attention_mask_v, attention_mask_l, p)
        out_v = out_v.transpose(1, 2).reshape(b, s, self.embed_dim)
        out_l = out_l.transpose(1, 2).reshape(b, t, self.embed_dim)
        return self.out_v_proj(out_v), self.out_l_proj(out_l)


class BiAttentionBlock(nn.Module):
    def __init__(self, v_dim, l_dim, embed_dim, num_heads, dropout=0.1, drop_path=0.0, init_values=1e-4,
                 cfg=None):
        super().__init__()
        self.layer_norm_v = nn.LayerNorm(v_dim)
        self.layer_norm_l = nn.LayerNorm(l_dim)
        self.attn = BiMultiHeadAttention(v_dim=v_dim, l_dim=l_dim, embed_dim=embed_dim, num_heads=num_heads,
                                         dropout=dropout)
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()
        self.gamma_v = nn.Parameter(init_values * torch.ones(v_dim), requires_grad=True)
        self.gamma_l = nn.Parameter(init_values * torch.ones(l_dim), requires_grad=True)

    def forward(self, v, l, attention_mask_v=None, attention_mask_l=None):
        v = layer_norm(self.layer_norm_v, v)  # HIP LayerNorm (+ bf16 copy for the projections)
        l = layer_norm(self.layer_norm_l, l)
        dv, dl = self.attn(v, l, attention_mask_v=attention_mask_v, attention_mask_l=attention_mask_l)
        # v + drop_path(gamma_v * dv) as one kernel each (misc.add_drop_path)
        dp = self.drop_path.drop_prob if isinstance(self.drop_path, DropPath) else 0.0
        return (add_drop_path(v, dv, dp, self.training, self.gamma_v),
                add_drop_path(l, dl, dp, self.training, self.gamma_l))
