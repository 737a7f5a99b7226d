"""Swin Transformer backbone (Swin-T/B/L) for Grounding DINO.

Architecture, parameter names and init follow the reference
(models/GroundingDINO/backbone/swin_transformer.py:24-791) so checkpoints load
unchanged; the window-attention core (q*scale @ k^T + relative-position bias
+ shifted-window mask, softmax, @ v — swin_transformer.py:134-174) runs through
``gdino_amd.kernels.window_attention``.

Host-side differences (behaviour-preserving): the shifted-window mask and the
gathered relative-position bias are computed once per (padded size, device)
and cached instead of being rebuilt on every forward (reference :402-426
rebuilds a [Hp, Wp] image mask with Python slicing each call).
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.utils.checkpoint as checkpoint

from gdino_amd.conv import GemmConv2d
from gdino_amd import castcache, kernels
from gdino_amd.layernorm import add_scaled_norm, layer_norm
from gdino_amd.misc import DropPath, NestedTensor, add_drop_path, to_2tuple, trunc_normal_


class Mlp(nn.Module):
    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.0):
        super().__init__()
        hidden_features = hidden_features or in_features
        out_features = out_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        return self.drop(self.fc2(self.drop(self.act(self.fc1(x)))))


def window_partition(x, ws):
    """[B, H, W, C] -> [B*nW, ws, ws, C] (windows of one image consecutive)."""
    b, h, w, c = x.shape
    x = x.view(b, h // ws, ws, w // ws, ws, c).permute(0, 1, 3, 2, 4, 5)
    return x.reshape(-1, ws, ws, c)


def window_reverse(windows, ws, h, w):
    """[B*nW, ws, ws, C] -> [B, H, W, C]."""
    b = windows.shape[0] // ((h // ws) * (w // ws))
    x = windows.view(b, h // ws, w // ws, ws, ws, -1).permute(0, 1, 3, 2, 4, 5)
    return x.reshape(b, h, w, -1)


def relative_position_index(wh: int, ww: int) -> torch.Tensor:
    """[wh*ww, wh*ww] index into the (2wh-1)(2ww-1) bias table."""
    ys, xs = torch.meshgrid(torch.arange(wh), torch.arange(ww), indexing="ij")
    pos = torch.stack([ys.flatten(), xs.flatten()])  # [2, N]
    rel = (pos[:, :, None] - pos[:, None, :]).permute(1, 2, 0)  # [N, N, 2]
    return (rel[..., 0] + wh - 1) * (2 * ww - 1) + (rel[..., 1] + ww - 1)


class WindowAttention(nn.Module):
    """W-MSA / SW-MSA with relative position bias (reference :77-174)."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=True, qk_scale=None, attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.dim = dim
        self.window_size = window_size
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * window_size[0] - 1) * (2 * window_size[1] - 1), num_heads))
        self.register_buffer("relative_position_index", relative_position_index(*window_size))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        trunc_normal_(self.relative_position_bias_table, std=0.02)

    def position_bias(self) -> torch.Tensor:
        n = self.window_size[0] * self.window_size[1]
        bias = self.relative_position_bias_table[self.relative_position_index.view(-1)]
        return bias.view(n, n, -1).permute(2, 0, 1).contiguous()  # [nH, N, N]

    def forward(self, x, mask=None):
        """x: [B*nW, N, C]; mask: [nW, N, N] (0 / -100) or None."""
        b_, n, c = x.shape
        qkv = self.qkv(x).view(b_, n, 3, self.num_heads, c // self.num_heads)
        if self.attn_drop.p > 0.0 and self.training:
            # attention-probability dropout (attn_drop_rate > 0; 0 in every
            # Grounding DINO config) is not fused: eager composition
            q, k, v = qkv.permute(2, 0, 3, 1, 4)
            attn = (q * self.scale) @ k.transpose(-2, -1) + self.position_bias().unsqueeze(0).to(q.dtype)
            if mask is not None:
                nw = mask.shape[0]
                attn = (attn.view(b_ // nw, nw, self.num_heads, n, n) + mask.to(attn.dtype)[None, :, None])
                attn = attn.view(b_, self.num_heads, n, n)
            out = (self.attn_drop(attn.softmax(-1)) @ v).transpose(1, 2).reshape(b_, n, c)
        else:
            # one fused kernel: bias gather, shift mask, softmax, both products
            # (gdino_amd/wattn.py, csrc/wattn.hip); reads qkv in place, writes
            # the [B_, N, C] layout proj reads
            out = kernels.window_attention_packed(qkv, self.relative_position_bias_table,
                                                  self.relative_position_index.view(-1), mask, self.scale)
        return self.proj_drop(self.proj(out))


class SwinTransformerBlock(nn.Module):
    def __init__(self, dim, num_heads, window_size=7, shift_size=0, mlp_ratio=4.0, qkv_bias=True,
                 qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0, act_layer=nn.GELU,
                 norm_layer=nn.LayerNorm):
        super().__init__()
        assert 0 <= shift_size < window_size, "shift_size must in 0-window_size"
        self.dim = dim
        self.num_heads = num_heads
        self.window_size = window_size
        self.shift_size = shift_size
        self.mlp_ratio = mlp_ratio
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(dim, to_2tuple(window_size), num_heads, qkv_bias, qk_scale, attn_drop, drop)
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(dim, int(dim * mlp_ratio), act_layer=act_layer, drop=drop)
        self.H = self.W = None

    def forward(self, x, mask_matrix, normed=None, next_norm=None):
        """normed: norm1(x) when the previous block computed it (its fused MLP
        residual + this block's norm1); next_norm: the following block's
        norm1, to return (x_out, next_norm(x_out)) from one fused kernel."""
        b, length, c = x.shape
        h, w = self.H, self.W
        assert length == h * w, "input feature has wrong size"
        ws, sh = self.window_size, self.shift_size
        shortcut = x
        x = layer_norm(self.norm1, x) if normed is None else normed
        attn = self.attn
        if attn.attn_drop.p > 0.0 and self.training:
            x = self._windowed_attention(x, mask_matrix)
        else:
            # the qkv Linear is per token, so it runs on the unpartitioned
            # image; pad, roll, partition, the attention, reverse, roll back
            # and crop are one kernel per direction (gdino_amd/wattn.py)
            qkv = attn.qkv(x)
            x = kernels.window_attention_image(qkv, attn.qkv.bias, attn.relative_position_bias_table,
                                               attn.relative_position_index.view(-1), mask_matrix, (h, w), ws, sh,
                                               attn.scale)
            x = attn.proj_drop(attn.proj(x))
        # x + drop_path(branch) as one kernel each (misc.add_drop_path); the
        # attention residual and norm2 as one kernel each way, whose backward
        # also sums the two gradients of x (layernorm.add_scaled_norm)
        dp = self.drop_path.drop_prob if isinstance(self.drop_path, DropPath) else 0.0
        fused = add_scaled_norm(self.norm2, shortcut, x, dp, self.training)
        if fused is not None:
            x, y = fused
            if next_norm is not None:
                # the MLP residual and the next block's norm1 likewise
                nxt = add_scaled_norm(next_norm, x, self.mlp(y), dp, self.training)
                if nxt is not None:
                    return nxt
                return add_drop_path(x, self.mlp(y), dp, self.training), None
            return add_drop_path(x, self.mlp(y), dp, self.training)
        x = add_drop_path(shortcut, x, dp, self.training)
        out = add_drop_path(x, self.mlp(layer_norm(self.norm2, x)), dp, self.training)
        return (out, None) if next_norm is not None else out

    def _windowed_attention(self, x, mask_matrix):
        """reference :250-290 step by step (the path with attention dropout)"""
        b, _, c = x.shape
        h, w = self.H, self.W
        ws, sh = self.window_size, self.shift_size
        dt = castcache.autocast_dtype(x)
        if dt is not None:
            # the qkv GEMM casts its input anyway: cast before the pad / roll /
            # window-partition copies (exact in either dtype) so they move half
            # the bytes; bit-identical to casting inside the Linear
            x = x.to(dt)
        x = x.view(b, h, w, c)
        pad_r, pad_b = (ws - w % ws) % ws, (ws - h % ws) % ws
        if pad_r or pad_b:
            x = F.pad(x, (0, 0, 0, pad_r, 0, pad_b))
        hp, wp = h + pad_b, w + pad_r
        if sh > 0:
            x = torch.roll(x, shifts=(-sh, -sh), dims=(1, 2))
        windows = window_partition(x, ws).reshape(-1, ws * ws, c)
        windows = self.attn(windows, mask=mask_matrix if sh > 0 else None)
        x = window_reverse(windows.view(-1, ws, ws, c), ws, hp, wp)
        if sh > 0:
            x = torch.roll(x, shifts=(sh, sh), dims=(1, 2))
        if pad_r or pad_b:
            x = x[:, :h, :w, :]
        return x.reshape(b, h * w, c)


class PatchMerging(nn.Module):
    def __init__(self, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = norm_layer(4 * dim)

    def forward(self, x, h, w):
        b, length, c = x.shape
        assert length == h * w, "input feature has wrong size"
        x = x.view(b, h, w, c)
        if h % 2 or w % 2:
            x = F.pad(x, (0, 0, 0, w % 2, 0, h % 2))
        # channel order (x0, x1, x2, x3) = (even,even), (odd,even), (even,odd), (odd,odd)
        x = torch.cat([x[:, 0::2, 0::2], x[:, 1::2, 0::2], x[:, 0::2, 1::2], x[:, 1::2, 1::2]], -1)
        return self.reduction(layer_norm(self.norm, x.view(b, -1, 4 * c)))


_MASK_CACHE: Dict[Tuple, torch.Tensor] = {}


def shifted_window_mask(hp: int, wp: int, ws: int, shift: int, device) -> torch.Tensor:
    """[nW, ws*ws, ws*ws] additive mask (0 / -100) for the cyclic shift
    (reference :402-426), cached per geometry."""
    key = (hp, wp, ws, shift, str(device))
    m = _MASK_CACHE.get(key)
    if m is None:
        region = np.zeros((hp, wp), dtype=np.float32)
        cuts = (0, hp - ws, hp - shift, hp), (0, wp - ws, wp - shift, wp)
        label = 0
        for i in range(3):
            for j in range(3):
                region[cuts[0][i]:cuts[0][i + 1], cuts[1][j]:cuts[1][j + 1]] = label
                label += 1
        t = torch.from_numpy(region).view(1, hp, wp, 1)
        win = window_partition(t, ws).reshape(-1, ws * ws)
        diff = win[:, None, :] - win[:, :, None]
        m = torch.where(diff != 0, torch.tensor(-100.0), torch.tensor(0.0)).to(device)
        # the window attention kernel computes this mask from the geometry
        # instead of reading it (gdino_amd/wattn.py)
        m._gd_region_mask = (hp, wp, ws, shift)
        _MASK_CACHE[key] = m
    return m


class BasicLayer(nn.Module):
    def __init__(self, dim, depth, num_heads, window_size=7, mlp_ratio=4.0, qkv_bias=True, qk_scale=None,
                 drop=0.0, attn_drop=0.0, drop_path=0.0, norm_layer=nn.LayerNorm, downsample=None,
                 use_checkpoint=False):
        super().__init__()
        self.window_size = window_size
        self.shift_size = window_size // 2
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(dim, num_heads, window_size, 0 if i % 2 == 0 else window_size // 2,
                                 mlp_ratio, qkv_bias, qk_scale, drop, attn_drop,
                                 drop_path[i] if isinstance(drop_path, list) else drop_path,
                                 norm_layer=norm_layer)
            for i in range(depth)])
        self.downsample = downsample(dim=dim, norm_layer=norm_layer) if downsample is not None else None

    def forward(self, x, h, w):
        ws = self.window_size
        hp, wp = -(-h // ws) * ws, -(-w // ws) * ws
        mask = shifted_window_mask(hp, wp, ws, self.shift_size, x.device)
        normed = None
        for i, blk in enumerate(self.blocks):
            blk.H, blk.W = h, w
            # block i's MLP residual also normalises for block i + 1 (one
            # fused kernel each way, layernorm.add_scaled_norm)
            nxt = self.blocks[i + 1].norm1 if i + 1 < len(self.blocks) else None
            if self.use_checkpoint and torch.is_grad_enabled():
                out = checkpoint.checkpoint(blk, x, mask, normed, nxt, use_reentrant=False)
            else:
                out = blk(x, mask, normed, nxt)
            x, normed = out if nxt is not None else (out, None)
        if self.downsample is not None:
            return x, h, w, self.downsample(x, h, w), (h + 1) // 2, (w + 1) // 2
        return x, h, w, x, h, w


class PatchEmbed(nn.Module):
    def __init__(self, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        self.patch_size = to_2tuple(patch_size)
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.proj = GemmConv2d(in_chans, embed_dim, kernel_size=self.patch_size, stride=self.patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):
        _, _, h, w = x.shape
        ph, pw = self.patch_size
        if w % pw or h % ph:
            x = F.pad(x, (0, (pw - w % pw) % pw, 0, (ph - h % ph) % ph))
        x = self.proj(x)
        if self.norm is not None:
            hh, ww = x.shape[2:]
            x = self.norm(x.flatten(2).transpose(1, 2)).transpose(1, 2).view(-1, self.embed_dim, hh, ww)
        return x


class SwinTransformer(nn.Module):
    """Reference :501-759 (frozen_stages, ape, dilation, out_indices kept)."""

    def __init__(self, pretrain_img_size=224, patch_size=4, in_chans=3, embed_dim=96, depths=(2, 2, 6, 2),
                 num_heads=(3, 6, 12, 24), window_size=7, mlp_ratio=4.0, qkv_bias=True, qk_scale=None,
                 drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.2, norm_layer=nn.LayerNorm, ape=False,
                 patch_norm=True, out_indices=(0, 1, 2, 3), frozen_stages=-1, dilation=False,
                 use_checkpoint=False):
        super().__init__()
        depths, num_heads = list(depths), list(num_heads)
        self.pretrain_img_size = pretrain_img_size
        self.num_layers = len(depths)
        self.embed_dim = embed_dim
        self.ape = ape
        self.patch_norm = patch_norm
        self.out_indices = out_indices
        self.frozen_stages = frozen_stages
        self.dilation = dilation
        self.patch_embed = PatchEmbed(patch_size, in_chans, embed_dim, norm_layer if patch_norm else None)
        if ape:
            ps, pi = to_2tuple(patch_size), to_2tuple(pretrain_img_size)
            self.absolute_pos_embed = nn.Parameter(torch.zeros(1, embed_dim, pi[0] // ps[0], pi[1] // ps[1]))
            trunc_normal_(self.absolute_pos_embed, std=0.02)
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [float(v) for v in torch.linspace(0, drop_path_rate, sum(depths))]
        downsample = [PatchMerging] * (self.num_layers - 1) + [None]
        num_features = [int(embed_dim * 2 ** i) for i in range(self.num_layers)]
        if dilation:
            downsample[-2] = None
            num_features[-1] = int(embed_dim * 2 ** (self.num_layers - 1)) // 2
        self.layers = nn.ModuleList()
        for i in range(self.num_layers):
            self.layers.append(BasicLayer(
                num_features[i], depths[i], num_heads[i], window_size, mlp_ratio, qkv_bias, qk_scale,
                drop_rate, attn_drop_rate, dpr[sum(depths[:i]):sum(depths[:i + 1])], norm_layer,
                downsample[i], use_checkpoint))
        self.num_features = num_features
        for i in out_indices:
            self.add_module(f"norm{i}", norm_layer(num_features[i]))
        self._freeze_stages()

    def _freeze_stages(self):
        if self.frozen_stages >= 0:
            self.patch_embed.eval()
            for p in self.patch_embed.parameters():
                p.requires_grad = False
        if self.frozen_stages >= 1 and self.ape:
            self.absolute_pos_embed.requires_grad = False
        if self.frozen_stages >= 2:
            self.pos_drop.eval()
            for i in range(0, self.frozen_stages - 1):
                self.layers[i].eval()
                for p in self.layers[i].parameters():
                    p.requires_grad = False

    def _stages(self, x):
        x = self.patch_embed(x)
        wh, ww = x.shape[2:]
        if self.ape:
            pe = F.interpolate(self.absolute_pos_embed, size=(wh, ww), mode="bicubic")
            x = x + pe
        x = self.pos_drop(x.flatten(2).transpose(1, 2))
        outs = []
        for i, layer in enumerate(self.layers):
            x_out, h, w, x, wh, ww = layer(x, wh, ww)
            if i in self.out_indices:
                y = layer_norm(getattr(self, f"norm{i}"), x_out, bf16_twin=False)  # feeds a permute, not a GEMM
                outs.append(y.view(-1, h, w, self.num_features[i]).permute(0, 3, 1, 2).contiguous())
        return outs

    def forward_raw(self, x):
        return tuple(self._stages(x))

    def forward(self, tensor_list):
        outs = self._stages(tensor_list.tensors)
        m = tensor_list.mask
        assert m is not None
        res = {}
        for idx, o in enumerate(outs):
            mask = F.interpolate(m[None].float(), size=o.shape[-2:]).to(torch.bool)[0]
            res[idx] = NestedTensor(o, mask)
        return res

    def train(self, mode=True):
        super().train(mode)
        self._freeze_stages()
        return self


SWIN_CONFIGS = {
    "swin_T_224_1k": dict(embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24], window_size=7),
    "swin_B_224_22k": dict(embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32], window_size=7),
    "swin_B_384_22k": dict(embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32], window_size=12),
    "swin_L_224_22k": dict(embed_dim=192, depths=[2, 2, 18, 2], num_heads=[6, 12, 24, 48], window_size=7),
    "swin_L_384_22k": dict(embed_dim=192, depths=[2, 2, 18, 2], num_heads=[6, 12, 24, 48], window_size=12),
}


def build_swin_transformer(modelname, pretrain_img_size, **kw):
    assert modelname in SWIN_CONFIGS, modelname
    cfg = dict(SWIN_CONFIGS[modelname])
    cfg.update(kw)
    return SwinTransformer(pretrain_img_size=pretrain_img_size, **cfg)
