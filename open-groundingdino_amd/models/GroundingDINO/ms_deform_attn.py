"""Multi-scale deformable attention modules on the HIP MSDA kernels.

Two module signatures exist in the reference and both are provided:

* ``MultiScaleDeformableAttention`` — the mmcv signature the training model
  actually instantiates (transformer.py:29 imports
  ``mmcv.ops.multi_scale_deform_attn.MultiScaleDeformableAttention``; built at
  transformer.py:761-767 and :827-833 with ``embed_dims=, num_levels=,
  num_heads=, num_points=, batch_first=True``).  mmcv's wrapper returns
  ``dropout(output) + identity`` with ``identity = query`` (as passed in, i.e.
  with the positional embedding already added by the caller) and
  ``dropout=0.1`` by default.  mmcv is not vendored in the reference, so these
  wrapper semantics are PARITY UNPINNED; ``identity_add=False`` gives the
  in-repo GroundingDINO wrapper semantics instead
  (models/GroundingDINO/ms_deform_attn.py:233-363: plain ``output_proj(out)``).
  ``embed_dim=`` / ``img2col_step=`` (that file's spelling) are accepted too.
* ``MSDeformAttn`` (in ``ops/modules``) — the Deformable-DETR signature of
  ops/modules/ms_deform_attn.py:30-126.

Parameter names (``sampling_offsets``, ``attention_weights``, ``value_proj``,
``output_proj``) and their init (ms_deform_attn.py:198-221) are those of the
reference so its checkpoints load unchanged.
"""
from __future__ import annotations

import math
import warnings
from typing import Optional

import torch
import torch.nn as nn
from torch.nn.init import constant_, xavier_uniform_

from gdino_amd import castcache, msda_prologue
from gdino_amd.misc import padding_free

from .ops.functions.ms_deform_attn_func import MSDeformAttnFunction


def _is_power_of_2(n):
    if (not isinstance(n, int)) or (n < 0):
        raise ValueError("invalid input for _is_power_of_2: {} (type: {})".format(n, type(n)))
    return (n & (n - 1) == 0) and n != 0


def init_msda_parameters(mod: nn.Module, num_heads: int, num_levels: int, num_points: int) -> None:
    """Deformable-DETR init: zero offset weights, per-head direction x (point
    index + 1) offset biases, uniform attention, xavier projections
    (reference ms_deform_attn.py:198-221)."""
    constant_(mod.sampling_offsets.weight.data, 0.0)
    ang = torch.arange(num_heads, dtype=torch.float32) * (2.0 * math.pi / num_heads)
    direction = torch.stack([ang.cos(), ang.sin()], -1)
    direction = direction / direction.abs().max(-1, keepdim=True)[0]
    scale = torch.arange(1, num_points + 1, dtype=torch.float32).view(1, 1, num_points, 1)
    bias = direction.view(num_heads, 1, 1, 2) * scale  # [heads, 1, points, 2]
    bias = bias.expand(num_heads, num_levels, num_points, 2).contiguous()
    with torch.no_grad():
        mod.sampling_offsets.bias = nn.Parameter(bias.view(-1))
    constant_(mod.attention_weights.weight.data, 0.0)
    constant_(mod.attention_weights.bias.data, 0.0)
    xavier_uniform_(mod.value_proj.weight.data)
    constant_(mod.value_proj.bias.data, 0.0)
    xavier_uniform_(mod.output_proj.weight.data)
    constant_(mod.output_proj.bias.data, 0.0)


def _loc_dtype(t: torch.Tensor) -> torch.dtype:
    """Sampling locations / weights are computed in fp32 (fp64 for fp64
    models), whatever the autocast dtype of the projections."""
    return torch.float64 if t.dtype == torch.float64 else torch.float32


def sampling_locations_from(reference_points, sampling_offsets, spatial_shapes, num_points):
    """Reference points + learned offsets -> normalized sampling locations
    [N, Lq, M, L, P, 2] in fp32 / fp64 (ms_deform_attn.py:310-329)."""
    ct = torch.promote_types(_loc_dtype(sampling_offsets), _loc_dtype(reference_points))
    off = sampling_offsets.to(ct)
    ref = reference_points.to(ct)
    if ref.shape[-1] == 2:
        normalizer = torch.stack([spatial_shapes[..., 1], spatial_shapes[..., 0]], -1).to(off.dtype)
        return ref[:, :, None, :, None, :] + off / normalizer[None, None, None, :, None, :]
    if ref.shape[-1] == 4:
        return ref[:, :, None, :, None, :2] + off / num_points * ref[:, :, None, :, None, 2:] * 0.5
    raise ValueError(
        "Last dim of reference_points must be 2 or 4, but get {} instead.".format(ref.shape[-1]))


def msda_attend(mod, query, value, reference_points, spatial_shapes, level_start_index,
                key_padding_mask, num_heads, num_levels, num_points, im2col_step):
    """Shared body (batch_first tensors): projections, softmax over L*P,
    sampling locations, HIP MSDA core, output projection."""
    bs, num_query, _ = query.shape
    _, num_value, _ = value.shape
    value = mod.value_proj(value)
    if key_padding_mask is not None and not padding_free():  # (an all-False mask: identity)
        value = value.masked_fill(key_padding_mask[..., None], 0.0)
    value = value.view(bs, num_value, num_heads, -1)
    offsets, attn = castcache.linear_shared_input(query, (mod.sampling_offsets, mod.attention_weights))
    if msda_prologue.supported(offsets, attn, reference_points, num_levels, num_points):
        # softmax + sampling-location math as one kernel each way
        # (gdino_amd/msda_prologue.py)
        loc, attn = msda_prologue.MSDAPrologue.apply(offsets, attn, reference_points, spatial_shapes, num_heads,
                                                     num_levels, num_points)
    else:
        offsets = offsets.reshape(bs, num_query, num_heads, num_levels, num_points, 2)
        attn = attn.reshape(bs, num_query, num_heads, num_levels * num_points)
        attn = attn.to(_loc_dtype(attn)).softmax(-1).view(bs, num_query, num_heads, num_levels, num_points)
        loc = sampling_locations_from(reference_points, offsets, spatial_shapes, num_points)
    if value.dtype == torch.float16:  # kernels run fp32 / bf16 / fp64 value
        value = value.float()
    out = MSDeformAttnFunction.apply(value.contiguous(), spatial_shapes, level_start_index,
                                     loc.contiguous(), attn.contiguous(), im2col_step)
    return mod.output_proj(out)


class MultiScaleDeformableAttention(nn.Module):
    """mmcv-signature MSDA module on the HIP kernels (see module docstring)."""

    def __init__(self, embed_dims: int = 256, num_heads: int = 8, num_levels: int = 4,
                 num_points: int = 4, im2col_step: int = 64, dropout: float = 0.1,
                 batch_first: bool = False, norm_cfg=None, init_cfg=None,
                 value_proj_ratio: float = 1.0, identity_add: bool = True,
                 embed_dim: Optional[int] = None, img2col_step: Optional[int] = None):
        super().__init__()
        if embed_dim is not None:  # GroundingDINO-copy spelling
            embed_dims = embed_dim
        if img2col_step is not None:
            im2col_step = img2col_step
        if embed_dims % num_heads != 0:
            raise ValueError(f"embed_dims must be divisible by num_heads, but got {embed_dims} and {num_heads}")
        head_dim = embed_dims // num_heads
        if not _is_power_of_2(head_dim):
            warnings.warn("You'd better set embed_dims in MultiScaleDeformableAttention to make the "
                          "dimension of each attention head a power of 2 (the fast kernel path is D=32).")
        self.embed_dims = self.embed_dim = embed_dims
        self.num_heads = num_heads
        self.num_levels = num_levels
        self.num_points = num_points
        self.im2col_step = im2col_step
        self.batch_first = batch_first
        self.identity_add = identity_add
        self.dropout = nn.Dropout(dropout)
        value_proj_size = int(embed_dims * value_proj_ratio)
        self.sampling_offsets = nn.Linear(embed_dims, num_heads * num_levels * num_points * 2)
        self.attention_weights = nn.Linear(embed_dims, num_heads * num_levels * num_points)
        self.value_proj = nn.Linear(embed_dims, value_proj_size)
        self.output_proj = nn.Linear(value_proj_size, embed_dims)
        self.init_weights()

    def init_weights(self):
        init_msda_parameters(self, self.num_heads, self.num_levels, self.num_points)

    _reset_parameters = init_weights

    def freeze_sampling_offsets(self):
        self.sampling_offsets.weight.requires_grad = False
        self.sampling_offsets.bias.requires_grad = False

    def freeze_attention_weights(self):
        self.attention_weights.weight.requires_grad = False
        self.attention_weights.bias.requires_grad = False

    def forward(self, query, key=None, value=None, identity=None, query_pos=None,
                key_padding_mask=None, reference_points=None, spatial_shapes=None,
                level_start_index=None, **kwargs):
        if value is None:
            value = query
        if identity is None:
            identity = query
        if query_pos is not None:
            query = query + query_pos
        if not self.batch_first:
            query = query.permute(1, 0, 2)
            value = value.permute(1, 0, 2)
        out = msda_attend(self, query, value, reference_points, spatial_shapes, level_start_index,
                          key_padding_mask, self.num_heads, self.num_levels, self.num_points,
                          self.im2col_step)
        if not self.batch_first:
            out = out.permute(1, 0, 2)
        if not self.identity_add:
            return out
        return self.dropout(out) + identity
