"""Deformable-DETR ``MSDeformAttn`` (reference ops/modules/ms_deform_attn.py:30-126)
on the HIP MSDA kernels.  Same constructor, parameter names, init and forward
signature; fp16 inputs run the kernel in fp32 as the reference does (:113-120)."""
import warnings

import torch.nn as nn

from ...ms_deform_attn import _is_power_of_2, init_msda_parameters, msda_attend


class MSDeformAttn(nn.Module):
    def __init__(self, d_model=256, n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        if d_model % n_heads != 0:
            raise ValueError("d_model must be divisible by n_heads, but got {} and {}".format(d_model, n_heads))
        if not _is_power_of_2(d_model // n_heads):
            warnings.warn("You'd better set d_model in MSDeformAttn to make the dimension of each "
                          "attention head a power of 2.")
        self.im2col_step = 64
        self.d_model = d_model
        self.n_levels = n_levels
        self.n_heads = n_heads
        self.n_points = n_points
        self.sampling_offsets = nn.Linear(d_model, n_heads * n_levels * n_points * 2)
        self.attention_weights = nn.Linear(d_model, n_heads * n_levels * n_points)
        self.value_proj = nn.Linear(d_model, d_model)
        self.output_proj = nn.Linear(d_model, d_model)
        self._reset_parameters()

    def _reset_parameters(self):
        init_msda_parameters(self, self.n_heads, self.n_levels, self.n_points)

    def forward(self, query, reference_points, input_flatten, input_spatial_shapes,
                input_level_start_index, input_padding_mask=None):
        N, Len_in, _ = input_flatten.shape
        assert int((input_spatial_shapes[:, 0] * input_spatial_shapes[:, 1]).sum()) == Len_in
        out = msda_attend(self, query, input_flatten, reference_points, input_spatial_shapes,
                          input_level_start_index, input_padding_mask, self.n_heads,
                          self.n_levels, self.n_points, self.im2col_step)
        return out
