"""Autograd wrapper of the HIP MSDA kernels.

Same contract as the reference ``MSDeformAttnFunction``
(/root/reference/models/GroundingDINO/ops/functions/ms_deform_attn_func.py:21-38):
``apply(value, value_spatial_shapes, value_level_start_index,
sampling_locations, attention_weights, im2col_step)``; the five tensors are
saved for backward; backward is once-differentiable and returns
``(grad_value, None, None, grad_sampling_loc, grad_attn_weight, None)``.

The reference's pure-PyTorch ``ms_deform_attn_core_pytorch`` (same file
:41-61, "for debug and test only") is deliberately NOT part of the product:
its restatement lives in ``oracle/msda_torch.py`` and is used only by tests.
"""
import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from gdino_amd import msda as MSDA


class MSDeformAttnFunction(Function):
    @staticmethod
    def forward(ctx, value, value_spatial_shapes, value_level_start_index, sampling_locations,
                attention_weights, im2col_step):
        ctx.im2col_step = im2col_step
        ctx.host_shapes = MSDA.host_level_shapes(value_spatial_shapes)
        output = MSDA.ms_deform_attn_forward(value, value_spatial_shapes, value_level_start_index,
                                             sampling_locations, attention_weights, im2col_step)
        ctx.save_for_backward(value, value_spatial_shapes, value_level_start_index,
                              sampling_locations, attention_weights)
        return output

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        value, shapes, lsi, loc, attn = ctx.saved_tensors
        # the sorted backward writes grad_value in value.dtype directly; the
        # atomic kernels keep their fp32 accumulation buffer, which autograd
        # casts to value.dtype (one pass either way)
        grad_value, grad_loc, grad_attn = MSDA.ms_deform_attn_backward(
            value, shapes, lsi, loc, attn, grad_output.contiguous(), ctx.im2col_step,
            grad_value_dtype=value.dtype if value.dtype == torch.bfloat16 else
            (torch.float64 if value.dtype == torch.float64 else torch.float32),
            host_shapes=ctx.host_shapes)
        return grad_value, None, None, grad_loc, grad_attn, None


# Name used by the GroundingDINO copy of the wrapper (ms_deform_attn.py:42).
MultiScaleDeformableAttnFunction = MSDeformAttnFunction
