"""Encoder-shape MSDA forward and backward (bs=2, 800x1333, bf16 value and
grad_value as the model calls it, init geometry), a few launches each: the program rocprofv3 --pmc runs to read the
SQ counters of the two kernels (tools/gpu_enc_pmc.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

import msda_microbench as mb  # noqa: E402
from gdino_amd import msda  # noqa: E402

S = sum(h * w for h, w in mb.LEVELS)
v, sh, ls, loc, attn, go = mb.inputs(S, torch.bfloat16)
loc = mb.init_geometry_loc(2)
for _ in range(3):
    msda.ms_deform_attn_forward(v, sh, ls, loc, attn, 64)
    msda.ms_deform_attn_backward(v, sh, ls, loc, attn, go, 64, grad_value_dtype=torch.bfloat16,
                                 host_shapes=mb.LEVELS)
torch.cuda.synchronize()
print("enc_pmc done")
