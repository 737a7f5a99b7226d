"""Model utilities (reference models/GroundingDINO/utils.py:1-273).

ContrastiveEmbed's logits go through ``gdino_amd.kernels.contrastive_logits``
(GEMM + pad-token mask + right-padding to max_text_len in one op)."""
import copy
import math

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from gdino_amd.misc import device_const

from gdino_amd import _lib, castcache, kernels
from gdino_amd.misc import sigmoid_focal_loss  # noqa: F401  (re-export, reference utils.py:152)


def _get_clones(module, N, layer_share=False):
    if layer_share:
        return nn.ModuleList([module for _ in range(N)])
    return nn.ModuleList([copy.deepcopy(module) for _ in range(N)])


def _dim_t(num_feats: int, temperature: float, device) -> Tensor:
    """temperature ** (2 * (i // 2) / num_feats), computed once per device
    with the device's own arithmetic (as the reference computes it per call)."""
    def make():
        idx = torch.arange(num_feats, dtype=torch.float32, device=device)
        return temperature ** (2 * torch.div(idx, 2, rounding_mode="floor") / num_feats)
    return device_const(("dim_t", num_feats, float(temperature)), make, device)


def _sin_cos(x: Tensor, dim_t: Tensor) -> Tensor:
    """x [...] -> [..., F] interleaved sin(even) / cos(odd)."""
    v = x[..., None] / dim_t
    return torch.stack((v[..., 0::2].sin(), v[..., 1::2].cos()), dim=-1).flatten(-2)


def get_sine_pos_embed(pos_tensor: Tensor, num_pos_feats: int = 128, temperature: int = 10000,
                       exchange_xy: bool = True) -> Tensor:
    """[..., n] -> [..., n*num_pos_feats]; exchange_xy swaps the first two
    coordinates' embeddings (reference utils.py:24-53)."""
    dim_t = _dim_t(num_pos_feats, temperature, pos_tensor.device)
    parts = [_sin_cos(pos_tensor[..., i] * (2 * math.pi), dim_t) for i in range(pos_tensor.shape[-1])]
    if exchange_xy:
        parts[0], parts[1] = parts[1], parts[0]
    return torch.cat(parts, dim=-1)


def gen_sineembed_for_position(pos_tensor: Tensor) -> Tensor:
    """[nq, bs, 2|4] -> [nq, bs, 256|512]: (y, x[, w, h]) 128 feats each, T=1e4
    (reference utils.py:204-230)."""
    n = pos_tensor.size(-1)
    if n not in (2, 4):
        raise ValueError("Unknown pos_tensor shape(-1):{}".format(n))
    dev = pos_tensor.device
    dim_t = _dim_t(128, 10000, dev)
    # all coordinates at once, in output order (y, x[, w, h]): same per-element
    # arithmetic as one embedding per coordinate + cat
    order = device_const(("sine_order", n), lambda: torch.tensor([1, 0, 2, 3][:n], device=dev), dev)
    coords = (pos_tensor * (2 * math.pi)).index_select(-1, order)
    v = coords[..., None] / dim_t
    return torch.stack((v[..., 0::2].sin(), v[..., 1::2].cos()), dim=-1).flatten(-3)


def query_anchors(reference_points: Tensor, vr: Tensor):
    """One decoder layer's anchors (reference transformer.py:660-672):
    ref_input = reference_points[:, :, None] * vr[None] ([nq, bs, L, 4]) and
    gen_sineembed_for_position(ref_input[:, :, 0]) ([nq, bs, 512]).  One HIP
    kernel (csrc/boxref.hip query_anchor_kernel) for the detached fp32 boxes
    of the two-stage decoder; the composition otherwise."""
    if (_lib.enabled("boxrefine") and _lib.on_device(reference_points) and not reference_points.requires_grad
            and not vr.requires_grad and reference_points.dim() == 3 and reference_points.shape[-1] == 4
            and reference_points.dtype == torch.float32 and vr.dtype == torch.float32 and vr.dim() == 3
            and vr.shape[-1] == 4 and vr.shape[0] == reference_points.shape[1]):
        nq, bs, _ = reference_points.shape
        L = vr.shape[1]
        vr = vr.contiguous()
        ref_input = torch.empty(nq, bs, L, 4, dtype=torch.float32, device=reference_points.device)
        sine = torch.empty(nq, bs, 512, dtype=torch.float32, device=reference_points.device)
        _lib.call("gd_query_anchor_forward", reference_points.data_ptr(), *reference_points.stride(), nq, bs,
                  vr.data_ptr(), L, _dim_t(128, 10000, vr.device).data_ptr(), ref_input.data_ptr(),
                  sine.data_ptr(), _lib.stream_of(vr))
        return ref_input, sine
    ref_input = reference_points[:, :, None] * vr[None, :]
    return ref_input, gen_sineembed_for_position(ref_input[:, :, 0, :])


def gen_encoder_output_proposals(memory: Tensor, memory_padding_mask: Tensor, spatial_shapes: Tensor,
                                 learnedwh=None):
    """Grid proposals per level in logit space + masked memory
    (reference utils.py:56-116).  -> (output_memory [N,S,C], proposals [N,S,4])."""
    n = memory.shape[0]
    proposals = []
    cur = 0
    shapes = spatial_shapes.tolist() if torch.is_tensor(spatial_shapes) else spatial_shapes
    for lvl, (h, w) in enumerate(shapes):
        m = memory_padding_mask[:, cur:cur + h * w].view(n, h, w)
        valid_h = (~m[:, :, 0]).sum(1).float()
        valid_w = (~m[:, 0, :]).sum(1).float()
        gy, gx = torch.meshgrid(torch.linspace(0, h - 1, h, dtype=torch.float32, device=memory.device),
                                torch.linspace(0, w - 1, w, dtype=torch.float32, device=memory.device),
                                indexing="ij")
        grid = torch.stack([gx, gy], -1)[None]  # [1, h, w, 2]
        scale = torch.stack([valid_w, valid_h], -1).view(n, 1, 1, 2)
        grid = (grid + 0.5) / scale
        if learnedwh is not None:
            wh = torch.ones_like(grid) * learnedwh.sigmoid() * (2.0 ** lvl)
        else:
            wh = torch.full_like(grid, 0.05 * (2.0 ** lvl))
        proposals.append(torch.cat((grid, wh), -1).view(n, -1, 4))
        cur += h * w
    props = torch.cat(proposals, 1)
    valid = ((props > 0.01) & (props < 0.99)).all(-1, keepdim=True)
    props = torch.log(props / (1 - props))
    invalid = memory_padding_mask.unsqueeze(-1) | ~valid
    props = props.masked_fill(invalid, float("inf"))
    out_memory = memory.masked_fill(invalid, 0.0)
    return out_memory, props


class RandomBoxPerturber:
    def __init__(self, x_noise_scale=0.2, y_noise_scale=0.2, w_noise_scale=0.2, h_noise_scale=0.2):
        self.noise_scale = torch.Tensor([x_noise_scale, y_noise_scale, w_noise_scale, h_noise_scale])

    def __call__(self, refanchors: Tensor) -> Tensor:
        nq, bs, qd = refanchors.shape
        noise = torch.rand_like(refanchors)
        scale = self.noise_scale.to(refanchors.device)[:qd]
        return (refanchors * (1 + (noise - 0.5) * scale)).clamp_(0, 1)


class MLP(nn.Module):
    """Linear-ReLU stack (reference utils.py:171-185)."""

    def __init__(self, input_dim, hidden_dim, output_dim, num_layers):
        super().__init__()
        self.num_layers = num_layers
        dims = [input_dim] + [hidden_dim] * (num_layers - 1)
        outs = [hidden_dim] * (num_layers - 1) + [output_dim]
        self.layers = nn.ModuleList(nn.Linear(a, b) for a, b in zip(dims, outs))

    def forward(self, x):
        # relu(layer(x)) with the ReLU in the GEMM epilogue on the token-linear
        # route (castcache.linear_relu; elsewhere the plain composition)
        last = self.num_layers - 1
        for i, layer in enumerate(self.layers):
            # (the MLP owns both layers: layer i's output feeds only layer i+1)
            x = castcache.linear_relu(x, layer, fold_into_consumer=True) if i < last else layer(x)
        return x


def _get_activation_fn(activation, d_model=256, batch_dim=0):
    table = {"relu": F.relu, "gelu": F.gelu, "glu": F.glu, "selu": F.selu}
    if activation in table:
        return table[activation]
    if activation == "prelu":
        return nn.PReLU()
    raise RuntimeError(f"activation should be relu/gelu, not {activation}.")


def ffn_act(linear1, activation, x):
    """activation(linear1(x)) of the FFN sublayers (reference transformer.py
    forward_ffn, transformer_vanilla.py:83).  With ReLU on the GPU training
    path the activation runs in the GEMM epilogue (castcache.linear_relu);
    the output is not offered to a consumer's dX fold (use ``ffn``)."""
    if activation is F.relu:
        from gdino_amd.castcache import linear_relu
        return linear_relu(x, linear1)
    return activation(linear1(x))


def ffn(linear1, activation, dropout, linear2, x):
    """linear2(dropout(activation(linear1(x)))), the FFN sublayer (reference
    transformer.py:803-806,931-934, transformer_vanilla.py:83).  With ReLU the
    sublayer owns both Linears, so linear2's dX kernel may apply the ReLU's
    backward mask (castcache.ffn)."""
    if activation is F.relu:
        from gdino_amd.castcache import ffn as _ffn
        return _ffn(x, linear1, linear2, dropout)
    return linear2(dropout(activation(linear1(x))))


class ContrastiveEmbed(nn.Module):
    """Text-alignment logits: x . encoded_text^T, -inf on padding tokens,
    right-padded with -inf to max_text_len (reference utils.py:233-273)."""

    def __init__(self, max_text_len=256):
        super().__init__()
        self.max_text_len = max_text_len

    def forward(self, x, text_dict):
        assert isinstance(text_dict, dict)
        return kernels.contrastive_logits(x, text_dict["encoded_text"], text_dict["text_token_mask"],
                                          self.max_text_len)
