"""Sine position embeddings for the image feature maps (reference
backbone/position_encoding.py:78-186).  Elementwise; stays in torch."""
import math

import torch
from torch import nn

from gdino_amd.misc import device_const


def _dim_t(num_feats: int, temperature: float, device) -> torch.Tensor:
    """temperature ** (2 * (i // 2) / num_feats), built once per device with
    the device's arithmetic (the reference rebuilds it on every call)."""
    def make():
        idx = torch.arange(num_feats, dtype=torch.float32, device=device)
        return temperature ** (2 * torch.div(idx, 2, rounding_mode="floor") / num_feats)
    return device_const(("pos_dim_t", num_feats, float(temperature)), make, device)


def _sine_yx(y: torch.Tensor, x: torch.Tensor, num_feats: int, temp_h: float, temp_w: float) -> torch.Tensor:
    """y, x [B, H, W] -> [B, H, W, 2*num_feats]: (pos_y, pos_x) interleaved
    sin/cos channels, both coordinates in one pass (same per-element math as
    one embedding per coordinate + cat)."""
    dims = torch.stack((_dim_t(num_feats, temp_h, y.device), _dim_t(num_feats, temp_w, y.device)))
    pos = torch.stack((y, x), dim=-1)[..., None] / dims          # [B, H, W, 2, F]
    return torch.stack((pos[..., 0::2].sin(), pos[..., 1::2].cos()), dim=-1).flatten(3)


class PositionEmbeddingSineHW(nn.Module):
    """Separate temperatures for y and x (pe_temperatureH/W, cfg 20/20)."""

    def __init__(self, num_pos_feats=64, temperatureH=10000, temperatureW=10000, normalize=False, scale=None):
        super().__init__()
        if scale is not None and normalize is False:
            raise ValueError("normalize should be True if scale is passed")
        self.num_pos_feats = num_pos_feats
        self.temperatureH = temperatureH
        self.temperatureW = temperatureW
        self.normalize = normalize
        self.scale = 2 * math.pi if scale is None else scale

    def forward(self, tensor_list):
        mask = tensor_list.mask
        assert mask is not None
        valid = (~mask).float()
        y = valid.cumsum(1)
        x = valid.cumsum(2)
        if self.normalize:
            eps = 1e-6
            y = y / (y[:, -1:, :] + eps) * self.scale
            x = x / (x[:, :, -1:] + eps) * self.scale
        return _sine_yx(y, x, self.num_pos_feats, self.temperatureH, self.temperatureW).permute(0, 3, 1, 2)


class PositionEmbeddingSine(PositionEmbeddingSineHW):
    def __init__(self, num_pos_feats=64, temperature=10000, normalize=False, scale=None):
        super().__init__(num_pos_feats, temperature, temperature, normalize, scale)


class PositionEmbeddingLearned(nn.Module):
    def __init__(self, num_pos_feats=256):
        super().__init__()
        self.row_embed = nn.Embedding(50, num_pos_feats)
        self.col_embed = nn.Embedding(50, num_pos_feats)
        nn.init.uniform_(self.row_embed.weight)
        nn.init.uniform_(self.col_embed.weight)

    def forward(self, tensor_list):
        x = tensor_list.tensors
        h, w = x.shape[-2:]
        xe = self.col_embed(torch.arange(w, device=x.device))
        ye = self.row_embed(torch.arange(h, device=x.device))
        pos = torch.cat([xe[None].expand(h, w, -1), ye[:, None].expand(h, w, -1)], -1)
        return pos.permute(2, 0, 1)[None].expand(x.shape[0], -1, -1, -1)


def build_position_encoding(args):
    n_steps = args.hidden_dim // 2
    if args.position_embedding in ("v2", "sine"):
        return PositionEmbeddingSineHW(n_steps, temperatureH=args.pe_temperatureH,
                                       temperatureW=args.pe_temperatureW, normalize=True)
    if args.position_embedding in ("v3", "learned"):
        return PositionEmbeddingLearned(n_steps)
    raise ValueError(f"not supported {args.position_embedding}")
