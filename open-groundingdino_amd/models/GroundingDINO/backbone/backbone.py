"""Backbone assembly (reference backbone/backbone.py:146-221): Joiner of the
Swin backbone and the sine position embedding.  ResNet backbones need
torchvision, which is not part of this image; asking for one raises."""
from typing import List

import torch
from torch import nn

from gdino_amd.misc import NestedTensor

from .position_encoding import build_position_encoding
from .swin_transformer import SWIN_CONFIGS, build_swin_transformer


class FrozenBatchNorm2d(nn.Module):
    """BatchNorm2d with fixed statistics and affine params (eps inside rsqrt)."""

    def __init__(self, n):
        super().__init__()
        self.register_buffer("weight", torch.ones(n))
        self.register_buffer("bias", torch.zeros(n))
        self.register_buffer("running_mean", torch.zeros(n))
        self.register_buffer("running_var", torch.ones(n))

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        state_dict.pop(prefix + "num_batches_tracked", None)
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    def forward(self, x):
        scale = self.weight * (self.running_var + 1e-5).rsqrt()
        shift = self.bias - self.running_mean * scale
        return x * scale[None, :, None, None] + shift[None, :, None, None]


class Joiner(nn.Sequential):
    def __init__(self, backbone, position_embedding):
        super().__init__(backbone, position_embedding)

    def forward(self, tensor_list):
        feats = self[0](tensor_list)
        outs: List[NestedTensor] = []
        pos = []
        for _, f in feats.items():
            outs.append(f)
            pos.append(self[1](f).to(f.tensors.dtype))
        return outs, pos


def build_backbone(args):
    position_embedding = build_position_encoding(args)
    rii = list(args.return_interm_indices)
    assert rii in [[0, 1, 2, 3], [1, 2, 3], [3]]
    use_checkpoint = getattr(args, "use_checkpoint", False)
    if args.backbone in SWIN_CONFIGS:
        pretrain = int(args.backbone.split("_")[-2])
        body = build_swin_transformer(args.backbone, pretrain_img_size=pretrain, out_indices=tuple(rii),
                                      dilation=False, use_checkpoint=use_checkpoint)
        channels = body.num_features[4 - len(rii):]
    elif args.backbone in ("resnet50", "resnet101"):
        raise NotImplementedError("ResNet backbones need torchvision, which this image does not ship")
    else:
        raise NotImplementedError("Unknown backbone {}".format(args.backbone))
    assert len(channels) == len(rii)
    model = Joiner(body, position_embedding)
    model.num_channels = list(channels)
    return model
