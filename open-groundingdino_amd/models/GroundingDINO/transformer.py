"""Grounding DINO deformable transformer (reference transformer.py:41-968).

Same module tree / parameter names / init as the reference so its checkpoints
load.  Hot ops go to the HIP path: MSDA (encoder self- and decoder
cross-attention) through ``MultiScaleDeformableAttention``, attention-family
ops through ``gdino_amd.kernels``.

Host-side changes, all behaviour-preserving:
* the level shapes travel as a Python list next to the device tensor, so
  reference points / proposals need no device->host copies;
* the decoder's per-layer ``isnan().any() | isinf().any()`` print
  (:711-718, one host sync per layer) runs only with GDINO_DEBUG_NAN=1;
* activation checkpointing uses the non-reentrant implementation.
"""
from __future__ import annotations

import contextlib
import os
from typing import List, Optional

import torch
import torch.utils.checkpoint as checkpoint
from torch import Tensor, nn

from gdino_amd import kernels
from gdino_amd.layernorm import add_norm, add_norm3
from gdino_amd.mha import MultiheadAttention
from gdino_amd.misc import add_with_twins, box_refine, device_const, inverted, no_padding, padding_free, topk_indices

from .fuse_modules import BiAttentionBlock
from .ms_deform_attn import MultiScaleDeformableAttention as MSDeformAttn
from .ms_deform_attn import msda_attend
from .transformer_vanilla import TransformerEncoderLayer
from .utils import (MLP, _get_activation_fn, _get_clones, ffn, gen_encoder_output_proposals,
                    get_sine_pos_embed, query_anchors)

_DEBUG_NAN = os.environ.get("GDINO_DEBUG_NAN", "0") == "1"
# mmcv MSDA wrapper semantics (identity add + dropout) — see ms_deform_attn.py
MSDA_IDENTITY_ADD = os.environ.get("GDINO_MSDA_SEMANTICS", "mmcv") == "mmcv"


def _ckpt(fn, *args):
    # the recompute (in backward, outside the forward's no_padding context)
    # must take the forward's masking decision: same ops, same saved tensors
    pf = padding_free()
    return checkpoint.checkpoint(fn, *args, use_reentrant=False,
                                 context_fn=lambda: (contextlib.nullcontext(), no_padding(pf)))


def _inert(m) -> bool:
    """An nn.Dropout that changes nothing now (p = 0 or eval), or Identity."""
    return isinstance(m, nn.Identity) or (isinstance(m, nn.Dropout) and (m.p == 0.0 or not m.training))


class Transformer(nn.Module):
    def __init__(self, d_model=256, nhead=8, num_queries=300, num_encoder_layers=6, num_unicoder_layers=0,
                 num_decoder_layers=6, dim_feedforward=2048, dropout=0.0, activation="relu",
                 normalize_before=False, return_intermediate_dec=False, query_dim=4, num_patterns=0,
                 num_feature_levels=1, enc_n_points=4, dec_n_points=4, learnable_tgt_init=False,
                 two_stage_type="no", embed_init_tgt=False, use_text_enhancer=False, use_fusion_layer=False,
                 use_checkpoint=False, use_transformer_ckpt=False, use_text_cross_attention=False,
                 text_dropout=0.1, fusion_dropout=0.1, fusion_droppath=0.0):
        super().__init__()
        self.num_feature_levels = num_feature_levels
        self.num_encoder_layers = num_encoder_layers
        self.num_unicoder_layers = num_unicoder_layers
        self.num_decoder_layers = num_decoder_layers
        self.num_queries = num_queries
        assert query_dim == 4
        enc_layer = DeformableTransformerEncoderLayer(d_model, dim_feedforward, dropout, activation,
                                                      num_feature_levels, nhead, enc_n_points)
        text_layer = TransformerEncoderLayer(d_model=d_model, nhead=nhead // 2,
                                             dim_feedforward=dim_feedforward // 2,
                                             dropout=text_dropout) if use_text_enhancer else None
        fusion_layer = BiAttentionBlock(v_dim=d_model, l_dim=d_model, embed_dim=dim_feedforward // 2,
                                        num_heads=nhead // 2, dropout=fusion_dropout,
                                        drop_path=fusion_droppath) if use_fusion_layer else None
        assert not normalize_before
        self.encoder = TransformerEncoder(enc_layer, num_encoder_layers, d_model=d_model, num_queries=num_queries,
                                          text_enhance_layer=text_layer, feature_fusion_layer=fusion_layer,
                                          use_checkpoint=use_checkpoint, use_transformer_ckpt=use_transformer_ckpt)
        dec_layer = DeformableTransformerDecoderLayer(d_model, dim_feedforward, dropout, activation,
                                                      num_feature_levels, nhead, dec_n_points,
                                                      use_text_cross_attention=use_text_cross_attention)
        self.decoder = TransformerDecoder(dec_layer, num_decoder_layers, nn.LayerNorm(d_model),
                                          return_intermediate=return_intermediate_dec, d_model=d_model,
                                          query_dim=query_dim, num_feature_levels=num_feature_levels)
        self.d_model = d_model
        self.nhead = nhead
        self.dec_layers = num_decoder_layers
        self.num_patterns = num_patterns if isinstance(num_patterns, int) else 0
        if num_feature_levels > 1:
            self.level_embed = nn.Parameter(torch.Tensor(num_feature_levels, d_model)) \
                if num_encoder_layers > 0 else None
        self.learnable_tgt_init = learnable_tgt_init
        assert learnable_tgt_init, "why not learnable_tgt_init"
        self.embed_init_tgt = embed_init_tgt
        if (two_stage_type != "no" and embed_init_tgt) or two_stage_type == "no":
            self.tgt_embed = nn.Embedding(num_queries, d_model)
            nn.init.normal_(self.tgt_embed.weight.data)
        else:
            self.tgt_embed = None
        self.two_stage_type = two_stage_type
        assert two_stage_type in ["no", "standard"], f"unknown param {two_stage_type} of two_stage_type"
        if two_stage_type == "standard":
            self.enc_output = nn.Linear(d_model, d_model)
            self.enc_output_norm = nn.LayerNorm(d_model)
            self.two_stage_wh_embedding = None
        if two_stage_type == "no":
            self.refpoint_embed = nn.Embedding(num_queries, 4)
        self.enc_out_class_embed = None
        self.enc_out_bbox_embed = None
        self._reset_parameters()

    def _reset_parameters(self):
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)
        for m in self.modules():
            if isinstance(m, MSDeformAttn):
                m.init_weights()
        if self.num_feature_levels > 1 and self.level_embed is not None:
            nn.init.normal_(self.level_embed)

    @staticmethod
    def get_valid_ratio(mask):
        _, h, w = mask.shape
        valid_h = (~mask[:, :, 0]).sum(1).float() / h
        valid_w = (~mask[:, 0, :]).sum(1).float() / w
        return torch.stack([valid_w, valid_h], -1)

    def init_ref_points(self, use_num_queries):
        self.refpoint_embed = nn.Embedding(use_num_queries, 4)

    def forward(self, srcs, masks, refpoint_embed, pos_embeds, tgt, attn_mask=None, text_dict=None):
        flat_src, flat_mask, flat_pos, shapes_list = [], [], [], []
        for lvl, (src, mask, pos) in enumerate(zip(srcs, masks, pos_embeds)):
            bs, c, h, w = src.shape
            shapes_list.append((h, w))
            flat_src.append(src.flatten(2).transpose(1, 2))
            flat_mask.append(mask.flatten(1))
            pos = pos.flatten(2).transpose(1, 2)
            if self.num_feature_levels > 1 and self.level_embed is not None:
                pos = pos + self.level_embed[lvl].view(1, 1, -1)
            flat_pos.append(pos)
        src_flatten = torch.cat(flat_src, 1)
        mask_flatten = torch.cat(flat_mask, 1)
        lvl_pos_embed_flatten = torch.cat(flat_pos, 1)
        device = src_flatten.device
        starts = [0]
        for h, w in shapes_list[:-1]:
            starts.append(starts[-1] + h * w)
        key = tuple(shapes_list)
        spatial_shapes = device_const(("shapes",) + key,
                                      lambda: torch.as_tensor(shapes_list, dtype=torch.long), device)
        # host copy for the MSDA backward's pixel-block tiling (no device sync)
        spatial_shapes.gd_host_shapes = key
        level_start_index = device_const(("lsi",) + key, lambda: torch.as_tensor(starts, dtype=torch.long), device)
        valid_ratios = torch.stack([self.get_valid_ratio(m) for m in masks], 1)

        memory, memory_text = self.encoder(
            src_flatten, pos=lvl_pos_embed_flatten, level_start_index=level_start_index,
            spatial_shapes=spatial_shapes, valid_ratios=valid_ratios, key_padding_mask=mask_flatten,
            memory_text=text_dict["encoded_text"], text_attention_mask=inverted(text_dict["text_token_mask"]),
            position_ids=text_dict["position_ids"],
            text_self_attention_masks=text_dict["text_self_attention_masks"], shapes_list=shapes_list)
        text_dict["encoded_text"] = memory_text

        if self.two_stage_type == "standard":
            output_memory, output_proposals = gen_encoder_output_proposals(memory, mask_flatten, shapes_list)
            output_memory = self.enc_output_norm(self.enc_output(output_memory))
            # enc_out_class_embed(output_memory, text_dict).max(-1)[0]
            # (reference :292-293), without the [bs, S, 256] logits: only the
            # top-k indices are used (gdino_amd/contrastive.py)
            topk_logits = kernels.contrastive_rowmax(output_memory, text_dict["encoded_text"],
                                                     text_dict["text_token_mask"])
            # (the bf16 head output widened first: a mixed bf16 + fp32 add of
            # this [B, S, 4] shape took 90 us in PyTorch's templated kernel)
            delta = self.enc_out_bbox_embed(output_memory)
            enc_coord = delta.to(torch.promote_types(delta.dtype, output_proposals.dtype)) + output_proposals
            topk_proposals = topk_indices(topk_logits, self.num_queries)  # [bs, nq]
            idx4 = topk_proposals.unsqueeze(-1).expand(-1, -1, 4)
            refpoint_embed_undetach = torch.gather(enc_coord, 1, idx4)
            refpoint_embed_ = refpoint_embed_undetach.detach()
            init_box_proposal = torch.gather(output_proposals, 1, idx4).sigmoid()
            tgt_undetach = torch.gather(output_memory, 1,
                                        topk_proposals.unsqueeze(-1).expand(-1, -1, self.d_model))
            if self.embed_init_tgt:
                tgt_ = self.tgt_embed.weight[None].expand(bs, -1, -1)
            else:
                tgt_ = tgt_undetach.detach()
            if refpoint_embed is not None:
                refpoint_embed = torch.cat([refpoint_embed, refpoint_embed_], dim=1)
                tgt = torch.cat([tgt, tgt_], dim=1)
            else:
                refpoint_embed, tgt = refpoint_embed_, tgt_
        elif self.two_stage_type == "no":
            tgt_ = self.tgt_embed.weight[None].expand(bs, -1, -1)
            refpoint_embed_ = self.refpoint_embed.weight[None].expand(bs, -1, -1)
            if refpoint_embed is not None:
                refpoint_embed = torch.cat([refpoint_embed, refpoint_embed_], dim=1)
                tgt = torch.cat([tgt, tgt_], dim=1)
            else:
                refpoint_embed, tgt = refpoint_embed_, tgt_
            if self.num_patterns > 0:
                tgt_embed = tgt.repeat(1, self.num_patterns, 1)
                refpoint_embed = refpoint_embed.repeat(1, self.num_patterns, 1)
                tgt = tgt_embed + self.patterns.weight[None, :, :].repeat_interleave(self.num_queries, 1)
            init_box_proposal = refpoint_embed_.sigmoid()
        else:
            raise NotImplementedError(f"unknown two_stage_type {self.two_stage_type}")

        hs, references = self.decoder(
            tgt=tgt.transpose(0, 1), memory=memory.transpose(0, 1), memory_key_padding_mask=mask_flatten,
            pos=lvl_pos_embed_flatten.transpose(0, 1), refpoints_unsigmoid=refpoint_embed.transpose(0, 1),
            level_start_index=level_start_index, spatial_shapes=spatial_shapes, valid_ratios=valid_ratios,
            tgt_mask=attn_mask, memory_text=text_dict["encoded_text"],
            text_attention_mask=inverted(text_dict["text_token_mask"]))
        if self.two_stage_type == "standard":
            hs_enc = tgt_undetach.unsqueeze(0)
            ref_enc = refpoint_embed_undetach.sigmoid().unsqueeze(0)
        else:
            hs_enc = ref_enc = None
        return hs, references, hs_enc, ref_enc, init_box_proposal


class TransformerEncoder(nn.Module):
    def __init__(self, encoder_layer, num_layers, d_model=256, num_queries=300, enc_layer_share=False,
                 text_enhance_layer=None, feature_fusion_layer=None, use_checkpoint=False,
                 use_transformer_ckpt=False):
        super().__init__()
        self.layers, self.text_layers, self.fusion_layers = [], [], []
        if num_layers > 0:
            self.layers = _get_clones(encoder_layer, num_layers, layer_share=enc_layer_share)
            if text_enhance_layer is not None:
                self.text_layers = _get_clones(text_enhance_layer, num_layers, layer_share=enc_layer_share)
            if feature_fusion_layer is not None:
                self.fusion_layers = _get_clones(feature_fusion_layer, num_layers, layer_share=enc_layer_share)
        self.query_scale = None
        self.num_queries = num_queries
        self.num_layers = num_layers
        self.d_model = d_model
        self.use_checkpoint = use_checkpoint
        self.use_transformer_ckpt = use_transformer_ckpt

    @staticmethod
    def get_reference_points(spatial_shapes, valid_ratios, device):
        """Pixel-centre reference points of every level, normalised by the
        valid (unpadded) extent, then re-scaled per target level
        (reference :471-485).  spatial_shapes: list of (H, W) or tensor."""
        shapes = spatial_shapes.tolist() if torch.is_tensor(spatial_shapes) else spatial_shapes
        refs = []
        for lvl, (h, w) in enumerate(shapes):
            ry, rx = torch.meshgrid(torch.linspace(0.5, h - 0.5, h, dtype=torch.float32, device=device),
                                    torch.linspace(0.5, w - 0.5, w, dtype=torch.float32, device=device),
                                    indexing="ij")
            ry = ry.reshape(-1)[None] / (valid_ratios[:, None, lvl, 1] * h)
            rx = rx.reshape(-1)[None] / (valid_ratios[:, None, lvl, 0] * w)
            refs.append(torch.stack((rx, ry), -1))
        ref = torch.cat(refs, 1)
        return ref[:, :, None] * valid_ratios[:, None]

    def forward(self, src: Tensor, pos: Tensor, spatial_shapes: Tensor, level_start_index: Tensor,
                valid_ratios: Tensor, key_padding_mask: Tensor, memory_text: Tensor = None,
                text_attention_mask: Tensor = None, pos_text: Tensor = None,
                text_self_attention_masks: Tensor = None, position_ids: Tensor = None,
                shapes_list: Optional[List] = None):
        output = src
        if self.num_layers > 0:
            reference_points = self.get_reference_points(shapes_list if shapes_list is not None
                                                         else spatial_shapes, valid_ratios, src.device)
        if self.text_layers:
            bs, n_text, _ = memory_text.shape
            if pos_text is None and position_ids is None:
                ar = torch.arange(n_text, device=memory_text.device).float()[None, :, None].repeat(bs, 1, 1)
                pos_text = get_sine_pos_embed(ar, num_pos_feats=256, exchange_xy=False)
            if position_ids is not None:
                pos_text = get_sine_pos_embed(position_ids[..., None], num_pos_feats=256, exchange_xy=False)
        train_ckpt = torch.is_grad_enabled()
        for layer_id, layer in enumerate(self.layers):
            if self.fusion_layers:
                fl = self.fusion_layers[layer_id]
                if self.use_checkpoint and train_ckpt:
                    output, memory_text = _ckpt(fl, output, memory_text, key_padding_mask, text_attention_mask)
                else:
                    output, memory_text = fl(v=output, l=memory_text, attention_mask_v=key_padding_mask,
                                             attention_mask_l=text_attention_mask)
            if self.text_layers:
                memory_text = self.text_layers[layer_id](
                    src=memory_text.transpose(0, 1), src_mask=inverted(text_self_attention_masks),
                    src_key_padding_mask=text_attention_mask,
                    pos=pos_text.transpose(0, 1) if pos_text is not None else None).transpose(0, 1)
            if self.use_transformer_ckpt and train_ckpt:
                output = _ckpt(layer, output, pos, reference_points, spatial_shapes, level_start_index,
                               key_padding_mask)
            else:
                output = layer(src=output, pos=pos, reference_points=reference_points,
                               spatial_shapes=spatial_shapes, level_start_index=level_start_index,
                               key_padding_mask=key_padding_mask)
        return output, memory_text


# GDINO_DEFER_BOX_REFINE=0: the per-layer anchor update with autograd (A/B)
DEFER_BOX_REFINE = os.environ.get("GDINO_DEFER_BOX_REFINE", "1") != "0"


def _uncached_autocast(dev: str):
    """The current autocast state with its cast cache disabled (a no-op
    context when autocast is off)."""
    if dev not in ("cuda", "cpu") or not torch.is_autocast_enabled(dev):
        return contextlib.nullcontext()
    return torch.autocast(device_type=dev, dtype=torch.get_autocast_dtype(dev), cache_enabled=False)


class _BatchedBoxRefine(torch.autograd.Function):
    """The decoder's refined anchors new_ref[l] = box_refine(bbox_embed(
    out[l]), ref[l]) of every layer (reference transformer.py
    :728-731) as ONE autograd node: the forward returns the values the layer
    loop computed without autograd (the same kernels, so the anchors each
    layer sampled with are exactly these), the backward recomputes the shared
    bbox_embed MLP once over all layers' queries [L, nq, bs, C] under the
    forward's autocast state and differentiates it -- one set of GEMMs and
    one gradient per parameter instead of L of each (plus L - 1
    accumulations of the shared weights' gradients)."""

    @staticmethod
    def forward(ctx, values, outs, refs, mlp, *params):
        dev = outs.device.type
        ctx.mlp = mlp
        ctx.amp = (torch.is_autocast_enabled(dev), torch.get_autocast_dtype(dev)) if dev in ("cuda", "cpu") else None
        ctx.save_for_backward(outs, refs)
        return values.clone()

    @staticmethod
    def backward(ctx, g):
        outs, refs = ctx.saved_tensors
        dev = outs.device.type
        params = [q for q in ctx.mlp.parameters() if q.requires_grad]
        amp = ctx.amp if ctx.amp is not None else (False, None)
        with torch.enable_grad(), torch.autocast(device_type=dev, enabled=amp[0], dtype=amp[1]):
            x = outs.detach().requires_grad_(True)
            y = box_refine(ctx.mlp(x), refs)
        grads = torch.autograd.grad(y, [x] + params, g, allow_unused=True)
        return (None, grads[0], None, None, *grads[1:])


class TransformerDecoder(nn.Module):
    def __init__(self, decoder_layer, num_layers, norm=None, return_intermediate=False, d_model=256,
                 query_dim=4, num_feature_levels=1):
        super().__init__()
        self.layers = _get_clones(decoder_layer, num_layers) if num_layers > 0 else []
        self.num_layers = num_layers
        self.norm = norm
        self.return_intermediate = return_intermediate
        assert return_intermediate, "support return_intermediate only"
        self.query_dim = query_dim
        assert query_dim in [2, 4], f"query_dim should be 2/4 but {query_dim}"
        self.num_feature_levels = num_feature_levels
        self.ref_point_head = MLP(query_dim // 2 * d_model, d_model, d_model, 2)
        self.query_pos_sine_scale = None
        self.query_scale = None
        self.bbox_embed = None
        self.class_embed = None
        self.d_model = d_model
        self.ref_anchor_head = None

    def forward(self, tgt, memory, tgt_mask: Optional[Tensor] = None, memory_mask: Optional[Tensor] = None,
                tgt_key_padding_mask: Optional[Tensor] = None, memory_key_padding_mask: Optional[Tensor] = None,
                pos: Optional[Tensor] = None, refpoints_unsigmoid: Optional[Tensor] = None,
                level_start_index: Optional[Tensor] = None, spatial_shapes: Optional[Tensor] = None,
                valid_ratios: Optional[Tensor] = None, memory_text: Optional[Tensor] = None,
                text_attention_mask: Optional[Tensor] = None):
        output = tgt
        intermediate = []
        reference_points = refpoints_unsigmoid.sigmoid()
        ref_points = [reference_points]
        vr = torch.cat([valid_ratios, valid_ratios], -1) if reference_points.shape[-1] == 4 else valid_ratios
        # one shared bbox_embed (dec_pred_bbox_embed_share, the cfg default)
        # and autograd on: the per-layer anchor updates' backward runs batched
        deferred = ([] if (DEFER_BOX_REFINE and self.bbox_embed is not None and torch.is_grad_enabled()
                           and all(m is self.bbox_embed[0] for m in self.bbox_embed)
                           and not refpoints_unsigmoid.requires_grad) else None)
        for layer_id, layer in enumerate(self.layers):
            # ref_input [nq, bs, nlevel, 4], query_sine_embed [nq, bs, 512]
            ref_input, query_sine_embed = query_anchors(reference_points, vr)
            raw_query_pos = self.ref_point_head(query_sine_embed)
            pos_scale = self.query_scale(output) if self.query_scale is not None else 1
            # (no multiply by the constant 1; and fp32 once per layer: the
            # layer adds it to the fp32 target three times, with_pos_embed,
            # and a bf16 + fp32 add takes PyTorch's slow mixed-dtype path --
            # the values are the ones the promotion would produce)
            query_pos = raw_query_pos if self.query_scale is None else pos_scale * raw_query_pos
            if query_pos.dtype != output.dtype and output.dtype == torch.float32:
                query_pos = query_pos.float()
            output = layer(tgt=output, tgt_query_pos=query_pos, tgt_query_sine_embed=query_sine_embed,
                           tgt_key_padding_mask=tgt_key_padding_mask, tgt_reference_points=ref_input,
                           memory_text=memory_text, text_attention_mask=text_attention_mask, memory=memory,
                           memory_key_padding_mask=memory_key_padding_mask,
                           memory_level_start_index=level_start_index, memory_spatial_shapes=spatial_shapes,
                           memory_pos=pos, self_attn_mask=tgt_mask, cross_attn_mask=memory_mask)
            if _DEBUG_NAN and bool(output.isnan().any() | output.isinf().any()):
                print(f"output layer_id {layer_id} is nan: num_nan {int(output.isnan().sum())}, "
                      f"num_inf {int(output.isinf().sum())}")
            if self.bbox_embed is not None:
                if deferred is not None:
                    # the anchor update without autograd; its gradient path
                    # is rebuilt for all layers at once below
                    # (autocast's weight-cast cache off: a cast made here,
                    # without autograd, would be reused by the model's box
                    # heads in the same autocast region and cut their
                    # gradient to bbox_embed's weights)
                    with torch.no_grad(), _uncached_autocast(output.device.type):
                        new_ref = box_refine(self.bbox_embed[layer_id](output), reference_points)
                    deferred.append((output, reference_points, new_ref))
                else:
                    new_ref = box_refine(self.bbox_embed[layer_id](output), reference_points)  # transformer.py:728-731
                ref_points.append(new_ref)
                reference_points = new_ref.detach()
            intermediate.append(self.norm(output))
        if deferred:
            # every layer's refined anchors through ONE batched bbox_embed on
            # the gradient path (_BatchedBoxRefine); the last layer's too (the
            # model's box heads read reference[:-1], other callers of the
            # module may use all of them)
            n = len(deferred)
            outs = torch.stack([d[0] for d in deferred])
            refs = torch.stack([d[1] for d in deferred])
            vals = torch.stack([d[2] for d in deferred])
            mlp = self.bbox_embed[0]
            params = [q for q in mlp.parameters() if q.requires_grad]
            ref_points[1:1 + n] = list(_BatchedBoxRefine.apply(vals, outs, refs, mlp, *params).unbind(0))
        return [[x.transpose(0, 1) for x in intermediate], [r.transpose(0, 1) for r in ref_points]]


class DeformableTransformerEncoderLayer(nn.Module):
    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu", n_levels=4, n_heads=8,
                 n_points=4):
        super().__init__()
        self.self_attn = MSDeformAttn(embed_dims=d_model, num_levels=n_levels, num_heads=n_heads,
                                      num_points=n_points, batch_first=True, identity_add=MSDA_IDENTITY_ADD)
        self.dropout1 = nn.Dropout(dropout)
        self.norm1 = nn.LayerNorm(d_model)
        self.linear1 = nn.Linear(d_model, d_ffn)
        self.activation = _get_activation_fn(activation, d_model=d_ffn)
        self.dropout2 = nn.Dropout(dropout)
        self.linear2 = nn.Linear(d_ffn, d_model)
        self.dropout3 = nn.Dropout(dropout)
        self.norm2 = nn.LayerNorm(d_model)

    @staticmethod
    def with_pos_embed(tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward_ffn(self, src, resid=None):
        """resid: a second handle on src (add_norm taps) for the residual"""
        src2 = ffn(self.linear1, self.activation, self.dropout2, self.linear2, src)
        return add_norm(self.norm2, src if resid is None else resid, self.dropout3(src2))

    def forward(self, src, pos, reference_points, spatial_shapes, level_start_index, key_padding_mask=None):
        # src + pos with the bf16 twins of query and src (the projections'
        # autocast inputs) in the same pass (gdino_amd.misc.add_with_twins)
        query = src if pos is None else add_with_twins(src, pos)
        sa = self.self_attn
        if sa.identity_add and sa.batch_first and _inert(self.dropout1):
            # norm1(src + dropout1(dropout(msda(query)) + query)) with dropout1
            # inert: the module's dropout and identity add folded into the
            # add + LayerNorm kernel (gdino_amd.layernorm.add_norm3)
            out = msda_attend(sa, query, src, reference_points, spatial_shapes, level_start_index,
                              key_padding_mask, sa.num_heads, sa.num_levels, sa.num_points, sa.im2col_step)
            # two handles on the output (FFN input, FFN residual): the two
            # gradients are summed in the add + LayerNorm backward kernel
            y = add_norm3(self.norm1, src, query, out, sa.dropout, taps=2)
            if y is None:
                y = add_norm(self.norm1, src, sa.dropout(out) + query, taps=2)
            return self.forward_ffn(*y)
        src2 = sa(query=query, reference_points=reference_points, value=src, spatial_shapes=spatial_shapes,
                  level_start_index=level_start_index, key_padding_mask=key_padding_mask)
        src = add_norm(self.norm1, src, self.dropout1(src2))
        return self.forward_ffn(src)


class DeformableTransformerDecoderLayer(nn.Module):
    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu", n_levels=4, n_heads=8,
                 n_points=4, use_text_feat_guide=False, use_text_cross_attention=False):
        super().__init__()
        self.cross_attn = MSDeformAttn(embed_dims=d_model, num_levels=n_levels, num_heads=n_heads,
                                       num_points=n_points, batch_first=True, identity_add=MSDA_IDENTITY_ADD)
        self.dropout1 = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
        self.norm1 = nn.LayerNorm(d_model)
        if use_text_cross_attention:
            self.ca_text = MultiheadAttention(d_model, n_heads, dropout=dropout)
            self.catext_dropout = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
            self.catext_norm = nn.LayerNorm(d_model)
        self.self_attn = MultiheadAttention(d_model, n_heads, dropout=dropout)
        self.dropout2 = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
        self.norm2 = nn.LayerNorm(d_model)
        self.linear1 = nn.Linear(d_model, d_ffn)
        self.activation = _get_activation_fn(activation, d_model=d_ffn, batch_dim=1)
        self.dropout3 = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
        self.linear2 = nn.Linear(d_ffn, d_model)
        self.dropout4 = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
        self.norm3 = nn.LayerNorm(d_model)
        self.key_aware_proj = None
        self.use_text_feat_guide = use_text_feat_guide
        assert not use_text_feat_guide
        self.use_text_cross_attention = use_text_cross_attention

    def rm_self_attn_modules(self):
        self.self_attn = None
        self.dropout2 = None
        self.norm2 = None

    @staticmethod
    def with_pos_embed(tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward_ffn(self, tgt, resid=None):
        # the reference runs the decoder FFN outside autocast (fp32, :870-875)
        with torch.autocast(device_type=tgt.device.type, enabled=False):
            t = tgt.float() if tgt.dtype in (torch.float16, torch.bfloat16) else tgt
            tgt2 = ffn(self.linear1, self.activation, self.dropout3, self.linear2, t)
        return add_norm(self.norm3, tgt if resid is None else resid, self.dropout4(tgt2))

    def forward(self, tgt, tgt_query_pos=None, tgt_query_sine_embed=None, tgt_key_padding_mask=None,
                tgt_reference_points=None, memory_text=None, text_attention_mask=None, memory=None,
                memory_key_padding_mask=None, memory_level_start_index=None, memory_spatial_shapes=None,
                memory_pos=None, self_attn_mask=None, cross_attn_mask=None):
        assert cross_attn_mask is None
        if self.self_attn is not None:
            # q = k = tgt + pos with the bf16 twins of the sum and of tgt
            # (the value) written in the same pass: the self-attention's
            # packed in-projection reads them instead of two cast kernels
            q = k = tgt if tgt_query_pos is None else add_with_twins(tgt, tgt_query_pos)
            tgt2 = self.self_attn(q, k, tgt, attn_mask=self_attn_mask)[0]
            if self.use_text_cross_attention:
                # two handles (the text cross-attention's query, its residual)
                tgt_q, tgt = add_norm(self.norm2, tgt, self.dropout2(tgt2), taps=2)
            else:
                tgt = tgt_q = add_norm(self.norm2, tgt, self.dropout2(tgt2))
        else:
            tgt_q = tgt
        if self.use_text_cross_attention:
            # key and value are the same tensor (reference :900-905 passes
            # two identical transposes): one object lets the MHA project them
            # with one GEMM
            text_kv = memory_text.transpose(0, 1)
            ca_q = tgt_q if tgt_query_pos is None else add_with_twins(tgt_q, tgt_query_pos)
            tgt2 = self.ca_text(ca_q, text_kv, text_kv,
                                key_padding_mask=text_attention_mask)[0]
            # two handles (the deformable attention's query, its residual)
            tgt_q, tgt = add_norm(self.catext_norm, tgt, self.catext_dropout(tgt2), taps=2)
        else:
            tgt_q = tgt
        query = self.with_pos_embed(tgt_q, tgt_query_pos)
        ca = self.cross_attn
        ref_t = tgt_reference_points.transpose(0, 1).contiguous()
        if ca.identity_add and ca.batch_first and _inert(self.dropout1):
            # the MSDA module's dropout and identity add folded into norm1
            # (as in the encoder layer; the output arrives batch-first)
            out = msda_attend(ca, query.transpose(0, 1), memory.transpose(0, 1), ref_t, memory_spatial_shapes,
                              memory_level_start_index, memory_key_padding_mask, ca.num_heads, ca.num_levels,
                              ca.num_points, ca.im2col_step).transpose(0, 1)
            y = add_norm3(self.norm1, tgt, query, out, ca.dropout, taps=2)
            if y is None:
                y = add_norm(self.norm1, tgt, ca.dropout(out) + query, taps=2)
            return self.forward_ffn(*y)
        tgt2 = ca(query=query.transpose(0, 1), reference_points=ref_t, value=memory.transpose(0, 1),
                  spatial_shapes=memory_spatial_shapes, level_start_index=memory_level_start_index,
                  key_padding_mask=memory_key_padding_mask).transpose(0, 1)
        tgt = add_norm(self.norm1, tgt, self.dropout1(tgt2))
        return self.forward_ffn(tgt)


def build_transformer(args):
    return Transformer(
        d_model=args.hidden_dim, dropout=args.dropout, nhead=args.nheads, num_queries=args.num_queries,
        dim_feedforward=args.dim_feedforward, num_encoder_layers=args.enc_layers,
        num_decoder_layers=args.dec_layers, normalize_before=args.pre_norm, return_intermediate_dec=True,
        query_dim=args.query_dim, activation=args.transformer_activation, num_patterns=args.num_patterns,
        num_feature_levels=args.num_feature_levels, enc_n_points=args.enc_n_points,
        dec_n_points=args.dec_n_points, learnable_tgt_init=True, two_stage_type=args.two_stage_type,
        embed_init_tgt=args.embed_init_tgt, use_text_enhancer=args.use_text_enhancer,
        use_fusion_layer=args.use_fusion_layer, use_checkpoint=args.use_checkpoint,
        use_transformer_ckpt=args.use_transformer_ckpt, use_text_cross_attention=args.use_text_cross_attention,
        text_dropout=args.text_dropout, fusion_dropout=args.fusion_dropout, fusion_droppath=args.fusion_droppath)
