"""Grounding DINO model, criterion, post-processing and builder.

Drop-in for the reference models/GroundingDINO/groundingdino.py:
``build_groundingdino(args) -> (model, criterion, {"bbox": PostProcess})``,
registered as "groundingdino" in ``models.registry.MODULE_BUILD_FUNCS``
(:726); ``model(samples, targets=None, captions=[...])`` returns the same
dict (pred_logits [B,900,256], pred_boxes [B,900,4], text_mask [B,256],
aux_outputs, token, interm_outputs, interm_outputs_for_matching_pre);
``criterion(outputs, targets, cat_list, captions)`` returns the same loss
names (loss_ce / loss_bbox / loss_giou / loss_xy / loss_hw, with _0.._4 and
_interm suffixes).

Host-path changes (same values, fewer syncs — SURVEY §7 hard part 5):
* phrase masks / position ids are built on the host from the CPU token ids
  and moved once (bertwarper.py);
* ``text_mask`` is one slice assignment, not a B x T loop of device reads
  (reference :343-349, 512 host syncs per step);
* the criterion builds every positive map once per image, matches all
  (layer, image) problems with ONE device->host copy of the cost matrices,
  builds the one-hot targets on the device, and keeps ``num_boxes`` a device
  tensor (no ``.item()``);
* the token focal loss masks instead of ``masked_select`` (no data-dependent
  shape sync); GIoU of matched pairs is computed pairwise instead of as the
  diagonal of an N x N matrix.
"""
from __future__ import annotations

import copy

import numpy as np
from typing import List

import torch
import torch.nn.functional as F
from torch import nn

from gdino_amd import box_ops, castcache
from gdino_amd.conv import GemmConv2d
from gdino_amd.misc import (NestedTensor, box_refine, collectives_enabled, no_padding, get_world_size,
                            is_dist_avail_and_initialized,
                            nested_tensor_from_tensor_list)
from gdino_amd.tokenizer import get_pretrained_language_model, get_tokenlizer

from ..registry import MODULE_BUILD_FUNCS
from .backbone import build_backbone
from .bertwarper import BertModelWarper, generate_masks_with_special_tokens_and_transfer_map
from .matcher import build_matcher
from .transformer import build_transformer
from .utils import MLP, ContrastiveEmbed


def prepare_text_host(tokenizer, special_tokens, max_text_len, captions):
    """Tokenize the captions and build the sub-sentence masks on the host
    (reference groundingdino.py:235-262: padding="longest", phrase-block
    self-attention masks and position ids, truncation to max_text_len).
    -> (dict of CPU tensors, tokenizer output)."""
    tokenized = tokenizer(captions, padding="longest", return_tensors="pt")
    self_masks, position_ids, _ = generate_masks_with_special_tokens_and_transfer_map(
        tokenized, special_tokens, tokenizer)
    tok = {k: v for k, v in tokenized.items()}
    if self_masks.shape[1] > max_text_len:
        self_masks = self_masks[:, :max_text_len, :max_text_len]
        position_ids = position_ids[:, :max_text_len]
        for k in ("input_ids", "attention_mask", "token_type_ids"):
            tok[k] = tok[k][:, :max_text_len]
    text = {"input_ids": tok["input_ids"], "token_type_ids": tok["token_type_ids"],
            "text_token_mask": tok["attention_mask"].bool(), "self_masks": self_masks,
            "position_ids": position_ids}
    return text, tokenized


def pad_text(text: dict, multiple: int, max_text_len: int) -> dict:
    """prepare_text_host's tensors with T padded to a multiple of
    ``multiple`` (at most max_text_len) by pad tokens, as the tokenizer's
    padding itself produces them: id 0, type 0, attention-mask False,
    position id 0 and a phrase-mask row / column that holds only the pad
    token's own diagonal entry (bertwarper.py:224-273 builds the blocks from
    the special tokens; tokens after the last one attend only to
    themselves).  No real token attends to a pad token anywhere (BERT's
    phrase masks, the text enhancer, BiAttention and the decoder's text
    cross-attention mask them, the contrastive head writes -inf), so every
    output of a real token is unchanged.  The step graph pads T this way so
    that batches of different caption lengths share a graph."""
    T = text["input_ids"].shape[1]
    Tb = min(max(-(-T // max(multiple, 1)) * max(multiple, 1), T), max(max_text_len, T))
    if Tb == T:
        return text
    pad = Tb - T
    out = {}
    for k in ("input_ids", "token_type_ids", "position_ids"):
        out[k] = torch.nn.functional.pad(text[k], (0, pad), value=0)
    out["text_token_mask"] = torch.nn.functional.pad(text["text_token_mask"], (0, pad), value=False)
    m = text["self_masks"]
    sm = torch.zeros(m.shape[0], Tb, Tb, dtype=m.dtype)
    sm[:, :T, :T] = m
    idx = torch.arange(T, Tb)
    sm[:, idx, idx] = True
    out["self_masks"] = sm
    return out


_STAGING = []  # (pinned host buffer, event recorded after its copy)


def to_device_async(t: torch.Tensor, device) -> torch.Tensor:
    """Host tensor -> device without a stream synchronisation: a pageable
    source copied with non_blocking=False makes torch wait for the whole
    stream (the queued forward included) before the copy; staging it through
    pinned memory keeps the copy async.  The staging buffer is held here
    until an event recorded after the copy has completed, so it cannot be
    reused while the copy still waits in the stream behind queued work."""
    device = torch.device(device)
    if device.type != "cuda" or t.device.type != "cpu":
        return t.to(device)
    while _STAGING and _STAGING[0][1].query():
        _STAGING.pop(0)
    pinned = t if t.is_pinned() else t.pin_memory()
    out = pinned.to(device, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    _STAGING.append((pinned, ev))
    return out


class GroundingDINO(nn.Module):
    def __init__(self, backbone, transformer, num_queries, aux_loss=False, iter_update=False, query_dim=2,
                 num_feature_levels=1, nheads=8, two_stage_type="no", dec_pred_bbox_embed_share=True,
                 two_stage_class_embed_share=True, two_stage_bbox_embed_share=True, num_patterns=0,
                 dn_number=100, dn_box_noise_scale=0.4, dn_label_noise_ratio=0.5, dn_labelbook_size=100,
                 text_encoder_type="bert-base-uncased", sub_sentence_present=True, max_text_len=256):
        super().__init__()
        self.num_queries = num_queries
        self.transformer = transformer
        self.hidden_dim = hidden_dim = transformer.d_model
        self.num_feature_levels = num_feature_levels
        self.nheads = nheads
        self.max_text_len = 256
        self.sub_sentence_present = sub_sentence_present
        self.query_dim = query_dim
        assert query_dim == 4
        self.num_patterns = num_patterns
        self.dn_number = dn_number
        self.dn_box_noise_scale = dn_box_noise_scale
        self.dn_label_noise_ratio = dn_label_noise_ratio
        self.dn_labelbook_size = dn_labelbook_size

        self.tokenizer = get_tokenlizer(text_encoder_type)
        bert = get_pretrained_language_model(text_encoder_type)
        bert.pooler.dense.weight.requires_grad_(False)
        bert.pooler.dense.bias.requires_grad_(False)
        self.bert = BertModelWarper(bert_model=bert)
        self.feat_map = nn.Linear(self.bert.config.hidden_size, hidden_dim, bias=True)
        nn.init.constant_(self.feat_map.bias.data, 0)
        nn.init.xavier_uniform_(self.feat_map.weight.data)
        self.specical_tokens = self.tokenizer.convert_tokens_to_ids(["[CLS]", "[SEP]", ".", "?"])

        if num_feature_levels > 1:
            projs = []
            chans = list(backbone.num_channels)
            for c in chans:
                projs.append(nn.Sequential(GemmConv2d(c, hidden_dim, kernel_size=1), nn.GroupNorm(32, hidden_dim)))
            in_c = chans[-1]
            for _ in range(num_feature_levels - len(chans)):
                projs.append(nn.Sequential(GemmConv2d(in_c, hidden_dim, kernel_size=3, stride=2, padding=1),
                                           nn.GroupNorm(32, hidden_dim)))
                in_c = hidden_dim
            self.input_proj = nn.ModuleList(projs)
        else:
            assert two_stage_type == "no", "two_stage_type should be no if num_feature_levels=1 !!!"
            self.input_proj = nn.ModuleList([nn.Sequential(
                GemmConv2d(backbone.num_channels[-1], hidden_dim, kernel_size=1), nn.GroupNorm(32, hidden_dim))])

        self.backbone = backbone
        self.aux_loss = aux_loss
        self.box_pred_damping = None
        self.iter_update = iter_update
        assert iter_update, "Why not iter_update?"

        self.dec_pred_bbox_embed_share = dec_pred_bbox_embed_share
        _class_embed = ContrastiveEmbed()
        _bbox_embed = MLP(hidden_dim, hidden_dim, 4, 3)
        nn.init.constant_(_bbox_embed.layers[-1].weight.data, 0)
        nn.init.constant_(_bbox_embed.layers[-1].bias.data, 0)
        n_dec = transformer.num_decoder_layers
        box_list = [_bbox_embed] * n_dec if dec_pred_bbox_embed_share else \
            [copy.deepcopy(_bbox_embed) for _ in range(n_dec)]
        self.bbox_embed = nn.ModuleList(box_list)
        self.class_embed = nn.ModuleList([_class_embed] * n_dec)
        self.transformer.decoder.bbox_embed = self.bbox_embed
        self.transformer.decoder.class_embed = self.class_embed

        self.two_stage_type = two_stage_type
        assert two_stage_type in ["no", "standard"], f"unknown param {two_stage_type} of two_stage_type"
        if two_stage_type != "no":
            if two_stage_bbox_embed_share:
                assert dec_pred_bbox_embed_share
                self.transformer.enc_out_bbox_embed = _bbox_embed
            else:
                self.transformer.enc_out_bbox_embed = copy.deepcopy(_bbox_embed)
            if two_stage_class_embed_share:
                assert dec_pred_bbox_embed_share
                self.transformer.enc_out_class_embed = _class_embed
            else:
                self.transformer.enc_out_class_embed = copy.deepcopy(_class_embed)
            self.refpoint_embed = None
        self._reset_parameters()

    def _reset_parameters(self):
        for proj in self.input_proj:
            nn.init.xavier_uniform_(proj[0].weight, gain=1)
            nn.init.constant_(proj[0].bias, 0)

    def init_ref_points(self, use_num_queries):
        self.refpoint_embed = nn.Embedding(use_num_queries, self.query_dim)

    # ------------------------------------------------------------------ text
    def prepare_text(self, captions, device, prepared=None, pad_multiple=1):
        """Host side of the text path (tokenize, phrase masks / position ids,
        truncate to max_text_len: prepare_text_host) and one move to the
        device.  ``prepared`` = prepare_text_host's result computed elsewhere
        (e.g. in DataLoader workers by gdino_amd.data.TextPreprocessor);
        pinned tensors are copied asynchronously.  ``pad_multiple`` > 1: T
        padded to a multiple of it (pad_text).
        -> (dict of device tensors, tokenizer output for the loss)."""
        text, tokenized = prepared if prepared is not None else prepare_text_host(
            self.tokenizer, self.specical_tokens, self.max_text_len, captions)
        if pad_multiple > 1:
            text = pad_text(text, pad_multiple, self.max_text_len)
        return {k: to_device_async(v, device) for k, v in text.items()}, tokenized

    def encode_text(self, input_ids, token_type_ids, text_token_mask, self_masks, position_ids):
        """BERT + feat_map -> text_dict (groundingdino.py:259-287)."""
        if self.sub_sentence_present:
            bert_out = self.bert(input_ids=input_ids, token_type_ids=token_type_ids,
                                 attention_mask=self_masks, position_ids=position_ids)
        else:
            bert_out = self.bert(input_ids=input_ids, token_type_ids=token_type_ids,
                                 attention_mask=text_token_mask)
        encoded_text = self.feat_map(bert_out["last_hidden_state"])
        n = self.max_text_len
        return {"encoded_text": encoded_text[:, :n], "text_token_mask": text_token_mask[:, :n],
                "position_ids": position_ids[:, :n], "text_self_attention_masks": self_masks[:, :n, :n]}

    # --------------------------------------------------------------- forward
    def forward_core(self, images, image_mask, input_ids, token_type_ids, text_token_mask, self_masks,
                     position_ids):
        """Tensor-in / tensor-out body of the forward (no host syncs, static
        shapes for a fixed batch geometry), the unit that gdino_amd.graphs
        captures into one HIP graph for forward and one for backward.
        -> (outputs_class [L,B,Q,256], outputs_coord [L,B,Q,4], text_mask [B,256],
            interm_class, interm_coord, init_box_proposal)"""
        castcache.refresh_shadows(self, images)  # this step's bf16 weights, one launch
        text_dict = self.encode_text(input_ids, token_type_ids, text_token_mask, self_masks, position_ids)
        samples = NestedTensor(images, image_mask)
        features, poss = self.backbone(samples)
        srcs, masks = [], []
        for lvl, feat in enumerate(features):
            src, mask = feat.decompose()
            srcs.append(self.input_proj[lvl](src))
            masks.append(mask)
            assert mask is not None
        if self.num_feature_levels > len(srcs):
            n_back = len(srcs)
            for lvl in range(n_back, self.num_feature_levels):
                src = self.input_proj[lvl](features[-1].tensors if lvl == n_back else srcs[-1])
                mask = F.interpolate(image_mask[None].float(), size=src.shape[-2:]).to(torch.bool)[0]
                pos_l = self.backbone[1](NestedTensor(src, mask)).to(src.dtype)
                srcs.append(src)
                masks.append(mask)
                poss.append(pos_l)

        hs, reference, hs_enc, ref_enc, init_box_proposal = self.transformer(
            srcs, masks, None, poss, None, None, text_dict)

        outputs_coord, outputs_class = self._heads_all_layers(hs, reference, text_dict)
        bs, len_td = text_dict["text_token_mask"].shape
        text_mask = torch.zeros(bs, self.max_text_len, dtype=torch.bool, device=images.device)
        text_mask[:, :len_td] = text_dict["text_token_mask"]
        if hs_enc is not None:
            interm_class = self.transformer.enc_out_class_embed(hs_enc[-1], text_dict)
            return outputs_class, outputs_coord, text_mask, interm_class, ref_enc[-1], init_box_proposal
        return outputs_class, outputs_coord, text_mask, None, None, None

    def _heads_all_layers(self, hs, reference, text_dict):
        """The per-layer box and class heads (reference groundingdino.py:
        325-337): box_refine(bbox_embed[l](hs[l]), reference[l]) and
        class_embed[l](hs[l], text).  When every layer shares one bbox_embed
        and one class_embed (dec_pred_bbox_embed_share, the cfg default)
        the heads run ONCE over all layers' queries, [B, L*Q, C], instead of
        once per layer: the same per-row arithmetic, one GEMM per MLP layer
        and one contrastive launch instead of L, and the shared weights'
        gradients summed inside one weight-gradient GEMM instead of L
        gradient accumulations.  -> (coords [L, B, Q, 4], logits [L, B, Q, 256])"""
        L = len(hs)
        shared = (all(m is self.bbox_embed[0] for m in self.bbox_embed)
                  and all(m is self.class_embed[0] for m in self.class_embed) and L > 1
                  and all(h.shape == hs[0].shape for h in hs))
        if not shared:
            coords = [box_refine(box_embed(layer_hs), ref_sig)
                      for ref_sig, box_embed, layer_hs in zip(reference[:-1], self.bbox_embed, hs)]
            return (torch.stack(coords),
                    torch.stack([emb(layer_hs, text_dict) for emb, layer_hs in zip(self.class_embed, hs)]))
        B, Q, C = hs[0].shape
        x = torch.stack(hs, 1)                                    # [B, L, Q, C]
        ref = torch.stack(reference[:-1], 1)                      # [B, L, Q, 4]
        delta = self.bbox_embed[0](x)                             # [B, L, Q, 4]
        coords = box_refine(delta.reshape(B, L * Q, 4), ref.reshape(B, L * Q, 4)).view(B, L, Q, 4)
        logits = self.class_embed[0](x.view(B, L * Q, C), text_dict)   # [B, L*Q, 256]
        return coords.transpose(0, 1), logits.view(B, L, Q, -1).transpose(0, 1)

    def forward(self, samples, targets: List = None, **kw):
        captions = kw["captions"] if targets is None else [t["caption"] for t in targets]
        if isinstance(samples, (list, torch.Tensor)):
            samples = nested_tensor_from_tensor_list(samples)
        device = samples.tensors.device
        text, one_hot_token = self.prepare_text(captions, device, kw.get("prepared_text"))
        core = self._graphed_core if getattr(self, "_graphed_core", None) is not None else self.forward_core
        # (a graphed core keeps the masking it was captured with)
        with no_padding(getattr(samples, "padding_free", False)):
            outs = core(samples.tensors, samples.mask, text["input_ids"], text["token_type_ids"],
                        text["text_token_mask"], text["self_masks"], text["position_ids"])
        return self.assemble_outputs(outs, one_hot_token)

    def assemble_outputs(self, core_outputs, one_hot_token=None):
        """forward_core's tuple -> the reference output dict (:343-392)."""
        (outputs_class, outputs_coord, text_mask, interm_class, interm_coord,
         init_box_proposal) = core_outputs
        out = {"pred_logits": outputs_class[-1], "pred_boxes": outputs_coord[-1], "text_mask": text_mask}
        if self.aux_loss:
            out["aux_outputs"] = self._set_aux_loss(outputs_class, outputs_coord)
        out["token"] = one_hot_token
        if interm_class is not None:
            out["interm_outputs"] = {"pred_logits": interm_class, "pred_boxes": interm_coord}
            out["interm_outputs_for_matching_pre"] = {"pred_logits": interm_class,
                                                      "pred_boxes": init_box_proposal}
        return out

    @torch.jit.unused
    def _set_aux_loss(self, outputs_class, outputs_coord):
        return [{"pred_logits": a, "pred_boxes": b} for a, b in zip(outputs_class[:-1], outputs_coord[:-1])]


class SetCriterion(nn.Module):
    def __init__(self, matcher, weight_dict, focal_alpha, focal_gamma, losses):
        super().__init__()
        self.matcher = matcher
        self.weight_dict = weight_dict
        self.losses = losses
        self.focal_alpha = focal_alpha
        self.focal_gamma = focal_gamma

    @torch.no_grad()
    def loss_cardinality(self, outputs, targets, indices, num_boxes):
        logits = outputs["pred_logits"]
        tgt_len = torch.as_tensor([len(v["labels"]) for v in targets], device=logits.device)
        card = (logits.argmax(-1) != logits.shape[-1] - 1).sum(1)
        return {"cardinality_error": F.l1_loss(card.float(), tgt_len.float())}

    def loss_boxes(self, outputs, targets, indices, num_boxes):
        assert "pred_boxes" in outputs
        idx = self._get_src_permutation_idx(indices)
        dev = outputs["pred_boxes"].device
        src = outputs["pred_boxes"][idx[0].to(dev), idx[1].to(dev)]
        tgt = torch.cat([t["boxes"][j.to(t["boxes"].device)] for t, (_, j) in zip(targets, indices)], 0).to(dev)
        l1 = F.l1_loss(src, tgt, reduction="none")
        giou = box_ops.paired_generalized_box_iou(box_ops.box_cxcywh_to_xyxy(src), box_ops.box_cxcywh_to_xyxy(tgt))
        losses = {"loss_bbox": l1.sum() / num_boxes, "loss_giou": (1 - giou).sum() / num_boxes}
        with torch.no_grad():
            losses["loss_xy"] = l1[..., :2].sum() / num_boxes
            losses["loss_hw"] = l1[..., 2:].sum() / num_boxes
        return losses

    def token_sigmoid_binary_focal_loss(self, outputs, targets, indices, num_boxes):
        logits = outputs["pred_logits"]
        tgt = outputs["one_hot"].to(logits.device)
        text_mask = outputs["text_mask"]
        assert tgt.dim() == 3 and logits.dim() == 3
        keep = text_mask[:, None, :].expand_as(logits)
        x = torch.where(keep, logits.float(), torch.zeros((), device=logits.device))
        t = tgt.float()
        p = torch.sigmoid(x)
        ce = F.binary_cross_entropy_with_logits(x, t, reduction="none")
        p_t = p * t + (1 - p) * (1 - t)
        loss = ce * ((1 - p_t) ** self.focal_gamma)
        if self.focal_alpha >= 0:
            loss = (self.focal_alpha * t + (1 - self.focal_alpha) * (1 - t)) * loss
        loss = (loss * keep).sum()
        n_pos = max(sum(len(i[0]) for i in indices), 1.0)
        return {"loss_ce": loss / n_pos}

    @staticmethod
    def _get_src_permutation_idx(indices):
        batch_idx = torch.cat([torch.full_like(src, i) for i, (src, _) in enumerate(indices)])
        src_idx = torch.cat([src for (src, _) in indices])
        return batch_idx, src_idx

    @staticmethod
    def _get_tgt_permutation_idx(indices):
        batch_idx = torch.cat([torch.full_like(tgt, i) for i, (_, tgt) in enumerate(indices)])
        tgt_idx = torch.cat([tgt for (_, tgt) in indices])
        return batch_idx, tgt_idx

    def get_loss(self, loss, outputs, targets, indices, num_boxes, **kwargs):
        loss_map = {"labels": self.token_sigmoid_binary_focal_loss, "cardinality": self.loss_cardinality,
                    "boxes": self.loss_boxes}
        assert loss in loss_map, f"do you really want to compute {loss} loss?"
        return loss_map[loss](outputs, targets, indices, num_boxes, **kwargs)

    @staticmethod
    def _one_hot(shape, indices, targets, label_maps, device):
        """[B, Q, 256] int64 token targets of the matched queries (device)."""
        oh = torch.zeros(shape, dtype=torch.int64, device=device)
        for i, (src, tgt) in enumerate(indices):
            if len(src):
                lab = targets[i]["labels"].to(device)[tgt.to(device)]
                oh[i, src.to(device)] = label_maps[i].to(device)[lab].long()
        return oh

    @staticmethod
    def _heads(outputs):
        heads = [("", outputs)]
        for i, aux in enumerate(outputs.get("aux_outputs", [])):
            heads.append((f"_{i}", aux))
        if "interm_outputs" in outputs:
            heads.append(("_interm", outputs["interm_outputs"]))
        return heads

    def forward(self, outputs, targets, cat_list, caption, return_indices=False):
        device = outputs["pred_logits"].device
        heads = self._heads(outputs)
        if self._device_matching_ok(heads, targets):
            # matching on the device (gdino_amd.lsap): no device->host copy,
            # no host wait anywhere in the loss
            prep = self.prepare_targets(targets, cat_list, caption, outputs["token"], device)
            losses, pairs = self.loss_prepared(outputs, prep)
            if return_indices:
                indices_list = self._pairs_to_indices(pairs, prep["sizes"], len(heads))
                return losses, indices_list[1:] + indices_list[:1]
            return losses
        token = outputs["token"]
        bs = len(cat_list)
        label_maps = []
        for j in range(bs):
            label_maps.append(create_positive_map(token[j], range(len(cat_list[j])), cat_list[j], caption[j])
                              .to(device))

        num_boxes = torch.as_tensor([float(sum(len(t["labels"]) for t in targets))], device=device)
        if collectives_enabled():
            torch.distributed.all_reduce(num_boxes)
        num_boxes = torch.clamp(num_boxes / get_world_size(), min=1)[0]

        if self._can_batch(heads, targets):
            losses, indices_list = self._forward_batched(heads, outputs, targets, label_maps, num_boxes, device)
        else:
            losses, indices_list = self._forward_per_head(heads, outputs, targets, label_maps, num_boxes, device)
        if return_indices:
            return losses, indices_list[1:] + indices_list[:1]
        return losses

    # ---------------------------------------------------- device matching
    # DEVICE_MATCHING = False: the host scipy path (_forward_batched) for A/B
    DEVICE_MATCHING = True

    def _device_matching_ok(self, heads, targets):
        from gdino_amd import _lib, lsap
        logits = heads[0][1]["pred_logits"]
        kmax = max((len(t["labels"]) for t in targets), default=0)
        return (self.DEVICE_MATCHING and self._can_batch(heads, targets) and _lib.on_device(logits)
                and _lib.enabled("lsap") and getattr(self.matcher, "device_matching", False)
                and lsap.supported(logits.shape[1], kmax))

    def prepare_targets(self, targets, cat_list, caption, token, device, kmax=None):
        """The host side of the loss (reference :553-574 before the matcher):
        positive maps of every caption's categories, each target's token map,
        targets padded to ``kmax`` (default: the batch maximum) -- all moved
        with async copies, no stream synchronisation.  -> dict:
          tgt_boxes [B, K, 4] f32, maps [B, K, 256] f32 (positive map of each
          target's label), valid [B, K] bool, sizes [B] int32 (device),
          num_boxes [1] f32 (device, this rank's target count), "sizes" is
          also kept as a host list under "sizes_host"."""
        bs = len(targets)
        sizes = [len(t["labels"]) for t in targets]
        k = max(max(sizes, default=0), 1) if kmax is None else int(kmax)
        if max(sizes, default=0) > k:
            raise ValueError(f"prepare_targets: {max(sizes)} targets > kmax {k}")
        label_maps = [create_positive_map(token[j], range(len(cat_list[j])), cat_list[j], caption[j])
                      for j in range(bs)]
        cmax = max(max(m.shape[0] for m in label_maps), 1)
        lm = torch.zeros(bs, cmax, label_maps[0].shape[1], dtype=torch.float32)
        for j, m in enumerate(label_maps):
            lm[j, :m.shape[0]] = m
        valid = torch.as_tensor(np.arange(k)[None, :] < np.asarray(sizes)[:, None])
        host = {"label_maps": lm, "valid": valid, "sizes": torch.as_tensor(sizes, dtype=torch.int32),
                "num_boxes": torch.as_tensor([float(sum(sizes))], dtype=torch.float32)}
        dev = {n: to_device_async(v, device) for n, v in host.items()}
        tgt_boxes = torch.zeros(bs, k, 4, dtype=torch.float32, device=device)
        labels = torch.zeros(bs, k, dtype=torch.int64, device=device)
        for j, t in enumerate(targets):
            n = sizes[j]
            if n:
                tgt_boxes[j, :n] = to_device_async(t["boxes"], device).float()
                labels[j, :n] = to_device_async(t["labels"], device)
        bidx = torch.arange(bs, device=device)[:, None].expand(bs, k)
        dev["maps"] = dev.pop("label_maps")[bidx, labels]  # [B, K, 256]
        dev["tgt_boxes"] = tgt_boxes
        dev["sizes_host"] = sizes
        return dev

    def loss_prepared(self, outputs, prep):
        """All heads' losses from prepare_targets' tensors, entirely on the
        device and free of host synchronisation (static shapes: capturable
        into the train-step HIP graph).  Same losses as _forward_batched
        (reference :553-636): one cost pass for all H x B problems, the
        Hungarian assignment of each on the device (gdino_amd.lsap, scipy's
        algorithm and tie-breaking), token focal / L1 / GIoU on the matched
        pairs.  Padded pair slots (images with fewer targets than K) are
        masked out exactly.  -> (losses, (rows, cols) [H*B, K])."""
        from gdino_amd import lsap
        heads = self._heads(outputs)
        device = outputs["pred_logits"].device
        H = len(heads)
        logits = torch.stack([o["pred_logits"] for _, o in heads])          # [H, B, Q, 256]
        boxes = torch.stack([o["pred_boxes"] for _, o in heads])            # [H, B, Q, 4]
        _, B, Q, _ = logits.shape
        tgt_boxes, maps, valid, sizes = prep["tgt_boxes"], prep["maps"], prep["valid"], prep["sizes"]
        K = maps.shape[1]

        num_boxes = prep["num_boxes"].clone()
        if collectives_enabled():
            torch.distributed.all_reduce(num_boxes)
        num_boxes = torch.clamp(num_boxes / get_world_size(), min=1)[0]

        cost = self.matcher.cost_batched(logits, boxes, tgt_boxes, maps, valid)   # [H, B, Q, K]
        rows, cols = lsap.linear_sum_assignment_batched(cost.reshape(H * B, Q, K), sizes.repeat(H))
        w = (rows >= 0).view(-1)                                            # [H*B*K] real pairs
        hi, bi = self._pair_heads(H, B, K, device)
        qi = rows.clamp(0, Q - 1).view(-1)  # (the solver writes every slot; the clamps keep any index in range)
        ki = cols.clamp(0, K - 1).view(-1)
        npos = torch.clamp(torch.minimum(sizes, torch.full_like(sizes, Q)).sum().float(), min=1.0)

        # token-level sigmoid focal loss (token_sigmoid_binary_focal_loss, :462-496); padded
        # slots write their (zero) rows into a spare query row Q that is sliced off
        t = torch.zeros((H, B, Q + 1, logits.shape[-1]), dtype=torch.float32, device=device)
        t[hi, bi, torch.where(w, qi, torch.full_like(qi, Q))] = maps[bi, ki].float()
        t = t[:, :, :Q]
        keep = outputs["text_mask"][None, :, None, :]
        x = torch.where(keep, logits.float(), torch.zeros((), device=device))
        p = torch.sigmoid(x)
        ce = F.binary_cross_entropy_with_logits(x, t, reduction="none")
        p_t = p * t + (1 - p) * (1 - t)
        fl = ce * ((1 - p_t) ** self.focal_gamma)
        if self.focal_alpha >= 0:
            fl = (self.focal_alpha * t + (1 - self.focal_alpha) * (1 - t)) * fl
        loss_ce = torch.where(keep, fl, torch.zeros((), device=device)).sum((1, 2, 3)) / npos

        # L1 + GIoU on the matched pairs (loss_boxes, :436-459); a padded slot
        # compares against a unit dummy box (finite GIoU) and is zeroed by where
        src = boxes[hi, bi, qi].float()
        wc = w[:, None]
        tgt = torch.where(wc, tgt_boxes[bi, ki].float(), torch.full((), 0.5, device=device))
        l1 = torch.where(wc, (src - tgt).abs(), torch.zeros((), device=device))
        giou = box_ops.paired_generalized_box_iou(box_ops.box_cxcywh_to_xyxy(src), box_ops.box_cxcywh_to_xyxy(tgt))
        one_m = torch.where(w, 1 - giou, torch.zeros((), device=device))
        zeros = torch.zeros(H, dtype=torch.float32, device=device)
        loss_bbox = zeros.index_add(0, hi, l1.sum(-1)) / num_boxes
        loss_giou = zeros.index_add(0, hi, one_m) / num_boxes
        with torch.no_grad():
            l1d = l1.detach()
            loss_xy = zeros.index_add(0, hi, l1d[:, :2].sum(-1)) / num_boxes
            loss_hw = zeros.index_add(0, hi, l1d[:, 2:].sum(-1)) / num_boxes

        per = {"loss_ce": loss_ce.unbind(0), "loss_bbox": loss_bbox.unbind(0), "loss_giou": loss_giou.unbind(0),
               "loss_xy": loss_xy.unbind(0), "loss_hw": loss_hw.unbind(0)}
        order = (["loss_ce"] if "labels" in self.losses else []) + \
                (["loss_bbox", "loss_giou", "loss_xy", "loss_hw"] if "boxes" in self.losses else [])
        losses = {}
        for h, (suffix, o) in enumerate(heads):
            for k in order:
                losses[k + suffix] = per[k][h]
            if suffix:
                o["text_mask"] = outputs["text_mask"]
        return losses, (rows, cols)

    _PAIR_IDX: dict = {}

    @classmethod
    def _pair_heads(cls, H, B, K, device):
        """head / image index of every pair slot ([H*B*K] each, cached)"""
        key = (H, B, K, str(device))
        v = cls._PAIR_IDX.get(key)
        if v is None:
            hb = torch.arange(H * B * K) // K
            v = cls._PAIR_IDX[key] = (to_device_async(hb // B, device), to_device_async(hb % B, device))
        return v

    @staticmethod
    def _pairs_to_indices(pairs, sizes, H):
        """device (rows, cols) -> the reference's [[(src, tgt)] * B] * H host lists"""
        rows, cols = (x.cpu() for x in pairs)
        B = len(sizes)
        out = []
        for h in range(H):
            per = []
            for b in range(B):
                r, c = rows[h * B + b], cols[h * B + b]
                m = r >= 0
                per.append((r[m].clone(), c[m].clone()))
            out.append(per)
        return out

    def _forward_per_head(self, heads, outputs, targets, label_maps, num_boxes, device):
        """The reference's loop (groundingdino.py:553-636): per head, match,
        build the one-hot token targets, compute each loss.  All (head, image)
        matching problems still share one device->host copy."""
        bs = len(targets)
        problems = []
        for _, o in heads:
            for j in range(bs):
                problems.append((o["pred_logits"][j], o["pred_boxes"][j], targets[j]["labels"],
                                 targets[j]["boxes"].to(device), label_maps[j]))
        all_indices = self.matcher.match_many(problems)
        losses, indices_list = {}, []
        for h, (suffix, o) in enumerate(heads):
            indices = all_indices[h * bs:(h + 1) * bs]
            o["one_hot"] = self._one_hot(outputs["pred_logits"].shape, indices, targets, label_maps, device)
            if suffix:
                o["text_mask"] = outputs["text_mask"]
            for loss in self.losses:
                ld = self.get_loss(loss, o, targets, indices, num_boxes)
                losses.update({k + suffix: v for k, v in ld.items()})
            indices_list.append(indices)
        return losses, indices_list

    def _can_batch(self, heads, targets):
        shp_l, shp_b = heads[0][1]["pred_logits"].shape, heads[0][1]["pred_boxes"].shape
        return (set(self.losses) <= {"labels", "boxes"} and getattr(self.matcher, "batched", False)
                and all(o["pred_logits"].shape == shp_l and o["pred_boxes"].shape == shp_b for _, o in heads)
                and max((len(t["labels"]) for t in targets), default=0) > 0)

    def _forward_batched(self, heads, outputs, targets, label_maps, num_boxes, device):
        """Every head at once (same losses as _forward_per_head, reference
        :553-636): the H heads are stacked to [H, B, Q, .], the matcher builds
        all H*B cost matrices in one pass (one device->host copy), and the
        focal / L1 / GIoU losses are computed for all heads together and
        reduced per head.  Replaces ~H x (matcher + 3 losses) small launches
        with one set."""
        H = len(heads)
        logits = torch.stack([o["pred_logits"] for _, o in heads])          # [H, B, Q, 256]
        boxes = torch.stack([o["pred_boxes"] for _, o in heads])            # [H, B, Q, 4]
        sizes = [len(t["labels"]) for t in targets]
        tgt_boxes = torch.nn.utils.rnn.pad_sequence([t["boxes"].to(device) for t in targets], batch_first=True)
        maps = torch.nn.utils.rnn.pad_sequence(
            [label_maps[b].index_select(0, t["labels"].to(device)) for b, t in enumerate(targets)], batch_first=True)
        kmax = maps.shape[1]
        valid = torch.as_tensor(np.arange(kmax)[None, :] < np.asarray(sizes)[:, None]).to(device, non_blocking=True)

        indices = self.matcher.match_batched(logits, boxes, tgt_boxes, maps, valid, sizes)
        flat = [(h, b, src, tgt) for h in range(H) for b, (src, tgt) in enumerate(indices[h])]
        h_idx = np.concatenate([np.full(len(src), h) for h, _, src, _ in flat])
        b_idx = np.concatenate([np.full(len(src), b) for _, b, src, _ in flat])
        q_idx = np.concatenate([src.numpy() for _, _, src, _ in flat])
        k_idx = np.concatenate([tgt.numpy() for _, _, _, tgt in flat])
        n_pos = [max(sum(len(src) for src, _ in indices[h]), 1) for h in range(H)]
        idx = torch.from_numpy(np.stack([h_idx, b_idx, q_idx, k_idx]).astype(np.int64)).to(device, non_blocking=True)
        npos = torch.as_tensor(n_pos, dtype=torch.float32).to(device, non_blocking=True)
        hi, bi, qi, ki = idx.unbind(0)

        # token-level sigmoid focal loss (token_sigmoid_binary_focal_loss, :462-496)
        t = torch.zeros(logits.shape, dtype=torch.float32, device=device)
        t[hi, bi, qi] = maps[bi, ki].float()
        keep = outputs["text_mask"][None, :, None, :]
        x = torch.where(keep, logits.float(), torch.zeros((), device=device))
        p = torch.sigmoid(x)
        ce = F.binary_cross_entropy_with_logits(x, t, reduction="none")
        p_t = p * t + (1 - p) * (1 - t)
        fl = ce * ((1 - p_t) ** self.focal_gamma)
        if self.focal_alpha >= 0:
            fl = (self.focal_alpha * t + (1 - self.focal_alpha) * (1 - t)) * fl
        loss_ce = torch.where(keep, fl, torch.zeros((), device=device)).sum((1, 2, 3)) / npos

        # L1 + GIoU on the matched pairs (loss_boxes, :436-459)
        src = boxes[hi, bi, qi].float()
        tgt = tgt_boxes[bi, ki].float()
        l1 = (src - tgt).abs()
        giou = box_ops.paired_generalized_box_iou(box_ops.box_cxcywh_to_xyxy(src), box_ops.box_cxcywh_to_xyxy(tgt))
        zeros = torch.zeros(H, dtype=torch.float32, device=device)
        loss_bbox = zeros.index_add(0, hi, l1.sum(-1)) / num_boxes
        loss_giou = zeros.index_add(0, hi, 1 - giou) / num_boxes
        with torch.no_grad():
            l1d = l1.detach()
            loss_xy = zeros.index_add(0, hi, l1d[:, :2].sum(-1)) / num_boxes
            loss_hw = zeros.index_add(0, hi, l1d[:, 2:].sum(-1)) / num_boxes

        per = {"loss_ce": loss_ce.unbind(0), "loss_bbox": loss_bbox.unbind(0), "loss_giou": loss_giou.unbind(0),
               "loss_xy": loss_xy.unbind(0), "loss_hw": loss_hw.unbind(0)}
        order = (["loss_ce"] if "labels" in self.losses else []) + \
                (["loss_bbox", "loss_giou", "loss_xy", "loss_hw"] if "boxes" in self.losses else [])
        losses = {}
        for h, (suffix, o) in enumerate(heads):
            for k in order:
                losses[k + suffix] = per[k][h]
            if suffix:
                o["text_mask"] = outputs["text_mask"]
        return losses, indices


def _nms(boxes, scores, iou_threshold):
    """Greedy NMS on xyxy boxes (torchvision.ops.nms semantics)."""
    order = scores.argsort(descending=True)
    iou = box_ops.box_iou(boxes[order], boxes[order])[0]
    keep = torch.ones(len(order), dtype=torch.bool, device=boxes.device)
    for i in range(len(order)):
        if keep[i]:
            keep[i + 1:] &= iou[i, i + 1:] <= iou_threshold
    return order[keep]


class PostProcess(nn.Module):
    """Model outputs -> per-image {scores, labels, boxes} in image coordinates
    (reference :642-723): token probabilities averaged over each label's
    positive tokens, top-k over (query, label)."""

    def __init__(self, num_select=100, text_encoder_type="text_encoder_type", nms_iou_threshold=-1,
                 use_coco_eval=False, args=None):
        super().__init__()
        self.num_select = num_select
        self.tokenizer = get_tokenlizer(text_encoder_type)
        if args is not None and getattr(args, "use_coco_eval", False):
            from pycocotools.coco import COCO  # noqa: F401 (optional; not in this image)
            coco = COCO(args.coco_val_path)
            cat_list = [c["name"] for c in coco.loadCats(coco.getCatIds())]
        else:
            cat_list = list(getattr(args, "label_list", None) or ["object"])
        caption = " . ".join(cat_list) + " ."
        tokenized = self.tokenizer(caption, padding="longest", return_tensors="pt")
        pos_map = create_positive_map(tokenized, torch.arange(len(cat_list)), cat_list, caption)
        if args is not None and getattr(args, "use_coco_eval", False):
            coco_ids = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 27,
                        28, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 46, 47, 48, 49, 50, 51, 52, 53,
                        54, 55, 56, 57, 58, 59, 60, 61, 62, 63, 64, 65, 67, 70, 72, 73, 74, 75, 76, 77, 78, 79, 80,
                        81, 82, 84, 85, 86, 87, 88, 89, 90]
            full = torch.zeros((91, 256))
            full[torch.as_tensor(coco_ids)] = pos_map[: len(coco_ids)]
            pos_map = full
        self.nms_iou_threshold = nms_iou_threshold
        self.positive_map = pos_map

    @torch.no_grad()
    def forward(self, outputs, target_sizes, not_to_xyxy=False, test=False):
        logits, boxes = outputs["pred_logits"], outputs["pred_boxes"]
        assert len(logits) == len(target_sizes) and target_sizes.shape[1] == 2
        prob_tok = logits.sigmoid()
        pos = self.positive_map.to(prob_tok.device)
        s = pos.sum(-1, keepdim=True)
        pos = torch.where(s != 0, pos / s.clamp(min=1e-12), pos)
        prob = prob_tok @ pos.T
        scores, topk = torch.topk(prob.view(prob.shape[0], -1), self.num_select, dim=1)
        qidx = torch.div(topk, prob.shape[2], rounding_mode="trunc")
        labels = topk % prob.shape[2]
        if not not_to_xyxy:
            boxes = box_ops.box_cxcywh_to_xyxy(boxes)
        boxes = torch.gather(boxes, 1, qidx.unsqueeze(-1).expand(-1, -1, 4))
        img_h, img_w = target_sizes.unbind(1)
        boxes = boxes * torch.stack([img_w, img_h, img_w, img_h], dim=1)[:, None, :]
        return [{"scores": sc, "labels": lb, "boxes": bx} for sc, lb, bx in zip(scores, labels, boxes)]


@MODULE_BUILD_FUNCS.registe_with_name(module_name="groundingdino")
def build_groundingdino(args):
    backbone = build_backbone(args)
    transformer = build_transformer(args)
    model = GroundingDINO(
        backbone, transformer, num_queries=args.num_queries, aux_loss=args.aux_loss, iter_update=True, query_dim=4,
        num_feature_levels=args.num_feature_levels, nheads=args.nheads,
        dec_pred_bbox_embed_share=args.dec_pred_bbox_embed_share, two_stage_type=args.two_stage_type,
        two_stage_bbox_embed_share=args.two_stage_bbox_embed_share,
        two_stage_class_embed_share=args.two_stage_class_embed_share, num_patterns=args.num_patterns,
        dn_number=0, dn_box_noise_scale=args.dn_box_noise_scale, dn_label_noise_ratio=args.dn_label_noise_ratio,
        dn_labelbook_size=args.dn_labelbook_size, text_encoder_type=args.text_encoder_type,
        sub_sentence_present=args.sub_sentence_present, max_text_len=args.max_text_len)
    matcher = build_matcher(args)
    base = {"loss_ce": args.cls_loss_coef, "loss_bbox": args.bbox_loss_coef, "loss_giou": args.giou_loss_coef}
    weight_dict = dict(base)
    if args.aux_loss:
        for i in range(args.dec_layers - 1):
            weight_dict.update({k + f"_{i}": v for k, v in base.items()})
    if args.two_stage_type != "no":
        no_interm_box = getattr(args, "no_interm_box_loss", False)
        coeff = {"loss_ce": 1.0, "loss_bbox": 0.0 if no_interm_box else 1.0,
                 "loss_giou": 0.0 if no_interm_box else 1.0}
        interm_coef = getattr(args, "interm_loss_coef", 1.0)
        weight_dict.update({k + "_interm": v * interm_coef * coeff[k] for k, v in base.items()})
    criterion = SetCriterion(matcher=matcher, weight_dict=weight_dict, focal_alpha=args.focal_alpha,
                             focal_gamma=args.focal_gamma, losses=["labels", "boxes"])
    criterion.to(torch.device(args.device))
    post = {"bbox": PostProcess(num_select=args.num_select, text_encoder_type=args.text_encoder_type,
                                nms_iou_threshold=args.nms_iou_threshold, args=args)}
    castcache.install(model)  # cached bf16 weight casts under autocast (bit-identical)
    return model, criterion, post


def create_positive_map(tokenized, tokens_positive, cat_list, caption):
    """positive_map[i, j] = 1 iff label i's phrase covers token j
    (reference :808-855: first/last character of the phrase's first
    occurrence in the caption, end falling back 1-2 characters)."""
    pm = np.zeros((len(tokens_positive), 256), dtype=np.float32)  # host array, one tensor at the end
    for j, label in enumerate(tokens_positive.tolist() if torch.is_tensor(tokens_positive) else tokens_positive):
        name = cat_list[int(label)]
        start = caption.find(name)
        end = start + len(name) - 1
        beg_pos = tokenized.char_to_token(start)
        end_pos = None
        for off in (0, 1, 2):
            try:
                end_pos = tokenized.char_to_token(end - off)
            except Exception:
                end_pos = None
            if end_pos is not None:
                break
        if beg_pos is None or end_pos is None or beg_pos < 0 or end_pos < 0 or beg_pos > end_pos:
            continue
        pm[j, beg_pos:end_pos + 1] = 1.0
    return torch.from_numpy(pm)
