"""Shared specification of the block-level golden cases (TEST INFRASTRUCTURE).

Used by tests/golden/make_block_golden.py (which runs the REFERENCE modules
in this container to produce the fixtures) and by the tests (which run the
product modules on the same inputs).  Weights are not stored in the fixtures:
both sides fill every parameter deterministically from its state-dict name
(`fill_params`), so the fixture only carries inputs, outputs, gradients and a
checksum of the weights.  Same names + same shapes => same weights, which is
also the state-dict compatibility check.
"""
from __future__ import annotations

import math
import zlib

import torch

SEED = 20240917

# Small but structurally complete configurations.  MSDA keeps M*D with D=32,
# L=P=4 so that the GPU runs the vectorised kernels, not only the generic ones.
BIATTN = dict(v_dim=64, l_dim=48, embed_dim=128, num_heads=4)
SWIN = dict(pretrain_img_size=224, embed_dim=32, depths=[2, 2, 2, 2], num_heads=[1, 2, 4, 8], window_size=7,
            out_indices=(1, 2, 3), drop_path_rate=0.0)
TRANSFORMER = dict(d_model=256, nhead=8, num_queries=30, num_encoder_layers=2, num_decoder_layers=2,
                   dim_feedforward=256, dropout=0.0, activation="relu", normalize_before=False,
                   return_intermediate_dec=True, query_dim=4, num_patterns=0, num_feature_levels=4,
                   enc_n_points=4, dec_n_points=4, learnable_tgt_init=True, two_stage_type="standard",
                   embed_init_tgt=True, use_text_enhancer=True, use_fusion_layer=True, use_checkpoint=False,
                   use_transformer_ckpt=False, use_text_cross_attention=True, text_dropout=0.0,
                   fusion_dropout=0.0, fusion_droppath=0.0)
SWIN_B = dict(pretrain_img_size=384, embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32],
              window_size=12, out_indices=(1, 2, 3), drop_path_rate=0.0)  # BASELINE config 5 backbone
LEVELS = [(6, 8), (3, 4), (2, 2), (1, 1)]

# real configurations for the state-dict compatibility fixture
STATE_DICT_SWINS = {
    "swin_T_224_1k": dict(pretrain_img_size=224, embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24],
                          window_size=7, out_indices=(1, 2, 3)),
    "swin_B_384_22k": dict(pretrain_img_size=384, embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32],
                           window_size=12, out_indices=(1, 2, 3)),
}
STATE_DICT_TRANSFORMER = dict(TRANSFORMER, num_encoder_layers=6, num_decoder_layers=6, dim_feedforward=2048,
                              num_queries=900)
TEXT_LEN = 13


def _gen(name: str, salt: int = 0) -> torch.Generator:
    return torch.Generator().manual_seed((zlib.crc32(name.encode()) ^ SEED ^ salt) & 0x7FFFFFFF)


def fill_params(module: torch.nn.Module, salt: int = 0) -> float:
    """Deterministic, name-keyed parameter values (fp64).  Matrices get
    N(0, 1/fan_in); 1-D 'weight'/'gamma' vectors 1 + N(0, 0.1^2) (LayerNorm
    scales, layer-scale gammas); other 1-D vectors N(0, 0.1^2).  Returns a
    checksum (sum of |p|) for the fixture."""
    total = 0.0
    with torch.no_grad():
        for name, p in module.named_parameters():
            g = _gen(name, salt)
            if p.dim() >= 2:
                fan_in = math.prod(p.shape[1:])
                v = torch.randn(p.shape, generator=g, dtype=torch.float64) / math.sqrt(fan_in)
            elif name.endswith("weight") or "gamma" in name:
                v = 1.0 + 0.1 * torch.randn(p.shape, generator=g, dtype=torch.float64)
            else:
                v = 0.1 * torch.randn(p.shape, generator=g, dtype=torch.float64)
            p.copy_(v.to(p.dtype))
            total += float(v.abs().sum())
    return total


def rand(shape, name, scale=1.0):
    return torch.randn(shape, generator=_gen("input:" + name), dtype=torch.float64) * scale


def biattn_inputs():
    v = rand((2, 50, BIATTN["v_dim"]), "v")
    l = rand((2, TEXT_LEN, BIATTN["l_dim"]), "l")
    mask_v = torch.zeros(2, 50, dtype=torch.bool)
    mask_v[1, 40:] = True
    mask_l = torch.zeros(2, TEXT_LEN, dtype=torch.bool)
    mask_l[0, 9:] = True
    gv = rand((2, 50, BIATTN["v_dim"]), "gv")
    gl = rand((2, TEXT_LEN, BIATTN["l_dim"]), "gl")
    return dict(v=v, l=l, mask_v=mask_v, mask_l=mask_l, gv=gv, gl=gl)


def swin_inputs():
    x = rand((2, 3, 96, 128), "img")
    mask = torch.zeros(2, 96, 128, dtype=torch.bool)
    mask[1, :, 96:] = True  # second image padded on the right
    mask[1, 80:, :] = True
    x = x.masked_fill(mask[:, None], 0.0)
    return dict(x=x, mask=mask)


def swin_b_inputs():
    """1 image 96x160: stage-0 tokens 24x40 -> the 12-window padding and
    shift-mask paths are exercised at every stage."""
    x = rand((1, 3, 96, 160), "img_swin_b")
    mask = torch.zeros(1, 96, 160, dtype=torch.bool)
    mask[0, :, 150:] = True
    return dict(x=x.masked_fill(mask[:, None], 0.0), mask=mask)


def phrase_text(bs=2, t=TEXT_LEN):
    """Token-level inputs as BertModelWarper / the model produce them:
    valid-token mask, per-phrase position ids, block-diagonal phrase
    self-attention masks (sample 0 has 3 phrases and 4 pad tokens, sample 1
    two phrases and no padding)."""
    token_mask = torch.ones(bs, t, dtype=torch.bool)
    token_mask[0, 9:] = False
    blocks = [[(0, 1), (1, 4), (4, 7), (7, 8), (8, 9)] + [(i, i + 1) for i in range(9, t)],
              [(0, 1), (1, 6), (6, 12), (12, 13)]]
    sa = torch.zeros(bs, t, t, dtype=torch.bool)
    pos = torch.zeros(bs, t, dtype=torch.long)
    for b, bl in enumerate(blocks):
        for s, e in bl:
            sa[b, s:e, s:e] = True
            pos[b, s:e] = torch.arange(e - s)
    return token_mask, pos, sa


def transformer_inputs():
    d = TRANSFORMER["d_model"]
    srcs, masks, poss = [], [], []
    for i, (h, w) in enumerate(LEVELS):
        srcs.append(rand((2, d, h, w), f"src{i}"))
        m = torch.zeros(2, h, w, dtype=torch.bool)
        if w > 1:
            m[1, :, w - max(1, w // 4):] = True
        masks.append(m)
        poss.append(rand((2, d, h, w), f"pos{i}", 0.5))
    token_mask, pos_ids, sa = phrase_text()
    text = rand((2, TEXT_LEN, d), "text")
    g_hs = rand((TRANSFORMER["num_decoder_layers"], 2, TRANSFORMER["num_queries"], d), "g_hs")
    g_ref = rand((TRANSFORMER["num_decoder_layers"] + 1, 2, TRANSFORMER["num_queries"], 4), "g_ref")
    g_enc = rand((1, 2, TRANSFORMER["num_queries"], d), "g_enc")
    return dict(srcs=srcs, masks=masks, poss=poss, text=text, token_mask=token_mask, pos_ids=pos_ids,
                text_sa=sa, g_hs=g_hs, g_ref=g_ref, g_enc=g_enc)


def wire_heads(transformer, mlp_cls, contrastive_cls):
    """GroundingDINO.__init__'s head wiring (groundingdino.py:165-201) with
    cfg_odvg's sharing flags: decoder bbox MLP shared over layers, separate
    two-stage bbox MLP, parameter-free contrastive heads."""
    d = transformer.d_model
    n = transformer.num_decoder_layers
    bbox = mlp_cls(d, d, 4, 3)
    ce = contrastive_cls()
    transformer.decoder.bbox_embed = torch.nn.ModuleList([bbox for _ in range(n)])
    transformer.decoder.class_embed = torch.nn.ModuleList([ce for _ in range(n)])
    transformer.enc_out_bbox_embed = mlp_cls(d, d, 4, 3)
    transformer.enc_out_class_embed = contrastive_cls()
    return transformer


def transformer_text_dict(inp, dtype=torch.float64, device="cpu"):
    return {"encoded_text": inp["text"].to(device, dtype), "text_token_mask": inp["token_mask"].to(device),
            "position_ids": inp["pos_ids"].to(device), "text_self_attention_masks": inp["text_sa"].to(device)}


# ---------------------------------------------------------------- criterion
# cfg_odvg.py:92-104 costs / coefficients; matcher call groundingdino.py:545
MATCHER = dict(cost_class=1.0, cost_bbox=5.0, cost_giou=2.0, focal_alpha=0.25)
FOCAL_ALPHA, FOCAL_GAMMA = 0.25, 2.0
CRIT_QUERIES = 30


def criterion_weight_dict(dec_layers=2):
    """build_groundingdino's weight dict (groundingdino.py:764-795) for
    cfg_odvg with dec_layers decoder layers and two-stage interm losses."""
    base = {"loss_ce": 2.0, "loss_bbox": 5.0, "loss_giou": 2.0}
    wd = dict(base)
    for i in range(dec_layers - 1):
        wd.update({f"{k}_{i}": v for k, v in base.items()})
    wd.update({f"{k}_interm": v for k, v in base.items()})
    return wd


def criterion_inputs(tokenizer):
    cat_list = [["cat", "traffic light", "dog"], ["person", "umbrella"]]
    captions = [" . ".join(c) + " ." for c in cat_list]
    token = tokenizer(captions, padding="longest", return_tensors="pt")
    t = token["input_ids"].shape[1]
    text_mask = torch.zeros(2, 256, dtype=torch.bool)
    text_mask[:, :t] = token["attention_mask"].bool()
    g = _gen("input:crit_boxes")
    targets = []  # fp32, as the data pipeline produces them
    for labels in ([0, 1, 2, 0], [0, 1, 1]):
        k = len(labels)
        c = 0.2 + 0.6 * torch.rand(k, 2, generator=g, dtype=torch.float64)
        wh = 0.05 + 0.25 * torch.rand(k, 2, generator=g, dtype=torch.float64)
        targets.append({"boxes": torch.cat([c, wh], 1).float(), "labels": torch.as_tensor(labels, dtype=torch.long)})
    return dict(cat_list=cat_list, captions=captions, token=token, text_mask=text_mask, targets=targets)


def criterion_outputs(inp, device="cpu", dtype=torch.float32):
    """Model-shaped outputs (final layer, one aux layer, two-stage interm)
    built from leaf tensors: logits are -inf on padded tokens as
    ContrastiveEmbed produces them, boxes are sigmoid(cxcywh)."""
    mask = inp["text_mask"].to(device)
    leaves = {}

    def head(tag):
        lg = rand((2, CRIT_QUERIES, 256), f"crit_logits_{tag}", 2.0).to(device, dtype).requires_grad_(True)
        bx = rand((2, CRIT_QUERIES, 4), f"crit_boxes_{tag}").to(device, dtype).requires_grad_(True)
        leaves[f"{tag}_logits"] = lg
        leaves[f"{tag}_boxes"] = bx
        return {"pred_logits": lg.masked_fill(~mask[:, None, :], float("-inf")), "pred_boxes": bx.sigmoid()}

    out = head("final")
    out["aux_outputs"] = [head("aux0")]
    out["interm_outputs"] = head("interm")
    out["text_mask"] = mask
    out["token"] = inp["token"]
    return out, leaves


# ---------------------------------------------------------------- full model
# build_groundingdino(make_args(**MODEL_OVERRIDES)) on both sides, with a
# small random BERT (TINY_BERT) instead of bert-base (same code path; keeps
# the fixture generation fast) and the offline tokenizer.
MODEL_OVERRIDES = dict(enc_layers=2, dec_layers=2, num_queries=30, dim_feedforward=256, use_checkpoint=False,
                       use_transformer_ckpt=False, label_list=["cat", "traffic light", "dog", "person", "umbrella"])
TINY_BERT = dict(hidden_size=96, num_hidden_layers=2, num_attention_heads=2, intermediate_size=192)
MODEL_PGRADS = ("backbone.0.patch_embed.proj.weight", "backbone.0.layers.1.blocks.0.attn.qkv.weight",
                "input_proj.0.0.weight", "input_proj.3.0.weight", "input_proj.3.1.weight", "feat_map.weight",
                "bert.encoder.layer.1.attention.self.query.weight", "transformer.level_embed",
                "transformer.encoder.layers.0.self_attn.value_proj.weight",
                "transformer.encoder.fusion_layers.0.attn.out_v_proj.weight",
                "transformer.decoder.layers.1.ca_text.in_proj_weight", "transformer.decoder.bbox_embed.0.layers.0.weight",
                "transformer.enc_out_bbox_embed.layers.2.weight", "transformer.tgt_embed.weight")


def model_inputs(tokenizer):
    inp = criterion_inputs(tokenizer)
    x = rand((2, 3, 64, 96), "model_img")
    mask = torch.zeros(2, 64, 96, dtype=torch.bool)
    mask[1, :, 80:] = True
    mask[1, 56:, :] = True
    inp["images"] = x.masked_fill(mask[:, None], 0.0)
    inp["mask"] = mask
    return inp


def model_surrogate(out, device="cpu", dtype=torch.float64):
    """Fixed random linear functional of every model output (gradient
    source that does not depend on Hungarian matching)."""
    terms = [("final", out["pred_logits"], out["pred_boxes"]),
             ("aux0", out["aux_outputs"][0]["pred_logits"], out["aux_outputs"][0]["pred_boxes"]),
             ("interm", out["interm_outputs"]["pred_logits"], out["interm_outputs"]["pred_boxes"])]
    total = 0.0
    for tag, lg, bx in terms:
        finite = torch.isfinite(lg)
        glg = rand(lg.shape, f"model_g_logits_{tag}").to(device, lg.dtype)
        total = total + (torch.where(finite, lg, torch.zeros((), device=device, dtype=lg.dtype)) * glg).sum().to(dtype)
        total = total + (bx * rand(bx.shape, f"model_g_boxes_{tag}").to(device, bx.dtype)).sum().to(dtype)
    return total
