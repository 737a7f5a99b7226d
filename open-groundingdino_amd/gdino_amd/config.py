"""Model/training hyper-parameters restated from the reference config
(config/cfg_odvg.py:1-124; executed there through SLConfig, which needs
addict/yapf) plus the main.py CLI defaults the builders read.  Returns an
argparse.Namespace with the exact field names build_groundingdino reads."""
from __future__ import annotations

import argparse

CFG_ODVG = dict(
    modelname="groundingdino", backbone="swin_T_224_1k", position_embedding="sine", pe_temperatureH=20,
    pe_temperatureW=20, return_interm_indices=[1, 2, 3], enc_layers=6, dec_layers=6, pre_norm=False,
    dim_feedforward=2048, hidden_dim=256, dropout=0.0, nheads=8, num_queries=900, query_dim=4,
    num_patterns=0, num_feature_levels=4, enc_n_points=4, dec_n_points=4, two_stage_type="standard",
    two_stage_bbox_embed_share=False, two_stage_class_embed_share=False, transformer_activation="relu",
    dec_pred_bbox_embed_share=True, dn_box_noise_scale=1.0, dn_label_noise_ratio=0.5, dn_label_coef=1.0,
    dn_bbox_coef=1.0, embed_init_tgt=True, dn_labelbook_size=91, max_text_len=256,
    text_encoder_type="bert-base-uncased", use_text_enhancer=True, use_fusion_layer=True, use_checkpoint=True,
    use_transformer_ckpt=True, use_text_cross_attention=True, text_dropout=0.0, fusion_dropout=0.0,
    fusion_droppath=0.1, sub_sentence_present=True, max_labels=50, lr=1e-5, backbone_freeze_keywords=None,
    freeze_keywords=["bert"], lr_backbone=1e-5, lr_backbone_names=["backbone.0", "bert"],
    lr_linear_proj_mult=1e-5, lr_linear_proj_names=["ref_point_head", "sampling_offsets"],
    weight_decay=1e-4, param_dict_type="ddetr_in_mmdet", ddetr_lr_param=False, epochs=15, lr_drop=4,
    clip_max_norm=0.1, batch_norm_type="FrozenBatchNorm2d", masks=False, aux_loss=True, set_cost_class=1.0,
    set_cost_bbox=5.0, set_cost_giou=2.0, cls_loss_coef=2.0, bbox_loss_coef=5.0, giou_loss_coef=2.0,
    enc_loss_coef=1.0, interm_loss_coef=1.0, no_interm_box_loss=False, focal_alpha=0.25, focal_gamma=2.0,
    decoder_sa_type="sa", matcher_type="HungarianMatcher", decoder_module_seq=["sa", "ca", "ffn"],
    nms_iou_threshold=-1, dec_pred_class_embed_share=True, match_unstable_error=True, use_ema=False,
    use_detached_boxes_dec_out=False, use_coco_eval=False, num_select=300, dilation=False,
    label_list=["dent", "scratch", "missing", "scraped", "broken", "others"],
    device="cuda", seed=42, amp=True,
)


def make_args(**overrides) -> argparse.Namespace:
    d = dict(CFG_ODVG)
    d.update(overrides)
    return argparse.Namespace(**d)


def swin_b_args(**overrides) -> argparse.Namespace:
    """BASELINE config 5 (tools/GroundingDINO_SwinB_cfg.py:3): Swin-B/384."""
    return make_args(backbone="swin_B_384_22k", **overrides)
