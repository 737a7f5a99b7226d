"""Generate block-level golden vectors by running the REFERENCE modules.

Run in the build container (where /root/reference exists):
    python tests/golden/make_block_golden.py

The reference's model files are imported by path inside a synthetic package
(``_refmodels.GroundingDINO``, __path__ = the reference model directory), bypassing its
package __init__ files, which pull in torchvision / mmcv / timm.  None of those
are installed, so this script registers minimal in-memory stand-ins before the
import:
  timm.models.layers      DropPath (stochastic depth), to_2tuple, trunc_normal_
                          (the published timm behaviour; identity in eval mode)
  torchvision             a version string (util/misc.py checks it) and an
                          ops namespace (not called by the blocks used here)
  mmcv.ops.multi_scale_deform_attn.MultiScaleDeformableAttention
                          the reference's own pure-PyTorch
                          ms_deform_attn.MultiScaleDeformableAttention, with
                          mmcv's constructor keywords and the mmcv wrapper
                          semantics: output_proj result -> dropout -> + identity
                          (query before query_pos).  The mmcv wheel is not on
                          disk, so this wrapper behaviour is "parity unpinned"
                          (SURVEY 8c); the MSDA core inside it is the reference's.
  groundingdino.util.misc the reference's own util/misc.py, loaded by path.

Every module runs in fp64, eval mode, with name-keyed deterministic weights
(block_spec.fill_params).  Output: data-only .npz fixtures (no pickle) next to
this script.  Nothing from the reference is copied into the repository.
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch
from torch import nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
# the product's offline tokenizer produces the token batches the criterion
# reads (bert-base-uncased cannot be fetched here); nothing else of the
# product is imported
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "open-groundingdino_amd"))
import block_spec as spec  # noqa: E402

REF = "/root/reference"
REF_GD = os.path.join(REF, "models", "GroundingDINO")


# ----------------------------------------------------------------------------
# third-party stand-ins (behaviour as published, written here, not copied)
# ----------------------------------------------------------------------------
class _DropPath(nn.Module):
    def __init__(self, drop_prob=None):
        super().__init__()
        self.drop_prob = drop_prob or 0.0

    def forward(self, x):
        if self.drop_prob == 0.0 or not self.training:
            return x
        keep = 1.0 - self.drop_prob
        mask = x.new_empty((x.shape[0],) + (1,) * (x.dim() - 1)).bernoulli_(keep)
        return x * mask / keep


def _to_2tuple(x):
    return tuple(x) if isinstance(x, (tuple, list)) else (x, x)


def _module(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def _load_path(name, path):
    spec_ = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec_)
    sys.modules[name] = mod
    spec_.loader.exec_module(mod)
    return mod


def _box_area(boxes):
    return (boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])


def _unavailable(what):
    def f(*a, **k):
        raise RuntimeError(f"{what} is not available in the golden generator")
    return f


def install_shims():
    import transformers  # noqa: F401  (must precede the torchvision stand-in: it probes find_spec)

    _module("timm")
    _module("timm.models")
    _module("timm.models.layers", DropPath=_DropPath, to_2tuple=_to_2tuple,
            trunc_normal_=lambda t, mean=0.0, std=1.0, a=-2.0, b=2.0: nn.init.trunc_normal_(t, mean, std, a, b))
    tv = _module("torchvision", __version__="0.20.0")
    tv.ops = _module("torchvision.ops")
    tv.ops.boxes = _module("torchvision.ops.boxes", box_area=_box_area, nms=_unavailable("torchvision nms"))
    tv.ops.misc = _module("torchvision.ops.misc")
    tv.models = _module("torchvision.models")  # backbone.py: ResNet path only
    tv.models._utils = _module("torchvision.models._utils", IntermediateLayerGetter=_unavailable("IntermediateLayerGetter"))
    tv._is_tracing = lambda: False  # misc.nested_tensor_from_tensor_list

    pkg = _module("groundingdino")
    pkg.__path__ = []
    util = _module("groundingdino.util")
    util.__path__ = []
    pkg.util = util
    util.misc = _load_path("groundingdino.util.misc", os.path.join(REF, "util", "misc.py"))
    util.box_ops = _load_path("groundingdino.util.box_ops", os.path.join(REF, "util", "box_ops.py"))
    util.get_tokenlizer = _load_path("groundingdino.util.get_tokenlizer", os.path.join(REF, "util", "get_tokenlizer.py"))
    # imported by groundingdino.py for inference / visualisation only; their
    # real modules need slconfig (addict, yapf), cv2, matplotlib, pycocotools
    util.utils = _module("groundingdino.util.utils", get_phrases_from_posmap=_unavailable("get_phrases_from_posmap"))
    util.visualizer = _module("groundingdino.util.visualizer", COCOVisualizer=_unavailable("COCOVisualizer"))
    util.vl_utils = _module("groundingdino.util.vl_utils",
                            create_positive_map_from_span=_unavailable("create_positive_map_from_span"))
    top_util = _module("util")  # matcher.py imports util.box_ops
    top_util.__path__ = []
    top_util.box_ops = util.box_ops
    sys.modules["util.box_ops"] = util.box_ops

    models = _module("_refmodels")
    models.__path__ = [os.path.join(REF, "models")]
    refgd = _module("_refmodels.GroundingDINO")
    refgd.__path__ = [REF_GD]
    bb = _module("_refmodels.GroundingDINO.backbone", build_backbone=_unavailable("build_backbone"))
    bb.__path__ = [os.path.join(REF_GD, "backbone")]
    local_msda = _load_path("_refmodels.GroundingDINO.ms_deform_attn", os.path.join(REF_GD, "ms_deform_attn.py"))

    class MMCVMultiScaleDeformableAttention(local_msda.MultiScaleDeformableAttention):
        def __init__(self, embed_dims=256, num_heads=8, num_levels=4, num_points=4, im2col_step=64,
                     dropout=0.1, batch_first=False, norm_cfg=None, init_cfg=None):
            super().__init__(embed_dim=embed_dims, num_heads=num_heads, num_levels=num_levels,
                             num_points=num_points, img2col_step=im2col_step, batch_first=batch_first)
            self.dropout = nn.Dropout(dropout)

        def forward(self, query, key=None, value=None, identity=None, query_pos=None, key_padding_mask=None,
                    reference_points=None, spatial_shapes=None, level_start_index=None, **kwargs):
            if identity is None:
                identity = query
            out = super().forward(query, key=key, value=value, query_pos=query_pos,
                                  key_padding_mask=key_padding_mask, reference_points=reference_points,
                                  spatial_shapes=spatial_shapes, level_start_index=level_start_index)
            return self.dropout(out) + identity

    _module("mmcv")
    _module("mmcv.ops")
    _module("mmcv.ops.multi_scale_deform_attn", MultiScaleDeformableAttention=MMCVMultiScaleDeformableAttention)


def _tiny_language_model(_name):
    """get_pretrained_language_model stand-in: a random-init HF BertModel of
    block_spec.TINY_BERT, given the two transformers-4.x methods the
    reference's BertModelWarper binds (bertwarper.py:24-30) and that 5.x
    removed / changed: get_head_mask (returns [None] * n_layers for
    head_mask=None) and get_extended_attention_mask(mask, shape, device)
    (3rd argument was the device; [B,T,T] -> additive [B,1,T,T])."""
    from transformers import BertConfig, BertModel
    m = BertModel(BertConfig(**spec.TINY_BERT, attn_implementation="eager"))
    orig = m.get_extended_attention_mask
    m.get_head_mask = lambda head_mask, n_layers, *a, **k: [None] * n_layers
    m.get_extended_attention_mask = lambda mask, shape, device=None: orig(mask, shape)
    return m


def load_reference():
    install_shims()
    import importlib
    from gdino_amd.tokenizer import OfflineBertTokenizer
    gtk = sys.modules["groundingdino.util.get_tokenlizer"]
    gtk.get_tokenlizer = lambda name: OfflineBertTokenizer()  # bert-base-uncased cannot be fetched here
    gtk.get_pretrained_language_model = _tiny_language_model
    bb = sys.modules["_refmodels.GroundingDINO.backbone"]
    bb.build_backbone = importlib.import_module("_refmodels.GroundingDINO.backbone.backbone").build_backbone
    p = "_refmodels.GroundingDINO."
    return types.SimpleNamespace(
        fuse=importlib.import_module(p + "fuse_modules"),
        utils=importlib.import_module(p + "utils"),
        transformer=importlib.import_module(p + "transformer"),
        swin=importlib.import_module(p + "backbone.swin_transformer"),
        pos=importlib.import_module(p + "backbone.position_encoding"),
        matcher=importlib.import_module(p + "matcher"),
        gd=importlib.import_module(p + "groundingdino"),
        misc=sys.modules["groundingdino.util.misc"],
    )


# ----------------------------------------------------------------------------
# cases
# ----------------------------------------------------------------------------
def _np(x):
    return x.detach().cpu().numpy()


def _pgrad(res, name, grad):
    """Parameter gradients are stored as their first 4096 elements (fp32)
    plus full-tensor sums (fp64), which keeps the fixtures small."""
    g = grad.detach().double()
    res["pgrad." + name] = g.flatten()[:4096].float().numpy()
    res["pgradsum." + name] = np.array([float(g.sum()), float(g.abs().sum())])


def case_biattn(ref):
    torch.manual_seed(0)
    m = ref.fuse.BiAttentionBlock(**spec.BIATTN, dropout=0.0, drop_path=0.0).double().eval()
    ck = spec.fill_params(m)
    inp = spec.biattn_inputs()
    v = inp["v"].clone().requires_grad_(True)
    l = inp["l"].clone().requires_grad_(True)
    ov, ol = m(v, l, attention_mask_v=inp["mask_v"], attention_mask_l=inp["mask_l"])
    ((ov * inp["gv"]).sum() + (ol * inp["gl"]).sum()).backward()
    out = {"out_v": _np(ov), "out_l": _np(ol), "grad_v": _np(v.grad), "grad_l": _np(l.grad)}
    for name, p in m.named_parameters():
        _pgrad(out, name, p.grad)
    return out, {"weights_checksum": ck}


def case_swin(ref, cfg=None, inputs=None, tag=""):
    torch.manual_seed(0)
    m = ref.swin.SwinTransformer(**(cfg or spec.SWIN)).double()
    m.eval()  # SwinTransformer.train returns None in the reference: no chaining
    ck = spec.fill_params(m)
    inp = (inputs or spec.swin_inputs)()
    x = inp["x"].clone().requires_grad_(True)
    outs = m(ref.misc.NestedTensor(x, inp["mask"]))
    res, loss = {}, 0.0
    for k, nt in outs.items():
        # Swin-B feature maps are stored in fp32 (fixture size); held to 1e-6
        res[f"feat{k}"] = nt.tensors.detach().float().numpy() if tag else _np(nt.tensors)
        res[f"mask{k}"] = _np(nt.mask)
        g = spec.rand(nt.tensors.shape, f"swin{tag}_g{k}")
        loss = loss + (nt.tensors * g).sum()
    loss.backward()
    res["grad_x"] = x.grad.float().numpy()
    for name in ("patch_embed.proj.weight", "layers.0.blocks.1.attn.relative_position_bias_table",
                 "layers.2.blocks.0.attn.qkv.weight", "layers.3.blocks.1.mlp.fc2.weight", "norm3.weight"):
        _pgrad(res, name, dict(m.named_parameters())[name].grad)
    return res, {"weights_checksum": ck, "keys": sorted(outs.keys())}


def case_pos(ref):
    inp = spec.swin_inputs()
    pe = ref.pos.PositionEmbeddingSineHW(num_pos_feats=64, temperatureH=20, temperatureW=20, normalize=True)
    nt = ref.misc.NestedTensor(inp["x"], inp["mask"])
    return {"pos": _np(pe(nt))}, {}


def case_contrastive(ref):
    x = spec.rand((2, 30, 64), "ce_x")
    text = spec.rand((2, spec.TEXT_LEN, 64), "ce_text")
    token_mask, _, _ = spec.phrase_text()
    ce = ref.utils.ContrastiveEmbed()
    out = ce(x, {"encoded_text": text, "text_token_mask": token_mask})
    return {"logits": _np(out)}, {}


def case_proposals(ref):
    d = 64
    shapes = torch.as_tensor(spec.LEVELS, dtype=torch.long)
    s = int(shapes.prod(1).sum())
    memory = spec.rand((2, s, d), "prop_mem")
    masks = []
    for h, w in spec.LEVELS:
        m = torch.zeros(2, h, w, dtype=torch.bool)
        if w > 1:
            m[1, :, w - max(1, w // 4):] = True
        if h > 1:
            m[1, h - 1:, :] = True
        masks.append(m.flatten(1))
    mask = torch.cat(masks, 1)
    om, op = ref.utils.gen_encoder_output_proposals(memory, mask, shapes)
    return {"output_memory": _np(om), "output_proposals": _np(op), "memory": _np(memory), "mask": _np(mask)}, {}


def case_transformer(ref):
    torch.manual_seed(0)
    t = ref.transformer.Transformer(**spec.TRANSFORMER)
    spec.wire_heads(t, ref.utils.MLP, ref.utils.ContrastiveEmbed)
    t = t.double().eval()
    ck = spec.fill_params(t)
    inp = spec.transformer_inputs()
    srcs = [s.clone().requires_grad_(True) for s in inp["srcs"]]
    text = inp["text"].clone().requires_grad_(True)
    td = spec.transformer_text_dict(inp)
    td["encoded_text"] = text
    hs, refs, hs_enc, ref_enc, init_box = t(srcs, inp["masks"], None, inp["poss"], None, None, td)
    loss = (torch.stack(hs) * inp["g_hs"]).sum() + (torch.stack(refs) * inp["g_ref"]).sum() \
        + (hs_enc * inp["g_enc"]).sum()
    loss.backward()
    res = {f"hs{i}": _np(h) for i, h in enumerate(hs)}
    res.update({f"ref{i}": _np(r) for i, r in enumerate(refs)})
    res["hs_enc"] = _np(hs_enc)
    res["ref_enc"] = _np(ref_enc)
    res["init_box_proposal"] = _np(init_box)
    res.update({f"grad_src{i}": _np(s.grad) for i, s in enumerate(srcs)})
    res["grad_text"] = _np(text.grad)
    named = dict(t.named_parameters())
    for name in ("level_embed", "encoder.layers.0.self_attn.sampling_offsets.weight",
                 "encoder.fusion_layers.1.attn.values_l_proj.weight", "encoder.text_layers.0.self_attn.in_proj_weight",
                 "decoder.layers.1.cross_attn.value_proj.weight", "decoder.layers.0.ca_text.in_proj_weight",
                 "decoder.bbox_embed.0.layers.2.weight", "enc_output.weight", "tgt_embed.weight"):
        if name in named and named[name].grad is not None:
            _pgrad(res, name, named[name].grad)
    return res, {"weights_checksum": ck, "param_names": sorted(named.keys()),
                 "msda_semantics": "mmcv (dropout(output_proj(.)) + identity), dropout inactive (eval)"}


def case_criterion(ref):
    from gdino_amd.tokenizer import OfflineBertTokenizer
    inp = spec.criterion_inputs(OfflineBertTokenizer())
    matcher = ref.matcher.HungarianMatcher(**spec.MATCHER)
    crit = ref.gd.SetCriterion(matcher, spec.criterion_weight_dict(), spec.FOCAL_ALPHA, spec.FOCAL_GAMMA,
                               ["labels", "boxes"])
    outputs, leaves = spec.criterion_outputs(inp, dtype=torch.float32)  # the label maps are fp32
    losses = crit(outputs, inp["targets"], inp["cat_list"], inp["captions"])
    wd = crit.weight_dict
    total = sum(losses[k] * wd[k] for k in losses if k in wd)
    total.backward()
    res = {"loss." + k: np.array(float(v)) for k, v in losses.items()}
    res["total"] = np.array(float(total))
    res.update({"grad." + k: _np(v.grad) for k, v in leaves.items()})
    return res, {"loss_keys": sorted(losses.keys())}


def case_statedict(ref):
    """State-dict keys and shapes (parameters and buffers) of the reference
    modules at the real configurations: Swin-T / Swin-B-384 backbones and the
    cfg_odvg Transformer (6+6 layers, 900 queries) with its heads wired."""
    res = {}
    meta = {}
    for name, cfg in spec.STATE_DICT_SWINS.items():
        sd = ref.swin.SwinTransformer(**cfg).state_dict()
        meta[name] = {k: list(v.shape) for k, v in sd.items()}
    t = ref.transformer.Transformer(**spec.STATE_DICT_TRANSFORMER)
    spec.wire_heads(t, ref.utils.MLP, ref.utils.ContrastiveEmbed)
    meta["transformer_cfg_odvg"] = {k: list(v.shape) for k, v in t.state_dict().items()}
    res["n_keys"] = np.array([len(v) for v in meta.values()])
    return res, {"state_dicts": meta}


def case_model(ref):
    """build_groundingdino -> forward (final / aux / interm outputs) ->
    reference criterion losses, and parameter gradients of a fixed surrogate
    of all outputs; fp64, eval mode."""
    from gdino_amd.config import make_args
    from gdino_amd.tokenizer import OfflineBertTokenizer
    torch.manual_seed(0)
    args = make_args(device="cpu", **spec.MODEL_OVERRIDES)
    model, crit, _ = ref.gd.build_groundingdino(args)
    model = model.double()
    model.eval()
    ck = spec.fill_params(model)
    inp = spec.model_inputs(OfflineBertTokenizer())
    out = model(ref.misc.NestedTensor(inp["images"], inp["mask"]), captions=inp["captions"])
    res = {"pred_logits": _np(out["pred_logits"]), "pred_boxes": _np(out["pred_boxes"]),
           "aux0_logits": _np(out["aux_outputs"][0]["pred_logits"]),
           "aux0_boxes": _np(out["aux_outputs"][0]["pred_boxes"]),
           "interm_logits": _np(out["interm_outputs"]["pred_logits"]),
           "interm_boxes": _np(out["interm_outputs"]["pred_boxes"]), "text_mask": _np(out["text_mask"])}
    spec.model_surrogate(out).backward()
    named = dict(model.named_parameters())
    for name in spec.MODEL_PGRADS:
        _pgrad(res, name, named[name].grad)
    with torch.no_grad():
        targets = [{"boxes": t["boxes"].double(), "labels": t["labels"]} for t in inp["targets"]]
        losses = crit(out, targets, inp["cat_list"], inp["captions"])
    res.update({"loss." + k: np.array(float(v)) for k, v in losses.items()})
    return res, {"weights_checksum": ck, "param_names": sorted(named.keys()), "loss_keys": sorted(losses.keys()),
                 "note": "BERT = random-init HF BertModel(TINY_BERT) behind the reference BertModelWarper"}


def case_swin_b(ref):
    return case_swin(ref, spec.SWIN_B, spec.swin_b_inputs, "_b")


CASES = {"biattn": case_biattn, "swin": case_swin, "pos": case_pos, "contrastive": case_contrastive,
         "proposals": case_proposals, "transformer": case_transformer, "criterion": case_criterion,
         "statedict": case_statedict, "model": case_model,
         "swin_b": case_swin_b}


def main(names=None):
    # default dtype stays fp32, as in training: tensors the reference creates
    # without an explicit dtype (e.g. ContrastiveEmbed's -inf padding) keep
    # their real precision; modules and inputs are fp64.
    ref = load_reference()
    for name in names or CASES:
        arrays, meta = CASES[name](ref)
        meta["generator"] = "tests/golden/make_block_golden.py"
        arrays["meta_json"] = np.array(json.dumps(meta))
        path = os.path.join(HERE, f"block_{name}.npz")
        np.savez_compressed(path, **arrays)
        print(f"{name}: {len(arrays)} arrays -> {os.path.basename(path)} ({os.path.getsize(path) / 1e3:.0f} kB)")


if __name__ == "__main__":
    main(sys.argv[1:] or None)
