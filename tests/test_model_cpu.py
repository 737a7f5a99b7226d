"""Host-logic tests on CPU: the drop-in model API, architecture parity
(parameter counts measured on the reference modules), the
torch-composed attention-family ops vs the oracle's literal restatements,
text masks vs the reference loop, and one full train step (MSDA routed to
the oracle through tests/oracle_hooks.py — the product raises on CPU)."""
import random

import pytest
import torch

from oracle.blocks import (attention_ref, bi_attention_ref, contrastive_ref, phrase_masks_ref,
                           window_attention_ref)
from oracle_hooks import oracle_msda


@pytest.fixture(scope="module")
def built():
    from gdino_amd.config import make_args
    from gdino_amd.train import build_training
    torch.manual_seed(0)
    args = make_args(device="cpu", num_queries=100)
    model, criterion, post, opt = build_training(args, "cpu")
    return args, model, criterion, post, opt


def test_registry_and_builder_contract():
    from models.registry import MODULE_BUILD_FUNCS
    import models  # noqa: F401
    assert MODULE_BUILD_FUNCS.get("groundingdino") is not None


def test_parameter_counts_match_reference(built):
    args, model, *_ = built
    total = sum(p.numel() for p in model.parameters())
    trainable = sum(p.numel() for p in model.parameters() if p.requires_grad)
    # reference modules, cfg_odvg, BERT frozen: 172.84M / 63.36M
    assert total == 172_839_682 + (100 - 900) * 256  # tgt_embed has num_queries rows
    assert trainable == 63_357_442 + (100 - 900) * 256


def test_state_dict_names_follow_reference(built):
    _, model, *_ = built
    keys = set(model.state_dict())
    for k in ("transformer.encoder.layers.0.self_attn.sampling_offsets.weight",
              "transformer.encoder.layers.5.self_attn.value_proj.bias",
              "transformer.decoder.layers.0.cross_attn.attention_weights.weight",
              "transformer.decoder.layers.0.ca_text.in_proj_weight",
              "transformer.decoder.layers.0.self_attn.out_proj.weight",
              "transformer.encoder.fusion_layers.0.attn.values_l_proj.weight",
              "transformer.encoder.fusion_layers.0.gamma_v",
              "transformer.encoder.text_layers.0.self_attn.in_proj_bias",
              "transformer.enc_output_norm.weight", "transformer.level_embed", "transformer.tgt_embed.weight",
              "transformer.decoder.ref_point_head.layers.1.weight", "transformer.enc_out_bbox_embed.layers.2.bias",
              "backbone.0.patch_embed.proj.weight", "backbone.0.layers.2.blocks.5.attn.relative_position_bias_table",
              "backbone.0.layers.0.blocks.1.attn.relative_position_index", "backbone.0.norm3.weight",
              "backbone.0.layers.1.downsample.reduction.weight", "input_proj.3.0.weight", "input_proj.3.1.bias",
              "bert.embeddings.word_embeddings.weight", "bert.encoder.layer.11.attention.self.query.weight",
              "bert.pooler.dense.weight", "feat_map.weight", "bbox_embed.0.layers.0.weight"):
        assert k in keys, k


def test_train_step_and_outputs(built):
    from gdino_amd.train import synthetic_batch, train_step
    args, model, criterion, post, opt = built
    samples, targets, caps, cats = synthetic_batch(2, 128, 160, n_boxes=3, n_tokens=40, seed=0, device="cpu")
    model.train()
    with oracle_msda():
        loss = train_step(model, criterion, opt, samples, targets, caps, cats, amp_dtype=None)
        assert torch.isfinite(loss)
        model.eval()
        with torch.no_grad():
            out = model(samples, captions=caps)
    assert out["pred_logits"].shape == (2, 100, 256)
    assert out["pred_boxes"].shape == (2, 100, 4)
    assert out["text_mask"].shape == (2, 256) and out["text_mask"][:, :40].all() and not out["text_mask"][:, 40:].any()
    assert len(out["aux_outputs"]) == 5
    assert out["interm_outputs"]["pred_logits"].shape == (2, 100, 256)
    assert ((out["pred_boxes"] >= 0) & (out["pred_boxes"] <= 1)).all()
    losses = criterion(out, targets, cats, caps)
    assert set(losses) >= set(criterion.weight_dict)
    res = post["bbox"](out, torch.tensor([[128, 160], [128, 160]]))
    assert res[0]["boxes"].shape == (300, 4)


def test_phrase_masks_match_reference_loop():
    from models.GroundingDINO.bertwarper import generate_masks_with_special_tokens
    from gdino_amd.tokenizer import OfflineBertTokenizer
    from gdino_amd.train import synthetic_caption
    tok = OfflineBertTokenizer()
    rng = random.Random(3)
    caps = [" . ".join(synthetic_caption(rng, n)) + " ." for n in (40, 25, 33)]
    enc = tok(caps, padding="longest", return_tensors="pt")
    special = tok.convert_tokens_to_ids(["[CLS]", "[SEP]", ".", "?"])
    m, p = generate_masks_with_special_tokens(enc, special, tok)
    rm, rp = phrase_masks_ref(enc["input_ids"], special)
    assert torch.equal(m, rm) and torch.equal(p, rp)


def test_bi_attention_matches_reference_math():
    from gdino_amd import kernels
    g = torch.Generator().manual_seed(0)
    b, h, s, t, hd = 2, 4, 57, 13, 16
    q = torch.randn(b, h, s, hd, generator=g) * 0.5
    k, vl = torch.randn(b, h, t, hd, generator=g), torch.randn(b, h, t, hd, generator=g)
    vv = torch.randn(b, h, s, hd, generator=g)
    pad_v = torch.zeros(b, s, dtype=torch.bool)
    pad_v[1, 40:] = True
    pad_l = torch.zeros(b, t, dtype=torch.bool)
    pad_l[0, 10:] = True
    # the SDPA composition (used for fusion_dropout > 0) on CPU; the HIP
    # kernels are compared with the same oracle in test_kernels_gpu.py
    ov, ol = kernels._bi_attention_torch(q, k, vv, vl, pad_v, pad_l, 0.0)
    rv, rl = bi_attention_ref(q, k, vv, vl, pad_v, pad_l)
    torch.testing.assert_close(ov, rv, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ol, rl, rtol=1e-5, atol=1e-5)


def test_window_attention_and_attention_and_contrastive():
    from gdino_amd import kernels
    from models.GroundingDINO.backbone.swin_transformer import shifted_window_mask
    g = torch.Generator().manual_seed(1)
    q, k, v = (torch.randn(8, 3, 49, 32, generator=g) for _ in range(3))
    bias = torch.randn(3, 49, 49, generator=g)
    mask = shifted_window_mask(14, 28, 7, 3, "cpu")  # 2 x 4 = 8 windows
    torch.testing.assert_close(kernels.window_attention(q, k, v, bias, mask, 32 ** -0.5),
                               window_attention_ref(q, k, v, bias, mask, 32 ** -0.5), rtol=1e-5, atol=1e-5)
    q2, k2, v2 = torch.randn(2, 4, 30, 64, generator=g), torch.randn(2, 4, 20, 64, generator=g), \
        torch.randn(2, 4, 20, 64, generator=g)
    keep = torch.rand(2, 1, 30, 20, generator=g) > 0.3
    keep[..., 0] = True
    # the SDPA composition (shapes the HIP kernel does not cover) on CPU; the
    # HIP kernel is compared with the same oracle in test_kernels_gpu.py and,
    # on the host-side emulator, in test_emu_kernels.py
    torch.testing.assert_close(kernels._attention_torch(q2, k2, v2, keep), attention_ref(q2, k2, v2, keep),
                               rtol=1e-5, atol=1e-5)
    with pytest.raises(RuntimeError, match="Not implemented on the CPU"):
        kernels.attention(q2, k2, v2, keep)
    x, txt = torch.randn(2, 50, 32, generator=g), torch.randn(2, 11, 32, generator=g)
    tm = torch.ones(2, 11, dtype=torch.bool)
    tm[1, 7:] = False
    torch.testing.assert_close(kernels._contrastive_torch(x, txt, tm, 256), contrastive_ref(x, txt, tm, 256))
    from gdino_amd.contrastive import contrastive_rowmax_torch
    torch.testing.assert_close(contrastive_rowmax_torch(x, txt, tm), contrastive_ref(x, txt, tm, 256).max(-1)[0])
    with pytest.raises(RuntimeError, match="Not implemented on the CPU"):
        kernels.contrastive_logits(x, txt, tm, 256)


def test_mha_matches_torch_multihead_attention():
    """gdino_amd.mha vs nn.MultiheadAttention (the reference's module) with
    shared weights, including the text enhancer's head-major mask tiling."""
    from gdino_amd.mha import MultiheadAttention
    torch.manual_seed(0)
    ref = torch.nn.MultiheadAttention(64, 4)
    mine = MultiheadAttention(64, 4)
    mine.load_state_dict(ref.state_dict())
    q, kv = torch.randn(12, 2, 64), torch.randn(9, 2, 64)
    kpm = torch.zeros(2, 9, dtype=torch.bool)
    kpm[1, 6:] = True
    torch.testing.assert_close(mine(q, kv, kv, key_padding_mask=kpm)[0], ref(q, kv, kv, key_padding_mask=kpm)[0])
    m3 = torch.rand(2, 12, 12) > 0.5
    m3 |= torch.eye(12, dtype=torch.bool)
    tiled = (~m3).repeat(4, 1, 1)
    torch.testing.assert_close(mine(q, q, q, attn_mask=tiled)[0], ref(q, q, q, attn_mask=tiled)[0])


def test_cast_cache_is_bit_identical_under_autocast(built):
    """gdino_amd.castcache (one bf16 cast per parameter per step, reused by the
    checkpoint recompute and by the frozen BERT) must not change a single bit
    of the loss or of any gradient relative to plain autocast casting."""
    from gdino_amd import castcache
    from gdino_amd.train import synthetic_batch
    args, model, criterion, *_ = built
    samples, targets, caps, cats = synthetic_batch(2, 128, 160, n_boxes=3, n_tokens=40, seed=1, device="cpu")
    model.train()
    assert any(isinstance(m, castcache.CachedCastLinear) for m in model.modules())

    def run(enabled, fuse=False, amp=True, shadows=True):
        castcache.ENABLED = enabled
        castcache.FUSE_SHARED_INPUT = fuse
        castcache.SHADOWS = shadows
        castcache.clear()
        torch.manual_seed(7)
        for p in model.parameters():
            p.grad = None
        with oracle_msda():  # the checkpoint recompute in backward runs MSDA again
            with torch.autocast("cpu", dtype=torch.bfloat16, enabled=amp):
                out = model(samples, captions=caps)
                ld = criterion(out, targets, cats, caps)
                loss = sum(ld[k] * criterion.weight_dict[k] for k in ld if k in criterion.weight_dict)
            loss.backward()
        # the step-shadow path (one multi-tensor cast per step) was taken
        assert (len(castcache._shadow) > 100) == (enabled and amp and shadows)
        return loss.detach().clone(), {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}

    try:
        l0, g0 = run(False)
        l1, g1 = run(True)
        ls, gs = run(True, shadows=False)
        l2, g2 = run(True, fuse=True)
        lf, gf = run(True, amp=False)
    finally:
        castcache.ENABLED = True
        castcache.FUSE_SHARED_INPUT = True
        castcache.SHADOWS = True
        castcache.clear()
    assert torch.equal(l0, l1) and torch.equal(l0, ls)
    assert g0.keys() == g1.keys() == g2.keys() == gs.keys() and len(g0) > 100
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n
        assert torch.equal(g0[n], gs[n]), n
    # shared-input projections as one GEMM: same math (pinned at 1e-9 in fp64
    # by test_blocks_golden), GEMM blocking may round differently in bf16 ->
    # must stay within the bf16-vs-fp32 noise of the unfused path
    def rel(a, b):
        return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))
    assert abs(float(l2) - float(l0)) <= 1e-2 * abs(float(l0))
    noise = max(rel(g0[n], gf[n]) for n in gf)
    fused = max(rel(g2[n], gf[n]) for n in gf)
    assert fused <= 1.25 * noise + 0.02, (fused, noise)


def test_window_attention_packed_torch_composition_matches_oracle():
    """The torch composition behind window_attention_packed (used for shapes
    the HIP kernel does not cover) equals the reference restatement (fp64)."""
    from gdino_amd.wattn import window_attention_packed_torch
    from models.GroundingDINO.backbone.swin_transformer import relative_position_index
    from oracle.blocks import window_attention_packed_ref
    g = torch.Generator().manual_seed(0)
    for ws, masked in ((7, True), (12, False)):
        n = ws * ws
        qkv = torch.randn(8, n, 3, 4, 32, generator=g, dtype=torch.float64)
        table = torch.randn((2 * ws - 1) ** 2, 4, generator=g, dtype=torch.float64)
        ridx = relative_position_index(ws, ws).reshape(-1)
        mask = torch.where(torch.rand(4, n, n, generator=g) < 0.3, -100.0, 0.0).double() if masked else None
        torch.testing.assert_close(window_attention_packed_torch(qkv, table, ridx, mask, 32 ** -0.5),
                                   window_attention_packed_ref(qkv, table, ridx, mask, 32 ** -0.5),
                                   rtol=1e-12, atol=1e-12)


def test_kernel_families_can_be_disabled(monkeypatch):
    """GDINO_DISABLE lists kernel families that fall back to their torch
    compositions (A/B runs and bisection on the box)."""
    from gdino_amd import _lib
    monkeypatch.setenv("GDINO_DISABLE", "wattn, attn")
    assert not _lib.enabled("wattn") and not _lib.enabled("attn") and _lib.enabled("addln")
    monkeypatch.delenv("GDINO_DISABLE")
    assert _lib.enabled("wattn")


def test_weighted_loss_matches_the_per_term_sum():
    """train.weighted_loss (stack x cached weights, one sum) vs the reference
    engine's sum(loss_dict[k] * weight_dict[k]): the same total to rounding,
    every term's gradient exactly its weight, keys outside weight_dict
    ignored, dtypes promoted (fp64 stays fp64)."""
    from gdino_amd.train import weighted_loss
    g = torch.Generator().manual_seed(0)
    wd = {f"loss_{i}": float(w) for i, w in enumerate(torch.rand(45, generator=g) * 5)}
    for dt in (torch.float32, torch.float64):
        ld = {k: torch.rand((), generator=g, dtype=dt).requires_grad_(True) for k in wd}
        ld["cardinality_error"] = torch.tensor(3.0, dtype=dt)
        ld["loss_2"] = ld["loss_2"].detach().to(torch.bfloat16).requires_grad_(True)
        ref = sum(ld[k] * wd[k] for k in ld if k in wd)
        ref_promoted = sum(ld[k].to(dt) * wd[k] for k in ld if k in wd)  # the bf16 term's product in dt
        tot = weighted_loss(ld, wd)
        assert tot.dtype == dt
        torch.testing.assert_close(tot, ref_promoted, rtol=1e-6, atol=0)
        torch.testing.assert_close(tot, ref.to(dt), rtol=1e-4, atol=0)
        grads = torch.autograd.grad(tot, [ld[k] for k in wd])
        for k, gk in zip(wd, grads):
            want = torch.tensor(wd[k], dtype=ld[k].dtype)
            assert torch.equal(gk, want), k


def test_cast_cache_follows_fused_adamw_updates(built):
    """Fused AdamW updates parameters in place without bumping their version
    counters; the cast cache must still serve the updated weights on the next
    step.  Two train steps with the cache on and off (fp32-exact casts: same
    bits) must give bit-identical second-step losses."""
    from gdino_amd import castcache
    from gdino_amd.train import synthetic_batch, train_step
    args, model0, criterion, *_ = built
    samples, targets, caps, cats = synthetic_batch(1, 128, 160, n_boxes=3, n_tokens=24, seed=2, device="cpu")
    p = torch.nn.Parameter(torch.ones(3))
    opt = torch.optim.AdamW([p], lr=0.1, fused=True)
    p.grad = torch.ones(3)
    v = p._version
    opt.step()
    assert p._version == v, "fused AdamW bumps versions now: the generation guard is still needed for foreach=False"
    losses = {}
    model = model0
    state = {k: v.clone() for k, v in model.state_dict().items()}
    drop = {id(m): (m.p if isinstance(m, torch.nn.Dropout) else m.drop_prob) for m in model.modules()
            if isinstance(m, torch.nn.Dropout) or hasattr(m, "drop_prob")}
    for enabled in (True, False):
        castcache.ENABLED = enabled
        castcache.FUSE_SHARED_INPUT = False  # same GEMMs both ways (bit-identical gradients)
        castcache.clear()
        model.load_state_dict(state)
        model.train()
        for m in model.modules():  # deterministic: no dropout / drop-path
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
            if hasattr(m, "drop_prob"):
                m.drop_prob = 0.0
        opt = torch.optim.AdamW([q for q in model.parameters() if q.requires_grad], lr=1e-2, fused=True)
        try:
            with oracle_msda():
                losses[enabled] = [float(train_step(model, criterion, opt, samples, targets, caps, cats))
                                   for _ in range(2)]
        finally:
            castcache.ENABLED = True
            castcache.FUSE_SHARED_INPUT = True
            castcache.clear()
            model.load_state_dict(state)
            model.zero_grad(set_to_none=True)
            for m in model.modules():
                if id(m) in drop:
                    if isinstance(m, torch.nn.Dropout):
                        m.p = drop[id(m)]
                    else:
                        m.drop_prob = drop[id(m)]
    assert losses[True][0] == losses[False][0]
    assert losses[True][1] == losses[False][1], losses
    assert losses[True][1] != losses[True][0]


def test_mixed_od_vg_batch_trains(built):
    """BASELINE config 5's mixed batch: one OD image (category-name caption)
    and one VG image (short caption of unique free-text phrases, several boxes
    per phrase, datasets/odvg.py:236-252) through one train step on the
    product's host logic (HIP-only ops routed to the oracle)."""
    from gdino_amd.train import synthetic_batch, train_step
    args, model, criterion, *_ = built
    samples, targets, caps, cats = synthetic_batch(2, 128, 160, n_boxes=5, n_tokens=40, seed=3, device="cpu",
                                                   vg_images=1)
    od, vg = targets
    assert len(cats[0]) > len(cats[1]) >= 1 and len(set(cats[1])) == len(cats[1])
    assert all(len(p.split()) >= 2 for p in cats[1])           # free-text phrases
    assert len(set(vg["labels"].tolist())) == len(cats[1]) < 5  # phrases shared by boxes, all used
    assert vg["caption"] == " . ".join(cats[1]) + " ."
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-5)
    model.train()
    with oracle_msda():
        loss = train_step(model, criterion, opt, samples, targets, caps, cats)
    assert torch.isfinite(loss)


def test_activation_checkpointing_does_not_change_the_step():
    """train.set_activation_checkpointing: the reference's checkpointing
    (Swin blocks, fusion layers, encoder layers) only trades recompute for
    memory -- with it off (the MI355X default: the activations stay in HBM)
    the loss is bitwise the same and every gradient agrees to fp32 rounding
    (summation order at the checkpoint boundaries), dropout / drop-path
    included (the recompute replays the RNG state)."""
    from gdino_amd.config import make_args
    from gdino_amd.train import (activation_checkpointing, build_training, set_activation_checkpointing,
                                 synthetic_batch, weighted_loss)
    torch.manual_seed(0)
    args = make_args(device="cpu", num_queries=60, enc_layers=2, dec_layers=2)
    model, criterion, _, _ = build_training(args, "cpu")
    model.train()
    assert activation_checkpointing(model)  # cfg_odvg: use_checkpoint / use_transformer_ckpt
    samples, targets, caps, cats = synthetic_batch(2, 96, 128, n_boxes=3, n_tokens=30, seed=3, device="cpu")
    res = {}
    for on in (True, False):
        assert set_activation_checkpointing(model, on) > 0
        model.zero_grad(set_to_none=True)
        torch.manual_seed(123)
        with oracle_msda():
            out = model(samples, captions=caps)
            loss = weighted_loss(criterion(out, targets, cats, caps), criterion.weight_dict)
            loss.backward()
        res[on] = (loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})
    assert torch.equal(res[True][0], res[False][0])
    assert set(res[True][1]) == set(res[False][1])
    for n, g in res[True][1].items():
        # a checkpoint boundary hands back its inputs' gradient contributions
        # (the residual stream, the level / position embeddings used by every
        # layer) in another summation order: fp32 rounding apart
        r = res[False][1][n]
        assert float((g - r).abs().max()) <= 1e-5 * float(r.abs().max().clamp_min(1e-30)), n
    set_activation_checkpointing(model, True)


def test_padding_free_batch_skips_only_an_identity_mask():
    """A batch whose images all fill the canvas (NestedTensor.padding_free:
    known on the host) skips the deformable attention's value masked_fill;
    the mask is all False there, so the loss is bitwise that of the masked run
    and every gradient agrees to fp32 summation order.  nested_tensor_from_tensor_list sets the flag
    only when no image was padded."""
    from gdino_amd.config import make_args
    from gdino_amd.misc import NestedTensor, nested_tensor_from_tensor_list
    from gdino_amd.train import build_training, synthetic_batch, weighted_loss
    torch.manual_seed(0)
    model, criterion, _, _ = build_training(make_args(device="cpu", num_queries=60, enc_layers=1, dec_layers=1),
                                            "cpu")
    model.train()
    samples, targets, caps, cats = synthetic_batch(2, 96, 128, n_boxes=3, n_tokens=30, seed=3, device="cpu")
    assert samples.padding_free and not bool(samples.mask.any())
    res = {}
    for pf in (True, False):
        model.zero_grad(set_to_none=True)
        torch.manual_seed(123)
        with oracle_msda():
            out = model(NestedTensor(samples.tensors, samples.mask, pf), captions=caps)
            loss = weighted_loss(criterion(out, targets, cats, caps), criterion.weight_dict)
            loss.backward()
        res[pf] = (loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})
    assert torch.equal(res[True][0], res[False][0])
    for n, g in res[True][1].items():
        # (the autograd engine may sum a tensor's incoming gradients in
        # another order without the masked_fill node, and the CPU's threaded
        # reductions -- e.g. a relative-position-bias table summed over every
        # window -- need not repeat their order: fp32 rounding apart, seen up
        # to 1.1e-6 of the tensor's max)
        r = res[False][1][n]
        assert float((g - r).abs().max()) <= 1e-5 * float(r.abs().max().clamp_min(1e-30)), n
    a, b = torch.zeros(3, 8, 8), torch.zeros(3, 6, 8)
    assert nested_tensor_from_tensor_list([a, a]).padding_free
    assert not nested_tensor_from_tensor_list([a, b]).padding_free


def test_group_shadows_make_the_fused_projection_cat_a_view(built):
    """castcache group shadows: the shadows of the parameters a fused
    projection concatenates (MSDA offsets | weights, BiAttention v | values_v,
    l | values_l) are laid out back to back, so the bf16 concatenation is a
    buffer view instead of a cat kernel per call -- bitwise the same loss
    and gradients as the cat path."""
    from gdino_amd import castcache
    from gdino_amd.train import synthetic_batch
    args, model, criterion, *_ = built
    samples, targets, caps, cats = synthetic_batch(2, 128, 160, n_boxes=3, n_tokens=40, seed=2, device="cpu")
    model.train()
    cat_calls = []

    def run(group):
        castcache.GROUP_SHADOWS = group
        castcache.clear()
        res = None
        for it in range(2):  # the first forward registers the groups, the next refresh lays them out
            torch.manual_seed(7)
            for p in model.parameters():
                p.grad = None
            cat_calls.clear()
            with oracle_msda(), torch.autocast("cpu", dtype=torch.bfloat16):
                castcache._cache.clear()  # as under capture: no per-call cache, every fused call concatenates
                orig_gs = castcache._GroupShadow.apply
                castcache._GroupShadow.apply = lambda *a: cat_calls.append("view") or orig_gs(*a)
                try:
                    out = model(samples, captions=caps)
                finally:
                    castcache._GroupShadow.apply = orig_gs
                ld = criterion(out, targets, cats, caps)
                loss = sum(ld[k] * criterion.weight_dict[k] for k in ld if k in criterion.weight_dict)
            with oracle_msda():  # the checkpoint recompute runs MSDA again
                loss.backward()
            res = (loss.detach().clone(), {n: p.grad.clone() for n, p in model.named_parameters()
                                           if p.grad is not None}, cat_calls.count("view"),
                   len(castcache._group_buf))
        return res

    try:
        lc, gc, ncat_c, nb_c = run(False)
        lg, gg, ncat_g, nb_g = run(True)
    finally:
        castcache.GROUP_SHADOWS = True
        castcache.clear()
    assert nb_c == 0 and nb_g >= 4
    assert ncat_c == 0 and ncat_g >= 4  # the fused projections took the buffer views
    assert torch.equal(lc, lg)
    assert gc.keys() == gg.keys()
    for n in gc:
        assert torch.equal(gc[n], gg[n]), n
