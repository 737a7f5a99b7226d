"""The product's HIP path end to end on the CPU: one Grounding DINO train
step (forward, criterion, backward) with every HIP op of the model reaching
the host-side SIMT emulator build of the kernel sources through the
product's own autograd functions and ctypes calls (tests/emu_product.py),
against the same step with the ops routed to the oracle restatements
(tests/oracle_hooks.py, pinned by the reference goldens).

fp32, eval mode (no dropout / drop-path randomness): loss, logits and every
parameter gradient agree to fp32 rounding.  Under bf16 autocast the
two-stage top-k and the Hungarian matching are discrete, so the bf16 check
compares the continuous part (backbone features, encoder memory) and the
TokenLinear weight-gradient path in isolation.
"""
import pytest
import torch

import emu_product
import oracle_hooks


def _off_cell_edges(model, std=0.01):
    """The reference MSDA init (ms_deform_attn.py:198-221: zero
    sampling_offsets weight, integer grid bias) puts every sampling point at
    init exactly on a bilinear cell edge (pixel-centre reference + integer
    pixel offset), where d(out)/d(loc) is one-sided and each implementation
    picks a side by its own rounding of loc*size - 0.5 (the reference CUDA
    kernel's, grid_sample's unnormalize, FMA contraction).  Both paths are
    compared at a generic point instead: a small seeded perturbation of the
    sampling_offsets weights (about 0.2 px), identical in both paths."""
    g = torch.Generator().manual_seed(7)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if n.endswith("sampling_offsets.weight"):
                p.copy_(torch.randn(p.shape, generator=g) * std)


def _step(mode, amp, hooks=None, size=(96, 128)):
    from gdino_amd import castcache, train
    from gdino_amd.config import make_args
    torch.manual_seed(0)
    args = make_args(device="cpu", num_queries=100)
    model, criterion, _, _ = train.build_training(args, "cpu")
    _off_cell_edges(model)
    model.eval()
    samples, targets, captions, cats = train.synthetic_batch(1, size[0], size[1], n_boxes=3, n_tokens=24, seed=0,
                                                             device="cpu")
    captured = {}
    handles = []
    for name in hooks or ():
        mod = dict(model.named_modules())[name]
        handles.append(mod.register_forward_hook(
            lambda m, i, o, name=name: captured.__setitem__(name, o)))
    castcache.clear()
    ctx = oracle_hooks.oracle_msda() if mode == "oracle" else emu_product.emulated_product(min_tokens=64)
    try:
        with ctx:
            with torch.autocast("cpu", dtype=torch.bfloat16, enabled=amp):
                out = model(samples, captions=captions)
                ld = criterion(out, targets, cats, captions)
                loss = sum(ld[k] * criterion.weight_dict[k] for k in ld if k in criterion.weight_dict)
            if not amp:
                loss.backward()
    finally:
        for h in handles:
            h.remove()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    return loss.detach(), out["pred_logits"].detach(), grads, captured


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.slow
def test_train_step_fp32_emulated_hip_path_matches_oracle_path():
    lo, po, go, _ = _step("oracle", False)
    le, pe, ge, _ = _step("emu", False)
    assert abs(float(le - lo)) <= 1e-5 * abs(float(lo))
    fin = torch.isfinite(po)
    assert torch.equal(fin, torch.isfinite(pe))
    assert _rel(pe[fin], po[fin]) < 1e-5
    assert set(go) == set(ge)
    worst = max((_rel(ge[n], go[n]), n) for n in go if go[n].norm() > 0)
    assert worst[0] < 1e-5, worst


def _flat(o):
    if torch.is_tensor(o):
        return [o]
    if isinstance(o, dict):
        return [t for v in o.values() for t in _flat(v)]
    if isinstance(o, (list, tuple)):
        return [t for v in o for t in _flat(v)]
    return [t for t in (getattr(o, "tensors", None),) if t is not None]


@pytest.mark.slow
def test_forward_bf16_emulated_hip_path_matches_oracle_path():
    names = ("backbone", "transformer.encoder")
    _, _, _, co = _step("oracle", True, hooks=names)
    _, _, _, ce = _step("emu", True, hooks=names)
    for n in names:
        for a, b in zip(_flat(ce[n]), _flat(co[n])):
            if a.is_floating_point():
                assert _rel(a.float(), b.float()) < 3e-2, n


def test_token_linear_emulated_matches_library_linear():
    """castcache.linear under bf16 autocast routed through TokenLinear (the
    split-K weight-gradient kernel) vs the plain autocast F.linear path."""
    from gdino_amd import castcache, wgrad
    torch.manual_seed(0)
    lin = torch.nn.Linear(128, 192)
    x = torch.randn(3, 300, 128)
    gy = torch.randn(3, 300, 192)
    res = {}
    for use in (True, False):
        castcache.clear()
        lin.zero_grad()
        xi = x.clone().requires_grad_(True)
        with emu_product.emulated_product(min_tokens=64):
            wgrad.ENABLED = use
            try:
                with torch.autocast("cpu", dtype=torch.bfloat16):
                    y = castcache.linear(xi, lin.weight, lin.bias)
                assert ("TokenLinear" in type(y.grad_fn).__name__) == use
                (y.float() * gy).sum().backward()
            finally:
                wgrad.ENABLED = True
        res[use] = (y.float(), lin.weight.grad.clone(), lin.bias.grad.clone(), xi.grad.clone())
    torch.testing.assert_close(res[True][0], res[False][0], rtol=0, atol=0)
    xd, wd, bd = (t.double().requires_grad_(True) for t in (x, lin.weight.detach(), lin.bias.detach()))
    (torch.nn.functional.linear(xd, wd, bd) * gy.double()).sum().backward()
    for k, ref in ((1, wd.grad), (2, bd.grad), (3, xd.grad)):
        assert _rel(res[True][k], ref) < 1e-2
        assert _rel(res[True][k], ref) <= _rel(res[False][k], ref) * 1.5 + 1e-6, k


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
def test_tn_matmul_batched(dtype, tol):
    """a^T b over 300 tokens, batched over [2, 3], bf16 / fp32 output."""
    from gdino_amd.wgrad import tn_matmul
    g = torch.Generator().manual_seed(0)
    a = torch.randn(2, 3, 300, 128, generator=g).to(dtype)
    b = torch.randn(2, 3, 300, 64, generator=g).to(dtype)
    with emu_product.emulated_product(min_tokens=64):
        out = tn_matmul(a, b)
    assert out.shape == (2, 3, 128, 64) and out.dtype == dtype
    assert _rel(out.float(), a.double().transpose(-1, -2) @ b.double()) < tol


def test_bi_attention_long_k_products_on_the_split_k_kernel():
    """BiAttention with its three image-token-long products (out_l = P_l^T v_v,
    dv_l = P_v^T dout_v, dk = dS^T q) on the split-K kernel, fp32, against the
    reference restatement with gradients."""
    from gdino_amd import biattn
    from oracle.blocks import bi_attention_ref
    g = torch.Generator().manual_seed(1)
    b, h, s, t, hd = 1, 2, 300, 64, 64
    q = torch.randn(b, h, s, hd, generator=g) * hd ** -0.5
    k, vl = torch.randn(b, h, t, hd, generator=g), torch.randn(b, h, t, hd, generator=g)
    vv = torch.randn(b, h, s, hd, generator=g)
    pad_v = torch.zeros(b, s, dtype=torch.bool)
    pad_v[0, 250:] = True
    pad_l = torch.zeros(b, t, dtype=torch.bool)
    pad_l[0, 40:] = True
    gv, gl = torch.randn(b, h, s, hd, generator=g), torch.randn(b, h, t, hd, generator=g)
    mine = [x.clone().requires_grad_(True) for x in (q, k, vv, vl)]
    with emu_product.emulated_product(min_tokens=64):
        assert biattn._long_k_ok(*mine[:2], *mine[2:])
        ov, ol = biattn.bi_attention_hip(*mine, pad_v, pad_l)
        ((ov * gv).sum() + (ol * gl).sum()).backward()
    ref = [x.double().requires_grad_(True) for x in (q, k, vv, vl)]
    rv, rl = bi_attention_ref(*ref, pad_v, pad_l)
    ((rv * gv.double()).sum() + (rl * gl.double()).sum()).backward()
    assert _rel(ov, rv) < 1e-5 and _rel(ol, rl) < 1e-5
    for a, r in zip(mine, ref):
        assert _rel(a.grad, r.grad) < 1e-5


def test_bi_attention_token_major_core_on_the_emulated_kernels():
    """biattn.BiAttnTokens (the model's path: joint projection outputs read
    through strided per-head views, the scale on k, one gradient tensor per
    joint output) with the softmax kernels and the split-K long-K products
    emulated, fp32, against the reference restatement with gradients."""
    from gdino_amd import biattn
    from oracle.blocks import bi_attention_ref
    g = torch.Generator().manual_seed(2)
    b, h, s, t, hd = 2, 2, 300, 64, 64
    e, scale = h * hd, hd ** -0.5
    qvv = torch.randn(b, s, 2 * e, generator=g)
    klv = torch.randn(b, t, 2 * e, generator=g)
    pad_v = torch.zeros(b, s, dtype=torch.bool)
    pad_v[1, 250:] = True
    pad_l = torch.zeros(b, t, dtype=torch.bool)
    pad_l[0, 40:] = True
    gv, gl = torch.randn(b, s, e, generator=g), torch.randn(b, t, e, generator=g)
    mine = [x.clone().requires_grad_(True) for x in (qvv, klv)]
    with emu_product.emulated_product(min_tokens=64):
        assert biattn.tokens_ok(*mine, h)
        ov, ol = biattn.BiAttnTokens.apply(mine[0], mine[1], pad_v, pad_l, h, scale)
        ((ov * gv).sum() + (ol * gl).sum()).backward()
    ref = [x.double().requires_grad_(True) for x in (qvv, klv)]
    hv = lambda x: x.unflatten(-1, (h, hd)).transpose(1, 2)  # noqa: E731
    rv, rl = bi_attention_ref(hv(ref[0][..., :e]) * scale, hv(ref[1][..., :e]), hv(ref[0][..., e:]),
                              hv(ref[1][..., e:]), pad_v, pad_l)
    tok = lambda x: x.transpose(1, 2).reshape(x.shape[0], x.shape[2], e)  # noqa: E731
    rv, rl = tok(rv), tok(rl)
    ((rv * gv.double()).sum() + (rl * gl.double()).sum()).backward()
    assert _rel(ov, rv) < 1e-5 and _rel(ol, rl) < 1e-5
    for a, r in zip(mine, ref):
        assert _rel(a.grad, r.grad) < 1e-5


def test_frozen_bert_fast_encoder_matches_the_layer_stack():
    """BertModelWarper._encode_frozen (fused Q/K/V GEMM, in-place q / k / v
    reads by the attention kernel, add + LayerNorm kernel with its bf16 twin
    feeding the next GEMM) against transformers' BertLayer stack on the same
    emulated kernels, bf16 autocast, train mode with the Dropout modules'
    rates zeroed (the fast path reads the modules, not the config, as the
    GPU parity tests zero them): one layer agrees to bf16 GEMM
    rounding flips (the fused Q/K/V product sums in another order); twelve
    random-init layers amplify those flips, still well inside the north
    star's bf16 1e-2.  Nothing is recorded for autograd (frozen encoder)."""
    from gdino_amd.config import make_args
    from gdino_amd.train import build_training
    from models.GroundingDINO.bertwarper import BertModelWarper
    torch.manual_seed(0)
    model, _, _, _ = build_training(make_args(device="cpu", enc_layers=1, dec_layers=1, num_queries=100),
                                    torch.device("cpu"))
    bert = model.bert
    bert.train()
    for m in bert.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    assert not any(p.requires_grad for p in bert.encoder.parameters())
    ids = torch.randint(1000, 2000, (2, 40))
    kw = dict(input_ids=ids, attention_mask=torch.ones(2, 40, 40, dtype=torch.bool),
              token_type_ids=torch.zeros_like(ids), position_ids=torch.arange(40)[None].repeat(2, 1))
    layers = bert.encoder.layer

    def run(fast, n):
        bert.encoder.layer = layers[:n]
        saved = BertModelWarper.FAST
        BertModelWarper.FAST = fast
        try:
            with emu_product.emulated_product(), torch.autocast("cpu", dtype=torch.bfloat16):
                return bert(**kw)["last_hidden_state"]
        finally:
            BertModelWarper.FAST = saved
            bert.encoder.layer = layers
    for n, tol in ((1, 2e-4), (12, 1e-2)):
        ref, fast = run(False, n), run(True, n)
        assert fast.grad_fn is None and fast.dtype == ref.dtype == torch.float32
        rel = float((fast - ref).norm() / ref.norm())
        assert rel < tol, (n, rel)


def test_frozen_bert_fast_path_keeps_trainable_embedding_gradients():
    """with the encoder frozen but the embeddings trainable
    (a partial freeze), the fast path (which runs under no_grad) is refused,
    so the output keeps its autograd graph back to the embeddings; with
    nothing upstream needing a gradient it is taken."""
    from gdino_amd.config import make_args
    from gdino_amd.train import build_training
    torch.manual_seed(0)
    model, _, _, _ = build_training(make_args(device="cpu", enc_layers=1, dec_layers=1, num_queries=100),
                                    torch.device("cpu"))
    bert = model.bert
    bert.train()
    for m in bert.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    assert not any(p.requires_grad for p in bert.encoder.parameters())
    bert.encoder.layer = bert.encoder.layer[:2]
    ids = torch.randint(1000, 2000, (2, 24))
    kw = dict(input_ids=ids, attention_mask=torch.ones(2, 24, 24, dtype=torch.bool),
              token_type_ids=torch.zeros_like(ids), position_ids=torch.arange(24)[None].repeat(2, 1))
    taken = []
    orig = type(bert)._fast_ok

    def spy(self, hidden, head_mask):
        r = orig(self, hidden, head_mask)
        taken.append(r)
        return r
    type(bert)._fast_ok = spy
    try:
        for trainable in (False, True):
            bert.embeddings.word_embeddings.weight.requires_grad_(trainable)
            with emu_product.emulated_product(), torch.autocast("cpu", dtype=torch.bfloat16):
                out = bert(**kw)["last_hidden_state"]
            assert (out.grad_fn is not None) == trainable
    finally:
        type(bert)._fast_ok = orig
    assert taken == [True, False]
