"""Bisect HIP-graph capture problems: capture one model piece per
subprocess (fwd+bwd via make_graphed_callables), replay, compare with eager.
Stops at the first failing piece."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

CASES = ["msda", "biattn", "swin", "bert", "enc_ckpt", "text_layer", "dec_layer"]


def build(case, dev):
    import torch
    from torch import nn
    torch.manual_seed(0)
    if case == "msda":
        from models.GroundingDINO.ms_deform_attn import MultiScaleDeformableAttention
        m = MultiScaleDeformableAttention(256, 8, 4, 4, batch_first=True, dropout=0.0).to(dev)
        shapes = torch.as_tensor([(32, 40), (16, 20), (8, 10), (4, 5)], device=dev)
        lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
        S = int(shapes.prod(1).sum())

        class W(nn.Module):
            def __init__(s):
                super().__init__()
                s.m = m

            def forward(s, x, ref):
                return s.m(query=x, value=x, reference_points=ref, spatial_shapes=shapes, level_start_index=lsi)
        return W(), (torch.randn(2, S, 256, device=dev, requires_grad=True), torch.rand(2, S, 4, 2, device=dev))
    if case == "biattn":
        from models.GroundingDINO.fuse_modules import BiAttentionBlock
        m = BiAttentionBlock(256, 256, 1024, 4, dropout=0.0, drop_path=0.0).to(dev)
        return m, (torch.randn(2, 3000, 256, device=dev, requires_grad=True),
                   torch.randn(2, 64, 256, device=dev, requires_grad=True),
                   torch.zeros(2, 3000, dtype=torch.bool, device=dev), torch.zeros(2, 64, dtype=torch.bool, device=dev))
    if case == "swin":
        from models.GroundingDINO.backbone.swin_transformer import build_swin_transformer
        m = build_swin_transformer("swin_T_224_1k", 224, out_indices=(1, 2, 3), use_checkpoint=True,
                                   drop_path_rate=0.0).to(dev)

        class W(nn.Module):
            def __init__(s):
                super().__init__()
                s.m = m

            def forward(s, x):
                return s.m.forward_raw(x)
        return W(), (torch.randn(2, 3, 256, 320, device=dev),)
    if case == "bert":
        from transformers import BertConfig, BertModel
        from models.GroundingDINO.bertwarper import BertModelWarper
        cfg = BertConfig()
        m = BertModelWarper(BertModel(cfg)).to(dev)

        class W(nn.Module):
            def __init__(s):
                super().__init__()
                s.m = m
                s.proj = nn.Linear(768, 256).to(dev)

            def forward(s, ids, mask, pos):
                return s.proj(s.m(input_ids=ids, attention_mask=mask, position_ids=pos)["last_hidden_state"])
        ids = torch.randint(1000, 2000, (2, 64), device=dev)
        mask = torch.ones(2, 64, 64, dtype=torch.bool, device=dev)
        pos = torch.arange(64, device=dev)[None].expand(2, -1).contiguous()
        return W(), (ids, mask, pos)
    if case in ("enc_ckpt",):
        import torch.utils.checkpoint as cp
        from models.GroundingDINO.transformer import DeformableTransformerEncoderLayer
        m = DeformableTransformerEncoderLayer(256, 2048, 0.0, "relu", 4, 8, 4).to(dev)
        m.self_attn.dropout.p = 0.0
        shapes = torch.as_tensor([(32, 40), (16, 20), (8, 10), (4, 5)], device=dev)
        lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
        S = int(shapes.prod(1).sum())

        class W(nn.Module):
            def __init__(s):
                super().__init__()
                s.m = m

            def forward(s, x, pos, ref):
                return cp.checkpoint(s.m, x, pos, ref, shapes, lsi, None, use_reentrant=False)
        return W(), (torch.randn(2, S, 256, device=dev, requires_grad=True), torch.randn(2, S, 256, device=dev),
                     torch.rand(2, S, 4, 2, device=dev))
    if case == "text_layer":
        from models.GroundingDINO.transformer_vanilla import TransformerEncoderLayer
        m = TransformerEncoderLayer(256, 4, 1024, dropout=0.0).to(dev)
        mask = torch.rand(2, 64, 64, device=dev) > 0.5
        mask |= torch.eye(64, dtype=torch.bool, device=dev)

        class W(nn.Module):
            def __init__(s):
                super().__init__()
                s.m = m

            def forward(s, x, msk):
                return s.m(x, src_mask=~msk)
        return W(), (torch.randn(64, 2, 256, device=dev, requires_grad=True), mask)
    if case == "dec_layer":
        from models.GroundingDINO.transformer import DeformableTransformerDecoderLayer
        m = DeformableTransformerDecoderLayer(256, 2048, 0.0, "relu", 4, 8, 4, use_text_cross_attention=True).to(dev)
        m.cross_attn.dropout.p = 0.0
        shapes = torch.as_tensor([(32, 40), (16, 20), (8, 10), (4, 5)], device=dev)
        lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
        S = int(shapes.prod(1).sum())

        class W(nn.Module):
            def __init__(s):
                super().__init__()
                s.m = m

            def forward(s, tgt, qpos, ref, text, tmask, mem):
                return s.m(tgt=tgt, tgt_query_pos=qpos, tgt_reference_points=ref, memory_text=text,
                           text_attention_mask=tmask, memory=mem, memory_level_start_index=lsi,
                           memory_spatial_shapes=shapes)
        return W(), (torch.randn(300, 2, 256, device=dev, requires_grad=True), torch.randn(300, 2, 256, device=dev),
                     torch.rand(300, 2, 4, 4, device=dev), torch.randn(2, 64, 256, device=dev),
                     torch.zeros(2, 64, dtype=torch.bool, device=dev), torch.randn(S, 2, 256, device=dev))
    raise ValueError(case)


def run_case(case):
    import torch
    dev = torch.device("cuda")
    mod, args = build(case, dev)
    mod.train()

    def loss_of(outs):
        outs = outs if isinstance(outs, (tuple, list)) else (outs,)
        return sum(o.float().pow(2).mean() for o in outs if o.is_floating_point())

    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        ref = loss_of(mod(*args))
    ref.backward()
    g_ref = [p.grad.clone() for p in mod.parameters() if p.grad is not None]
    for p in mod.parameters():
        p.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        graphed = torch.cuda.make_graphed_callables(mod, args, num_warmup_iters=3)
    torch.cuda.synchronize()
    print(f"{case}: captured", flush=True)
    for p in mod.parameters():
        p.grad = None
    for _ in range(2):
        for p in mod.parameters():
            p.grad = None
        out = graphed(*args)
        loss_of(out).backward()
        torch.cuda.synchronize()
    g = [p.grad for p in mod.parameters() if p.grad is not None]
    err = max(float((a - b).abs().max() / (b.abs().max() + 1e-12)) for a, b in zip(g, g_ref))
    print(f"{case}: replay ok, loss {float(ref):.4f} vs {float(loss_of(out)):.4f}, max rel grad err {err:.2e}",
          flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run_case(sys.argv[1])
        sys.exit(0)
    for c in CASES:
        r = subprocess.run([sys.executable, "-X", "faulthandler", __file__, c], timeout=240)
        if r.returncode != 0:
            print(f"FAILED at {c} (rc={r.returncode}); stopping", flush=True)
            sys.exit(1)
    print("all cases ok")
