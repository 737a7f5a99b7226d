"""MFMA kernel families at the train step's production shapes (bf16,
800x1333, bs=2): masked attention (BERT self, text enhancer, decoder self,
decoder text cross), Swin-T window attention (stages 0-3, W-MSA and SW-MSA),
the token-linear GEMM (Swin stage 0, encoder FFN) and the contrastive head.

Each case runs forward + backward ``--iters`` times behind _lib.CallTimer
(HIP events on the launch stream around every C-ABI call) and prints one
JSON line per case: per entry point the calls, average device time, and
TFLOP/s against the dense bf16 peak from the algorithmic flop count.  It is
also the short program the rocprofv3 --pmc passes of tools/mfma_counters.py
run (``--iters 3``): every launch is a production-shape launch.

    python tools/attn_microbench.py [--iters 20] [--cases attn,wattn,tlin,contrastive]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "open-groundingdino_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

DEV = torch.device("cuda:0")
BF = torch.bfloat16


def _attn_case(b, h, lq, lk, hd, mask_kind, dropout):
    from gdino_amd.attn import AttnFunction
    g = torch.Generator(device=DEV).manual_seed(lq + lk)
    # the MHA projections' [L, B, H*hd] layout, read in place
    q = torch.randn(lq, b, h, hd, generator=g, device=DEV).to(BF).permute(1, 2, 0, 3).requires_grad_()
    k = torch.randn(lk, b, h, hd, generator=g, device=DEV).to(BF).permute(1, 2, 0, 3).requires_grad_()
    v = torch.randn(lk, b, h, hd, generator=g, device=DEV).to(BF).permute(1, 2, 0, 3).requires_grad_()
    if mask_kind == "add":
        mask = torch.where(torch.rand(b, 1, lq, lk, generator=g, device=DEV) < 0.2, -1e4, 0.0)
    elif mask_kind == "bool":
        mask = torch.rand(b, h, lq, lk, generator=g, device=DEV) < 0.7
    elif mask_kind == "keypad":
        mask = torch.ones(b, 1, 1, lk, dtype=torch.bool, device=DEV)
        mask[-1, ..., lk // 2:] = False
    else:
        mask = None
    go = torch.randn(b, h, lq, hd, generator=g, device=DEV).to(BF)

    def run():
        out = AttnFunction.apply(q, k, v, mask, hd ** -0.5, dropout)
        out.backward(go)
    return run


def _wattn_case(b, hh, ww, nh, ws, shift):
    from gdino_amd.wattn import WindowAttnImageFunction
    from models.GroundingDINO.backbone.swin_transformer import relative_position_index, shifted_window_mask
    g = torch.Generator(device=DEV).manual_seed(hh * ww + nh)
    c = 32 * nh
    qkv = torch.randn(b, hh * ww, 3 * c, generator=g, device=DEV).to(BF).requires_grad_()
    qb = (torch.randn(3 * c, generator=g, device=DEV) * 0.5).requires_grad_()
    table = (torch.randn((2 * ws - 1) ** 2, nh, generator=g, device=DEV) * 0.5).requires_grad_()
    ridx = relative_position_index(ws, ws).reshape(-1).to(DEV)
    hp, wp = -(-hh // ws) * ws, -(-ww // ws) * ws
    mask = shifted_window_mask(hp, wp, ws, shift, DEV) if shift else None
    go = torch.randn(b, hh * ww, c, generator=g, device=DEV).to(BF)

    def run():
        out = WindowAttnImageFunction.apply(qkv, qb, table, ridx, mask, (hh, ww), ws, shift, 32 ** -0.5)
        out.backward(go)
    return run


def _tlin_case(m, k, n, relu):
    from gdino_amd.wgrad import tlin_forward
    g = torch.Generator(device=DEV).manual_seed(m + k + n)
    x = torch.randn(m, k, generator=g, device=DEV).to(BF)
    w = (torch.randn(n, k, generator=g, device=DEV) * k ** -0.5).to(BF)
    bias = torch.randn(n, generator=g, device=DEV).to(BF)

    def run():
        tlin_forward(x, w, bias, relu=relu)
    return run


def _contrastive_case(b, q, t, rowmax):
    from gdino_amd.contrastive import ContrastiveFunction, contrastive_rowmax_hip
    g = torch.Generator(device=DEV).manual_seed(q + t)
    x = torch.randn(b, q, 256, generator=g, device=DEV).to(BF).requires_grad_()
    text = torch.randn(b, t, 256, generator=g, device=DEV).to(BF).requires_grad_()
    mask = torch.rand(b, t, generator=g, device=DEV) < 0.8
    mask[:, 0] = True
    gout = torch.randn(b, q, 256, generator=g, device=DEV)

    def run():
        if rowmax:
            with torch.no_grad():
                contrastive_rowmax_hip(x, text, mask)
        else:
            ContrastiveFunction.apply(x, text, mask, 256).backward(gout)
    return run


# name -> (family, factory); Swin-T at 800x1333 bs=2: stage resolutions
# 200x334, 100x167, 50x84, 25x42 with 3 / 6 / 12 / 24 heads
CASES = {
    "attn_bert_self": ("attn", lambda: _attn_case(2, 12, 256, 256, 64, "add", 0.1)),
    "attn_text_enhancer": ("attn", lambda: _attn_case(2, 4, 256, 256, 64, "bool", 0.0)),
    "attn_decoder_self": ("attn", lambda: _attn_case(2, 8, 900, 900, 32, "none", 0.0)),
    "attn_decoder_text_cross": ("attn", lambda: _attn_case(2, 8, 900, 256, 32, "keypad", 0.0)),
    "wattn_stage0_wmsa": ("wattn", lambda: _wattn_case(2, 200, 334, 3, 7, 0)),
    "wattn_stage0_swmsa": ("wattn", lambda: _wattn_case(2, 200, 334, 3, 7, 3)),
    "wattn_stage1_swmsa": ("wattn", lambda: _wattn_case(2, 100, 167, 6, 7, 3)),
    "wattn_stage2_swmsa": ("wattn", lambda: _wattn_case(2, 50, 84, 12, 7, 3)),
    "wattn_stage3_swmsa": ("wattn", lambda: _wattn_case(2, 25, 42, 24, 7, 3)),
    "tlin_swin0_qkv": ("tlin", lambda: _tlin_case(2 * 200 * 334, 96, 288, False)),
    "tlin_swin0_fc1": ("tlin", lambda: _tlin_case(2 * 200 * 334, 96, 384, False)),
    "tlin_enc_ffn1_relu": ("tlin", lambda: _tlin_case(2 * 22223, 256, 2048, True)),
    "contrastive_decoder": ("contrastive", lambda: _contrastive_case(2, 900, 256, False)),
    "contrastive_enc_rowmax": ("contrastive", lambda: _contrastive_case(2, 22223, 256, True)),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cases", default="attn,wattn,tlin,contrastive",
                    help="families or case names, comma-separated")
    a = ap.parse_args()
    from gdino_amd import _lib
    sel = set(a.cases.split(","))
    for name, (fam, make) in CASES.items():
        if fam not in sel and name not in sel:
            continue
        run = make()
        for _ in range(a.warmup):
            run()
        torch.cuda.synchronize()
        _lib.call_timer = _lib.CallTimer()
        for _ in range(a.iters):
            run()
        summ = _lib.call_timer.summary()
        _lib.call_timer = None
        print(json.dumps({"case": name, "family": fam, "iters": a.iters,
                          "entry_points": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv)
                                               for kk, vv in v.items()} for k, v in summ.items()}}), flush=True)
    print("attn_microbench done", flush=True)


if __name__ == "__main__":
    main()
