"""Probe: hipBLASLt time for the train step's token-linear GEMM shapes vs the
HBM / MFMA rooflines (bf16 operands; bf16 or fp32 output)."""
import json
import os
import sys

import torch

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                             "open-groundingdino_amd")]
from gdino_amd import wgrad  # noqa: E402

dev = torch.device("cuda")
M = 44446
shapes = [  # (name, M, K, N, out dtype)
    ("enc 256->256", M, 256, 256, torch.bfloat16),
    ("enc 256->384", M, 256, 384, torch.bfloat16),
    ("enc 256->1024", M, 256, 1024, torch.bfloat16),
    ("enc 256->2048", M, 256, 2048, torch.bfloat16),
    ("enc 2048->256", M, 2048, 256, torch.bfloat16),
    ("enc 1024->256", M, 1024, 256, torch.bfloat16),
    ("dgrad 256->256 f32", M, 256, 256, torch.float32),
    ("dgrad 2048->256 f32", M, 2048, 256, torch.float32),
    ("swin0 96->288", 133600, 96, 288, torch.bfloat16),
    ("swin0 96->96", 133600, 96, 96, torch.bfloat16),
    ("swin0 96->384", 133600, 96, 384, torch.bfloat16),
    ("swin0 384->96", 133600, 384, 96, torch.bfloat16),
    ("swin1 192->576", 33400, 192, 576, torch.bfloat16),
    ("swin1 192->192", 33400, 192, 192, torch.bfloat16),
    ("swin1 192->768", 33400, 192, 768, torch.bfloat16),
    ("swin1 768->192", 33400, 768, 192, torch.bfloat16),
    ("swin2 384->1152", 8400, 384, 1152, torch.bfloat16),
    ("swin2 384->384", 8400, 384, 384, torch.bfloat16),
    ("swin2 384->1536", 8400, 384, 1536, torch.bfloat16),
    ("swin2 1536->384", 8400, 1536, 384, torch.bfloat16),
    ("swin3 768->2304", 2100, 768, 2304, torch.bfloat16),
    ("text 256->256", 512, 256, 256, torch.bfloat16),
    ("dec 256->256", 1800, 256, 256, torch.bfloat16),
]
res = []
for name, m, k, n, odt in shapes:
    a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, device=dev, dtype=torch.bfloat16)

    def lib():
        if odt == torch.float32:
            return torch.mm(a, w.t(), out_dtype=torch.float32)
        return torch.addmm(b, a, w.t())

    def mine():
        return wgrad.tlin_forward(a, w, b)
    def timed(run):
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                run()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 100 * 1e3
    us = timed(lib)
    byts = m * k * 2 + n * k * 2 + m * n * (4 if odt == torch.float32 else 2)
    fl = 2.0 * m * k * n
    r = {"name": name, "us": round(us, 1), "GBps": round(byts / us / 1e3, 0), "TFLOPs": round(fl / us / 1e6, 1),
         "hbm_floor_us": round(byts / 8e6, 1), "mfma_floor_us": round(fl / 2.5e9, 1)}
    if odt == torch.bfloat16:
        ref = lib().float()
        got = mine().float()
        r["tlin_us"] = round(timed(mine), 1)
        r["tlin_maxrel"] = float(((got - ref).abs() / ref.abs().clamp_min(1e-2)).max())
    res.append(r)
    print(json.dumps(r), flush=True)
