"""Token-linear GEMM shapes of the train step (bf16, 800x1333, bs=2): the
library GEMM (torch.addmm / _addmm_activation -> hipBLASLt) against
csrc/tlin.hip's kernels, forward y = x W^T + b (ReLU), and the masked dX
(the FFN's second Linear with the ReLU backward folded in) against the
library GEMM + threshold_backward.

Device time per call from HIP events around one replay of ``--iters`` calls
captured in a HIP graph;
also the largest difference from the library result in bf16 ulps of the
result magnitude.  The measured table behind ``wgrad.tlin_wins``.

    python tools/tlin_microbench.py [--iters 50]
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
ENC, S0, S1, S2 = 2 * 22223, 2 * 200 * 334, 2 * 100 * 167, 2 * 50 * 84
SHAPES = [  # name, tokens, K, N, relu
    ("enc 256->256", ENC, 256, 256, False),
    ("enc 256->384", ENC, 256, 384, False),
    ("enc 256->128", ENC, 256, 128, False),
    ("enc 256->1024", ENC, 256, 1024, False),
    ("enc ffn1 256->2048 relu", ENC, 256, 2048, True),
    ("swin0 96->288", S0, 96, 288, False),
    ("swin0 96->96", S0, 96, 96, False),
    ("swin0 96->384", S0, 96, 384, False),
    ("swin1 192->576", S1, 192, 576, False),
    ("swin1 192->192", S1, 192, 192, False),
    ("swin1 192->768", S1, 192, 768, False),
    ("swin1 768->192", S1, 768, 192, False),
    ("swin2 384->1152", S2, 384, 1152, False),
    ("swin2 384->384", S2, 384, 384, False),
    ("swin2 384->1536", S2, 384, 1536, False),
    ("swin2 1536->384", S2, 1536, 384, False),
    ("enc 2048->256", ENC, 2048, 256, False),
    ("enc 1024->256", ENC, 1024, 256, False),
    ("dec 256->256", 1800, 256, 256, False),
]


def _time(fn, iters, warmup=3):
    """Device time per call: ``iters`` calls captured in one HIP graph and
    replayed (no host launch cost in the measurement, as in the step graph)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warmup):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(iters):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    graph.replay()
    b.record()
    b.synchronize()
    del graph
    return a.elapsed_time(b) * 1e3 / iters


def _ulps(y, ref):
    d = (y.float() - ref.float()).abs()
    return float((d / (ref.float().abs().clamp_min(1e-2) * 2 ** -7)).max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from gdino_amd.wgrad import masked_dx, tlin_forward
    g = torch.Generator(device=DEV).manual_seed(0)
    for name, m, k, n, relu in SHAPES:
        x = torch.randn(m, k, generator=g, device=DEV).to(BF)
        w = (torch.randn(n, k, generator=g, device=DEV) * k ** -0.5).to(BF)
        b = torch.randn(n, generator=g, device=DEV).to(BF)

        def lib():
            return torch._addmm_activation(b, x, w.t(), use_gelu=False) if relu else torch.addmm(b, x, w.t())

        def own():
            return tlin_forward(x, w, b, relu=relu)
        t_lib, t_own = _time(lib, a.iters), _time(own, a.iters)
        hbm = (m * k + n * k + m * n) * 2
        print(json.dumps({"name": name, "lib_us": round(t_lib, 2), "tlin_us": round(t_own, 2),
                          "hbm_floor_us": round(hbm / 8e12 * 1e6, 2), "tlin_TBps": round(hbm / t_own / 1e6, 3),
                          "ulps_vs_lib": round(_ulps(own(), lib()), 3)}), flush=True)
        del x, w, b
    # the FFN's second Linear's dX with the first's ReLU mask: [T, 256] . [256, 2048]
    dy = torch.randn(ENC, 256, generator=g, device=DEV).to(BF)
    w2 = (torch.randn(256, 2048, generator=g, device=DEV) * 0.06).to(BF)  # [N_out, K_in] of the Linear
    h = torch.randn(ENC, 2048, generator=g, device=DEV).clamp_min(0).to(BF)

    def lib_m():
        return torch.ops.aten.threshold_backward(torch.mm(dy, w2), h, 0)

    def own_m():
        return masked_dx(dy, w2, h)
    t_lib, t_own = _time(lib_m, a.iters), _time(own_m, a.iters)
    hbm = (ENC * 256 + 256 * 2048 + 2 * ENC * 2048) * 2
    print(json.dumps({"name": "enc ffn2 dX masked 256->2048", "lib_us": round(t_lib, 2),
                      "tlin_us": round(t_own, 2), "hbm_floor_us": round(hbm / 8e12 * 1e6, 2),
                      "tlin_TBps": round(hbm / t_own / 1e6, 3), "ulps_vs_lib": round(_ulps(own_m(), lib_m()), 3)}),
          flush=True)
    print("tlin_microbench done", flush=True)


if __name__ == "__main__":
    main()
