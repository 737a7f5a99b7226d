"""MSDA kernel microbenchmark at the 800x1333 bs=2 shapes (encoder Lq=22223,
decoder Lq=900): device time per launch via HIP events on the launch stream,
algorithmic bytes -> GB/s and fraction of 8 TB/s."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402

from gdino_amd import msda  # noqa: E402

LEVELS = [(100, 167), (50, 84), (25, 42), (13, 21)]
PEAK = 8.0e12


def inputs(lq, vdtype, n=2, seed=0):
    dev = "cuda"
    shapes = torch.as_tensor(LEVELS, dtype=torch.long, device=dev)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    S = int(shapes.prod(1).sum())
    g = torch.Generator(device=dev).manual_seed(seed)
    M, D, L, P = 8, 32, 4, 4
    value = torch.randn(n, S, M, D, generator=g, device=dev).to(vdtype)
    if lq == S:  # encoder: points around each query's own position (+- a few px)
        ys, xs = [], []
        for (h, w) in LEVELS:
            yy, xx = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
            ys.append((yy.reshape(-1) + 0.5) / h)
            xs.append((xx.reshape(-1) + 0.5) / w)
        ref = torch.stack([torch.cat(xs), torch.cat(ys)], -1)  # [S, 2]
        sh = torch.as_tensor([(w, h) for (h, w) in LEVELS], device=dev, dtype=torch.float32)
        off = torch.randn(n, lq, M, L, P, 2, generator=g, device=dev) * 2.0 / sh[None, None, None, :, None, :]
        loc = ref[None, :, None, None, None, :] + off
    else:
        loc = torch.rand(n, lq, M, L, P, 2, generator=g, device=dev)
    attn = torch.rand(n, lq, M, L, P, generator=g, device=dev) + 1e-5
    attn = attn / attn.sum((-1, -2), keepdim=True)
    go = torch.randn(n, lq, M * D, generator=g, device=dev).to(vdtype)
    return value.contiguous(), shapes, lsi, loc.contiguous(), attn.contiguous(), go


def algo_bytes(n, S, lq, sv, sf=4, so=None, bwd=False):
    so = sv if so is None else so
    M, D, L, P = 8, 32, 4, 4
    if not bwd:
        return sv * n * S * M * D + 3 * sf * n * lq * M * L * P + so * n * lq * M * D
    return sv * n * S * M * D + 4 * n * S * M * D + 2 * 3 * sf * n * lq * M * L * P + so * n * lq * M * D


def time_it(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    S = sum(h * w for h, w in LEVELS)
    res = []
    for lq, tag in ((S, "enc"), (900, "dec")):
        for vd in (torch.float32, torch.bfloat16):
            v, sh, ls, loc, attn, go = inputs(lq, vd)
            sv = v.element_size()
            tf = time_it(lambda: msda.ms_deform_attn_forward(v, sh, ls, loc, attn, 64), args.iters)
            tb = time_it(lambda: msda.ms_deform_attn_backward(v, sh, ls, loc, attn, go, 64,
                                                              grad_value_dtype=torch.float32), args.iters)
            bf, bb = algo_bytes(2, S, lq, sv), algo_bytes(2, S, lq, sv, bwd=True)
            r = dict(shape=tag, dtype=str(vd).split(".")[-1], fwd_us=tf * 1e6, bwd_us=tb * 1e6,
                     fwd_GBps=bf / tf / 1e9, bwd_GBps=bb / tb / 1e9,
                     fwd_frac=bf / tf / PEAK, bwd_frac=bb / tb / PEAK)
            res.append(r)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
