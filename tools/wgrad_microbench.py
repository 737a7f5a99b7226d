"""Split-K weight-gradient kernel (csrc/wgrad.hip) vs the library GEMM on the
train step's token-heavy Linear shapes: dW = dY^T X (+ db), bf16 in, fp32
out.  Device time per call via HIP events on the launch stream; TFLOP/s
against the 2.5 PFLOP/s dense bf16 peak; max relative error vs fp64."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402

from gdino_amd import wgrad  # noqa: E402

PEAK = 2.5e15
# (name, T, O, I): encoder (800x1333 bs=2: T = 44 446), Swin-T stages 0-2 (T = 133 600 / 33 400 / 8 350)
SHAPES = [("enc value/output proj", 44446, 256, 256), ("enc offsets+weights", 44446, 384, 256),
          ("enc ffn1", 44446, 2048, 256), ("enc ffn2", 44446, 256, 2048),
          ("swin0 qkv", 133600, 288, 96), ("swin0 fc1", 133600, 384, 96), ("swin0 fc2", 133600, 96, 384),
          ("swin1 qkv", 33400, 576, 192), ("swin1 fc1", 33400, 768, 192), ("swin2 fc1", 8350, 1536, 384),
          # below the split-K threshold today (library GEMM + fp32 sum): decoder (1 800 query tokens), text (512)
          ("dec proj", 1800, 256, 256), ("dec offsets+weights", 1800, 384, 256), ("dec ffn1", 1800, 2048, 256),
          ("dec ffn2", 1800, 256, 2048), ("text proj", 512, 256, 256), ("text ffn1", 512, 1024, 256)]


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
    ap.add_argument("--no-lib", action="store_true", help="skip the library GEMM timings")
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, t, o, i in SHAPES:
        dy = torch.randn(t, o, generator=g, device="cuda").to(torch.bfloat16)
        x = torch.randn(t, i, generator=g, device="cuda").to(torch.bfloat16)
        flops = 2.0 * t * o * i
        mine = time_it(lambda: wgrad.weight_grad(dy, x, True), a.iters)
        lib = (float("nan") if a.no_lib else  # bf16 x bf16 -> fp32 GEMM + fp32 sum
               time_it(lambda: wgrad.weight_grad_lib(dy, x, True), a.iters))
        dw, db = wgrad.weight_grad(dy, x, True)
        ref = dy.double().t() @ x.double()
        err = float((dw.double() - ref).abs().max() / ref.abs().max())
        berr = float((db.double() - dy.double().sum(0)).abs().max() / dy.double().sum(0).abs().max())
        nbytes = 2.0 * t * (o + i) + 4.0 * o * (i + 1)  # bf16 dY and X once, fp32 dW and db
        print(json.dumps(dict(variant=os.environ.get("GD_WGRAD_CHUNK", "32") + "/" +
                              os.environ.get("GD_WGRAD_WGS", "384"),
                              shape=name, T=t, O=o, I=i, splits=wgrad._splits(t, o, i), mine_us=mine * 1e6,
                              mine_tbs=nbytes / mine / 1e12, lib_us=lib * 1e6, mine_tflops=flops / mine / 1e12, lib_tflops=flops / lib / 1e12,
                              mfma_frac=flops / mine / PEAK, rel_err_w=err, rel_err_b=berr)), flush=True)
    # BiAttention's batched long-K products (biattn.py: 8 (b, h) x 22 223 tokens x 256 x 256)
    a_ = torch.randn(8, 22223, 256, generator=g, device="cuda").to(torch.bfloat16)
    b_ = torch.randn(8, 22223, 256, generator=g, device="cuda").to(torch.bfloat16)
    flops = 2.0 * 8 * 22223 * 256 * 256
    mine = time_it(lambda: wgrad.tn_matmul(a_, b_), a.iters)
    lib = time_it(lambda: torch.matmul(a_.transpose(-1, -2), b_), a.iters)
    print(json.dumps(dict(shape="biattn tn batched 8x22223x256x256", mine_us=mine * 1e6, lib_us=lib * 1e6,
                          mine_tflops=flops / mine / 1e12, lib_tflops=flops / lib / 1e12)), flush=True)


if __name__ == "__main__":
    main()
