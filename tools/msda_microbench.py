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


def init_geometry_loc(n, dev="cuda"):
    """Encoder sampling locations of the reference initialisation
    (ms_deform_attn.py:198-221: zero offset weights, per-head direction x
    (point + 1) pixel biases on every level) -- the step-0 geometry the
    train-step bench runs at."""
    import math
    M, L, P = 8, 4, 4
    ys, xs = [], []
    for (h, w) in LEVELS:
        yy, xx = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
        ys.append((yy.reshape(-1) + 0.5) / h)
        xs.append((xx.reshape(-1) + 0.5) / w)
    ref = torch.stack([torch.cat(xs), torch.cat(ys)], -1)  # [S, 2]
    ang = torch.arange(M, device=dev, dtype=torch.float32) * (2 * math.pi / M)
    d = torch.stack([ang.cos(), ang.sin()], -1)
    d = d / d.abs().max(-1, keepdim=True).values
    off = d[:, None, :] * torch.arange(1, P + 1, device=dev, dtype=torch.float32)[None, :, None]  # [M, P, 2]
    wh = torch.as_tensor([(w, h) for (h, w) in LEVELS], device=dev, dtype=torch.float32)  # [L, 2]
    loc = ref[:, None, None, None, :] + off[None, :, None, :, :] / wh[None, None, :, None, :]
    return loc[None].expand(n, -1, -1, -1, -1, -1).contiguous()


ENC_VARIANTS = [
    ("lane32", {"GD_MSDA_BWD": "lane32"}),
    ("enc default", {"GD_MSDA_BWD": "enc"}),
    ("enc 8x8 r256", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "8x8,8x8,4x8,4x8", "GD_MSDA_ENC_CAP": "128,64,32,32"}),
    ("enc 8x16 r256", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "8x16,8x8,4x8,4x8",
                       "GD_MSDA_ENC_CAP": "160,48,24,24"}),
    ("enc 4x8 r256", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "4x8,4x8,4x4,4x4", "GD_MSDA_ENC_CAP": "96,64,48,48"}),
    ("enc 4x8 r160", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "4x8,4x8,4x4,4x4", "GD_MSDA_ENC_CAP": "76,32,24,24"}),
    ("enc 4x16 r160", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "4x16,4x8,4x4,4x4",
                       "GD_MSDA_ENC_CAP": "92,32,16,16"}),
    ("enc 8x8 r160", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "8x8,4x8,4x4,4x4", "GD_MSDA_ENC_CAP": "92,32,16,16"}),
    ("enc 4x4 r160", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "4x4,4x4,4x4,4x4", "GD_MSDA_ENC_CAP": "64,40,24,28"}),
    ("enc 4x8 r160 rmax4", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "4x8,4x8,4x4,4x4",
                            "GD_MSDA_ENC_CAP": "76,32,24,24", "GD_MSDA_ENC_RMAX": "4"}),
    ("enc 2x8 r160", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "2x8,2x8,2x4,2x4", "GD_MSDA_ENC_CAP": "60,40,28,28"}),
]
# where the time goes: each probe drops one phase (wrong gradients; timing only)
ENC_PROBES = [
    ("enc depth2", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_DEPTH": "2"}),
    ("enc no-direct", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_MODE": "4"}),
    ("enc no-flush", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_MODE": "8"}),
    ("enc no-lds-acc", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_MODE": "16"}),
    ("enc no-zero", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_MODE": "32"}),
    ("enc no-atomics", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_MODE": "12"}),
    ("enc gathers+reduce only", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_MODE": "60"}),
]
# larger level boxes: fewer corners outside the box (direct 128-B atomics);
# simulated atomic bytes at the init geometry 572 (default) / 448 / 403 / 393 MB
ENC_CAPS = [
    ("enc 4x4 cap96", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "4x4,4x4,4x4,4x4", "GD_MSDA_ENC_CAP": "96,48,32,32"}),
    ("enc 4x4 cap128", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "4x4,4x4,4x4,4x4",
                        "GD_MSDA_ENC_CAP": "128,64,40,40"}),
    ("enc 4x4 cap160", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "4x4,4x4,4x4,4x4",
                        "GD_MSDA_ENC_CAP": "160,64,48,48"}),
    ("enc 4x8 cap160", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "4x8,4x8,4x8,4x8",
                        "GD_MSDA_ENC_CAP": "160,64,40,40"}),
    ("enc 8x8 cap320", {"GD_MSDA_BWD": "enc", "GD_MSDA_ENC_TILE": "8x8,8x8,8x8,8x8",
                        "GD_MSDA_ENC_CAP": "320,128,48,48"}),
]


def enc_variants(iters, variants=None):
    """Encoder-shape backward (bs=2, 800x1333, bf16 value) under every
    kernel variant, on the init geometry and on a 2-px random spread; each
    variant checked against lane32 on the same inputs."""
    S = sum(h * w for h, w in LEVELS)
    variants = variants or ENC_VARIANTS
    for geom in ("init", "spread2"):
        v, sh, ls, loc, attn, go = inputs(S, torch.bfloat16)
        if geom == "init":
            loc = init_geometry_loc(2)
        ref = None
        for name, env in variants:
            saved = {k: os.environ.get(k) for k in ("GD_MSDA_BWD", "GD_MSDA_ENC_RMAX", "GD_MSDA_ENC_CAP",
                                                    "GD_MSDA_ENC_TILE", "GD_MSDA_ENC_MODE", "GD_MSDA_ENC_DEPTH")}
            for k in saved:
                os.environ.pop(k, None)
            os.environ.update(env)
            try:
                fn = lambda: msda.ms_deform_attn_backward(v, sh, ls, loc, attn, go, 64,  # noqa: E731
                                                          grad_value_dtype=torch.float32, host_shapes=LEVELS)
                out = fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = [t.clone() for t in out]
                err = [float((a - b).abs().max() / b.abs().max()) for a, b in zip(out, ref)]
                t = time_it(fn, iters)
            finally:
                for k, val in saved.items():
                    os.environ.pop(k, None)
                    if val is not None:
                        os.environ[k] = val
            bb = algo_bytes(2, S, S, 2, bwd=True)
            print(json.dumps(dict(geom=geom, variant=name, bwd_us=t * 1e6, bwd_GBps=bb / t / 1e9,
                                  frac=bb / t / PEAK, rel_err_vs_lane32=err)), flush=True)


def fwd_gs(iters):
    """bf16 forward: the geometry-shared kernel (msda_fwd_gs, default) vs the
    per-lane kernel (GD_MSDA_FWD_GS=0), encoder shape at the init geometry
    and a 2-px spread, decoder shape; max relative difference between them."""
    S = sum(h * w for h, w in LEVELS)
    for lq, geom in ((S, "init"), (S, "spread2"), (900, "uniform")):
        v, sh, ls, loc, attn, go = inputs(lq, torch.bfloat16)
        if geom == "init":
            loc = init_geometry_loc(2)
        outs = {}
        for gs in ("0", "1"):
            os.environ["GD_MSDA_FWD_GS"] = gs
            fn = lambda: msda.ms_deform_attn_forward(v, sh, ls, loc, attn, 64)  # noqa: E731
            outs[gs] = fn().float()
            torch.cuda.synchronize()
            t = time_it(fn, iters)
            bf = algo_bytes(2, S, lq, 2)
            d = float((outs[gs] - outs["0"]).abs().max() / outs["0"].abs().max())
            print(json.dumps(dict(lq=lq, geom=geom, kernel="msda_fwd_gs" if gs == "1" else "msda_fwd_vec",
                                  fwd_us=t * 1e6, GBps=bf / t / 1e9, frac=bf / t / PEAK, rel_diff_vs_vec=d)),
                  flush=True)
        os.environ.pop("GD_MSDA_FWD_GS", None)


def fwd_variants(iters):
    """Forward (bs=2, 800x1333) under each gather batching of msda_fwd_vec
    (GD_MSDA_FWD_SB), encoder shape on the init geometry and a 2-px spread,
    decoder shape on uniform random locations; outputs compared with the
    first variant (bit-identical expected: same arithmetic order)."""
    S = sum(h * w for h, w in LEVELS)
    for vd in (torch.bfloat16, torch.float32):
        for lq, geom in ((S, "init"), (S, "spread2"), (900, "uniform")):
            v, sh, ls, loc, attn, go = inputs(lq, vd)
            if geom == "init":
                loc = init_geometry_loc(2)
            ref = None
            for sb in ("4", "8", "40", "80"):
                os.environ["GD_MSDA_FWD_SB"] = sb
                fn = lambda: msda.ms_deform_attn_forward(v, sh, ls, loc, attn, 64)  # noqa: E731
                out = fn()
                torch.cuda.synchronize()
                ref = out.clone() if ref is None else ref
                same = bool(torch.equal(out, ref))
                t = time_it(fn, iters)
                bf = algo_bytes(2, S, lq, v.element_size())
                print(json.dumps(dict(dtype=str(vd).split(".")[-1], lq=lq, geom=geom, sb=sb, fwd_us=t * 1e6,
                                      GBps=bf / t / 1e9, frac=bf / t / PEAK, identical=same)), flush=True)
            os.environ.pop("GD_MSDA_FWD_SB", None)


BWD_VARIANTS = [
    ("sorted", {"GD_MSDA_BWD": "sorted"}),
    ("sorted per-lane-geometry", {"GD_MSDA_BWD": "sorted", "GD_MSDA_SORTED_GS": "0"}),
    ("sorted cellsum", {"GD_MSDA_BWD": "sorted", "GD_MSDA_SORTED_K4": "1"}),
    ("sorted k1-level-by-level", {"GD_MSDA_BWD": "sorted", "GD_MSDA_SORTED_K1": "2"}),
    ("sorted one-head-per-wave", {"GD_MSDA_BWD": "sorted", "GD_MSDA_SORTED_HP": "1"}),
    ("sorted locations-held", {"GD_MSDA_BWD": "sorted", "GD_MSDA_SORTED_LL": "0"}),
    ("sorted sweep-prefetch", {"GD_MSDA_BWD": "sorted", "GD_MSDA_SWEEP_PF": "1"}),
    ("sorted no-lds-histogram", {"GD_MSDA_BWD": "sorted", "GD_MSDA_COUNT_PRIV": "0"}),
    ("sorted forced-lds-histogram", {"GD_MSDA_BWD": "sorted", "GD_MSDA_COUNT_PRIV": "2"}),
    ("sorted count-r1", {"GD_MSDA_BWD": "sorted", "GD_MSDA_COUNT_R": "1"}),
    ("sorted count-r8", {"GD_MSDA_BWD": "sorted", "GD_MSDA_COUNT_R": "8"}),
    ("sorted F1", {"GD_MSDA_BWD": "sorted-all", "GD_MSDA_SORTED_F": "1"}),
    ("sorted F4", {"GD_MSDA_BWD": "sorted-all", "GD_MSDA_SORTED_F": "4"}),
    ("sorted-all", {"GD_MSDA_BWD": "sorted-all"}),
    ("sorted deterministic", {"GD_MSDA_BWD": "sorted", "GD_MSDA_DETERMINISTIC": "1"}),
    ("enc", {"GD_MSDA_BWD": "enc"}),
    ("lane32", {"GD_MSDA_BWD": "lane32"}),
]


def bwd_variants(iters, only_geom=None, only_variant=None):
    """The backward as the model calls it (bf16 value, host level shapes,
    grad_value returned in bf16) under each kernel, encoder shape at the init
    geometry and a 2-px spread, and the decoder shape; checked against lane32."""
    S = sum(h * w for h, w in LEVELS)
    for geom in ("enc-init", "enc-spread2", "dec"):
        if only_geom and geom != only_geom:
            continue
        v, sh, ls, loc, attn, go = inputs(900 if geom == "dec" else S, torch.bfloat16)
        if geom == "enc-init":
            loc = init_geometry_loc(2)
        lq = loc.shape[1]
        ref = None
        for name, env in reversed(BWD_VARIANTS):
            if only_variant and name not in only_variant.split(","):
                continue
            saved = {k: os.environ.get(k) for k in ("GD_MSDA_BWD", "GD_MSDA_DETERMINISTIC", "GD_MSDA_SORTED_PROBE",
                                                    "GD_MSDA_SORTED_F", "GD_MSDA_SORTED_K1PIPE",
                                                    "GD_MSDA_SORTED_K4", "GD_MSDA_SORTED_K1",
                                                    "GD_MSDA_SORTED_HP", "GD_MSDA_SWEEP_PF",
                                                    "GD_MSDA_COUNT_PRIV", "GD_MSDA_SORTED_LL",
                                                    "GD_MSDA_SORTED_GS", "GD_MSDA_COUNT_R")}
            for k in saved:
                os.environ.pop(k, None)
            os.environ.update(env)
            try:
                fn = lambda: msda.ms_deform_attn_backward(v, sh, ls, loc, attn, go, 64,  # noqa: E731
                                                          grad_value_dtype=torch.bfloat16, host_shapes=LEVELS)
                out = fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = [t.float().clone() for t in out]
                err = [float((a.float() - b).abs().max() / b.abs().max()) for a, b in zip(out, ref)]
                t = time_it(fn, iters)
            finally:
                for k, val in saved.items():
                    os.environ.pop(k, None)
                    if val is not None:
                        os.environ[k] = val
            sg = 2 if name.startswith("sorted") else 4
            bb = msda.algorithmic_bytes("bwd", 2, S, 8, 32, 4, lq, 4, 2, sg=sg)
            print(json.dumps(dict(geom=geom, variant=name, bwd_us=t * 1e6, algo_MB=bb / 1e6, bwd_GBps=bb / t / 1e9,
                                  frac=bb / t / PEAK, rel_err_vs_lane32=err)), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fwd-variants", action="store_true")
    ap.add_argument("--fwd-gs", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--enc-variants", action="store_true")
    ap.add_argument("--enc-probes", action="store_true")
    ap.add_argument("--enc-caps", action="store_true")
    ap.add_argument("--bwd-variants", action="store_true")
    ap.add_argument("--geom", default=None, help="with --bwd-variants: enc-init | enc-spread2 | dec only")
    ap.add_argument("--variant", default=None, help="with --bwd-variants: one variant name only")
    args = ap.parse_args()
    if args.bwd_variants:
        bwd_variants(args.iters, args.geom, args.variant)
        return
    if args.fwd_variants:
        fwd_variants(args.iters)
        return
    if args.fwd_gs:
        fwd_gs(args.iters)
        return
    if args.enc_caps:
        enc_variants(args.iters, [ENC_VARIANTS[0], ENC_VARIANTS[1]] + ENC_CAPS)
        return
    if args.enc_variants or args.enc_probes:
        enc_variants(args.iters, [ENC_VARIANTS[0], ENC_VARIANTS[1]] + ENC_PROBES if args.enc_probes else None)
        return
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
