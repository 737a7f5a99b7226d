"""How much would LDS pre-aggregation cut the MSDA backward's grad_value
atomics?  A CPU study on the real encoder geometry (no GPU).

The encoder-shape backward (800x1333, bs=2) issues 2*22223*8*16*4 = 22.8 M
corner taps, each a 32-channel 128-B atomic add into grad_value
[N, S, M, D]; it is atomic-rate bound.  If one
workgroup handled a tile of queries of ONE head, corner contributions that
land on the same value row could be summed in LDS first and written with
one atomic per distinct (row, head) per tile.  This script counts, for tile
shapes, total taps / distinct (n, row, head) addresses per tile = the atomic
reduction factor.

Sampling locations are the Deformable-DETR initialisation
(ms_deform_attn.py:198-221: zero offset weights, per-head direction x
(point+1) biases), i.e. exactly the step-0 geometry; during training the
offsets drift, so the factor is an estimate of the start-of-training case.

    python tools/probes/msda_atomic_study.py
"""
import math

import numpy as np

LEVELS = [(100, 167), (50, 84), (25, 42), (13, 21)]
M, L, P = 8, 4, 4


def init_offsets():
    ang = np.arange(M) * (2 * math.pi / M)
    d = np.stack([np.cos(ang), np.sin(ang)], -1)
    d = d / np.abs(d).max(-1, keepdims=True)
    return d[:, None, :] * np.arange(1, P + 1)[None, :, None]  # [M, P, 2] (x, y) in pixels of each level


def taps_for_queries(qs, ref, shapes, starts, off):
    """value-row indices [len(qs), M, L*P*4] (-1 = outside) of the corners."""
    out = np.full((len(qs), M, L * P * 4), -1, dtype=np.int64)
    for li, (h, w) in enumerate(shapes):
        for m in range(M):
            lx = ref[qs, 0][:, None] + off[m, :, 0][None] / w     # [q, P]
            ly = ref[qs, 1][:, None] + off[m, :, 1][None] / h
            him, wim = ly * h - 0.5, lx * w - 0.5
            inside = (him > -1) & (wim > -1) & (him < h) & (wim < w)
            h0, w0 = np.floor(him).astype(np.int64), np.floor(wim).astype(np.int64)
            for c, (dh, dw) in enumerate(((0, 0), (0, 1), (1, 0), (1, 1))):
                hh, ww = h0 + dh, w0 + dw
                ok = inside & (hh >= 0) & (ww >= 0) & (hh < h) & (ww < w)
                idx = np.where(ok, starts[li] + hh * w + ww, -1)
                out[:, m, (li * P) * 4 + c::4][:, :P] = idx
    return out


def main():
    shapes = LEVELS
    sizes = [h * w for h, w in shapes]
    starts = np.cumsum([0] + sizes[:-1])
    S = sum(sizes)
    # encoder reference points: pixel centres of every level (valid ratio 1)
    refs = []
    for h, w in shapes:
        yy, xx = np.meshgrid((np.arange(h) + 0.5) / h, (np.arange(w) + 0.5) / w, indexing="ij")
        refs.append(np.stack([xx.ravel(), yy.ravel()], -1))
    ref = np.concatenate(refs)  # [S, 2] (x, y), same for every level (valid ratios 1)
    off = init_offsets()
    taps = taps_for_queries(np.arange(S), ref, shapes, starts, off)  # [S, M, 64]
    total_valid = int((taps >= 0).sum())
    print(f"encoder 800x1333 per image: S={S}, corner taps in range {total_valid} "
          f"({total_valid / taps.size:.1%} of {taps.size}); x2 images, x32 channels per atomic tap")
    print("tile (queries x heads) -> atomics per tile = distinct (row, head); reduction = taps / distinct")
    for tq in (1, 8, 32, 64, 128, 256):
        for th in (1,):
            n_tiles, distinct = 0, 0
            for q0 in range(0, S, tq):
                blk = taps[q0:q0 + tq]                       # [tq, M, 64]
                for m in range(M):
                    v = blk[:, m].ravel()
                    v = v[v >= 0]
                    distinct += len(np.unique(v))
                    n_tiles += 1
            print(f"  {tq:4d} queries x 1 head: {total_valid / distinct:6.2f}x fewer atomics "
                  f"({distinct * 2 / 1e6:.2f} M per launch at bs=2 vs {total_valid * 2 / 1e6:.2f} M)")


def kernel_policy(taps, tiles, shapes, starts, nrows=384):
    """Global atomics of msda_bwd_tiled's policy (msda_tiled.inc): per tile
    and head, each level's bounding box of corner rows is packed smallest
    first into an nrows-row LDS accumulator; taps in a packed box cost one
    flush atomic per distinct touched row, the others one atomic each."""
    sizes = [h * w for h, w in shapes]
    glob = 0
    for qs in tiles:
        blk = taps[qs]
        for m in range(M):
            v = blk[:, m].ravel()
            v = v[v >= 0]
            boxes = []
            for li, (h, w) in enumerate(shapes):
                vl = v[(v >= starts[li]) & (v < starts[li] + sizes[li])] - starts[li]
                if len(vl) == 0:
                    continue
                y, x = vl // w, vl % w
                boxes.append(((y.max() - y.min() + 1) * (x.max() - x.min() + 1), len(vl), len(np.unique(vl))))
            used = 0
            for area, n_taps, n_rows in sorted(boxes):
                if used + area <= nrows:
                    used += area
                    glob += n_rows
                else:
                    glob += n_taps
    return glob


def policy_main():
    shapes = LEVELS
    sizes = [h * w for h, w in shapes]
    starts = np.cumsum([0] + sizes[:-1])
    S = sum(sizes)
    refs = []
    for h, w in shapes:
        yy, xx = np.meshgrid((np.arange(h) + 0.5) / h, (np.arange(w) + 0.5) / w, indexing="ij")
        refs.append(np.stack([xx.ravel(), yy.ravel()], -1))
    ref = np.concatenate(refs)
    taps = taps_for_queries(np.arange(S), ref, shapes, starts, init_offsets())
    total = int((taps >= 0).sum())
    strips = [np.arange(q0, min(q0 + 32, S)) for q0 in range(0, S, 32)]
    blocks = []
    for li, (h, w) in enumerate(shapes):
        for y0 in range(0, h, 4):
            for x0 in range(0, w, 8):
                yy, xx = np.meshgrid(np.arange(y0, min(y0 + 4, h)), np.arange(x0, min(x0 + 8, w)), indexing="ij")
                blocks.append(starts[li] + (yy * w + xx).ravel())
    print("msda_bwd_tiled policy (384-row LDS boxes, global atomics per launch at bs=2):")
    for name, tiles in (("32 consecutive queries (gd_msda_backward)", strips),
                        ("4 x 8 pixel blocks (gd_msda_backward_geom)", blocks)):
        g = kernel_policy(taps, tiles, shapes, starts)
        print(f"  {name:44s} {g * 2 / 1e6:6.2f} M  ({total / g:.2f}x fewer than the direct kernel's "
              f"{total * 2 / 1e6:.2f} M)")


if __name__ == "__main__":
    main()
    policy_main()
