"""Per-step kernel breakdown from a rocprofv3 kernel-trace CSV: steps are
delimited by the fused AdamW kernel (one multi_tensor_apply chain per step);
only steps after --skip optimizer steps are summarised."""
import argparse
import collections
import csv
import re


def short(name):
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    for key, lab in (("msda_fwd", "gd::msda_fwd"), ("msda_bwd", "gd::msda_bwd"), ("attn_fwd", "sdpa attn_fwd"),
                     ("bwd_kernel_dq", "sdpa bwd_dq"), ("bwd_kernel_dk_dv", "sdpa bwd_dk_dv"),
                     ("Cijk_", "hipBLASLt GEMM"), ("layer_norm", "layer_norm"), ("LayerNorm", "layer_norm"),
                     ("GammaBeta", "layer_norm bwd"), ("ComputeGradInput", "layer_norm bwd"),
                     ("conv", "conv"), ("reduce_kernel", "reduce"), ("softmax", "softmax"),
                     ("FusedOpti", "adamw"), ("multi_tensor", "multi_tensor"), ("copy", "copy/cast"),
                     ("elementwise", "elementwise"), ("index", "index/gather"), ("fill", "fill"),
                     ("Fill", "fill"), ("scatter", "index/gather"), ("gather", "index/gather"),
                     ("group_norm", "group_norm"), ("GroupNorm", "group_norm"), ("topk", "topk"),
                     ("sort", "sort"), ("cat", "cat")):
        if key in n:
            return lab
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # step boundary = first fused AdamW kernel of a chain
    bounds, last = [], -1
    for i, r in enumerate(rows):
        if "FusedOpti" in r["Kernel_Name"] or "fused_adam" in r["Kernel_Name"].lower():
            if last < 0 or i - last > 1000:  # one chain per step (param groups launch separately)
                bounds.append(i)
            last = i
    if len(bounds) <= a.skip:
        raise SystemExit(f"only {len(bounds)} optimizer steps found")
    start = bounds[a.skip - 1] + 1 if a.skip > 0 else 0
    sel = rows[start:]
    nsteps = len(bounds) - a.skip
    print(f"# optimizer chains found at kernel indices {bounds}")
    t_first = int(sel[0]["Start_Timestamp"])
    t_last = int(sel[-1]["End_Timestamp"])
    by = collections.defaultdict(lambda: [0, 0.0])
    by_full = collections.defaultdict(lambda: [0, 0.0])
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        s = short(r["Kernel_Name"])
        by[s][0] += 1
        by[s][1] += d
        by_full[r["Kernel_Name"][:100]][0] += 1
        by_full[r["Kernel_Name"][:100]][1] += d
    busy = sum(v[1] for v in by.values())
    print(f"steps={nsteps} wall(first..last kernel)={((t_last - t_first) / 1e6) / nsteps:.1f} ms/step "
          f"kernel-busy={busy / nsteps:.1f} ms/step kernels/step={len(sel) / nsteps:.0f}")
    for k, (n, ms) in sorted(by.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {ms / nsteps:8.2f} ms/step {100 * ms / busy:5.1f}%  n/step={n / nsteps:7.1f}  {k}")
    print("--- gd:: kernels by launch grid (steady-state steps)")
    gd = collections.defaultdict(lambda: [0, 0.0])
    for r in sel:
        if "gd::" not in r["Kernel_Name"]:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        key = (re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", ""),
               int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]))
        gd[key][0] += 1
        gd[key][1] += d
    for (k, gx, gy), (n, us) in sorted(gd.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:45s} grid=({gx},{gy}) launches/step={n / nsteps:5.1f} avg={us / n:9.1f}us "
              f"total={us / nsteps / 1e3:7.2f} ms/step")
    # one replayed graph step: the interval between two optimizer chains
    # whose kernel count is the most common one (the capture step and the
    # eager per-entry-point step have other counts)
    ivs = [(bounds[i] + 1, bounds[i + 1] + 1) for i in range(len(bounds) - 1)]
    if ivs:
        counts = collections.Counter(b - a for a, b in ivs)
        mode = counts.most_common(1)[0][0]
        a0, b0 = [iv for iv in ivs if iv[1] - iv[0] == mode][-1]
        one = rows[a0:b0]
        busy1 = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in one)
        wall1 = (int(one[-1]["End_Timestamp"]) - int(one[0]["Start_Timestamp"])) / 1e6
        print(f"--- one graph step (kernel indices {a0}..{b0}, {counts[mode]} steps of this count): "
              f"kernels {len(one)} busy {busy1:.2f} ms wall {wall1:.2f} ms")
        g1 = collections.defaultdict(lambda: [0, 0.0])
        for r in one:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            g1[re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))[:90]][0] += 1
            g1[re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))[:90]][1] += d
        for k, (n, us) in sorted(g1.items(), key=lambda kv: -kv[1][1])[:60]:
            print(f"  {us:9.1f} us n={n:4d} avg={us / n:7.1f}  {k}")
    print("--- top individual kernels")
    for k, (n, ms) in sorted(by_full.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {ms / nsteps:8.2f} ms/step  n/step={n / nsteps:6.1f} avg={ms / n * 1e3:8.1f}us  {k}")


if __name__ == "__main__":
    main()
