"""MFMA utilisation and limiter counters of the MFMA kernel families, reduced
per kernel from rocprofv3 --pmc passes over tools/attn_microbench.py.

    python tools/mfma_counters.py --pass gpurun_out/pmc_a --pass gpurun_out/pmc_b \
        --bench gpurun_out/attn_mb.jsonl --out profiles/r06_mfma_counters.json

Each pass is its own rocprofv3 run (one counter group per run: at most 8 SQ
and 2 GRBM counters, MI355X_MICROARCH.md "rocprofv3 PMC").  Per (kernel,
grid) the mean per-dispatch value of every counter and the mean dispatch
duration, then:

  mfma_busy_frac   SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
                   -- the busy cycles are summed over SIMDs (32 per
                   32x32x16 bf16 MFMA, 16 per 16x16x32), GRBM_GUI_ACTIVE over
                   the 8 XCDs (reads high on dispatches shorter than ~0.3 ms,
                   which makes this fraction read LOW there)
  clock_ghz        GRBM_GUI_ACTIVE / 8 / duration
  valu_per_mfma    SQ_INSTS_VALU / SQ_INSTS_MFMA (wave instructions)
  active_valu / active_lds / wait_lds / wait_any
                   SQ_ACTIVE_INST_VALU, SQ_ACTIVE_INST_LDS, SQ_WAIT_INST_LDS,
                   SQ_WAIT_ANY as fractions of SQ_WAVE_CYCLES (all in
                   quad-cycles): where a resident wave's time goes
  lds_conflict     SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  flop_frac        (from --bench) the algorithmic TFLOP/s of the kernel's
                   entry point over the 2.5 PFLOP/s dense bf16 peak
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re

N_SIMD = 1024  # 256 CUs x 4 SIMDs
N_XCD = 8


def _rows(path):
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*counter_collection*.csv"),
                                                          recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection CSV under {path}")
    for f in files:
        with open(f) as fh:
            yield from csv.DictReader(fh)


def _short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)


def _grid(r):
    for k in ("Grid_Size", "Grid_Size_X", "grid_size"):
        if k in r and r[k]:
            return int(float(r[k]))
    return -1


def collect(paths, match):
    """-> {(kernel, grid): {"n": dispatches, "dur_us": mean, counter: mean}}"""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for pi, path in enumerate(paths):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        meta = {}
        for r in _rows(path):
            name = _short(r.get("Kernel_Name", "?"))
            if match not in name:
                continue
            did = (pi, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            per[did][r["Counter_Name"]] += float(r["Counter_Value"])
            try:
                dur = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-3
            except (KeyError, ValueError):
                dur = None
            meta[did] = ((name, _grid(r)), dur)
        for did, cs in per.items():
            key, dur = meta[did]
            for c, v in cs.items():
                acc[key][c].append(v)
            if dur is not None:
                acc[key]["_dur_us"].append(dur)
    out = {}
    for key, cs in acc.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["n"] = max(len(v) for v in cs.values())
        out[key] = d
    return out


def derive(d):
    g = d.get("GRBM_GUI_ACTIVE")
    wc = d.get("SQ_WAVE_CYCLES")
    r = {}
    if g and d.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
        r["mfma_busy_frac"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * g / N_XCD)
    if g and d.get("_dur_us"):
        r["clock_ghz"] = g / N_XCD / (d["_dur_us"] * 1e3)
    if d.get("SQ_INSTS_MFMA"):
        r["valu_per_mfma"] = d.get("SQ_INSTS_VALU", 0.0) / d["SQ_INSTS_MFMA"]
        r["lds_per_mfma"] = d.get("SQ_INSTS_LDS", 0.0) / d["SQ_INSTS_MFMA"]
    if wc:
        for k, c in (("active_valu", "SQ_ACTIVE_INST_VALU"), ("active_lds", "SQ_ACTIVE_INST_LDS"),
                     ("active_vmem", "SQ_ACTIVE_INST_VMEM"), ("wait_lds", "SQ_WAIT_INST_LDS"),
                     ("wait_any", "SQ_WAIT_ANY"), ("wait_inst_any", "SQ_WAIT_INST_ANY")):
            if c in d:
                r[k] = d[c] / wc
    if d.get("SQ_LDS_IDX_ACTIVE"):
        r["lds_conflict"] = d.get("SQ_LDS_BANK_CONFLICT", 0.0) / d["SQ_LDS_IDX_ACTIVE"]
    if d.get("SQ_WAVES") and d.get("_dur_us"):
        r["waves"] = d["SQ_WAVES"]
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pass", dest="passes", action="append", required=True)
    ap.add_argument("--bench", help="attn_microbench.py JSON lines (algorithmic TFLOP/s per entry point)")
    ap.add_argument("--match", default="gd::")
    ap.add_argument("--note", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    res = collect(a.passes, a.match)
    bench = []
    if a.bench and os.path.exists(a.bench):
        for line in open(a.bench):
            line = line.strip()
            if line.startswith("{"):
                bench.append(json.loads(line))
    rows = []
    for (name, grid), d in sorted(res.items(), key=lambda kv: -kv[1].get("_dur_us", 0) * kv[1]["n"]):
        row = {"kernel": name, "grid": grid, "dispatches": d["n"], "avg_us": round(d.get("_dur_us", 0.0), 2)}
        row.update({k: round(v, 4) for k, v in derive(d).items()})
        row["counters"] = {k: v for k, v in d.items() if not k.startswith("_") and k != "n"}
        rows.append(row)
    out = {"note": a.note, "passes": a.passes, "kernels": rows, "microbench": bench,
           "definitions": __doc__.split("\n\n", 2)[2].strip()}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for r in rows:
        print(f"{r['kernel'][:60]:60s} grid {r['grid']:>9d} n {r['dispatches']:3d} {r['avg_us']:8.1f} us "
              f"mfma {r.get('mfma_busy_frac', float('nan')):.3f} valu/mfma {r.get('valu_per_mfma', float('nan')):.1f} "
              f"act_valu {r.get('active_valu', float('nan')):.2f} wait_lds {r.get('wait_lds', float('nan')):.2f} "
              f"wait_any {r.get('wait_any', float('nan')):.2f} ldsconf {r.get('lds_conflict', float('nan')):.3f}")


if __name__ == "__main__":
    main()
