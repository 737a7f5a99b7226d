"""Per-launch HBM traffic of the path's kernels from rocprofv3 PMC passes.

    python tools/pmc_traffic.py --fetch gpurun_out/s_pmc_fetch --write gpurun_out/s_pmc_write \
        --out profiles/rNN_pmc_traffic.json

Input: the counter-collection CSVs of two separate passes (FETCH_SIZE and
WRITE_SIZE do not fit one TCC pass on gfx950).  Output: for each (kernel,
grid) the mean per-launch bytes read / written and their sum, with the
MI355X_MICROARCH.md "HBM" corrections:

  * FETCH_SIZE / WRITE_SIZE are in KiB;
  * FETCH_SIZE counts half the bytes of wide (16 B/lane) coalesced
    streaming reads on gfx950 -> `fetch_bytes_corrected` doubles it.  Other
    access widths (e.g. the MSDA gathers) are uncalibrated: both the raw and
    the corrected figure are kept, and ratios between variants of one kernel
    are unaffected;
  * WRITE_SIZE is exact for 16 B/lane stores and float atomics.

bench.py reads the resulting JSON (if present under profiles/) to fill the
roofline line's `traffic` for the dominant kernel at the same launch grid.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def _rows(path):
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*counter_collection*.csv"),
                                                          recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection CSV under {path}")
    for f in files:
        with open(f) as fh:
            yield from csv.DictReader(fh)


def _grid(r):
    for k in ("Grid_Size", "Grid_Size_X", "grid_size"):
        if k in r and r[k]:
            return int(float(r[k]))
    return -1


def collect(path, counter):
    """-> {(kernel short name, grid): [per-dispatch values in bytes]}"""
    per_dispatch = collections.defaultdict(float)
    meta = {}
    for r in _rows(path):
        if r.get("Counter_Name") != counter:
            continue
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per_dispatch[did] += float(r["Counter_Value"]) * 1024.0  # KiB -> B
        name = re.sub(r"\(.*", "", r.get("Kernel_Name", "?").replace("(anonymous namespace)::", ""))
        meta[did] = (name.replace("void ", ""), _grid(r))
    out = collections.defaultdict(list)
    for did, v in per_dispatch.items():
        out[meta[did]].append(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--match", default="gd::", help="kernel-name substring to keep")
    a = ap.parse_args()
    fetch, write = collect(a.fetch, "FETCH_SIZE"), collect(a.write, "WRITE_SIZE")
    res = []
    for key in sorted(set(fetch) | set(write)):
        name, grid = key
        if a.match not in name:
            continue
        f = fetch.get(key, [])
        w = write.get(key, [])
        fm = sum(f) / len(f) if f else None
        wm = sum(w) / len(w) if w else None
        res.append({"kernel": name, "grid": grid, "launches": max(len(f), len(w)),
                    "fetch_bytes_raw": fm, "fetch_bytes_corrected": None if fm is None else 2 * fm,
                    "write_bytes": wm,
                    "traffic_bytes": None if fm is None or wm is None else 2 * fm + wm})
    with open(a.out, "w") as fh:
        json.dump({"source": [a.fetch, a.write], "kernels": res}, fh, indent=1)
    for r in res:
        print(f"{r['kernel']:50s} grid={r['grid']:>10d} n={r['launches']:3d} "
              f"read={r['fetch_bytes_corrected'] or 0:12.3e} write={r['write_bytes'] or 0:12.3e}")


if __name__ == "__main__":
    main()
