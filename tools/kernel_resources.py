"""Static resource usage of every HIP kernel (compile-time, no GPU):
VGPRs / AGPRs / SGPRs / scratch / LDS / occupancy per kernel, from the
compiler's kernel-resource-usage remarks for gfx950.

    python tools/kernel_resources.py > profiles/rNN_kernel_resources.txt
"""
import concurrent.futures
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "open-groundingdino_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics"]
KEYS = ("VGPRs", "AGPRs", "SGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]")


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return out.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return names


def _remarks(src):
    """The device-side compile of one source (no host pass: the remarks are
    per kernel), its stderr."""
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run(["hipcc", *FLAGS, "--cuda-device-only", "-c", os.path.join(CSRC, src), "-o",
                            os.path.join(d, "x.o"), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
    return src, r.stderr


def main():
    rows = []
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    # one compiler process per source, in parallel (the serial loop took
    # ~3 minutes of the CPU test suite)
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        results = list(ex.map(_remarks, srcs))
    for src, err in results:
        cur = None
        for line in err.splitlines():
            m = re.search(r"remark: (Function Name|[A-Za-z \[\]/]+): (.*?) \[-Rpass", line)
            if not m:
                continue
            k, v = m.group(1).strip(), m.group(2).strip()
            if k == "Function Name":
                cur = {"src": src, "name": v}
                rows.append(cur)
            elif cur is not None and k in KEYS:
                cur[k] = v
    names = demangle([r["name"] for r in rows])
    print(f"{'kernel':80s} {'VGPR':>5s} {'AGPR':>5s} {'SGPR':>5s} {'scratch':>8s} {'LDS':>6s} {'occ':>4s}")
    for r, n in zip(rows, names):
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = re.sub(r"\(.*", "", n)[:80]
        print(f"{n:80s} {r.get('VGPRs', '?'):>5s} {r.get('AGPRs', '?'):>5s} {r.get('SGPRs', '?'):>5s} "
              f"{r.get('ScratchSize [bytes/lane]', '?'):>8s} {r.get('LDS Size [bytes/block]', '?'):>6s} "
              f"{r.get('Occupancy [waves/SIMD]', '?'):>4s}")


if __name__ == "__main__":
    sys.exit(main())
