"""Static instruction mix of the gfx950 kernels of one source file (no GPU):
per kernel the instruction count, VALU count and a few classes (packed /
dot-product math, global loads / stores, atomics, waitcnts, LDS ops).

    python tools/isa_stats.py msda.hip [name-substring ...]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "open-groundingdino_amd", "csrc")


def kernels(asm):
    for m in re.finditer(r"^(_Z\w+):", asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        body = asm[m.end():end]
        ins = []
        for line in body.split("\n"):
            t = line.split(";")[0].strip()
            if not t or t.startswith(".") or t.endswith(":"):
                continue
            ins.append(t.split()[0])
        yield m.group(1), ins


def main():
    src = sys.argv[1]
    pats = sys.argv[2:]
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
                        "--cuda-device-only", "-S", os.path.join(CSRC, src), "-I", CSRC, "-o", out],
                       check=True, capture_output=True)
        asm = open(out).read()
    names = dict(zip([n for n, _ in kernels(asm)], subprocess.run(
        ["c++filt"], input="\n".join(n for n, _ in kernels(asm)), capture_output=True, text=True).stdout.split("\n")))
    for name, ins in kernels(asm):
        dn = names.get(name, name)
        if pats and not any(p in dn for p in pats):
            continue
        c = collections.Counter(ins)
        cls = lambda f: sum(n for k, n in c.items() if f(k))  # noqa: E731
        print(f"{dn[:90]:90s} total {len(ins):5d} valu {cls(lambda k: k.startswith('v_')):5d} "
              f"pk/dot {cls(lambda k: k.startswith('v_pk_') or 'dot2' in k):4d} "
              f"gload {cls(lambda k: k.startswith(('global_load', 'buffer_load'))):4d} "
              f"gstore {cls(lambda k: k.startswith(('global_store', 'buffer_store'))):4d} "
              f"atomic {cls(lambda k: 'atomic' in k):3d} ds {cls(lambda k: k.startswith('ds_')):4d} "
              f"waitcnt {c.get('s_waitcnt', 0):4d}")


if __name__ == "__main__":
    main()
