"""No kernel on the product path uses scratch (private) memory.

A kernel with a nonzero private segment needs the runtime to back it with a
scratch allocation on the queue it runs on.  Eager launches get it (the
runtime grows a queue's scratch before such a dispatch); inside a replayed
HIP graph the round-4 step graph faulted with illegal addresses while its
eager warm-ups ran clean, and the one kernel of the step with a private
segment was the contrastive head's v2 kernel (a runtime-indexed register
double buffer, placed in scratch by the compiler).  Compile-time resource
remarks (tools/kernel_resources.py, no GPU) pin every kernel at 0 bytes,
except variants that only A/B switches or non-default modes reach (listed,
with the switch)."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# kernel-name patterns allowed a private segment: never launched by the
# default train step (and so never inside the step graph)
ALLOWED = {
    r"msda_bwd_samples<[^,]+, true,": "GD_MSDA_SORTED_K1PIPE=1 (A/B)",
    r"msda_bwd_sort_cells": "GD_MSDA_DETERMINISTIC=1 (deterministic mode)",
    r"wattn_bwd_kernel<[^,]+, \d+, 2,": "mask mode 2: a custom, non-region window mask",
    r"wattn_bwd_kernel<float, 4, 2,": "mask mode 2",
    r"wattn_bwd_kernel<float, 9, [01], false>": "fp32 window attention of 12 x 12 windows (Swin-B/384 without "
                                                 "autocast); the bf16 train step runs the bf16 kernels",
}


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_no_product_kernel_uses_scratch():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kernel_resources.py")], capture_output=True,
                         text=True, timeout=1200, check=True).stdout
    rows = []
    for line in out.splitlines()[1:]:
        cols = line.split()
        if len(cols) < 7:
            continue
        name = line[:80].strip()
        rows.append((name, cols[-3]))
    assert len(rows) > 50, out[:2000]
    bad = [(n, s) for n, s in rows if s not in ("0", "?") and not any(re.search(p, n) for p in ALLOWED)]
    assert not bad, bad
    # the production contrastive kernels in particular
    assert all(s == "0" for n, s in rows if "contrastive" in n), [r for r in rows if "contrastive" in r[0]]
