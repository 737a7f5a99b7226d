"""Per-call times (HIP events, median of 50) of the encoder FFN's second-Linear
input gradient: library GEMM + threshold pass vs csrc/tlin.hip's masked dX,
and the unmasked kernel for reference.  python tools/probes/tlin_masked_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]
import torch  # noqa: E402
from gdino_amd.wgrad import masked_dx, tlin_forward  # noqa: E402


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[n // 2]


m, k, n = int(os.environ.get("M", 44446)), 256, 2048
dev = "cuda"
dy = torch.randn(m, k, device=dev).to(torch.bfloat16)
w2 = (torch.randn(k, n, device=dev) * n ** -0.5).to(torch.bfloat16)
w2t = w2.t().contiguous()
h = torch.randn(m, n, device=dev).clamp_min(0).to(torch.bfloat16)
res = {
    "lib_mm": timeit(lambda: torch.mm(dy, w2)),
    "lib_mm+threshold": timeit(lambda: torch.ops.aten.threshold_backward(torch.mm(dy, w2), h, 0)),
    "threshold": timeit(lambda: torch.ops.aten.threshold_backward(h, h, 0)),
    "tlin_masked": timeit(lambda: masked_dx(dy, w2, h)),
    "tlin_plain": timeit(lambda: tlin_forward(dy, w2t)),
    "transpose_w": timeit(lambda: w2.t().contiguous()),
}
res["floor_masked_us"] = (m * k * 2 + 2 * m * n * 2) / 8e12 * 1e6
print(json.dumps({k_: round(v, 1) for k_, v in res.items()}))
