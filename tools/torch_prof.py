"""Device time of one eager train step by ATen op, input shapes and source
line (torch.profiler on the ROCm device), to find the glue worth fusing.

    python tools/torch_prof.py [--out gpurun_out/t_prof] [--steps 1]

Writes <out>_by_shape.txt (device time per (op, input shapes)) and
<out>_by_stack.txt (device time per op and the innermost package frames).
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from gdino_amd.config import make_args  # noqa: E402
from gdino_amd.train import build_training, synthetic_batch, train_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/t_prof")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=80)
    ap.add_argument("--checkpointing", choices=("on", "off"), default="off")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model, crit, _, opt = build_training(make_args(device="cuda"), dev)
    model.train()
    from gdino_amd.train import set_activation_checkpointing
    set_activation_checkpointing(model, a.checkpointing == "on")
    samples, targets, caps, cats = synthetic_batch(2, 800, 1333, n_boxes=8, n_tokens=256, seed=1000, device=dev)
    for _ in range(a.warmup):
        train_step(model, crit, opt, samples, targets, caps, cats)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=True) as prof:
        for _ in range(a.steps):
            train_step(model, crit, opt, samples, targets, caps, cats)
        torch.cuda.synchronize()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    key = "self_cuda_time_total"
    with open(a.out + "_by_shape.txt", "w") as f:
        f.write(prof.key_averages(group_by_input_shape=True).table(sort_by=key, row_limit=a.rows,
                                                                   max_name_column_width=60,
                                                                   max_shapes_column_width=90))
    with open(a.out + "_by_stack.txt", "w") as f:
        f.write(prof.key_averages(group_by_stack_n=6).table(sort_by=key, row_limit=a.rows,
                                                            max_name_column_width=60))
    # per ATen op: device time by (op, input shapes, innermost package frame);
    # backward ops carry no Python stack (autograd engine thread)
    import collections
    agg = collections.Counter()
    cnt = collections.Counter()
    def site(e):
        """innermost product frame (forward ops), else the autograd node whose
        backward issued the op (backward ops run on the engine's thread
        without a Python stack), else the nearest named parent range"""
        frame = next((f for f in (e.stack or []) if "open-groundingdino_amd" in f or "bench.py" in f), "")
        if frame:
            return frame.split("open-groundingdino_amd/")[-1]
        p = e.cpu_parent
        while p is not None:
            if p.name.startswith("autograd::engine::evaluate_function: "):
                return "bwd " + p.name.split(": ", 1)[1]
            p = p.cpu_parent
        p = e.cpu_parent
        while p is not None and p.name.startswith("aten::"):
            p = p.cpu_parent
        return ("in " + p.name) if p is not None else ""

    for e in prof.events():
        t = getattr(e, "self_device_time_total", None)
        if t is None:
            t = e.self_cuda_time_total
        if not t or not e.name.startswith("aten::"):
            continue
        k = (e.name, str(e.input_shapes)[:110], site(e)[:90])
        agg[k] += t
        cnt[k] += 1
    tot = sum(agg.values())
    with open(a.out + "_by_site.txt", "w") as f:
        f.write(f"aten self device time {tot / 1e3:.2f} ms over {a.steps} step(s)\n")
        for k, v in agg.most_common(150):
            f.write(f"{v / 1e3 / a.steps:8.3f} ms  n={cnt[k] // a.steps:4d}  {k[0]:28s} {k[2]:90s} {k[1]}\n")
    print(prof.key_averages().table(sort_by=key, row_limit=25, max_name_column_width=60))


if __name__ == "__main__":
    main()
