"""Where does a train step's wall time go?  Host enqueue time vs device time
per phase of the bench's train step (forward, criterion incl. the Hungarian
host sync, backward, clip + AdamW), without a profiler: host clock marks and
HIP events at the same four boundaries, averaged over steady-state steps.

A phase whose host time exceeds its device time starves the GPU (launch
bound); the criterion's device->host copy for the matching makes the GPU wait
for the host's LSA and for the first backward launches.

    python tools/probes/step_phases.py [--steps 8] [--warmup 3] [--graphs]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402

from gdino_amd.config import make_args  # noqa: E402
from gdino_amd.train import build_training, synthetic_batch, weighted_loss  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--graphs", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model, crit, _, opt = build_training(make_args(device="cuda"), dev)
    model.train()
    samples, targets, caps, cats = synthetic_batch(2, 800, 1333, n_boxes=8, n_tokens=256, seed=1000, device=dev)
    if a.graphs:
        from gdino_amd import graphs
        text, _ = model.prepare_text(caps, dev)
        graphs.capture(model, (samples.tensors, samples.mask, text["input_ids"], text["token_type_ids"],
                               text["text_token_mask"], text["self_masks"], text["position_ids"]))
    names = ["forward", "criterion", "backward", "clip+adamw"]
    acc_h = [0.0] * 4
    acc_d = [0.0] * 4
    for it in range(a.warmup + a.steps):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        hs = [time.perf_counter()]
        evs[0].record()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(samples, captions=caps)
            hs.append(time.perf_counter())
            evs[1].record()
            ld = crit(out, targets, cats, caps)
            loss = weighted_loss(ld, crit.weight_dict)
        hs.append(time.perf_counter())
        evs[2].record()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        hs.append(time.perf_counter())
        evs[3].record()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.1, foreach=True)
        opt.step()
        hs.append(time.perf_counter())
        evs[4].record()
        torch.cuda.synchronize()
        if it >= a.warmup:
            for i in range(4):
                acc_h[i] += (hs[i + 1] - hs[i]) * 1e3
                acc_d[i] += evs[i].elapsed_time(evs[i + 1])
    res = {n: {"host_ms": round(acc_h[i] / a.steps, 2), "device_ms": round(acc_d[i] / a.steps, 2)}
           for i, n in enumerate(names)}
    res["total"] = {"host_ms": round(sum(acc_h) / a.steps, 2), "device_ms": round(sum(acc_d) / a.steps, 2)}
    res["graphs"] = a.graphs
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
