"""Capture the whole-step graph (gdino_amd.stepgraph) WITHOUT replaying it
and dump its node list (hipGraphDebugDotPrint through CUDAGraph.debug_dump):
node types (kernel / memcpy / memset / host / event), copy directions and
sizes -- the nodes a replay executes that the eager warm-ups did not show.

    python tools/graph_dump.py [--full] [--out gpurun_out/graph.dot]
"""
import argparse
import collections
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true", help="the bench's shapes (default: the step-graph test's)")
    ap.add_argument("--ckpt", type=int, default=1)
    ap.add_argument("--out", default="gpurun_out/graph.dot")
    a = ap.parse_args()
    from gdino_amd.config import make_args
    from gdino_amd.stepgraph import TrainStepGraph
    from gdino_amd.train import build_training, set_activation_checkpointing, synthetic_batch
    dev = torch.device("cuda")
    torch.manual_seed(0)
    args = make_args(device="cuda") if a.full else make_args(device="cuda", enc_layers=2, dec_layers=2,
                                                               num_queries=300)
    model, crit, _, opt = build_training(args, dev)
    set_activation_checkpointing(model, bool(a.ckpt))
    model.train()
    b = (synthetic_batch(2, 800, 1333, n_boxes=8, n_tokens=256, seed=1000, device=dev) if a.full else
         synthetic_batch(2, 320, 384, n_boxes=5, n_tokens=40, seed=11, device=dev))
    g = TrainStepGraph(model, crit, opt, warmup=2)
    inputs = g._prepare(*b)
    key = g._signature(inputs) + (("padding_free", True),)
    # capture exactly as TrainStepGraph._capture, with the debug mode on
    orig_graph = torch.cuda.CUDAGraph

    class DebugGraph(orig_graph):
        def __init__(self, *x, **k):
            super().__init__(*x, **k)
            self.enable_debug_mode()
    import gdino_amd.stepgraph as sg
    sg.torch.cuda.CUDAGraph = DebugGraph
    try:
        c = g._capture(key, inputs, True)
    finally:
        sg.torch.cuda.CUDAGraph = orig_graph
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    c.graph.debug_dump(a.out)
    txt = open(a.out).read()
    kinds = collections.Counter()
    names = collections.Counter()
    for m in re.finditer(r'\[\s*(?:shape|style|label)[^\]]*\]', txt):
        pass
    for line in txt.splitlines():
        low = line.lower()
        if "label" not in low:
            continue
        if "memcpy" in low:
            kinds["memcpy"] += 1
            d = re.search(r"(HtoD|DtoH|DtoD|HtoH|hipMemcpy\w+)", line)
            names["memcpy " + (d.group(1) if d else line.strip()[:120])] += 1
        elif "memset" in low:
            kinds["memset"] += 1
            names["memset " + line.strip()[:160]] += 1
        elif "host" in low and "kernel" not in low:
            kinds["host"] += 1
            names["host " + line.strip()[:160]] += 1
        elif "event" in low:
            kinds["event"] += 1
            names["event " + line.strip()[:160]] += 1
        elif "kernel" in low or "func" in low:
            kinds["kernel"] += 1
    print("graph nodes by kind:", dict(kinds), flush=True)
    for k, v in names.most_common(60):
        print(f"{v:5d}  {k}")
    print(f"dot: {a.out} ({len(txt) / 1e6:.1f} MB)")


if __name__ == "__main__":
    main()
