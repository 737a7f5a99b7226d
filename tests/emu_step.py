"""One whole train-step body (gdino_amd.stepgraph.TrainStepGraph._body:
forward, loss_prepared with the device LSA, backward, clipping) with every
HIP entry point executed by the host-side emulator of the kernel sources
(tests/emu) -- TEST INFRASTRUCTURE ONLY.  Under the ASan build of the
emulator (GD_EMU_ASAN=1 + the clang ASan runtime preloaded) an out-of-bounds
global or LDS access of any kernel, at the shapes the model really hands it,
aborts with its stack.

    python tests/emu_step.py [--height 320 --width 384 --queries 300 --layers 2 --boxes 5 --tokens 40]
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "open-groundingdino_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=320)
    ap.add_argument("--width", type=int, default=384)
    ap.add_argument("--queries", type=int, default=300)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--boxes", type=int, default=5)
    ap.add_argument("--tokens", type=int, default=40)
    ap.add_argument("--ckpt", type=int, default=1)
    a = ap.parse_args()
    from emu_product import emulated_product
    from gdino_amd.config import make_args
    from gdino_amd.stepgraph import TrainStepGraph
    from gdino_amd.train import build_training, set_activation_checkpointing, synthetic_batch

    torch.manual_seed(0)
    args = make_args(device="cpu", enc_layers=a.layers, dec_layers=a.layers, num_queries=a.queries)
    model, crit, _, _ = build_training(args, torch.device("cpu"))
    set_activation_checkpointing(model, bool(a.ckpt))
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
        if hasattr(m, "drop_prob"):
            m.drop_prob = 0.0
    model.train()

    class NoStep:
        def step(self):
            pass

        def zero_grad(self, set_to_none=True):
            model.zero_grad(set_to_none=set_to_none)

    g = TrainStepGraph(model, crit, NoStep(), clip_max_norm=0.1, amp_dtype=torch.bfloat16)
    b = synthetic_batch(2, a.height, a.width, n_boxes=a.boxes, n_tokens=a.tokens, seed=11, device="cpu")
    t0 = time.time()
    with emulated_product():
        inputs, pf = g._prepare(*b)
        loss, _ = g._body(inputs, pf)
    print(f"emu step: loss {float(loss):.4f} in {time.time() - t0:.0f} s", flush=True)
    print("emu-step-ok", flush=True)


if __name__ == "__main__":
    main()
