"""Tune the train step's GEMMs with PyTorch TunableOp on the GPU and write
the solution table that ``bench.py --tunableop CSV`` reads.

    python tools/tune_gemms.py --out tunableop/gdino_train_gfx950.csv [--steps 2]

TunableOp times every hipBLASLt (and rocBLAS) solution for each GEMM shape the
step issues, including split-K variants. The default heuristic misses those
for the long-K weight-gradient GEMMs (dW = dY^T X over 44k tokens with a
256x256 output). Tuning is bounded per shape (--ms), so a full step's ~100
distinct shapes tune in a few minutes. Results are validated against the
running PyTorch / ROCm / hipBLASLt versions and GPU arch when read back.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402


def main():
    # Round 5: the tuning run faulted the GPU a second time (an illegal
    # address while TunableOp timed candidate solutions for the encoder's
    # Linear, profiles/r05e_tunableop_fault.log) after round 4's fix for the
    # strided BiAttention operands.  Refused unless explicitly forced.
    if os.environ.get("GDINO_ALLOW_TUNING") != "1":
        raise SystemExit("tune_gemms.py: TunableOp tuning faulted the GPU twice (rounds 3 and 5); "
                         "set GDINO_ALLOW_TUNING=1 to run it anyway")
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "tunableop", "gdino_train_gfx950.csv"))
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--ms", type=int, default=30, help="max tuning time per GEMM shape")
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--width", type=int, default=1333)
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    t = torch.cuda.tunable
    t.enable(True)
    t.tuning_enable(True)
    t.set_filename(a.out, False)
    t.set_max_tuning_duration(a.ms)
    t.set_max_tuning_iterations(30)

    from gdino_amd.config import make_args
    from gdino_amd.train import build_training, synthetic_batch, train_step
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model, crit, _, opt = build_training(make_args(device="cuda"), dev)
    model.train()
    batch = synthetic_batch(2, a.height, a.width, n_boxes=8, n_tokens=256, seed=0, device=dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        train_step(model, crit, opt, *batch)
        torch.cuda.synchronize()
        print(f"step {i}: {time.perf_counter() - t0:.1f}s, {len(t.get_results())} tuned shapes", flush=True)
    # TunableOp writes the table when the process exits normally
    print(f"tuned {len(t.get_results())} GEMM shapes -> {a.out} (written at exit)", flush=True)


if __name__ == "__main__":
    main()
