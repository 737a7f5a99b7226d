"""Probe: eager vs HIP-graph-replayed train step (correctness + timing)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402

from gdino_amd import graphs  # noqa: E402
from gdino_amd.config import make_args  # noqa: E402
from gdino_amd.train import build_training, synthetic_batch, train_step  # noqa: E402


def run(mode, args, steps=5, warm=2, h=800, w=1333, check=False):
    torch.manual_seed(0)
    dev = torch.device("cuda")
    model, crit, _, opt = build_training(args, dev)
    model.train()
    if check:  # deterministic comparison: no dropout / drop-path anywhere
        from gdino_amd.misc import DropPath
        for m in model.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
            if isinstance(m, DropPath):
                m.drop_prob = 0.0
    samples, targets, caps, cats = synthetic_batch(2, h, w, n_boxes=8, n_tokens=256, seed=1, device=dev)
    if mode == "graph":
        text, _ = model.prepare_text(caps, dev)
        t0 = time.perf_counter()
        graphs.capture(model, (samples.tensors, samples.mask, text["input_ids"], text["token_type_ids"],
                               text["text_token_mask"], text["self_masks"], text["position_ids"]))
        torch.cuda.synchronize()
        print(f"[{mode}] capture {time.perf_counter() - t0:.1f}s", flush=True)
    if check:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(samples, captions=caps)
            ld = crit(out, targets, cats, caps)
            loss = sum(ld[k] * crit.weight_dict[k] for k in ld if k in crit.weight_dict)
        opt.zero_grad()
        loss.backward()
        g = {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}
        return float(loss), g
    for _ in range(warm):
        train_step(model, crit, opt, samples, targets, caps, cats)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = train_step(model, crit, opt, samples, targets, caps, cats)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"[{mode}] {dt * 1e3:.1f} ms/step  {2 / dt:.2f} img/s  loss={float(loss):.2f}  "
          f"mem={torch.cuda.max_memory_allocated() / 2**30:.1f} GiB", flush=True)


if __name__ == "__main__":
    import subprocess
    what = sys.argv[1] if len(sys.argv) > 1 else "both"
    if what == "check1":  # one mode per process
        mode = sys.argv[2]
        hw = [int(v) for v in sys.argv[3:5]] if len(sys.argv) > 4 else [512, 640]
        loss, g = run(mode, make_args(device="cuda", fusion_droppath=0.0), check=True, h=hw[0], w=hw[1])
        torch.save({"loss": loss, "g": {k: v.cpu() for k, v in g.items()}}, f"/tmp/gp_{mode}.pt")
        sys.exit(0)
    if what == "traj1":  # per-step loss trajectory of one mode (same seeds as the other)
        mode = sys.argv[2]
        torch.manual_seed(0)
        dev = torch.device("cuda")
        model, crit, _, opt = build_training(make_args(device="cuda"), dev)
        model.train()
        samples, targets, caps, cats = synthetic_batch(2, 800, 1333, n_boxes=8, n_tokens=256, seed=1000, device=dev)
        if mode == "graph":
            text, _ = model.prepare_text(caps, dev)
            graphs.capture(model, (samples.tensors, samples.mask, text["input_ids"], text["token_type_ids"],
                                   text["text_token_mask"], text["self_masks"], text["position_ids"]))
        losses = [float(train_step(model, crit, opt, samples, targets, caps, cats)) for _ in range(12)]
        print(f"[{mode}] losses " + " ".join(f"{v:.1f}" for v in losses), flush=True)
        sys.exit(0)
    if what == "traj":
        for mode in ("eager", "graph"):
            subprocess.run([sys.executable, __file__, "traj1", mode], check=True, timeout=400)
        sys.exit(0)
    if what == "time1":
        kw = {}
        if "nockpt" in sys.argv[3:]:
            kw.update(use_checkpoint=False, use_transformer_ckpt=False)
        if "norng" in sys.argv[3:]:
            kw.update(fusion_droppath=0.0)
        a = make_args(device="cuda", **kw)
        if "norng" in sys.argv[3:]:
            import models.GroundingDINO.backbone.swin_transformer as sw
            _orig = sw.SwinTransformer.__init__

            def _init(self, *args, **kwargs):
                kwargs["drop_path_rate"] = 0.0
                _orig(self, *args, **kwargs)
            sw.SwinTransformer.__init__ = _init
            import models.GroundingDINO.ms_deform_attn as md
            _morig = md.MultiScaleDeformableAttention.__init__

            def _minit(self, *args, **kwargs):
                kwargs["dropout"] = 0.0
                _morig(self, *args, **kwargs)
            md.MultiScaleDeformableAttention.__init__ = _minit
        run(sys.argv[2], a)
        sys.exit(0)
    if what == "hyp":
        for extra in (["nockpt"], ["norng"]):
            r = subprocess.run([sys.executable, __file__, "time1", "graph"] + extra, timeout=600)
            print("hyp", extra, "rc", r.returncode, flush=True)
            if r.returncode != 0:
                sys.exit(1)
        sys.exit(0)
    if what in ("check", "both"):
        hw = sys.argv[2:4] if len(sys.argv) > 3 else ["512", "640"]
        for mode in ("eager", "graph"):
            subprocess.run([sys.executable, __file__, "check1", mode] + hw, check=True, timeout=400)
        e, g = torch.load("/tmp/gp_eager.pt"), torch.load("/tmp/gp_graph.pt")
        worst = max(((e["g"][n] - g["g"][n]).abs().max() / (e["g"][n].abs().max() + 1e-12)).item() for n in e["g"])
        print(f"check: loss eager {e['loss']:.4f} graph {g['loss']:.4f}; max rel grad diff {worst:.3e}", flush=True)
    if what in ("time", "both"):
        for mode in ("eager", "graph"):
            subprocess.run([sys.executable, __file__, "time1", mode], check=True, timeout=600)
