"""Which part of the whole-step graph refuses HIP-graph capture?

    python tools/probes/capture_probe.py

1. One eager train step under torch.cuda.set_sync_debug_mode("warn"): every
   host-synchronising op (the usual capture breakers) is reported with its
   stack.
2. Captures of growing pieces, each in its own graph: the criterion alone
   (forward + backward on leaf outputs), the model forward + loss, forward +
   loss + backward, the full step.  Prints OK / the error per piece.
"""
from __future__ import annotations

import os
import contextlib
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402


NODE_LOG = []


class OpLog(TorchDispatchMode):
    """Remembers the last ATen ops dispatched (also on the autograd engine's
    threads, which inherit the mode) and the last C-ABI entry points."""

    def __init__(self):
        super().__init__()
        self.last = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        self.last.append(str(func))
        del self.last[:-40]
        return func(*args, **(kwargs or {}))


def main():
    from gdino_amd.config import make_args
    from gdino_amd.stepgraph import TrainStepGraph
    from gdino_amd.train import build_training, set_activation_checkpointing, synthetic_batch, train_step, \
        weighted_loss
    dev = torch.device("cuda")
    torch.manual_seed(0)
    full = os.environ.get("PROBE_FULL") == "1"  # the bench's shapes
    args = make_args(device="cuda") if full else make_args(device="cuda", enc_layers=2, dec_layers=2,
                                                           num_queries=300)
    model, crit, _, opt = build_training(args, dev)
    model.train()
    ckpt = os.environ.get("PROBE_CKPT", "off") == "on"
    set_activation_checkpointing(model, ckpt)
    b = (synthetic_batch(2, 800, 1333, n_boxes=8, n_tokens=256, seed=1000, device=dev) if full else
         synthetic_batch(2, 320, 384, n_boxes=5, n_tokens=40, seed=11, device=dev))
    train_step(model, crit, opt, *b)
    torch.cuda.synchronize()
    print(f"checkpointing={ckpt}; eager step under sync debug mode:", flush=True)
    oplog = OpLog()
    torch.cuda.set_sync_debug_mode("error")
    try:
        with oplog:
            train_step(model, crit, opt, *b)
    except Exception as e:  # noqa: BLE001
        print(f"  SYNC at op {oplog.last[-3:]}: {str(e)[:160]}", flush=True)
        traceback.print_exc(limit=12)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    print("  (sync probe done)", flush=True)

    g = TrainStepGraph(model, crit, opt, warmup=1)
    inputs = g._prepare(*b)
    for k, v in inputs.items():
        inputs[k] = v.clone()
    # eager pieces run once (library handles / caches)
    g._body(inputs)
    torch.cuda.synchronize()

    def fwd_loss():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            core = model.forward_core(inputs["images"], inputs["mask"], inputs["input_ids"],
                                      inputs["token_type_ids"], inputs["text_token_mask"], inputs["self_masks"],
                                      inputs["position_ids"])
            out = model.assemble_outputs(core)
            prep = {n: inputs[n] for n in ("tgt_boxes", "maps", "valid", "sizes", "num_boxes")}
            ld, _ = crit.loss_prepared(out, prep)
            return weighted_loss(ld, crit.weight_dict), out

    def crit_only():
        with torch.no_grad():
            _, out = fwd_loss()
        leaves = {}

        def leaf(t):
            if not t.is_floating_point():
                return t
            x = t.detach().clone().requires_grad_(True)
            leaves[id(x)] = x
            return x
        out2 = {"pred_logits": leaf(out["pred_logits"]), "pred_boxes": leaf(out["pred_boxes"]),
                "text_mask": out["text_mask"], "aux_outputs": [{k: leaf(v) for k, v in a.items()}
                                                               for a in out["aux_outputs"]],
                "interm_outputs": {k: leaf(v) for k, v in out["interm_outputs"].items()}}
        prep = {n: inputs[n] for n in ("tgt_boxes", "maps", "valid", "sizes", "num_boxes")}
        crit.loss_prepared(out2, prep)  # eager once

        def body():
            ld, _ = crit.loss_prepared(out2, prep)
            loss = weighted_loss(ld, crit.weight_dict)
            node_log = NODE_LOG
            seen, stack = set(), [loss.grad_fn]
            while stack:  # a pre-hook on every backward node: the last name printed ran last
                n = stack.pop()
                if n is None or n in seen:
                    continue
                seen.add(n)
                n.register_prehook((lambda name: lambda *a: node_log.append(name))(n.name()))
                stack.extend(f for f, _ in n.next_functions)
            loss.backward()
        return body

    if os.environ.get("PROBE_STEPGRAPH") == "1":
        g2 = TrainStepGraph(model, crit, opt, warmup=2)
        try:
            g2(*b)
            torch.cuda.synchronize()
            print("CAPTURE TrainStepGraph: OK", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"CAPTURE TrainStepGraph: FAILED {type(e).__name__}: {str(e)[:200]}", flush=True)
        return
    pieces = [("criterion fwd+bwd", crit_only()),
              ("forward + loss", lambda: fwd_loss()),
              ("forward + loss + backward", lambda: fwd_loss()[0].backward()),
              ("full step body", lambda: g._body(inputs))]
    for name, fn in pieces:
        opt.zero_grad(set_to_none=True)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()  # eager warm-up of this piece on a side stream
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        opt.zero_grad(set_to_none=True)
        graph = torch.cuda.CUDAGraph()
        oplog = OpLog() if os.environ.get("PROBE_OPLOG", "1") == "1" else contextlib.nullcontext()
        try:
            with torch.cuda.graph(graph, stream=s), oplog:
                fn()
            print(f"CAPTURE {name}: captured, replaying", flush=True)
            for i in range(int(os.environ.get("PROBE_REPLAYS", "1"))):
                graph.replay()
                torch.cuda.synchronize()
                print(f"  replay {i} done", flush=True)
            print(f"CAPTURE {name}: OK", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"CAPTURE {name}: FAILED {type(e).__name__}: {str(e)[:200]}", flush=True)
            print(f"  last ops before the failure: {getattr(oplog, 'last', [])[-8:]}", flush=True)
            print(f"  last backward nodes: {NODE_LOG[-6:]}", flush=True)
            traceback.print_exc(limit=6)
            break


if __name__ == "__main__":
    main()
