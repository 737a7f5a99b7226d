"""Probe: the same fp32 forward/backward at T = 40 and with the text padded to
the 64-token bucket; prints the first modules (execution order) whose outputs
differ on the real-token slice, and the matchings."""
import sys
import torch
sys.path[:0] = ["tests", ".", "open-groundingdino_amd"]
import test_stepgraph_gpu as t
from gdino_amd.stepgraph import TrainStepGraph

b = t._batch(11, 5)
runs = {}
for mult in (1, 64):
    model, crit, opt = t._model()
    rec = []
    def hook(name):
        def f(m, i, o):
            x = o[0] if isinstance(o, (tuple, list)) else o
            if isinstance(x, dict):
                x = next((v for v in x.values() if torch.is_tensor(v)), None)
            if torch.is_tensor(x) and x.is_floating_point():
                rec.append((name, x.detach().float().clone()))
        return f
    for n, m in model.named_modules():
        if n and n.count(".") <= 4:
            m.register_forward_hook(hook(n))
    g = TrainStepGraph(model, crit, opt, amp_dtype=None, text_multiple=mult)
    inputs, pf = g._prepare(*b)
    captured = {}
    orig = crit.loss_prepared
    def lp(outputs, prep):
        losses, pairs = orig(outputs, prep)
        captured["pairs"] = [p.clone() for p in pairs]
        captured["logits"] = outputs["pred_logits"].detach().clone()
        captured["boxes"] = outputs["pred_boxes"].detach().clone()
        return losses, pairs
    crit.loss_prepared = lp
    loss, d = g._forward_loss(inputs, pf)
    loss.backward()
    torch.cuda.synchronize()
    runs[mult] = (rec, captured, {k: float(v) for k, v in d.items()})

ra, ca, da = runs[1]
rb, cb, db = runs[64]
print("n hooks", len(ra), len(rb))
nb = dict()
for n, x in rb:
    nb.setdefault(n, []).append(x)
seen = {}
shown = 0
for n, x in ra:
    k = seen.get(n, 0); seen[n] = k + 1
    if n not in nb or k >= len(nb[n]):
        continue
    y = nb[n][k]
    if x.dim() != y.dim():
        continue
    sl = tuple(slice(0, min(a, c)) for a, c in zip(x.shape, y.shape))
    xs, ys = x[sl], y[sl]
    r = float((xs - ys).norm() / xs.norm().clamp_min(1e-30))
    if r > 1e-5 and shown < 40:
        print(f"{n}[{k}] shapes {tuple(x.shape)} {tuple(y.shape)} rel {r:.3e}")
        shown += 1
print("pairs equal:", all(torch.equal(p, q) for p, q in zip(ca["pairs"], cb["pairs"])))
print("logits rel", float((ca["logits"][..., :40] - cb["logits"][..., :40]).nan_to_num(0, 0, 0).norm()
                          / ca["logits"][..., :40].nan_to_num(0, 0, 0).norm()))
print("boxes rel", float((ca["boxes"] - cb["boxes"]).norm() / ca["boxes"].norm()))
for k in da:
    if abs(da[k] - db[k]) > 1e-5 * abs(da[k]) + 1e-7:
        print("loss term", k, da[k], db[k])
