"""Fine-grained probe: MSDA C-ABI calls under HIP stream capture."""
import faulthandler
import os
import subprocess
import sys

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]


def inputs(dev):
    import torch
    shapes = torch.as_tensor([(32, 40), (16, 20), (8, 10), (4, 5)], device=dev)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    S = int(shapes.prod(1).sum())
    v = torch.randn(2, S, 8, 32, device=dev)
    loc = torch.rand(2, S, 8, 4, 4, 2, device=dev)
    a = torch.rand(2, S, 8, 4, 4, device=dev)
    return v, shapes, lsi, loc, a


def step(name):
    import torch
    from gdino_amd import msda
    dev = torch.device("cuda")
    v, sh, ls, loc, a = inputs(dev)
    print(name, "start", flush=True)
    if name == "fwd_graph":
        ref = msda.ms_deform_attn_forward(v, sh, ls, loc, a, 64)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            msda.ms_deform_attn_forward(v, sh, ls, loc, a, 64)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = msda.ms_deform_attn_forward(v, sh, ls, loc, a, 64)
        print(name, "captured", flush=True)
        g.replay()
        torch.cuda.synchronize()
        print(name, "replayed; equal:", bool(torch.equal(out, ref)), flush=True)
    elif name == "bwd_graph":
        go = torch.randn(v.shape[0], loc.shape[1], 256, device=dev)
        ref = msda.ms_deform_attn_backward(v, sh, ls, loc, a, go, 64)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            msda.ms_deform_attn_backward(v, sh, ls, loc, a, go, 64)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = msda.ms_deform_attn_backward(v, sh, ls, loc, a, go, 64)
        print(name, "captured", flush=True)
        g.replay()
        torch.cuda.synchronize()
        print(name, "replayed; close:", [bool(torch.allclose(x, y, atol=1e-5)) for x, y in zip(out, ref)],
              flush=True)
    elif name == "func_graphed":
        from models.GroundingDINO.ops.functions.ms_deform_attn_func import MSDeformAttnFunction

        class M(torch.nn.Module):
            def forward(self, v, loc, a):
                return MSDeformAttnFunction.apply(v, sh, ls, loc, a, 64)
        vv = v.clone().requires_grad_(True)
        ll = loc.clone().requires_grad_(True)
        aa = a.clone().requires_grad_(True)
        gm = torch.cuda.make_graphed_callables(M(), (vv, ll, aa), num_warmup_iters=2)
        print(name, "captured", flush=True)
        out = gm(vv, ll, aa)
        out.sum().backward()
        torch.cuda.synchronize()
        print(name, "replayed", float(out.sum()), float(vv.grad.abs().sum()), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        step(sys.argv[1])
        sys.exit(0)
    for c in ["fwd_graph", "bwd_graph", "func_graphed"]:
        r = subprocess.run([sys.executable, "-X", "faulthandler", __file__, c], timeout=200)
        if r.returncode != 0:
            print(f"FAILED at {c} rc={r.returncode}", flush=True)
            sys.exit(1)
    print("all ok")
