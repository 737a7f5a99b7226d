"""Where does msda_bwd_enc differ from msda_bwd_lane32?  (diagnostic, GPU)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

from gdino_amd import _lib, msda  # noqa: E402
import msda_microbench as mb  # noqa: E402

LV = mb.LEVELS
S = sum(h * w for h, w in LV)


def run(v, sh, ls, loc, attn, go, fill):
    N, _, M, D = v.shape
    Lq, L, P = loc.shape[1], loc.shape[3], loc.shape[4]
    gv = torch.empty(N, S, M, D, device="cuda")
    gl = torch.full((N, Lq, M, L, P, 2), fill, device="cuda")
    ga = torch.full((N, Lq, M, L, P), fill, device="cuda")
    hs = (ctypes.c_int64 * (2 * L))(*[int(x) for hw in LV for x in hw])
    _lib.call("gd_msda_backward_geom", _lib.dtype_code(v), v.data_ptr(), sh.data_ptr(), ls.data_ptr(),
              loc.data_ptr(), attn.data_ptr(), go.data_ptr(), N, S, M, D, L, Lq, P, gv.data_ptr(),
              gl.data_ptr(), ga.data_ptr(), hs, _lib.stream_of(v))
    torch.cuda.synchronize()
    return gv.cpu(), gl.cpu(), ga.cpu()


for vd in ():
    v, sh, ls, loc, attn, go = mb.inputs(S, vd)
    for geom in ("spread2", "init"):
        if geom == "init":
            loc = mb.init_geometry_loc(2)
        os.environ["GD_MSDA_BWD"] = "lane32"
        ref = run(v, sh, ls, loc, attn, go, 0.0)
        os.environ["GD_MSDA_BWD"] = "enc"
        out = run(v, sh, ls, loc, attn, go, float("nan"))
        ga, rga = out[2], ref[2]
        nan = ga.isnan()
        bad = ((ga - rga).abs() > 1e-4 * rga.abs().max()) & ~nan
        print(vd, geom, "unwritten", int(nan.sum()), "wrong", int(bad.sum()), "of", ga.numel(),
              "gv err", float((out[0] - ref[0]).abs().max() / ref[0].abs().max()), flush=True)
        for name, msk in (("unwritten", nan), ("wrong", bad)):
            if msk.any():
                st = [0]
                for h, w in LV:
                    st.append(st[-1] + h * w)
                bq = msk.any(-1).any(-1).any(-1)[0]
                print(f"  {name}: by level {msk.sum((0, 1, 2, 4)).tolist()} by head {msk.sum((0, 1, 3, 4)).tolist()}"
                      f" queries per query level {[int(bq[st[i]:st[i + 1]].sum()) for i in range(4)]}"
                      f" first {msk.nonzero()[:4].tolist()}")

# init geometry against the fp64 oracle (test infrastructure, diagnostic only)
import numpy as np  # noqa: E402
import oracle  # noqa: E402

v, sh, ls, loc, attn, go = mb.inputs(S, torch.float32)
loc = mb.init_geometry_loc(2)
cpu = [t.cpu() for t in (v, sh, ls, loc, attn, go)]
rgv, rgl, rga = oracle.msda_backward(cpu[0].double().numpy(), cpu[1], cpu[2], cpu[3].double(), cpu[4].double(),
                                     cpu[5].double().numpy())
rga = torch.from_numpy(np.asarray(rga))
for var, mode in (("lane32", "0"), ("enc", "0"), ("enc", "1")):
    os.environ["GD_MSDA_BWD"] = var
    os.environ["GD_MSDA_ENC_MODE"] = mode
    out = run(v, sh, ls, loc, attn, go, float("nan"))
    bad = (out[2].double() - rga).abs() > 1e-4 * rga.abs().max()
    badl = (out[1].double() - torch.from_numpy(np.asarray(rgl))).abs() > 1e-3 * float(np.abs(rgl).max())
    print("oracle vs", var, mode, "grad_attn wrong", int(bad.sum()), "grad_loc wrong", int(badl.sum()),
          "first", bad.nonzero()[:3].tolist(), flush=True)
    i = tuple(bad.nonzero()[0].tolist()) if bad.any() else None
    if i:
        print("   value", float(out[2][i]), "oracle", float(rga[i]), "loc", out and loc.cpu()[i].tolist())
        vv = v.cpu()
        print("   value rows (0,0),(0,1),(0,2) ch0-3:", vv[0, 0, 0, :4].tolist(), vv[0, 1, 0, :4].tolist(),
              vv[0, 2, 0, :4].tolist(), "grad_out ch0-3", go.cpu()[0, 0, :4].tolist(), "attn", attn.cpu()[0, 0, 0, 0].tolist())
