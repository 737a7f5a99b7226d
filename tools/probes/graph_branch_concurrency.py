"""Probe: does a HIP graph run independent branches (captured on two forked
streams) concurrently on this ROCm?  Chains of small kernels on one stream vs
the same kernels split over two forked streams, captured and replayed."""
import time
import torch

dev = torch.device("cuda")
N = 200
a = [torch.randn(1 << 16, device=dev) for _ in range(4)]
big = [torch.randn(1 << 24, device=dev) for _ in range(4)]


def chain(x, n, t):
    for _ in range(n):
        torch.add(x, 1.0, out=t)
        torch.add(t, 1.0, out=x)


def capture(fn):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        fn()
    return g


def serial(xs):
    def fn():
        chain(xs[0], N, xs[1])
        chain(xs[2], N, xs[3])
    return fn


def forked(xs):
    def fn():
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        chain(xs[0], N, xs[1])
        with torch.cuda.stream(side):
            chain(xs[2], N, xs[3])
        cur.wait_stream(side)
    return fn


def timeit(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


for name, xs in (("small", a), ("big", big)):
    gs, gf = capture(serial(xs)), capture(forked(xs))
    print(f"{name}: serial {timeit(gs):.3f} ms  forked {timeit(gf):.3f} ms  ({4 * N} kernels)", flush=True)
