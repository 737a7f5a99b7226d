"""bench.py — Grounding DINO (Swin-T + BERT-base) training throughput on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1 under torchrun: one rank per process from RANK / LOCAL_RANK / WORLD_SIZE;
     N > 1 without a torchrun environment: bench.py starts the N ranks itself)

A step is one full training iteration of BASELINE config 3 (the metric's
"train images/sec"): synthetic odvg batch of bs=2 images per GPU at 800x1333
with 256-token captions, forward (Swin-T, BERT-base, 6+6 layer deformable
transformer with fusion, 900 queries) -> SetCriterion (Hungarian matching,
token focal + L1 + GIoU on 7 heads) -> backward -> clip_grad_norm(0.1) ->
AdamW, under bf16 autocast, random weights; activation checkpointing off by
default (--checkpointing on: cfg_odvg's recompute of the Swin blocks, fusion
and encoder layers; same losses and gradients, see --checkpointing).  Multi-GPU: one process per GPU, DDP over RCCL (all-reduce bucketed
and overlapped with backward), per-GPU batch fixed -> weak scaling.

Rank 0 prints ONE JSON line with the contract fields plus
  roofline      live HIP-event timing of the dominant MSDA launch (the
                encoder-shape backward) inside the timed region, priced with
                SURVEY §8d algorithmic bytes against 8 TB/s;
  cpu_baseline  the reference's pure-PyTorch MSDA fallback (oracle
                restatement) on this host's cores, a bounded sample of the same
                per-step MSDA work, converted to images/s.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-groundingdino_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md chip table (spec)
LEVELS_800 = [(100, 167), (50, 84), (25, 42), (13, 21)]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bs", type=int, default=2, help="images per GPU")
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--width", type=int, default=1333)
    ap.add_argument("--backbone", default="swin_T_224_1k")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--bucket-mb", type=float, default=25,
                    help="gradient all-reduce bucket size (MB; the first bucket is 1 MB so the first collective "
                         "starts early in the backward)")
    ap.add_argument("--forward-only", action="store_true",
                    help="BASELINE config 2: eval-mode forward (no autograd) instead of the train step")
    ap.add_argument("--graphs", dest="graphs", action="store_true", default=None,
                    help="replay the whole train step (forward, device Hungarian matching + loss, backward with "
                         "the overlapped gradient all-reduce, clip, AdamW) as ONE HIP graph (default for the train "
                         "step on the GPU; DESIGN.md section 7)")
    ap.add_argument("--no-graphs", dest="graphs", action="store_false", help="eager train step")
    ap.add_argument("--checkpointing", choices=("on", "off"), default="off",
                    help="the reference's activation checkpointing (cfg_odvg use_checkpoint / use_transformer_ckpt: "
                         "Swin blocks, fusion and encoder layers recomputed in the backward). Default off: the "
                         "bs=2 step's activations fit a 288 GB MI355X many times over, and the loss and gradients "
                         "are the same either way (train.set_activation_checkpointing)")
    ap.add_argument("--tunableop", default=None, metavar="CSV",
                    help="use pre-tuned hipBLASLt GEMM solutions from CSV (tools/tune_gemms.py); no tuning at run time")
    ap.add_argument("--output-dir", default=None,
                    help="reference main.py:347-434: resume from DIR/checkpoint.pth when present, save it after "
                         "the timed steps (rank 0); outside the timed region")
    ap.add_argument("--ckpt-compare", choices=("auto", "on", "off"), default="auto",
                    help="also time the reference configuration (activation checkpointing on) in the same run and "
                         "report it under config.value_ckpt_on (auto: with HIP graphs)")
    ap.add_argument("--timeout", type=float, default=600.0,
                    help="bound (s) on every device wait and host barrier: a stuck collective or kernel ends the "
                         "run with an error line instead of a hang")
    ap.add_argument("--device", choices=("cuda", "cpu"), default=None,
                    help=argparse.SUPPRESS)  # cpu: the CPU contract tests only (HIP ops routed by the test)
    return ap.parse_args(argv)


def use_tunableop(path):
    """PyTorch TunableOp with a committed solution table (tools/tune_gemms.py
    writes it): picks per-shape hipBLASLt solutions, e.g. split-K for the
    long-K weight-gradient GEMMs, instead of the default heuristic's first
    choice.  Must run before the first GEMM."""
    t = torch.cuda.tunable
    t.enable(True)
    t.tuning_enable(False)
    t.set_filename(path, False)
    if not t.read_file(path):
        raise RuntimeError(f"TunableOp could not read {path}")


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, script=None):
    """``--gpus N`` (N > 1) without a torchrun environment: start the N ranks
    as children of ``torch.distributed.run`` on 127.0.0.1 and return their
    exit code.  The parent never touches the GPU (it only imports torch), so
    no HIP context exists here when the children start; rank 0's JSON line
    reaches stdout directly.  ``script`` (default: this file) is what each
    rank runs with ``argv``."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", script or os.path.abspath(__file__),
           *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    return subprocess.call(cmd, env=env)


def setup_dist(n, on_gpu=True, capture=False):
    if n <= 1 and "RANK" not in os.environ:
        return 0, 1, 0
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    if on_gpu:
        torch.cuda.set_device(local)  # bind the device before RCCL creates its communicator
        if capture:  # collectives inside the step graph (gdino_amd.stepgraph.RCCL_CAPTURE_ENV)
            from gdino_amd.stepgraph import RCCL_CAPTURE_ENV
            for k, v in RCCL_CAPTURE_ENV.items():
                os.environ.setdefault(k, v)
    dist.init_process_group("nccl" if on_gpu else "gloo")  # gloo: CPU contract test only
    return dist.get_rank(), dist.get_world_size(), local


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(bs, recompute=False):
    """The reference's pure-PyTorch MSDA CPU fallback (oracle restatement of
    ms_deform_attn_core_pytorch, oracle/msda_torch.py) timed on this host by
    BASELINE.md section 3's protocol: cfg1 (N=1, 512x512 levels, Lq=100) fwd
    and fwd+bwd with 5 warmups + 20 reps; the bs=2 800x1333 encoder layer
    (Lq = S = 22 223) fwd and fwd+bwd and the decoder layer (Lq=900) fwd+bwd
    with fewer reps (the encoder case is 0.4-2.5 s per call: 2 warmups + 5
    reps); median and p90 of each, at 1 thread and at the process's thread
    count.  `value` converts the all-thread medians to images/s of the train
    step's MSDA share (6 encoder fwd+bwd + 6 decoder fwd+bwd per step, plus
    6 encoder fwd recomputed when the step runs with activation
    checkpointing).  Thread counts: 1, the process's torch threads and the
    affinity's full core count (all host cores); ``value`` is
    the best of them, ``cores`` its thread count."""
    import statistics

    from oracle.msda_torch import msda_grid_sample

    M, D, L, P = 8, 32, 4, 4

    def make(levels, n, lq, seed):
        g = torch.Generator().manual_seed(seed)
        shapes = torch.as_tensor(levels, dtype=torch.long)
        S = int(shapes.prod(1).sum())
        v = torch.rand(n, S, M, D, generator=g)
        loc = torch.rand(n, lq, M, L, P, 2, generator=g)
        a = torch.rand(n, lq, M, L, P, generator=g) + 1e-5
        a = a / a.sum((-1, -2), keepdim=True)
        return shapes, v, loc, a

    def timed(inputs, bwd, warm, reps):
        shapes, v0, loc0, a0 = inputs
        ts = []
        for i in range(warm + reps):
            v, loc, a = (t.clone().requires_grad_(bwd) for t in (v0, loc0, a0))
            t0 = time.perf_counter()
            out = msda_grid_sample(v, shapes, loc, a)
            if bwd:
                out.backward(torch.ones_like(out))
            dt = time.perf_counter() - t0
            if i >= warm:
                ts.append(dt)
        ts.sort()
        return {"median_s": statistics.median(ts), "p90_s": ts[min(len(ts) - 1, int(0.9 * len(ts)))],
                "reps": reps, "warmup": warm}

    cfg1 = make([(64, 64), (32, 32), (16, 16), (8, 8)], 1, 100, 0)
    enc = make(LEVELS_800, bs, sum(h * w for h, w in LEVELS_800), 1)
    dec = make(LEVELS_800, bs, 900, 2)
    cases = [("cfg1_fwd", cfg1, False, 5, 20), ("cfg1_fwd_bwd", cfg1, True, 5, 20),
             ("enc_fwd", enc, False, 2, 5), ("enc_fwd_bwd", enc, True, 2, 5), ("dec_fwd_bwd", dec, True, 3, 10)]
    # the process's torch thread count is the host share this GPU gets (16 on
    # the MI355X boxes: OMP_NUM_THREADS); the affinity mask there lists all
    # 256 cores of the machine, and 256 threads on a 16-core share ran ~9x
    # slower than 16 (profiles/r04b_bench.json of round 4, 4.5 min of bench)
    threads = torch.get_num_threads()
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    res = {}
    for nt in sorted({threads, 1}, reverse=True):
        torch.set_num_threads(nt)
        try:
            res[nt] = {}
            for name, inp, bwd, w, r in cases:
                res[nt][name] = timed(inp, bwd, w, r)
                _progress(f"cpu baseline {nt} threads {name}: median {res[nt][name]['median_s'] * 1e3:.1f} ms")
        finally:
            torch.set_num_threads(threads)

    def per_step(r):
        return 6 * ((r["enc_fwd"]["median_s"] if recompute else 0.0) + r["enc_fwd_bwd"]["median_s"]
                    + r["dec_fwd_bwd"]["median_s"])

    best = min(res, key=lambda nt: per_step(res[nt]))
    return {
        "value": bs / per_step(res[best]),
        "unit": "images/s (MSDA fwd+bwd share of the train step only)",
        "cores": best,
        "kind": "port",
        "by_threads": {f"{nt}": round(bs / per_step(r), 4) for nt, r in res.items()},
        "single_thread": {"value": bs / per_step(res[1]), "cores": 1},
        "cases": {f"{nt}thr": {k: {kk: round(vv, 6) if isinstance(vv, float) else vv for kk, vv in d.items()}
                               for k, d in r.items()} for nt, r in res.items()},
        "sample": (f"reference pure-PyTorch MSDA fallback (grid_sample restatement, oracle/msda_torch.py) on "
                   f"{_cpu_model()}, torch threads={threads}, affinity cpus={affinity}, "
                   f"os.cpu_count()={os.cpu_count()}: cfg1 (N=1, 512x512, Lq=100) and bs={bs} 800x1333 encoder / "
                   f"decoder layers, median of timed reps after warmups, at {sorted(res)} threads; value (best, "
                   f"{best} threads) = {bs} images / (6 x ({'enc fwd + ' if recompute else ''}enc fwd+bwd + "
                   f"dec fwd+bwd)) = {per_step(res[best]):.2f} s of MSDA per step"),
    }


def _dist_stats(ms):
    """p50 / p90 / min / max of per-step times (ms) plus the first and last
    steps, so a drift over the timed steps is visible."""
    if not ms:
        return None
    s = sorted(ms)
    q = lambda f: s[min(len(s) - 1, int(f * len(s)))]  # noqa: E731
    return {"p50": s[len(s) // 2], "p90": q(0.9), "min": s[0], "max": s[-1], "first": ms[0], "last": ms[-1],
            "n": len(ms)}


def pmc_traffic(kname, bs):
    """HBM bytes per launch of the dominant MSDA kernel from the newest
    profiles/*_pmc_traffic.json (tools/pmc_traffic.py over separate
    FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this bench), matched by
    kernel and launch grid; None when no such profile is committed."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None
    kind, lq = kname
    with open(files[-1]) as f:
        allrows = json.load(f)["kernels"]
    rows = [k for k in allrows if f"msda_{kind}" in k["kernel"] and k["traffic_bytes"] is not None]
    if not rows:
        return None
    # the launch grid is chosen inside the C-ABI (direct, lane32 or pixel-tiled
    # backward), so match by size: the encoder call (Lq = S, tens of
    # thousands of queries) has the largest grid of its kernel, the decoder
    # call (Lq = 900) the smallest
    pick = max if lq > 900 else min
    if kind == "bwd" and any("msda_bwd_samples" in k["kernel"] for k in rows):
        # the sorted backward is several kernels per call (cell count, scan,
        # per-sample pass, [sort], per-cell and per-pixel sums): sum one row
        # per kernel, each at the encoder's (largest) or decoder's grid
        single = ("msda_bwd_lane32", "msda_bwd_enc", "msda_bwd_generic", "msda_bwd_tiled")
        fam = [k for k in allrows if k["traffic_bytes"] is not None and
               (("msda_bwd_" in k["kernel"] and not any(t in k["kernel"] for t in single)) or
                any(t in k["kernel"] for t in ("scan_block_sums", "scan_bsums", "scan_finish")))]
        by = {}
        for k in fam:
            by.setdefault(k["kernel"], []).append(k)
        return sum(pick(v, key=lambda k: k["grid"])["traffic_bytes"] for v in by.values())
    return pick(rows, key=lambda k: k["grid"])["traffic_bytes"]


def _progress(msg):
    """one stderr line per bench phase (a silent GPU run is taken for hung)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


METRIC = "train images/sec GroundingDINO-SwinT 800x1333 bs=2/GPU"


class BenchError(RuntimeError):
    pass


def _bounded_sync(on_gpu, timeout_s, what):
    """torch.cuda.synchronize() with a deadline: a replay stuck in a
    collective (or a hung kernel) becomes an error line instead of a silent
    hang."""
    if not on_gpu:
        return
    ev = torch.cuda.Event()
    ev.record()
    deadline = time.monotonic() + timeout_s
    while not ev.query():
        if time.monotonic() > deadline:
            raise BenchError(f"device did not finish within {timeout_s:.0f} s: {what}")
        time.sleep(2e-4)
    torch.cuda.synchronize()


def _barrier(world, ctrl):
    """host barrier over the gloo control group (its timeout bounds it)"""
    if world > 1:
        dist.barrier(group=ctrl)


def _max_over_ranks(x, world, ctrl):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctrl)
    return float(t)


def _timed(step, a, on_gpu, world, ctrl, what):
    """W warm-up steps, then K timed steps bracketed by a barrier and a device
    synchronisation on both sides; per-step device boundaries from one event
    per step (no host sync inside the loop); the max elapsed over ranks."""
    for _ in range(a.warmup):
        step()
    _bounded_sync(on_gpu, a.timeout, f"{what}: warm-up steps")
    _barrier(world, ctrl)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)] if on_gpu else None
    host_marks = []
    loss = None
    t0 = time.perf_counter()
    if evs:
        evs[0].record()
    for i in range(a.steps):
        loss = step()
        if evs:
            evs[i + 1].record()
        host_marks.append(time.perf_counter())
    _bounded_sync(on_gpu, a.timeout, f"{what}: timed steps")
    _barrier(world, ctrl)
    elapsed = time.perf_counter() - t0
    if evs:
        step_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(a.steps)]
    else:
        step_ms = [(b - a_) * 1e3 for a_, b in zip([t0] + host_marks[:-1], host_marks)]
    return _max_over_ranks(elapsed, world, ctrl), _dist_stats(step_ms), float(loss)


def _roofline(kern, bs, timed_note):
    """dominant MSDA launch of a per-launch timing summary -> roofline dict"""
    if not kern:
        return None
    kname, kd = max(kern.items(), key=lambda kv: kv[1]["ms"])
    avg_s = kd["ms"] / kd["n"] * 1e-3
    achieved = kd["bytes"] / avg_s
    return {"bound": "hbm", "kernel": f"msda_{kname[0]} (Lq={kname[1]})",
            "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / HBM_PEAK, "traffic": pmc_traffic(kname, bs),
            "avg_launch_us": avg_s * 1e6, "algo_bytes_per_launch": kd["bytes"], "timed": timed_note}


def main(argv=None, device_type="cuda", child_script=None):
    """device_type="cpu" exists for tests/test_bench_contract.py only (the
    HIP ops are then routed to the oracle by the test); the bench itself
    always runs on cuda.  ``--gpus N`` with no RANK in the environment
    launches the N ranks itself (launch_ranks; ``child_script`` lets the CPU
    test wrap each rank in its oracle routing)."""
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    device_type = a.device or device_type
    if a.gpus > 1 and "RANK" not in os.environ:
        if device_type != "cuda" and "--device" not in argv:
            argv += ["--device", device_type]
        rc = launch_ranks(a.gpus, argv, child_script)
        if rc:
            raise SystemExit(rc)
        return
    on_gpu = device_type == "cuda"
    rank, world, local = setup_dist(a.gpus, on_gpu,
                                    capture=(a.graphs is not False) and on_gpu and not a.forward_only)
    ctrl = None
    if world > 1:
        from gdino_amd.stepgraph import make_control_group
        ctrl = make_control_group(a.timeout)
    try:
        _run(a, on_gpu, rank, world, local, ctrl)
    except BenchError as e:
        _error_line(a, world, rank, str(e))
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)  # a rank stuck in a collective cannot be joined: leave now


def _error_line(a, world, rank, msg):
    print(f"bench error on rank {rank}: {msg}", file=sys.stderr, flush=True)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "images/s", "n_gpus": world, "steps": a.steps,
                          "warmup": a.warmup, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                          "dtype": "bf16", "error": msg}), flush=True)


def _run(a, on_gpu, rank, world, local, ctrl):
    device = torch.device("cuda", local) if on_gpu else torch.device("cpu")
    if on_gpu:
        torch.cuda.set_device(device)
    if a.tunableop:
        use_tunableop(a.tunableop)
    torch.manual_seed(1234 + rank)

    from gdino_amd import _lib, msda
    from gdino_amd.config import make_args
    from gdino_amd.train import build_training, forward_step, set_activation_checkpointing, synthetic_batch, \
        train_step

    args = make_args(device=str(device), backbone=a.backbone)
    model, criterion, _, optimizer = build_training(args, device)
    model.train(not a.forward_only)
    set_activation_checkpointing(model, a.checkpointing == "on")
    _progress("model built")
    start_epoch = 0
    # reference main.py:339 (the cfg_odvg default: StepLR every lr_drop epochs)
    sched = torch.optim.lr_scheduler.StepLR(optimizer, args.lr_drop)
    if a.output_dir and not a.forward_only:
        from gdino_amd import checkpoint as ckpt
        path = ckpt.resume_path(a.output_dir)
        if path is not None:
            start_epoch = ckpt.resume(path, model, optimizer, sched)
    # HIP graphs: the default for the train step on the
    # GPU; the forward-only line and CPU contract runs stay eager
    use_graphs = (a.graphs if a.graphs is not None else True) and on_gpu and not a.forward_only
    core = model
    grad_sync = None
    if world > 1 and not a.forward_only:
        if use_graphs:
            # DDP's reducer cannot follow graph replays: BucketedGradSync does
            # the same bucketed, backward-overlapped all-reduce from
            # post-accumulate hooks, captured into the step graph
            from gdino_amd.train import BucketedGradSync
            grad_sync = BucketedGradSync(model.parameters(), a.bucket_mb, control_group=ctrl)
        else:
            # reference main.py:258-261 (DDP + static graph); buckets sized for
            # xGMI rings (fewer, larger all-reduces), launched as backward
            # produces them so RCCL overlaps the rest of the backward pass
            model = torch.nn.parallel.DistributedDataParallel(
                model, device_ids=[local] if on_gpu else None, bucket_cap_mb=a.bucket_mb, static_graph=True)
    samples, targets, captions, cats = synthetic_batch(a.bs, a.height, a.width, n_boxes=8, n_tokens=256,
                                                       seed=1000 + rank, device=device)
    if a.forward_only:
        def step():
            out = forward_step(model, samples, captions)
            return out["pred_logits"].float().nan_to_num(0.0, 0.0, 0.0).abs().mean()
    else:
        def step():
            return train_step(model, criterion, optimizer, samples, targets, captions, cats, grad_sync=grad_sync)

    eager_step = step
    step_graph = None

    def make_graph_step():
        from gdino_amd.stepgraph import TrainStepGraph
        g = TrainStepGraph(core, criterion, optimizer, grad_sync=grad_sync, control_group=ctrl)
        return g, (lambda: g(samples, targets, captions, cats))

    if use_graphs:
        # GEMM library inside the captured region (GDINO_GRAPH_BLAS: "hipblaslt"
        # or "cublas" = rocBLAS on ROCm)
        blas = os.environ.get("GDINO_GRAPH_BLAS")
        if blas:
            torch.backends.cuda.preferred_blas_library(blas)
        # a capture failure on any rank sends EVERY rank to the eager step
        # (TrainStepGraph's rank agreement); the line records each rank's mode
        step_graph, step = make_graph_step()
        step()  # capture (+ its rolled-back warm-up steps) and one replay
        _bounded_sync(on_gpu, a.timeout, "first step (capture)")
        _progress(f"step graph: {step_graph.stats()}")

    # MSDA launch timing over the timed region (eager); with graphs the
    # launches are inside the replays, where ROCm refuses timing events: they
    # are timed in the eager step that follows the timed region
    msda.timer = None if use_graphs else msda.LaunchTimer()
    elapsed, step_stats, loss_v = _timed(step, a, on_gpu, world, ctrl, "headline")
    kern = msda.timer.summary() if msda.timer is not None else {}
    msda.timer = None
    _progress(f"{a.steps} timed steps done: {elapsed / a.steps * 1e3:.1f} ms/step")
    graph_stats = step_graph.agree.gather(step_graph.stats()) if step_graph is not None else None

    # one extra step, outside the timed region, with HIP events around every
    # C-ABI call: device time per HIP entry point (all kernel families, not
    # only the MSDA launches the roofline prices)
    # (single GPU only: under DDP a rank that failed here would leave the
    # others blocked in the gradient all-reduce, and the extra step would
    # also move the weights)
    hip_calls = None
    timed_note = ("HIP events on the launch stream in one eager step right after the timed graph replays (ROCm "
                  "refuses timing events inside a graph capture)" if use_graphs else
                  "HIP events on the launch stream over the timed region")
    if on_gpu and world == 1:
        if use_graphs:  # the extra step runs eagerly: every C-ABI call is a Python call
            msda.timer = msda.LaunchTimer()
        _lib.call_timer = _lib.CallTimer()
        try:
            eager_step()
            hip_calls = _lib.call_timer.summary()
            if use_graphs:
                kern = msda.timer.summary()
        except Exception as e:  # diagnostics only: never cost the bench line
            hip_calls = {"error": repr(e)[:300]}
        finally:
            _lib.call_timer = None
            msda.timer = None
        _progress("per-entry-point timing step done")
    roofline = _roofline(kern, a.bs, timed_note)
    kernels = {f"msda_{k}_lq{lq}": {"launches": d["n"], "avg_us": d["ms"] / d["n"] * 1e3,
                                     "algo_bytes": d["bytes"], "GBps": d["bytes"] / (d["ms"] / d["n"] * 1e-3) / 1e9}
               for (k, lq), d in sorted(kern.items())}

    # the reference's own configuration, measured in the same run: cfg_odvg's
    # activation checkpointing (use_checkpoint / use_transformer_ckpt,
    # config/cfg_odvg.py:41-42) recomputes the Swin blocks, fusion and
    # encoder layers in the backward
    ckpt_on = None
    compare = a.ckpt_compare == "on" or (a.ckpt_compare == "auto" and use_graphs)
    if compare and not a.forward_only and a.checkpointing == "off":
        if step_graph is not None:
            step_graph.release()
        set_activation_checkpointing(core, True)
        if use_graphs:
            step_graph, step2 = make_graph_step()
            step2()
            _bounded_sync(on_gpu, a.timeout, "first checkpoint-on step (capture)")
        else:
            step2 = eager_step
        e2, st2, loss2 = _timed(step2, a, on_gpu, world, ctrl, "checkpointing on")
        kern2 = {}
        if on_gpu and world == 1:
            msda.timer = msda.LaunchTimer()
            try:
                eager_step()
                kern2 = msda.timer.summary()
            finally:
                msda.timer = None
        ckpt_on = {"activation_checkpointing": True, "value": a.bs * world * a.steps / e2,
                   "ms_per_step": e2 / a.steps * 1e3, "step_ms": st2, "loss": loss2,
                   "roofline": _roofline(kern2, a.bs, timed_note),
                   "step_graph": step_graph.stats() if step_graph is not None else None}
        set_activation_checkpointing(core, False)
        _progress(f"checkpointing on: {ckpt_on['ms_per_step']:.1f} ms/step")

    images = a.bs * world * a.steps
    value = images / elapsed
    device_check = None
    if on_gpu:
        try:  # the MSDA kernels' device-side guards (csrc/msda.hip g_device_err)
            msda.check_device_status(device)
        except _lib.GdError as e:
            device_check = str(e)[:300]

    if a.output_dir and not a.forward_only:
        from gdino_amd import checkpoint as ckpt
        ckpt.save_checkpoint(os.path.join(a.output_dir, "checkpoint.pth"), core, optimizer, sched, start_epoch,
                             args)

    if rank == 0:
        mode = "forward (eval, no autograd)" if a.forward_only else "train step (fwd+bwd+AdamW)"
        res = {
            "metric": ("forward images/sec GroundingDINO-SwinT 800x1333 bs=2/GPU" if a.forward_only else METRIC),
            "value": value,
            "unit": "images/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            # per-step device time between consecutive step boundaries (HIP
            # events on the launch stream; rank 0), p50 / p90 / max
            "step_ms": step_stats,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (odvg-shaped batch, random weights, 256-token captions, 8 boxes/image)",
            "config": {"workload": f"GroundingDINO-{a.backbone} + BERT-base {mode}, "
                                   f"{a.height}x{a.width}, 900 queries, 4 levels",
                       "global_batch": a.bs * world, "per_gpu_batch": a.bs, "image": [a.height, a.width],
                       "text_tokens": 256, "parallelism": f"dp{world}",
                       "activation_checkpointing": a.checkpointing == "on",
                       "peak_hbm_gb": (round(torch.cuda.max_memory_allocated(device) / 2 ** 30, 1) if on_gpu
                                       else None)},
            "roofline": roofline,
            "kernels": kernels,
            "hip_entry_points_one_step": hip_calls,
            "options": {"hip_graphs": bool(use_graphs), "tunableop": a.tunableop,
                        "step_graph": ("whole train step (forward, device Hungarian matching + loss, backward, "
                                       "all-reduce, clip, AdamW) as one HIP graph" if use_graphs else None),
                        # per rank: graph / eager mode, captures, replays, eager steps
                        "step_graph_by_rank": graph_stats,
                        "grad_sync": (f"bucketed RCCL all-reduce overlapped with the backward (post-accumulate "
                                      f"hooks, gradients as bucket views, buckets launched in index order, "
                                      f"captured in the step graph), buckets "
                                      f"{[round(x, 1) for x in grad_sync.bucket_sizes_mb()]} MB"
                                      if grad_sync is not None else
                                      ("DDP (overlapped, eager step)" if world > 1 and not a.forward_only else None)),
                        # HIP kernel families on this run (GDINO_DISABLE turns them off for A/B)
                        "hip_families": ["msda", "biattn"] + [f for f in ("wattn", "attn", "contrastive", "prologue",
                                                                         "wgrad", "addln") if _lib.enabled(f)],
                        "msda_bwd": os.environ.get("GD_MSDA_BWD", "sorted")},
            "loss": loss_v,
        }
        if ckpt_on is not None:
            # the reference configuration (cfg_odvg: checkpointing on), same run
            res["config"]["value_ckpt_on"] = ckpt_on["value"]
            res["config"]["ms_per_step_ckpt_on"] = ckpt_on["ms_per_step"]
            res["config"]["roofline_ckpt_on"] = ckpt_on["roofline"]
            res["config"]["ckpt_on"] = ckpt_on
        if not math.isfinite(loss_v):
            res["error"] = f"non-finite loss {loss_v}: the step diverged, the throughput is not a valid measurement"
        if device_check is not None:
            res["error"] = f"device-side check failed: {device_check}"
        if not a.no_cpu_baseline and world == 1:
            _progress("cpu baseline (host cores)")
            res["cpu_baseline"] = cpu_baseline(a.bs, recompute=a.checkpointing == "on")
        print(json.dumps(res), flush=True)
    # free the step graph (and its shared memory pool) and drain the device
    # while the HIP runtime and any profiler are still up, at every world
    # size: left to interpreter teardown, a one-GPU graph was destroyed after
    # the runtime began finalising (a SIGSEGV in a non-main thread under
    # rocprofv3, profiles/r05p_pmc_write_segv.log).  Under DDP the captured
    # step also holds RCCL collectives, and destroying a process group under
    # a live graph that references it aborts.
    if step_graph is not None:
        step_graph.release()
        step_graph = None
    import gc
    gc.collect()
    _bounded_sync(on_gpu, a.timeout, "teardown")
    if world > 1:
        _barrier(world, ctrl)
        dist.destroy_process_group()
    if not math.isfinite(loss_v):
        raise SystemExit(1)


if __name__ == "__main__":
    main()
