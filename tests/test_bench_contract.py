"""bench.py's driver contract, exercised end to end on CPU: argument
parsing, the warmup / timed loop around the real train step, and the one JSON
line with every field the driver and the judge read (metric, value, unit,
n_gpus, steps, warmup, ms_per_step, higher_is_better, scaling, vs_baseline,
dtype, data, config, roofline, cpu_baseline).  Tiny image, HIP-only ops
routed to the oracle (tests/oracle_hooks.py); the GPU run itself happens on
the MI355X."""
import json

import torch

from oracle_hooks import oracle_msda


def test_bench_prints_the_contract_json_line(capsys):
    import bench
    # 256x320: the smallest image whose encoder tokens (1 700) cover the 900
    # queries' top-k; the full Swin-T + BERT-base model as in the bench
    argv = ["--steps", "1", "--warmup", "0", "--height", "256", "--width", "320"]
    torch.manual_seed(0)
    with oracle_msda():
        bench.main(argv, device_type="cpu")
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, "rank 0 must print exactly one JSON line"
    res = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in res, k
    assert res["metric"].startswith("train images/sec GroundingDINO-SwinT")
    assert res["unit"] == "images/s" and res["higher_is_better"] is True and res["scaling"] == "weak"
    assert res["n_gpus"] == 1 and res["steps"] == 1 and res["warmup"] == 0
    assert res["value"] > 0 and res["ms_per_step"] > 0
    assert abs(res["value"] - 2 / (res["ms_per_step"] / 1e3)) < 1e-6 * res["value"]  # bs=2 images per step
    assert res["vs_baseline"] is None and res["dtype"] == "bf16"
    assert res["config"]["parallelism"] == "dp1" and res["config"]["global_batch"] == 2
    assert res["roofline"] is None  # MSDA ran through the oracle hook: no HIP launches were timed
    cb = res["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1 and cb["sample"]
    assert cb["unit"].startswith("images/s")
    st = cb["single_thread"]
    assert st["cores"] == 1 and 0 < st["value"]


def _rank_worker(rank, world, port, q):
    import contextlib
    import io
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "open-groundingdino_amd")]
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(3)
    import bench
    from oracle_hooks import oracle_msda
    buf = io.StringIO()
    try:
        with oracle_msda(), contextlib.redirect_stdout(buf):
            bench.main(["--gpus", str(world), "--steps", "1", "--warmup", "1", "--height", "256", "--width", "320"],
                       device_type="cpu")
        q.put((rank, "ok", buf.getvalue()))
    except Exception as e:  # noqa: BLE001 (reported to the parent)
        q.put((rank, repr(e), buf.getvalue()))


def test_bench_two_ranks_contract():
    """The torchrun path the driver's scaling runs take (--gpus N, one rank per
    device, DDP, barrier + max-over-ranks timing): two gloo ranks on CPU.
    Rank 0 alone prints the line; value counts the images of all ranks."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=900)
    res = dict((r, (st, out)) for r, st, out in (q.get(timeout=5) for _ in range(2)))
    assert all(p.exitcode == 0 for p in procs)
    assert res[0][0] == "ok" and res[1][0] == "ok", res
    assert not [ln for ln in res[1][1].splitlines() if ln.startswith("{")], "only rank 0 prints"
    lines = [ln for ln in res[0][1].splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    r0 = json.loads(lines[0])
    assert r0["n_gpus"] == 2 and r0["config"]["parallelism"] == "dp2" and r0["config"]["global_batch"] == 4
    assert abs(r0["value"] - 4 / (r0["ms_per_step"] / 1e3)) < 1e-6 * r0["value"]  # 2 images x 2 ranks per step
    assert "cpu_baseline" not in r0  # rank 0 at N=1 only


def test_bench_self_launches_ranks_from_a_bare_environment(capfd, monkeypatch):
    """``python bench.py --gpus 2`` as the driver may call it, with no torchrun
    environment: bench.main starts the 2 ranks itself (torch.distributed.run on
    127.0.0.1) and rank 0 prints the one line.  Here the ranks run on
    CPU/gloo with the HIP-only ops routed to the oracle (tests/bench_cpu_rank.py)."""
    import os
    import bench
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench_cpu_rank.py")
    bench.main(["--gpus", "2", "--steps", "1", "--warmup", "1", "--height", "256", "--width", "320"],
               device_type="cpu", child_script=child)
    out = capfd.readouterr().out
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    r0 = json.loads(lines[0])
    assert r0["n_gpus"] == 2 and r0["config"]["parallelism"] == "dp2" and r0["config"]["global_batch"] == 4
    assert abs(r0["value"] - 4 / (r0["ms_per_step"] / 1e3)) < 1e-6 * r0["value"]
    assert r0["step_ms"]["n"] == 1 and r0["step_ms"]["max"] > 0
    assert "cpu_baseline" not in r0


def test_pmc_traffic_matches_the_encoder_and_decoder_launch_by_grid(tmp_path, monkeypatch):
    """roofline.traffic: the committed PMC summary is matched by kernel name,
    the encoder call to its kernel's largest grid, the decoder call to the
    smallest (the C-ABI picks the backward variant, hence the grid)."""
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    rows = [{"kernel": "gd::msda_bwd_tiled<unsigned short, 64, 8>", "grid": 2_850_000, "traffic_bytes": 3.0e8},
            {"kernel": "gd::msda_bwd_lane32<unsigned short, 4, 4>", "grid": 460_800, "traffic_bytes": 1.1e7},
            {"kernel": "gd::msda_fwd_vec<unsigned short, 32, 4, 4>", "grid": 1_422_336, "traffic_bytes": 1.6e8},
            {"kernel": "gd::msda_fwd_vec<unsigned short, 32, 4, 4>", "grid": 57_600, "traffic_bytes": None}]
    (prof / "r01_pmc_traffic.json").write_text(json.dumps({"kernels": rows}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_traffic(("bwd", 22223), 2) == 3.0e8
    assert bench.pmc_traffic(("bwd", 900), 2) == 1.1e7
    assert bench.pmc_traffic(("fwd", 22223), 2) == 1.6e8
    assert bench.pmc_traffic(("fwd", 900), 2) == 1.6e8  # only the measured row
    (prof / "r01_pmc_traffic.json").write_text(json.dumps({"kernels": rows[2:3]}))
    assert bench.pmc_traffic(("bwd", 22223), 2) is None


def test_bench_output_dir_resumes_and_saves(tmp_path, capsys):
    """--output-dir (reference main.py:347-362, 414-434): the first run saves
    DIR/checkpoint.pth after its timed steps; the second run resumes model,
    optimizer and scheduler state from it and saves the next epoch."""
    import bench
    from gdino_amd.checkpoint import load_checkpoint
    argv = ["--steps", "1", "--warmup", "0", "--height", "256", "--width", "320", "--no-cpu-baseline",
            "--output-dir", str(tmp_path)]
    torch.manual_seed(0)
    with oracle_msda():
        bench.main(argv, device_type="cpu")
        ck0 = load_checkpoint(str(tmp_path / "checkpoint.pth"))
        assert ck0["epoch"] == 0 and {"model", "optimizer", "lr_scheduler", "args"} <= set(ck0)
        bench.main(argv, device_type="cpu")
    ck1 = load_checkpoint(str(tmp_path / "checkpoint.pth"))
    assert ck1["epoch"] == 1
    # the optimizer state continued from the first run: AdamW's step counter is 2
    steps = {int(v["step"]) for v in ck1["optimizer"]["state"].values()}
    assert steps == {2}, steps
    capsys.readouterr()
