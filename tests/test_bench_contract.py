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
