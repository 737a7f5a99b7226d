"""Test-only rank script for tests/test_bench_contract.py: bench.py's own
launcher (``--gpus N`` with no RANK in the environment) starts N copies of
this file under torch.distributed.run; each routes the HIP-only ops to their
oracle restatements (tests/oracle_hooks.py) and runs bench.main on CPU/gloo."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "open-groundingdino_amd")]

import torch  # noqa: E402

torch.set_num_threads(3)

import bench  # noqa: E402
from oracle_hooks import oracle_msda  # noqa: E402

if __name__ == "__main__":
    with oracle_msda():
        bench.main(sys.argv[1:], device_type="cpu")
