"""pytest plugin (TEST INFRASTRUCTURE ONLY): dry-run the GPU test files on a
machine without a GPU, with the product's HIP calls served by the host-side
SIMT emulator (tests/emu_product.py), to catch mistakes in the tests and in
the kernels' integration before a GPU session:

    python -m pytest -p emu_gpu_dryrun tests/test_kernels_gpu.py -m gpu -k "not rejects"

(run from the repo root with tests/ on PYTHONPATH, e.g. PYTHONPATH=tests).
"cuda" tensors become host tensors: tests that assert the product refuses
host tensors ("rejects") fail by design, and large shapes are slow.  It
proves nothing about the GPU itself; the same tests run on the box.
"""
import os

import torch

os.environ.setdefault("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
torch.cuda.synchronize = lambda *a, **k: None
_ctx = None


def pytest_sessionstart(session):
    global _ctx
    import emu_product
    _ctx = emu_product.emulated_product(min_tokens=64)
    _ctx.__enter__()


def pytest_sessionfinish(session, exitstatus):
    if _ctx is not None:
        _ctx.__exit__(None, None, None)


def pytest_collection_modifyitems(session, config, items):
    for it in items:
        if hasattr(it.module, "DEV"):
            it.module.DEV = "cpu"


def pytest_collection_finish(session):
    import block_harness
    orig = block_harness.compare

    def compare(name, device, *a, **k):
        return orig(name, "cpu" if device == "cuda" else device, *a, **k)

    for it in session.items:
        if hasattr(it.module, "compare"):
            it.module.compare = compare
