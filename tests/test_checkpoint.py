"""Checkpoint save / resume / partial load (gdino_amd/checkpoint.py) against
the reference's contract (main.py:347-434, util/misc.py:620-626).

The "reference state dict" is the block-golden model case's parameter set:
its names come from the reference's own build_groundingdino (stored in
tests/golden/block_model.npz by make_block_golden.py) and its values from the
name-keyed deterministic fill both sides use (block_spec.fill_params)."""
import argparse

import pytest
import torch

from block_harness import fixture
from conftest import GOLDEN  # noqa: F401  (puts tests/golden on sys.path)
import block_spec as spec


def _tiny_model(seed=0):
    import models.GroundingDINO.groundingdino as gd
    from gdino_amd.config import make_args

    def tiny_lm(_name):
        from transformers import BertConfig, BertModel
        return BertModel(BertConfig(**spec.TINY_BERT))

    prev = gd.get_pretrained_language_model
    gd.get_pretrained_language_model = tiny_lm
    try:
        torch.manual_seed(seed)
        model, _, _ = gd.build_groundingdino(make_args(device="cpu", **spec.MODEL_OVERRIDES))
    finally:
        gd.get_pretrained_language_model = prev
    return model


@pytest.fixture(scope="module")
def reference_state():
    """{reference parameter name: value} of the block-golden model case."""
    _, meta = fixture("model")
    m = _tiny_model()
    ck = spec.fill_params(m.double())
    assert abs(ck - meta["weights_checksum"]) <= 1e-9 * meta["weights_checksum"]
    params = dict(m.named_parameters())
    assert sorted(params) == meta["param_names"]
    return {n: params[n].detach().float().clone() for n in meta["param_names"]}


def _train_state(model):
    from gdino_amd.config import make_args
    from gdino_amd.train import build_optimizer
    opt = build_optimizer(make_args(device="cpu"), model)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=4)
    return opt, sched


def test_reference_state_dict_loads_strict(reference_state):
    m = _tiny_model(seed=1)
    own = m.state_dict()
    sd = dict(own)
    sd.update(reference_state)  # every reference parameter, by its reference name
    res = m.load_state_dict(sd, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
    for n, v in reference_state.items():
        assert torch.equal(m.state_dict()[n], v), n


def test_save_resume_round_trip(tmp_path, reference_state):
    from gdino_amd import checkpoint as C
    m = _tiny_model(seed=1)
    m.load_state_dict(reference_state, strict=False)
    opt, sched = _train_state(m)
    # one optimizer step so AdamW has moments to save
    loss = sum((p.float() ** 2).sum() for p in m.parameters() if p.requires_grad)
    loss.backward()
    opt.step()
    sched.step()
    args = argparse.Namespace(lr=1e-4, epochs=15)
    path = str(tmp_path / "out" / "checkpoint.pth")
    C.save_checkpoint(path, m, opt, sched, epoch=3, args=args)

    m2 = _tiny_model(seed=2)
    opt2, sched2 = _train_state(m2)
    assert C.resume_path(str(tmp_path / "out"), "elsewhere.pth") == path  # main.py:347-348
    start = C.resume(path, m2, opt2, sched2)
    assert start == 4
    for (n, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), n
    s1, s2 = opt.state_dict(), opt2.state_dict()
    assert s1["param_groups"] == s2["param_groups"]
    for k in s1["state"]:
        for kk in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(s1["state"][k][kk], s2["state"][k][kk])
    assert sched2.state_dict() == sched.state_dict()
    # evaluation: model only, training state untouched (main.py:358)
    m3 = _tiny_model(seed=3)
    opt3, sched3 = _train_state(m3)
    assert C.resume(path, m3, opt3, sched3, eval_only=True) == 0
    assert not opt3.state_dict()["state"]


def test_ddp_prefixed_checkpoint_and_pickled_namespace(tmp_path, reference_state):
    """A checkpoint as the reference writes it: DDP 'module.' keys and the
    args Namespace pickled in (main.py:425-431) -- loaded without executing
    anything from the file (weights_only + the Namespace allow-list)."""
    from gdino_amd import checkpoint as C
    path = str(tmp_path / "ref_style.pth")
    torch.save({"model": {"module." + k: v for k, v in reference_state.items()},
                "args": argparse.Namespace(lr=1e-4, finetune_ignore=None)}, path)
    m = _tiny_model(seed=4)
    assert C.resume(path, m) == 0
    for n, v in reference_state.items():
        assert torch.equal(m.state_dict()[n], v), n


def test_pretrained_partial_load_with_finetune_ignore(tmp_path, reference_state):
    """main.py:364-381: keys containing a finetune_ignore keyword keep the
    model's own values."""
    from gdino_amd import checkpoint as C
    path = str(tmp_path / "pretrained.pth")
    torch.save({"model": reference_state}, path)
    m = _tiny_model(seed=5)
    own = {k: v.clone() for k, v in m.state_dict().items()}
    ignore = ["bert", "class_embed", "label_enc.weight"]
    res, dropped = C.load_pretrained(path, m, ignore)
    assert dropped and all(any(w in k for w in ignore) for k in dropped)
    assert set(dropped) == {k for k in reference_state if any(w in k for w in ignore)}
    assert not res.unexpected_keys
    sd = m.state_dict()
    for k, v in reference_state.items():
        if k in dropped:
            assert torch.equal(sd[k], own[k]), k
        else:
            assert torch.equal(sd[k], v), k
