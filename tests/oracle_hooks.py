"""Test-only: run the model's host logic on CPU by routing the HIP-only ops
(MSDA, BiAttention softmax, window attention, masked attention, contrastive head) to their oracle restatements.  The product raises on CPU tensors; this hook
is the only way CPU tests execute MSDA."""
import contextlib

from oracle.msda_torch import msda_gather


class _OracleMSDA:
    @staticmethod
    def apply(value, shapes, lsi, loc, attn, im2col_step):
        return msda_gather(value, shapes, lsi, loc.to(value.dtype), attn.to(value.dtype))


@contextlib.contextmanager
def oracle_msda():
    """Route every HIP-only op to its oracle restatement (CPU tests)."""
    import models.GroundingDINO.ms_deform_attn as mod
    from gdino_amd import kernels
    from oracle.blocks import (attention_ref, bi_attention_ref, contrastive_ref, window_attention_image_ref,
                               window_attention_packed_ref)

    prev = mod.MSDeformAttnFunction
    mod.MSDeformAttnFunction = _OracleMSDA
    try:
        with kernels.override("bi_attention", lambda q, k, vv, vl, pv=None, pl=None, p=0.0:
                              bi_attention_ref(q, k, vv, vl, pv, pl)), \
                kernels.override("window_attention_packed", window_attention_packed_ref), \
                kernels.override("window_attention_image", window_attention_image_ref), \
                kernels.override("attention", lambda q, k, v, m=None, sc=None, p=0.0:
                                 attention_ref(q, k, v, m, sc)), \
                kernels.override("contrastive_logits", contrastive_ref), \
                kernels.override("contrastive_rowmax", lambda x, t, m:
                                 contrastive_ref(x, t, m, t.shape[1]).detach().max(-1)[0]):
            yield
    finally:
        mod.MSDeformAttnFunction = prev


@contextlib.contextmanager
def scipy_lsap():
    """Route the device Hungarian solver (gdino_amd.lsap, csrc/lsap.hip) to
    scipy's linear_sum_assignment -- the reference's own solver and the
    kernel's oracle -- so SetCriterion.loss_prepared runs on CPU tensors."""
    import numpy as np
    import torch
    from scipy.optimize import linear_sum_assignment

    from gdino_amd import lsap

    def host(cost, sizes, status=None):
        p, q, k = cost.shape
        rows = torch.full((p, k), -1, dtype=torch.int64)
        cols = torch.full((p, k), -1, dtype=torch.int64)
        c = cost.detach().double().cpu().numpy()
        for i, n in enumerate(sizes.tolist()):
            r, cc = linear_sum_assignment(np.asarray(c[i, :, :n]))
            rows[i, :len(r)], cols[i, :len(r)] = torch.from_numpy(r), torch.from_numpy(cc)
        return rows.to(cost.device), cols.to(cost.device)

    saved = lsap.linear_sum_assignment_batched
    lsap.linear_sum_assignment_batched = host
    try:
        yield
    finally:
        lsap.linear_sum_assignment_batched = saved
