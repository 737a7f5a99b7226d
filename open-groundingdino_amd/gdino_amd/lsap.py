"""Hungarian matching on the device (csrc/lsap.hip, gd_linear_sum_assignment).

The reference's HungarianMatcher copies every cost matrix to the host and
calls ``scipy.optimize.linear_sum_assignment`` per image
(models/GroundingDINO/matcher.py:104-110): a device->host copy and a host
wait in the middle of every train step, after which the loss and the whole
backward can only start once the host has solved all problems.  Here the
same algorithm -- scipy 1.15's rectangular LSAP, float64 on the float32
costs, same tie-breaking -- runs as one kernel over all (head, image)
problems of a step, so matching costs the stream a few tens of
microseconds, the host nothing, and the whole train step can be captured
into one HIP graph (gdino_amd.stepgraph).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

_p, _i, _i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
_lib.register("gd_linear_sum_assignment", [_p, _i, _i, _i, _i64, _p, _p, _p, _p, _p])

MAX_COLS, MAX_ROWS = 2048, 1024


def supported(q: int, k: int) -> bool:
    """Shapes the device solver takes (max(Q, n) <= 2048, min(Q, n) <= 1024)."""
    return q <= MAX_COLS and k <= MAX_COLS and (q <= MAX_ROWS or k <= MAX_ROWS)


def linear_sum_assignment_batched(cost: torch.Tensor, sizes: torch.Tensor, status: torch.Tensor | None = None):
    """cost [P, Q, K] float32 on the device; sizes [P] int32 on the device
    (problem p uses columns :sizes[p]).  -> (rows, cols) [P, K] int64:
    scipy's linear_sum_assignment(cost[p, :, :n_p]) in its first min(Q, n_p)
    slots (ascending rows), -1 after.  ``status`` [P] int32 (optional): 1
    where scipy would raise (then the pairs are the reference's argmin
    fallback).  No host synchronisation."""
    _lib.require_device(cost, sizes, what="linear_sum_assignment")
    if cost.dtype != torch.float32:
        cost = cost.float()
    cost = cost.contiguous()
    p, q, k = cost.shape
    if sizes.dtype != torch.int32:
        sizes = sizes.to(torch.int32)
    sizes = sizes.contiguous()
    if not supported(q, k):
        raise _lib.GdError(f"linear_sum_assignment: Q={q} K={k} exceed the device solver")
    rows = torch.empty(p, k, dtype=torch.int64, device=cost.device)
    cols = torch.empty(p, k, dtype=torch.int64, device=cost.device)
    _lib.call("gd_linear_sum_assignment", cost.data_ptr(), p, q, k, q * k, sizes.data_ptr(), rows.data_ptr(),
              cols.data_ptr(), _lib.ptr(status), _lib.stream_of(cost))
    return rows, cols
