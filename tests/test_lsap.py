"""Device Hungarian matching (csrc/lsap.hip) against the algorithm the
reference calls: scipy.optimize.linear_sum_assignment (scipy 1.15.3 here;
reference call site models/GroundingDINO/matcher.py:104-110).  scipy is the
oracle: the kernel restates its rectangular LSAP with the same float64
operation order and tie-breaking, so the pairs must be IDENTICAL -- also on
tie-heavy integer and constant cost matrices, where any other exact solver
may return a different optimal assignment.

CPU: the kernel source on the host-side SIMT emulator (tests/emu).
GPU: the gfx950 build through the C ABI (gdino_amd.lsap)."""
import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment


def _cases(seed, n_cases, qs, ks):
    rng = np.random.default_rng(seed)
    for c in range(n_cases):
        q, k = int(rng.choice(qs)), int(rng.choice(ks))
        kind = c % 5
        shape = (3, q, k)
        if kind == 0:
            cost = rng.random(shape)
        elif kind == 1:
            cost = rng.integers(0, 3, shape)        # many ties
        elif kind == 2:
            cost = np.zeros(shape)                  # all tied: scipy's identity-like pick
        elif kind == 3:
            cost = rng.integers(0, 50, shape) / 7.0
        else:                                       # matcher-like: L1 + focal + GIoU magnitudes
            cost = rng.normal(0.0, 1.0, shape) * 2.0 + 3.0
        sizes = rng.integers(0, k + 1, 3)
        sizes[0] = k                                # the full width at least once
        yield cost.astype(np.float32), sizes


def _check(cost, sizes, rows, cols, status):
    P, Q, K = cost.shape
    for p in range(P):
        n = int(sizes[p])
        i, j = linear_sum_assignment(cost[p, :, :n])
        m = len(i)
        assert m == min(Q, n)
        np.testing.assert_array_equal(rows[p, :m], i, err_msg=f"rows of problem {p} (Q={Q}, n={n})")
        np.testing.assert_array_equal(cols[p, :m], j, err_msg=f"cols of problem {p} (Q={Q}, n={n})")
        assert (rows[p, m:] == -1).all() and (cols[p, m:] == -1).all()
        assert status[p] == 0


@pytest.mark.parametrize("seed", [0, 1])
def test_emulated_lsap_matches_scipy_small(seed):
    import emu_lib as E
    for cost, sizes in _cases(seed, 40, qs=[1, 2, 5, 9, 17, 33], ks=[1, 2, 4, 9, 17, 40]):
        rows, cols, status = E.linear_sum_assignment(torch.from_numpy(cost), sizes)
        _check(cost, sizes, rows.numpy(), cols.numpy(), status.numpy())


def test_emulated_lsap_matches_scipy_matcher_shapes():
    """900 queries x up to 64 targets (the criterion's problems), and wide
    matrices (more targets than queries: no transpose)."""
    import emu_lib as E
    for cost, sizes in _cases(5, 16, qs=[64, 300, 900], ks=[1, 8, 23, 64]):
        rows, cols, status = E.linear_sum_assignment(torch.from_numpy(cost), sizes)
        _check(cost, sizes, rows.numpy(), cols.numpy(), status.numpy())


def test_emulated_lsap_infeasible_falls_back_to_argmin():
    """+inf everywhere in one column: scipy raises, the reference then takes
    the argmin query per target (matcher.py:111-119); status says so."""
    import emu_lib as E
    cost = torch.rand(1, 6, 3)
    cost[0, :, 1] = float("inf")
    with pytest.raises(ValueError):
        linear_sum_assignment(cost[0].numpy())
    rows, cols, status = E.linear_sum_assignment(cost, [3])
    assert int(status[0]) == 1
    np.testing.assert_array_equal(rows[0].numpy(), cost[0].argmin(0).numpy())
    np.testing.assert_array_equal(cols[0].numpy(), np.arange(3))


def test_emulated_lsap_rejects_oversized():
    import emu_lib as E
    with pytest.raises(RuntimeError, match="exceed"):
        E.linear_sum_assignment(torch.zeros(1, 3000, 4), [4])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_lsap_gpu_matches_scipy(seed):
    from gdino_amd.lsap import linear_sum_assignment_batched
    cases = list(_cases(seed, 30, qs=[1, 5, 33, 300, 900], ks=[1, 4, 8, 17, 64]))
    for cost, sizes in cases:
        dev = torch.from_numpy(cost).cuda()
        st = torch.full((cost.shape[0],), 7, dtype=torch.int32, device="cuda")
        rows, cols = linear_sum_assignment_batched(dev, torch.from_numpy(sizes).cuda(), st)
        _check(cost, sizes, rows.cpu().numpy(), cols.cpu().numpy(), st.cpu().numpy())


@pytest.mark.gpu
def test_lsap_gpu_criterion_batch_shape():
    """All 7 heads x 2 images of a train step (900 queries, 8 and 13
    targets), matcher-like costs; also captured and replayed in a HIP graph
    on new costs (static shapes, device-side sizes)."""
    from gdino_amd.lsap import linear_sum_assignment_batched
    g = torch.Generator().manual_seed(0)
    cost = (torch.randn(14, 900, 13, generator=g) * 2 + 3).float()
    sizes = torch.tensor([8, 13] * 7, dtype=torch.int32)
    dc, ds = cost.cuda(), sizes.cuda()
    rows, cols = linear_sum_assignment_batched(dc, ds)
    _check(cost.numpy(), sizes.numpy(), rows.cpu().numpy(), cols.cpu().numpy(), np.zeros(14, np.int32))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        gr, gc = linear_sum_assignment_batched(dc, ds)
    cost2 = (torch.randn(14, 900, 13, generator=g) * 2 + 3).float()
    dc.copy_(cost2.cuda())
    graph.replay()
    torch.cuda.synchronize()
    _check(cost2.numpy(), sizes.numpy(), gr.cpu().numpy(), gc.cpu().numpy(), np.zeros(14, np.int32))
