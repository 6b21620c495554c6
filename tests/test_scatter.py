"""Fixed-order scatter sums of the solver (ipm._ScatterSum, ipm._GatherMv): equal to the atomic
index_put_(accumulate=True) they replace, on patterns with repeated indices, batched, empty."""
import numpy as np
import torch

from awebox_amd.ipm import _GatherMv, _ScatterSum


def test_scatter_sum_matches_index_put_accumulate():
    rng = np.random.default_rng(3)
    for n_out, n_src in ((1, 1), (7, 50), (100, 3000), (5, 0)):
        dst = rng.integers(0, n_out, n_src)
        if n_src > 10:
            dst[:n_src // 3] = 0                               # one destination with a long run
        vals = torch.tensor(rng.standard_normal(n_src))
        ref = torch.zeros(n_out, dtype=torch.float64).index_put_((torch.tensor(dst, dtype=torch.int64),), vals,
                                                                   accumulate=True)
        out = _ScatterSum(dst, "cpu").add_into(torch.zeros(n_out, dtype=torch.float64), vals)
        assert torch.allclose(out, ref, rtol=1e-13, atol=1e-13)


def test_scatter_sum_batched_and_repeatable():
    rng = np.random.default_rng(4)
    dst = rng.integers(0, 40, 900)
    sc = _ScatterSum(dst, "cpu")
    vals = torch.tensor(rng.standard_normal((3, 900)))
    out = sc.add_into(torch.zeros(3, 40, dtype=torch.float64), vals)
    for b in range(3):
        one = sc.add_into(torch.zeros(40, dtype=torch.float64), vals[b])
        assert torch.equal(out[b], one)                        # same order per batch member
    assert torch.equal(out, sc.add_into(torch.zeros(3, 40, dtype=torch.float64), vals))


def test_gather_mv_matches_dense():
    rng = np.random.default_rng(5)
    rows = rng.integers(0, 30, 400)
    cols = rng.integers(0, 20, 400)
    rows[:100] = 2                                            # a long row (J^T's t_f column)
    vals = torch.tensor(rng.standard_normal(400))
    A = torch.zeros(30, 20, dtype=torch.float64).index_put_(
        (torch.tensor(rows, dtype=torch.int64), torch.tensor(cols, dtype=torch.int64)), vals, accumulate=True)
    x = torch.tensor(rng.standard_normal(20))
    y = _GatherMv(rows, cols, (30, 20), "cpu").mv(vals, x)
    assert torch.allclose(y, A @ x, rtol=1e-12, atol=1e-12)
