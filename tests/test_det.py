"""Batch-invariant reductions (awebox_amd/det.py), host side.

The restatements det.py runs on host tensors define the order the libawelu kernels follow
(tests/test_det_gpu.py checks the kernels against them bitwise): here they are checked against a
plain-Python statement of that order, and the batched CPU-harness homotopy is checked to return
bitwise the single solves (the property DESIGN.md section 9 asks of the GPU solver)."""
import numpy as np
import pytest
import torch

from awebox_amd import det


def _row_sum_python(row):
    """awelu_row_sum's order in plain Python: 256 sequential partial sums, adjacent-pair tree."""
    T = det.ROW_SUM_THREADS
    part = []
    for t in range(T):
        acc = 0.0
        for j in range(t, len(row), T):
            acc = acc + float(row[j])
        part.append(acc)
    while len(part) > 1:
        part = [part[i] + part[i + 1] for i in range(0, len(part), 2)]
    return part[0]


def _spread(rng, shape):
    return torch.tensor(rng.standard_normal(shape) * np.exp(rng.uniform(-30, 30, shape)))


@pytest.mark.parametrize("n", [0, 1, 5, 255, 256, 257, 1000, 3001])
def test_row_sum_order(n):
    rng = np.random.default_rng(n)
    x = _spread(rng, (3, n))
    got = det.row_sum(x)
    for r in range(3):
        assert got[r].item() == _row_sum_python(x[r].tolist())


def test_row_sum_does_not_depend_on_rows():
    rng = np.random.default_rng(2)
    x = _spread(rng, (9, 777))
    full = det.row_sum(x)
    for r in range(9):
        assert torch.equal(det.row_sum(x[r:r + 1]), full[r:r + 1])
    assert torch.equal(det.row_sum(x.view(3, 3, 777)), full.view(3, 3))


def test_tree_sum_order():
    x = torch.tensor([[1e17, 1.0, -1e17, 1.0, 3.0, 0.5, 0.25, 2.0]])
    # ((1e17 + 1) + (-1e17 + 1)) + ((3 + 0.5) + (0.25 + 2)) = 0 + 5.75
    assert det.tree_sum(x).item() == ((1e17 + 1.0) + (-1e17 + 1.0)) + ((3.0 + 0.5) + (0.25 + 2.0))
    with pytest.raises(ValueError):
        det.tree_sum(torch.zeros(2, 6, dtype=torch.float64))


@pytest.mark.parametrize("M,N,K", [(7, 5, 11), (1, 1, 1), (64, 1, 300), (3, 40, 0)])
def test_bmm_order_and_values(M, N, K):
    rng = np.random.default_rng(M * 100 + N)
    A = _spread(rng, (4, K, M)).transpose(1, 2)              # a transposed view, as ipm uses it
    B = _spread(rng, (4, K, N))
    C = det.bmm(A, B)
    assert C.shape == (4, M, N)
    for b in range(4):
        for i in range(min(M, 3)):
            for j in range(min(N, 3)):
                acc = 0.0
                for k in range(K):
                    acc = acc + float(A[b, i, k]) * float(B[b, k, j])
                assert C[b, i, j].item() == acc
    ref = A @ B
    assert torch.allclose(C, ref, rtol=1e-12, atol=1e-12 * float(ref.abs().max()) if ref.numel() else 0.0)
    for b in range(4):
        assert torch.equal(det.bmm(A[b:b + 1], B[b:b + 1]), C[b:b + 1])
    assert torch.equal(det.bmv(A, B[..., 0]) if N else C[..., 0], C[..., 0])


def test_batched_homotopy_is_bitwise_the_single_solves_on_cpu_port():
    """ipm.solve_batch on the CPU harness: two wind speeds solved side by side through the whole
    homotopy return bitwise the V, multipliers and iteration counts of the two separate solves (every
    reduction and product in the solver has an order independent of the batch, det.py)."""
    from awebox_amd import problem as pb
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.trajectory import optimize, optimize_batch
    from oracle.cpu_device import CpuDeviceEvaluator
    consts = pb.build_constants(pb.Ap2Config(n_k=4, d=2))
    ev = CpuDeviceEvaluator(consts)
    u_refs = [9.5, 10.5]
    Vb, summary, outs, res = optimize_batch(consts, ev, u_refs, IpmOptions(max_iter=400), device="cpu")
    for b, u in enumerate(u_refs):
        V1, s1, o1, r1 = optimize(consts, ev, IpmOptions(max_iter=400), device="cpu", u_ref=u)
        assert [r["iterations"] for r in s1] == [r["iterations"][b] for r in summary]
        assert np.array_equal(Vb[b], V1)
        assert np.array_equal(res[b].lam_g, r1.lam_g)
