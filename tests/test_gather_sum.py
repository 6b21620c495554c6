"""ipm._ScatterSum's gather-sums: the lane layout of the native kernel (CPU) and, on MI355X, the
kernel against the torch reduction it replaces -- bitwise, for plain sums, selected sources and
products, with lists of every width from 1 to 256 (the ones above 64 stay on the torch path)."""
import numpy as np
import pytest
import torch

from awebox_amd import ipm


def _pattern(rng, n_dst=300, max_mult=200):
    mult = np.concatenate([rng.integers(1, 9, n_dst - 6), [16, 33, 64, 65, 130, max_mult]])
    dst = np.repeat(rng.permutation(4 * n_dst)[:n_dst], mult)
    return rng.permutation(dst)


def test_lane_layout_covers_every_source_once_with_aligned_lists():
    rng = np.random.default_rng(0)
    dst = _pattern(rng)
    sc = ipm._ScatterSum(dst, "cpu")
    lsrc, lw, ldst = sc.lanes_host
    L = len(lsrc)
    seen = np.zeros(len(dst), dtype=int)
    l = 0
    while l < L:
        w = int(lw[l])
        assert l % w == 0 and np.all(lw[l:l + w] == w) and w <= 64
        assert ldst[l] >= 0 and np.all(ldst[l + 1:l + w] == -1)
        src = lsrc[l:l + w]
        src = src[src >= 0]
        assert len(src) > w // 2 or w == 1                 # a list fills more than half its width
        assert np.all(dst[src] == ldst[l])
        seen[src] += 1
        l += w
    wide = {int(d) for dd, t in sc.buckets if t.shape[1] > 64 for d in dd.tolist()}
    assert wide                                             # the pattern has lists beyond 64
    for i, d in enumerate(dst):
        assert seen[i] == (0 if int(d) in wide else 1)
    # the host model of the kernel's sums (adjacent-pair trees, then the wide buckets by torch)
    # agrees with the torch path (whose CPU summation order differs: to rounding)
    vals = rng.standard_normal(len(dst))
    ref = sc.add_into(torch.zeros(4 * 300, dtype=torch.float64), torch.tensor(vals)).numpy()
    emu = np.zeros(4 * 300)
    l = 0
    while l < L:
        w = int(lw[l])
        v = np.where(lsrc[l:l + w] >= 0, vals[np.clip(lsrc[l:l + w], 0, None)], 0.0)
        while len(v) > 1:
            v = v[0::2] + v[1::2]
        emu[ldst[l]] += v[0]
        l += w
    for d, t in sc.buckets:
        if t.shape[1] > 64:
            ext = np.concatenate([vals, [0.0]])
            emu[d.numpy()] += ext[t.numpy()].sum(-1)
    assert np.allclose(emu, ref, rtol=1e-13, atol=1e-13)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 7, 64])
def test_native_gather_sum_is_bitwise_the_torch_reduction(B):
    rng = np.random.default_rng(B)
    dst = _pattern(rng)
    n_out = 4 * 300
    sc = ipm._ScatterSum(dst, "cuda")
    assert sc.native and sc.lsrc.numel() > 0 and sc.wide
    vals = torch.tensor(rng.standard_normal((B, len(dst))) * np.exp(rng.uniform(-15, 15, (B, len(dst)))),
                        device="cuda")
    base = torch.tensor(rng.standard_normal((B, n_out)), device="cuda")
    ref = sc._torch_buckets(base.clone(), vals, sc.buckets)
    got = sc.add_into(base.clone(), vals)
    assert torch.equal(got.view(torch.int64), ref.view(torch.int64))
    # selected sources: vals[:, sel]
    sel = torch.tensor(rng.permutation(len(dst) + 50)[:len(dst)], device="cuda")
    big = torch.tensor(rng.standard_normal((B, len(dst) + 50)), device="cuda")
    ref = sc._torch_buckets(base.clone(), big[:, sel], sc.buckets)
    got = sc.add_into_sel(base.clone(), big, sel)
    assert torch.equal(got.view(torch.int64), ref.view(torch.int64))
    # products vals * x[cols]
    cols = torch.tensor(rng.integers(0, 500, len(dst)), device="cuda")
    x = torch.tensor(rng.standard_normal((B, 500)), device="cuda")
    ref = sc._torch_buckets(base.clone(), vals * x[:, cols], sc.buckets)
    got = sc.add_products(base.clone(), vals, x, cols, cols.to(torch.int32))
    assert torch.equal(got.view(torch.int64), ref.view(torch.int64))
