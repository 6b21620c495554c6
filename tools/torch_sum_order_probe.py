"""Which summation order does torch's CUDA/HIP `x.sum(dim=-1)` use for float64 [..., w] rows?

ipm._ScatterSum sums the duplicates of every destination as rows of power-of-two width; a native
gather-sum kernel can only replace it without changing the solver's rounding (the homotopy's final
step is sensitive to it) if it adds in torch's order.  For every width the probe compares
torch's result bitwise with candidate orders evaluated on the host in IEEE double: sequential,
adjacent-pair tree, and k strided accumulators (k = 2, 4, 8) combined sequentially or as a tree.

    python tools/torch_sum_order_probe.py  (on the GPU box)
"""
import json

import numpy as np
import torch


def seq(a):
    s = a[..., 0].copy()
    for i in range(1, a.shape[-1]):
        s = s + a[..., i]
    return s


def tree(a):
    while a.shape[-1] > 1:
        if a.shape[-1] % 2:
            a = np.concatenate([a, np.zeros(a.shape[:-1] + (1,))], -1)
        a = a[..., 0::2] + a[..., 1::2]
    return a[..., 0]


def strided(a, k, comb):
    w = a.shape[-1]
    if w < k or w % k:
        return None
    acc = [seq(a[..., j::k]) for j in range(k)]
    acc = np.stack(acc, -1)
    return seq(acc) if comb == "seq" else tree(acc)


def halving(a):
    """shuffle-down tree: x[t] += x[t + n/2], n halving"""
    while a.shape[-1] > 1:
        h = a.shape[-1] // 2
        a = a[..., :h] + a[..., h:2 * h]
    return a[..., 0]


def threaded(a, T, vec, vcomb, tcomb, layout):
    """T threads; thread t takes vec-wide loads at (j T + t) vec (layout 'strided') or the
    contiguous chunk t (layout 'chunk'); per-lane accumulators summed sequentially over j, combined
    over the vec lanes by vcomb, then over the threads by tcomb."""
    w = a.shape[-1]
    if w % (T * vec):
        return None
    J = w // (T * vec)
    if layout == "strided":
        r = a.reshape(a.shape[:-1] + (J, T, vec))              # [.., j, t, v]
        r = np.moveaxis(r, -3, -1)                             # [.., t, v, j]
    else:
        r = a.reshape(a.shape[:-1] + (T, J, vec))              # [.., t, j, v]
        r = np.swapaxes(r, -1, -2)                             # [.., t, v, j]
    acc = seq(r)                                               # [.., t, v]
    acc = {"seq": seq, "tree": tree}[vcomb](acc) if vec > 1 else acc[..., 0]
    return {"tree": tree, "halving": halving}[tcomb](acc)


def wide(dev, rng):
    res = {}
    for w in (128, 256, 512, 1024, 4096):
        a = rng.standard_normal((3, w)) * np.exp(rng.uniform(-20, 20, (3, w)))
        t = torch.tensor(a, device=dev).sum(dim=-1).cpu().numpy()
        ok = []
        for T in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512):
            for vec in (1, 2, 4):
                for vcomb in ("seq", "tree"):
                    for tcomb in ("tree", "halving"):
                        for layout in ("strided", "chunk"):
                            if vec == 1 and vcomb == "tree":
                                continue
                            r = threaded(a, T, vec, vcomb, tcomb, layout)
                            if r is not None and np.array_equal(r.view(np.int64), t.view(np.int64)):
                                ok.append(f"T{T}_v{vec}_{vcomb}_{tcomb}_{layout}")
        res[w] = ok
        print("wide", w, ok[:12], flush=True)
    return res


def main():
    dev = torch.device("cuda")
    rng = np.random.default_rng(0)
    out = {}
    for w in (4, 16, 64):
        for rows in (7, 64 * 37):
            a = rng.standard_normal((rows, w)) * np.exp(rng.uniform(-20, 20, (rows, w)))
            t = torch.tensor(a, device=dev).sum(dim=-1).cpu().numpy()
            cands = {"seq": seq(a), "tree": tree(a)}
            for k in (2, 4, 8):
                for comb in ("seq", "tree"):
                    r = strided(a, k, comb)
                    if r is not None:
                        cands[f"strided{k}_{comb}"] = r
            match = [n for n, r in cands.items() if np.array_equal(r.view(np.int64), t.view(np.int64))]
            # also through the gather the solver uses: ext[..., table].sum(-1) on a 3-D tensor
            B = 64
            src = rng.standard_normal((B, rows * w // B + 1)) if rows * w >= B else rng.standard_normal((B, w))
            table = rng.integers(0, src.shape[1], (max(1, rows // B), w))
            g = torch.tensor(src, device=dev)[:, torch.tensor(table, device=dev)].sum(-1).cpu().numpy()
            ga = src[:, table]
            gm = [n for n, f in (("seq", seq), ("tree", tree)) if np.array_equal(f(ga).view(np.int64), g.view(np.int64))]
            for k in (2, 4, 8):
                for comb in ("seq", "tree"):
                    r = strided(ga, k, comb)
                    if r is not None and np.array_equal(r.view(np.int64), g.view(np.int64)):
                        gm.append(f"strided{k}_{comb}")
            out[f"w{w}_rows{rows}"] = {"match_2d": match, "match_gather_3d": gm}
            print(w, rows, match, gm, flush=True)
    out["wide"] = wide(dev, rng)
    json.dump(out, open("gpurun_out/torch_sum_order.json", "w"), indent=1)


if __name__ == "__main__":
    main()
