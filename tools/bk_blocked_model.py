"""Host model of sym_inertia_blocked_kernel's algorithm (batched_lu.hip), for checking the delayed-
update Bunch-Kaufman logic on the CPU before it runs on the GPU: the same storage (the lower
triangle kept column-major, i.e. in the upper triangle of the row-major array), the same panel
bookkeeping (W = L D columns, the L coefficients of each column, the symmetric interchanges applied
to the un-updated trailing matrix) and the same decisions; the counts are compared with eigenvalue
counts.  Not used by the product or the tests."""
import numpy as np

ALPHA = (1.0 + np.sqrt(17.0)) / 8.0


def inertia_blocked(A0, ztol=1e-13, nb=16):
    n = A0.shape[0]
    M = np.array(A0, dtype=np.float64).copy()
    for c in range(n):                       # lower triangle into the upper storage
        M[c, c + 1:] = M[c + 1:, c]
    amax = np.abs(np.tril(A0)).max()
    zlim = ztol * amax
    W = np.zeros((nb, n))
    ca = np.zeros(nb); cb = np.zeros(nb); cp = np.zeros(nb, dtype=int)
    pos = neg = zero = 0

    def Lrow(s, j):
        return np.array([ca[c] * W[c, s] + cb[c] * W[cp[c], s] for c in range(j)])

    def gather_k(k, j, slot):               # column k of the current Schur complement, rows >= k
        Lk = Lrow(k, j)
        W[slot, k:] = M[k, k:] - (W[:j, k:].T @ Lk if j else 0.0)

    def gather_imax(im, k, j, slot):
        Li = Lrow(im, j)
        col = np.empty(n - k)
        col[im - k:] = M[im, im:]            # rows >= imax: column imax (contiguous)
        col[:im - k] = M[k:im, im]           # rows k..imax-1: row imax of the lower triangle
        W[slot, k:] = col - (W[:j, k:].T @ Li if j else 0.0)

    k = 0
    while k < n:
        j = 0
        while k < n and j < nb - 1:
            gather_k(k, j, j)
            absakk = abs(W[j, k])
            if k + 1 < n:
                v = np.abs(W[j, k + 1:])
                imax = k + 1 + int(np.argmax(v))
                colmax = v.max()
            else:
                imax, colmax = k, 0.0
            if max(absakk, colmax) <= zlim:
                zero += 1
                k += 1
                continue
            kp, kstep = k, 1
            if absakk < ALPHA * colmax:
                gather_imax(imax, k, j, j + 1)
                v = np.abs(W[j + 1, k:]).copy()
                v[imax - k] = -1.0
                rowmax = v.max()
                if absakk >= ALPHA * colmax * (colmax / rowmax):
                    kp = k
                elif abs(W[j + 1, imax]) >= ALPHA * rowmax:
                    kp = imax
                else:
                    kp, kstep = imax, 2
            kk = k + kstep - 1
            if kp != kk:
                # symmetric interchange kk <-> kp of the un-updated matrix (lower triangle, stored
                # at M[col, row])
                t = M[kk, kp + 1:].copy(); M[kk, kp + 1:] = M[kp, kp + 1:]; M[kp, kp + 1:] = t
                for jj in range(kk + 1, kp):
                    t = M[kk, jj]; M[kk, jj] = M[jj, kp]; M[jj, kp] = t
                t = M[kk, kk]; M[kk, kk] = M[kp, kp]; M[kp, kp] = t
                if kstep == 2:
                    t = M[k, k + 1]; M[k, k + 1] = M[k, kp]; M[k, kp] = t
                for c in range(j):
                    t = W[c, kk]; W[c, kk] = W[c, kp]; W[c, kp] = t
                if kstep == 1:
                    W[j, k:] = W[j + 1, k:]
                    t = W[j, k]; W[j, k] = W[j, kp]; W[j, kp] = t
                else:
                    for s in (j, j + 1):
                        t = W[s, kk]; W[s, kk] = W[s, kp]; W[s, kp] = t
            if kstep == 1:
                d = W[j, k]
                if d > 0: pos += 1
                elif d < 0: neg += 1
                else: zero += 1
                ca[j], cb[j], cp[j] = 1.0 / d, 0.0, j
            else:
                d11, d21, d22 = W[j, k], W[j, k + 1], W[j + 1, k + 1]
                det = d11 * d22 - d21 * d21
                if det < 0: pos += 1; neg += 1
                elif det > 0:
                    if d11 + d22 > 0: pos += 2
                    else: neg += 2
                else:
                    zero += 1
                    tr = d11 + d22
                    if tr > 0: pos += 1
                    elif tr < 0: neg += 1
                    else: zero += 1
                ca[j], cb[j], cp[j] = d22 / det, -d21 / det, j + 1
                ca[j + 1], cb[j + 1], cp[j + 1] = d11 / det, -d21 / det, j
            j += kstep
            k += kstep
        if k < n and j > 0:                  # trailing update of columns s >= k, rows r >= s
            for s in range(k, n):
                Ls = Lrow(s, j)
                M[s, s:] -= W[:j, s:].T @ Ls
    return pos, neg, zero


def eig_counts(A, ztol=1e-13):
    ev = np.linalg.eigvalsh(A)
    s = np.abs(A).max()
    p = int((ev > ztol * s).sum()); m = int((ev < -ztol * s).sum())
    return p, m, len(ev) - p - m


def kkt(rng, nx, nc, zero_diag=0.3):
    H = rng.standard_normal((nx, nx)); H = H + H.T
    H[np.diag_indices(nx)] += rng.uniform(0, 3, nx)
    Aj = rng.standard_normal((nc, nx))
    Aj[rng.random((nc, nx)) < 0.7] = 0.0
    K = np.zeros((nx + nc, nx + nc))
    K[:nx, :nx] = H; K[nx:, :nx] = Aj; K[:nx, nx:] = Aj.T
    K[nx:, nx:] = -1e-9 * np.eye(nc)
    p = rng.permutation(nx + nc)
    return K[np.ix_(p, p)]


if __name__ == "__main__":
    rng = np.random.default_rng(0)
    bad = 0
    for trial in range(60):
        nx, nc = int(rng.integers(3, 60)), int(rng.integers(1, 40))
        nc = min(nc, nx)
        K = kkt(rng, nx, nc)
        nb = int(rng.choice([4, 5, 8, 16]))
        got = inertia_blocked(K, nb=nb)
        want = eig_counts(K)
        if got != want:
            bad += 1
            print("MISMATCH", trial, nx, nc, nb, got, want)
    for trial in range(20):                  # plain indefinite and singular matrices
        n = int(rng.integers(2, 50))
        A = rng.standard_normal((n, n)); A = A + A.T
        if trial % 3 == 0:
            r = max(1, n // 2)
            B = rng.standard_normal((n, r)); A = B @ np.diag(rng.choice([-1.0, 1.0], r)) @ B.T
        got = inertia_blocked(A, nb=int(rng.choice([4, 16])))
        want = eig_counts(A, ztol=1e-10)
        got2 = inertia_blocked(A, ztol=1e-10, nb=8)
        if got2 != want:
            bad += 1
            print("MISMATCH plain", trial, n, got2, want)
    print("mismatches:", bad)
