"""Collocation coefficients for the awebox direct-collocation transcription.

Restates ``awebox/ocp/collocation.py:67-200`` (``Collocation.__poly_coeffs`` and
``Collocation.__quadrature_weights``) without CasADi:

* ``tau_root = [0, collocation_points(d, scheme)]`` (``collocation.py:76``).  CasADi's
  ``collocation_points`` returns the Radau IIA / Gauss-Legendre nodes; they are computed
  here from their defining polynomials in exact arithmetic (sympy) and rounded to fp64,
  so the right Radau end point is exactly ``1.0``.
* ``C[j, r] = l_j'(tau_r)`` (``coeff_collocation``, ``collocation.py:113-115``)
* ``D[j] = l_j(1)`` (``coeff_continuity``, ``collocation.py:108``)
* ``w = C[1:, 1:]^{-1} D[1:]`` (``quad_weights``, ``collocation.py:185-200``)
"""
from __future__ import annotations

import functools

import numpy as np


@functools.lru_cache(maxsize=None)
def collocation_points(d: int, scheme: str = "radau") -> tuple:
    import sympy as sp

    x = sp.Symbol("x")
    if scheme == "radau":
        # Radau IIA nodes on (0, 1]: roots of P_d(2t-1) - P_{d-1}(2t-1)
        poly = sp.legendre(d, 2 * x - 1) - sp.legendre(d - 1, 2 * x - 1)
    elif scheme == "legendre":
        poly = sp.legendre(d, 2 * x - 1)
    else:
        raise ValueError(f"unknown collocation scheme {scheme!r}")
    roots = sp.Poly(sp.expand(poly), x).nroots(n=40, maxsteps=200)
    vals = sorted(float(sp.re(r)) for r in roots)
    if scheme == "radau":
        vals[-1] = 1.0
    return tuple(vals)


@functools.lru_cache(maxsize=None)
def coefficients(d: int, scheme: str = "radau"):
    """Return (tau_root[d+1], C[d+1, d+1], D[d+1], w[d]) as float64 numpy arrays."""
    tau = np.array((0.0,) + collocation_points(d, scheme), dtype=np.float64)
    n = d + 1
    C = np.zeros((n, n))
    D = np.zeros(n)
    for j in range(n):
        # l_j(t) = prod_{r != j} (t - tau_r) / (tau_j - tau_r)   (collocation.py:99-102)
        others = [r for r in range(n) if r != j]
        val = 1.0
        for r in others:
            val *= (1.0 - tau[r]) / (tau[j] - tau[r])
        D[j] = val
        # derivative by the product rule, evaluated at every node
        for m in range(n):
            t = tau[m]
            deriv = 0.0
            for skip in others:
                term = 1.0 / (tau[j] - tau[skip])
                for r in others:
                    if r != skip:
                        term *= (t - tau[r]) / (tau[j] - tau[r])
                deriv += term
            C[j, m] = deriv
    w = np.linalg.solve(C[1:, 1:], D[1:])
    return tau, C, D, w
