"""Drop-in for ``casadi.nlpsol``'s NLP functions -- active only where ``import casadi`` works.

In the reference the NLP handed to IPOPT is ``{'x': V, 'p': P, 'f': f_fun(V, P), 'g': g_fun(V, P)}``
(awebox/opti/preparation.py:366-400) and CasADi generates nlp_f / nlp_g / nlp_grad_f / nlp_jac_g
from the expanded SX graph.  Here ``f`` and ``g`` are ``casadi.Callback`` objects backed by the HIP
evaluator, following the in-tree Callback idiom (awebox/tools/callback.py:31-60:
get_n_in / get_sparsity_in / eval) plus ``has_jacobian`` / ``get_jacobian`` so that CasADi asks the
evaluator for J_g (in its fixed CCS pattern) and grad f instead of differentiating.

Use (inside awebox.opti.preparation, in place of the MX expressions):

    from awebox_amd.casadi_bridge import make_nlp
    nlp = make_nlp(evaluator)             # {'x','p','f','g'} built from Callbacks
    solver = cas.nlpsol('solver', 'ipopt', nlp, {**opts, 'expand': False,
                        'ipopt.hessian_approximation': 'limited-memory'})

The exact Hessian of the Lagrangian (default in awebox, default.py:323) is the next kernel
(DESIGN.md, row f1); until then IPOPT runs with L-BFGS through this bridge.
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - casadi is absent in this container
    import casadi as cas
except ImportError:  # pragma: no cover
    cas = None


def available() -> bool:
    return cas is not None


def _require():
    if cas is None:
        raise ImportError("casadi is not importable here; the bridge is only needed where IPOPT runs via CasADi")


def make_nlp(evaluator):
    """Return {'x': V, 'p': P, 'f': f(V,P), 'g': g(V,P)} with MX symbols and Callback outputs."""
    _require()
    n_v, n_p = evaluator.n_v, evaluator.n_p
    V = cas.MX.sym("V", n_v)
    P = cas.MX.sym("P", n_p)
    F = _FCallback("awe_f", evaluator)
    G = _GCallback("awe_g", evaluator)
    keep = [F, G]
    nlp = {"x": V, "p": P, "f": F(V, P), "g": G(V, P)}
    nlp["_callbacks"] = keep  # callbacks must outlive the solver
    return nlp


if cas is not None:  # pragma: no cover - exercised only where casadi is installed

    class _Base(cas.Callback):
        def __init__(self, name, ev, opts=None):
            cas.Callback.__init__(self)
            self.ev = ev
            self.construct(name, opts or {})

        def get_n_in(self):
            return 2

        def get_sparsity_in(self, i):
            return cas.Sparsity.dense(self.ev.n_v if i == 0 else self.ev.n_p)

        def _call(self, arg):
            x = np.asarray(arg[0]).reshape(-1)
            p = np.asarray(arg[1]).reshape(-1)
            return self.ev.eval_nlp(x.reshape(1, -1), p.reshape(1, -1))

    class _GCallback(_Base):
        def get_n_out(self):
            return 1

        def get_sparsity_out(self, i):
            return cas.Sparsity.dense(self.ev.n_g)

        def eval(self, arg):
            return [self._call(arg)["g"][0]]

        def has_jacobian(self):
            return True

        def get_jacobian(self, name, inames, onames, opts):
            self._jac = _JacGCallback(name, self.ev, opts)
            return self._jac

    class _JacGCallback(_Base):
        # inputs: x, p, g (nominal output); outputs: d g/d x (CCS), d g/d p (structurally zero)
        def get_n_in(self):
            return 3

        def get_sparsity_in(self, i):
            if i == 2:
                return cas.Sparsity.dense(self.ev.n_g)
            return _Base.get_sparsity_in(self, i)

        def get_n_out(self):
            return 2

        def get_sparsity_out(self, i):
            if i == 0:
                colind, row = self.ev.sparsity_jac()
                return cas.Sparsity(self.ev.n_g, self.ev.n_v, colind.tolist(), row.tolist())
            return cas.Sparsity(self.ev.n_g, self.ev.n_p)

        def eval(self, arg):
            out = self._call(arg)
            colind, row = self.ev.sparsity_jac()
            J = cas.DM(cas.Sparsity(self.ev.n_g, self.ev.n_v, colind.tolist(), row.tolist()), out["jac"][0])
            return [J, cas.DM(cas.Sparsity(self.ev.n_g, self.ev.n_p))]

    class _FCallback(_Base):
        def get_n_out(self):
            return 1

        def get_sparsity_out(self, i):
            return cas.Sparsity.dense(1)

        def eval(self, arg):
            return [self._call(arg)["f"][0]]

        def has_jacobian(self):
            return True

        def get_jacobian(self, name, inames, onames, opts):
            self._jac = _GradFCallback(name, self.ev, opts)
            return self._jac

    class _GradFCallback(_Base):
        def get_n_in(self):
            return 3

        def get_sparsity_in(self, i):
            if i == 2:
                return cas.Sparsity.dense(1)
            return _Base.get_sparsity_in(self, i)

        def get_n_out(self):
            return 2

        def get_sparsity_out(self, i):
            return cas.Sparsity.dense(1, self.ev.n_v) if i == 0 else cas.Sparsity(1, self.ev.n_p)

        def eval(self, arg):
            out = self._call(arg)
            return [cas.DM(out["grad_f"][0]).T, cas.DM(cas.Sparsity(1, self.ev.n_p))]
else:
    _FCallback = _GCallback = None
