"""Drop-in for ``casadi.nlpsol``'s NLP functions -- active only where ``import casadi`` works.

In the reference the NLP handed to IPOPT is ``{'x': V, 'p': P, 'f': f_fun(V, P), 'g': g_fun(V, P)}``
(awebox/opti/preparation.py:366-400) and CasADi generates nlp_f / nlp_g / nlp_grad_f / nlp_jac_g /
nlp_hess_l from the expanded SX graph.  Here ``f`` and ``g`` are ``casadi.Callback`` objects backed
by the HIP evaluator, following the in-tree Callback idiom (awebox/tools/callback.py:31-60:
get_n_in / get_sparsity_in / eval):

* f and g values come from the value-only kernel (``awe_eval_f_host`` / ``awe_eval_g_host``: the
  model in plain double, no derivatives) -- IPOPT's line-search trials;
* ``has_jacobian`` / ``get_jacobian`` make CasADi ask the evaluator for grad f and J_g (the fused
  derivative kernel, J_g in its fixed CCS pattern) instead of differentiating;
* the exact Hessian of the Lagrangian (IPOPT's default, awebox/opts/default.py:323 and
  preparation.py:272-273) comes from the hyper-dual Hessian kernel through the ``hess_lag``
  option of nlpsol: a Callback (x, p, lam_f, lam_g) -> upper triangle of sigma f + lam^T g.

The reference's P struct is fed unchanged: ``make_nlp`` takes the reference's P *layout* through
``p_from_reference`` -- by default problem.pack_p_from_reference, which reads the struct entry by
entry by name (discretization.py:168-179) -- so ``solver(x0=..., p=p_fix_num, ...)`` at
optimization.py:363 keeps working.

Use (inside awebox.opti.preparation, in place of the MX expressions):

    from awebox_amd.casadi_bridge import make_nlp, solver_options
    nlp = make_nlp(evaluator, P_struct=nlp.P)       # {'x','p','f','g'} built from Callbacks
    solver = cas.nlpsol('solver', 'ipopt', nlp, {**opts, **solver_options(nlp)})
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


def p_packer_for(layout):
    """The by-name reader of the reference's parameter struct for an evaluator's layout: the
    periodic-OCP P (AP2 ``NlpLayout`` and multi-kite ``MultiLayout``: problem.pack_p_from_reference)
    or Pmpc's p (``MpcLayout``: kite3.pack_p_from_reference)."""
    from . import kite3 as k3
    from . import problem as pb
    if isinstance(layout, k3.MpcLayout):
        return k3.pack_p_from_reference
    return pb.pack_p_from_reference


def reference_p_reader(P_struct):
    """A function turning the reference's numeric P (a DM of P_struct's size) into this library's
    flat P, reading P_struct's entries by name (p_packer_for the evaluator's layout)."""

    def convert(p_num, layout):
        s = P_struct(p_num)

        def get(path):
            try:
                return np.asarray(s[path]).ravel()
            except Exception as exc:                           # missing entry name in the struct
                raise KeyError(path) from exc
        return p_packer_for(layout)(get, layout)
    return convert


def make_nlp(evaluator, P_struct=None):
    """Return {'x': V, 'p': P, 'f': f(V,P), 'g': g(V,P)} with MX symbols and Callback outputs.
    With ``P_struct`` (the reference's casadi.tools P struct) the p input has the reference's size
    and is converted by name on every call; without it, p is this library's flat P."""
    _require()
    n_v = evaluator.n_v
    convert = None
    n_p = evaluator.n_p
    if P_struct is not None:
        convert = reference_p_reader(P_struct)
        n_p = P_struct.size
    V = cas.MX.sym("V", n_v)
    P = cas.MX.sym("P", n_p)
    F = _FCallback("awe_f", evaluator, convert, n_p)
    G = _GCallback("awe_g", evaluator, convert, n_p)
    nlp = {"x": V, "p": P, "f": F(V, P), "g": G(V, P)}
    nlp["_callbacks"] = [F, G]  # callbacks must outlive the solver
    if hasattr(evaluator, "eval_hess"):
        H = _HessCallback("awe_hess_l", evaluator, convert, n_p)
        nlp["_callbacks"].append(H)
        nlp["_hess_lag"] = H
    return nlp


def solver_options(nlp):
    """nlpsol options that keep IPOPT's exact Hessian with the HIP Hessian kernel (evaluators
    without a Hessian kernel leave the Hessian to CasADi's default)."""
    if "_hess_lag" not in nlp:
        return {"expand": False}
    return {"hess_lag": nlp["_hess_lag"], "expand": False}


if cas is not None:  # pragma: no cover - exercised only where casadi is installed

    class _Base(cas.Callback):
        def __init__(self, name, ev, convert, n_p, opts=None):
            cas.Callback.__init__(self)
            self.ev, self.convert, self.n_p = ev, convert, n_p
            self.construct(name, opts or {})

        def get_n_in(self):
            return 2

        def get_sparsity_in(self, i):
            return cas.Sparsity.dense(self.ev.n_v if i == 0 else self.n_p)

        def _xp(self, arg):
            x = np.asarray(arg[0]).reshape(1, -1)
            p = np.asarray(arg[1]).reshape(-1)
            if self.convert is not None:
                p = self.convert(p, self.ev.layout)
            return x, p.reshape(1, -1)

        def _call(self, arg):
            return self.ev.eval_nlp(*self._xp(arg))

    class _GCallback(_Base):
        def get_n_out(self):
            return 1

        def get_sparsity_out(self, i):
            return cas.Sparsity.dense(self.ev.n_g)

        def eval(self, arg):
            return [self.ev.eval_g(*self._xp(arg))[0]]

        def has_jacobian(self):
            return True

        def get_jacobian(self, name, inames, onames, opts):
            self._jac = _JacGCallback(name, self.ev, self.convert, self.n_p, opts)
            return self._jac

    class _JacGCallback(_Base):
        # inputs: x, p, g (nominal output); outputs: d g/d x (CCS), d g/d p (not needed by IPOPT)
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
            return cas.Sparsity(self.ev.n_g, self.n_p)

        def eval(self, arg):
            out = self._call(arg)
            colind, row = self.ev.sparsity_jac()
            J = cas.DM(cas.Sparsity(self.ev.n_g, self.ev.n_v, colind.tolist(), row.tolist()), out["jac"][0])
            return [J, cas.DM(cas.Sparsity(self.ev.n_g, self.n_p))]

    class _FCallback(_Base):
        def get_n_out(self):
            return 1

        def get_sparsity_out(self, i):
            return cas.Sparsity.dense(1)

        def eval(self, arg):
            return [self.ev.eval_f(*self._xp(arg))[0]]

        def has_jacobian(self):
            return True

        def get_jacobian(self, name, inames, onames, opts):
            self._jac = _GradFCallback(name, self.ev, self.convert, self.n_p, opts)
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
            return cas.Sparsity.dense(1, self.ev.n_v) if i == 0 else cas.Sparsity(1, self.n_p)

        def eval(self, arg):
            out = self._call(arg)
            return [cas.DM(out["grad_f"][0]).T, cas.DM(cas.Sparsity(1, self.n_p))]

    class _HessCallback(_Base):
        """nlp_hess_l: (x, p, lam_f, lam_g) -> upper triangle of lam_f f + lam_g^T g in the
        kernel's fixed CCS pattern (nlpsol's hess_lag option)."""

        def get_n_in(self):
            return 4

        def get_name_in(self, i):
            return ["x", "p", "lam_f", "lam_g"][i]

        def get_name_out(self, i):
            return "hess_gamma_x_x"

        def get_sparsity_in(self, i):
            if i == 2:
                return cas.Sparsity.dense(1)
            if i == 3:
                return cas.Sparsity.dense(self.ev.n_g)
            return _Base.get_sparsity_in(self, i)

        def get_n_out(self):
            return 1

        def get_sparsity_out(self, i):
            colind, row = self.ev.sparsity_hess()
            return cas.Sparsity(self.ev.n_v, self.ev.n_v, colind.tolist(), row.tolist())

        def eval(self, arg):
            x, p = self._xp(arg)
            lam_f = float(np.asarray(arg[2]).reshape(-1)[0])
            lam_g = np.asarray(arg[3]).reshape(1, -1)
            H = self.ev.eval_hess(x, p, lam_f, lam_g)[0]
            colind, row = self.ev.sparsity_hess()
            return [cas.DM(cas.Sparsity(self.ev.n_v, self.ev.n_v, colind.tolist(), row.tolist()), H)]
else:
    _FCallback = _GCallback = _HessCallback = None
