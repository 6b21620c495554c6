"""Extract the reference's parameter tree (P['theta0', ...]) for the AP2 trajectory example into
tests/golden/reference_params.json -- the names, values and defining file:line of every entry,
read from the reference's source *as text* (Python's ast; no reference module is imported or run:
they all import casadi, which is absent).

Sources, in the order the reference applies them:

* ``awebox/opts/default.py``: the option tuples ``('params', a, b, name, value, ...)``;
* ``awebox/opts/model_funcs.py``: entries appended as ``options_tree.append(('params', a, b, name,
  ...))`` (values computed there are taken from the option they copy, e.g. wind.u_ref);
  geometry (``build_geometry_options``, :87-97: every kite-data geometry entry whose overwrite
  option is flagged 's' in default.py:148-164) and the stability derivatives
  (``:470-493``: ``('params', 'aero', coeff, input)`` for every derivative of the kite data);
* ``awebox/opts/kite_data/ampyx_data.py``: ``geometry()`` and ``aero()`` assignments;
* ``awebox/opts/kite_data/ampyx_ap2_settings.py`` and ``examples/ampyx_ap2_trajectory.py``:
  ``options['params.a.b'] = value`` overrides (and ``user_options.wind.u_ref``, which
  model_funcs.py:927 copies into params.wind.u_ref).

Expressions are evaluated by a small literal evaluator (numbers, lists, ``np.array``,
``np.zeros``, ``np.pi``, arithmetic, and the dict entries already assigned); anything else is
recorded with value null.  Run from the repository root (needs /root/reference):

    python tests/golden/make_reference_params.py
"""
import ast
import json
import math
import os

import numpy as np

REF = os.environ.get("AWEBOX_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "reference_params.json")


class _Eval:
    """Evaluate a literal-arithmetic expression; raise ValueError for anything else."""

    def __init__(self, names=None):
        self.names = names or {}

    def __call__(self, node):
        m = getattr(self, "_" + type(node).__name__, None)
        if m is None:
            raise ValueError(type(node).__name__)
        return m(node)

    def _Constant(self, n):
        return n.value

    def _List(self, n):
        return [self(e) for e in n.elts]

    _Tuple = _List

    def _UnaryOp(self, n):
        v = self(n.operand)
        if isinstance(n.op, ast.USub):
            return -np.asarray(v) if isinstance(v, (list, np.ndarray)) else -v
        if isinstance(n.op, ast.UAdd):
            return v
        raise ValueError("unary")

    def _BinOp(self, n):
        a, b = self(n.left), self(n.right)
        a = np.asarray(a) if isinstance(a, list) else a
        b = np.asarray(b) if isinstance(b, list) else b
        ops = {ast.Add: lambda x, y: x + y, ast.Sub: lambda x, y: x - y, ast.Mult: lambda x, y: x * y,
               ast.Div: lambda x, y: x / y, ast.Pow: lambda x, y: x ** y}
        for k, f in ops.items():
            if isinstance(n.op, k):
                return f(a, b)
        raise ValueError("binop")

    def _Attribute(self, n):
        if isinstance(n.value, ast.Name) and n.value.id in ("np", "ca", "cas") and n.attr == "pi":
            return math.pi
        if isinstance(n.value, ast.Name) and n.value.id in ("ca", "cas") and n.attr == "inf":
            return math.inf
        raise ValueError("attribute")

    def _Call(self, n):
        f = n.func
        if isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name) and f.value.id == "np":
            args = [self(a) for a in n.args]
            if f.attr == "array":
                return np.asarray(args[0], dtype=np.float64)
            if f.attr == "zeros":
                return np.zeros(args[0])
        raise ValueError("call")

    def _Subscript(self, n):
        if isinstance(n.value, ast.Name) and n.value.id in self.names:
            key = self(n.slice)
            return self.names[n.value.id][key]
        raise ValueError("subscript")

    def _Name(self, n):
        if n.id in self.names:
            return self.names[n.id]
        raise ValueError("name " + n.id)


def _val(node, ev=None):
    try:
        v = (ev or _Eval())(node)
    except (ValueError, KeyError, TypeError):
        return None
    if isinstance(v, (bool, str)) or v is None:
        return None
    return np.asarray(v, dtype=np.float64).ravel().tolist()


def _rel(path):
    return os.path.relpath(path, REF)


def default_params():
    """('params', a, b, name, value, ...) tuples of default.py -> {theta0 path: (value, source)}."""
    fn = os.path.join(REF, "awebox/opts/default.py")
    tree = ast.parse(open(fn).read())
    out = {}
    geometry_s = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Tuple) and len(node.elts) >= 5 and isinstance(node.elts[0], ast.Constant):
            head = [e.value if isinstance(e, ast.Constant) else "?" for e in node.elts[:4]]
            if head[0] == "params":
                path = ("theta0",) + tuple(x for x in head[1:4] if x is not None)
                out[path] = (_val(node.elts[4]), f"{_rel(fn)}:{node.lineno}")
            if head[:3] == ["model", "geometry", "overwrite"] and isinstance(node.elts[-1], ast.Constant) \
                    and node.elts[-1].value == "s":
                geometry_s.append((head[3], node.lineno))
    return out, geometry_s


def model_funcs_params():
    """options_tree.append(('params', a, b, name, ...)) sites of model_funcs.py."""
    fn = os.path.join(REF, "awebox/opts/model_funcs.py")
    tree = ast.parse(open(fn).read())
    out = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute) and node.func.attr == "append" \
                and node.args and isinstance(node.args[0], ast.Tuple):
            elts = node.args[0].elts
            if elts and isinstance(elts[0], ast.Constant) and elts[0].value == "params":
                head = [e.value if isinstance(e, ast.Constant) else "?" for e in elts[1:4]]
                if "?" not in head:
                    out[("theta0",) + tuple(x for x in head if x is not None)] = f"{_rel(fn)}:{node.lineno}"
    return out


def kite_data():
    """geometry() and aero() of ampyx_data.py: {name: value}, {coeff: {input: values}} with lines."""
    fn = os.path.join(REF, "awebox/opts/kite_data/ampyx_data.py")
    tree = ast.parse(open(fn).read())
    funcs = {n.name: n for n in tree.body if isinstance(n, ast.FunctionDef)}
    geometry, geo_line = {}, {}
    ev = _Eval({"geometry": geometry})
    for st in funcs["geometry"].body:
        if isinstance(st, ast.Assign) and isinstance(st.targets[0], ast.Subscript):
            key = st.targets[0].slice.value
            try:
                geometry[key] = ev(st.value)
            except (ValueError, KeyError, TypeError):
                geometry[key] = None
            geo_line[key] = f"{_rel(fn)}:{st.lineno}"
    derivs = {}
    for st in funcs["aero"].body:
        if isinstance(st, ast.Assign) and isinstance(st.targets[0], ast.Subscript):
            t = st.targets[0]
            if isinstance(t.value, ast.Subscript) and isinstance(t.value.value, ast.Name) \
                    and t.value.value.id == "stab_derivs":
                coeff, inp = t.value.slice.value, t.slice.value
                if coeff != "frame":
                    derivs.setdefault(coeff, {})[inp] = (_val(st.value), f"{_rel(fn)}:{st.lineno}")
    return geometry, geo_line, derivs


def option_overrides(relpath):
    """options['params.a.b'] = value and options['user_options.wind.u_ref'] = value assignments."""
    fn = os.path.join(REF, relpath)
    tree = ast.parse(open(fn).read())
    out = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.Assign) and isinstance(node.targets[0], ast.Subscript):
            t = node.targets[0]
            if isinstance(t.value, ast.Name) and t.value.id == "options" and isinstance(t.slice, ast.Constant):
                key = t.slice.value
                if isinstance(key, str) and (key.startswith("params.") or key == "user_options.wind.u_ref"):
                    out[key] = (_val(node.value), f"{relpath}:{node.lineno}")
    return out


def main():
    entries = {}
    defaults, geometry_s = default_params()
    for path, (v, src) in defaults.items():
        entries[path] = {"value": v, "source": src}
    appended = model_funcs_params()
    for path, src in appended.items():
        entries.setdefault(path, {"value": None, "source": src})
    geometry, geo_line, derivs = kite_data()
    mf = "awebox/opts/model_funcs.py"
    for name, line in geometry_s:
        if name in geometry:
            v = geometry[name]
            entries[("theta0", "geometry", name)] = {
                "value": None if v is None else np.asarray(v, dtype=np.float64).ravel().tolist(),
                "source": f"{geo_line[name]} via {mf}:87-97 (default.py:{line} flag 's')"}
    for coeff, d in derivs.items():
        for inp, (v, src) in d.items():
            entries[("theta0", "aero", coeff, inp)] = {"value": v, "source": f"{src} via {mf}:470-493"}
    for rel in ("awebox/opts/kite_data/ampyx_ap2_settings.py", "examples/ampyx_ap2_trajectory.py"):
        for key, (v, src) in option_overrides(rel).items():
            if key == "user_options.wind.u_ref":
                path = ("theta0", "wind", "u_ref")
                src = f"{src} via {appended.get(path, mf)}"
            else:
                path = ("theta0",) + tuple(key.split(".")[1:])
            entries[path] = {"value": v, "source": src}
    rows = [{"path": list(p), **e} for p, e in sorted(entries.items(), key=lambda kv: kv[0])]
    with open(OUT, "w") as fh:
        json.dump({"reference": "rcleuthold/awebox (read as text)", "config": "examples/ampyx_ap2_trajectory.py",
                   "entries": rows}, fh, indent=1)
    print(f"{len(rows)} theta0 entries -> {OUT}")


if __name__ == "__main__":
    main()
