"""The evaluation paths of awe_eval_nlp on MI355X return the same f, g, grad f and J_g:

* the instance-minor path (ap2_soa_shoot / ap2_soa_radau kernels, one lane per instance, tangents
  stored straight into J_g through the destination table; the default) agrees BITWISE with the
  node + gather path in g and J_g (the same generated node code), in both J_g layouts -- per
  instance (awe_eval_nlp) and instance-minor (awe_eval_nlp_im, the solver's layout) -- and to 1e-12
  in f and grad f (its interval kernel sums the objective per lane, the gather kernel across a
  wavefront);
* the node + gather path agrees with the colour path (compressed forward mode) to rounding.

At B = 128 (two full instance blocks; the instance-minor path is the default from here on), a
ragged batch (B = 70: a partial block, lanes past the batch idle) and B = 1 (the solver's
single-instance calls, where the colour path is the default).  Oracle parity of the
default path is tests/test_gpu_parity.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _close(a, b, rtol=1e-9):
    scale = np.max(np.abs(b))
    assert np.all(np.abs(a - b) <= rtol * np.abs(b) + 1e-11 * scale), float(np.max(np.abs(a - b)))


def _inputs(B):
    import torch

    from awebox_amd import problem as pb
    from awebox_amd.initial_guess import batch_member, initial_guess
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    V = torch.tensor(np.stack([batch_member(v0, lay, b) for b in range(B)]), device="cuda")
    P = torch.tensor(np.stack([pb.pack_p(lay, consts, v0, u_ref=5.0 + 0.05 * b) for b in range(B)]), device="cuda")
    return consts, V, P


def _eval(ev, V, P, path, instance_minor):
    import torch
    B = ev.batch
    ev.path = path
    f = torch.empty(B, dtype=torch.float64, device="cuda")
    g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
    gr = ev.alloc_grad("cuda", instance_minor=instance_minor)
    jac = ev.alloc_jac("cuda", instance_minor=instance_minor)
    jac.fill_(np.nan)
    gr.fill_(np.nan)
    ev.eval_nlp_device(V, P, f, g, gr, jac)
    torch.cuda.synchronize()
    return [x.cpu().numpy() for x in (f, g, gr, jac)]


@pytest.mark.parametrize("B", [128, 70, 1])
def test_instance_minor_path_is_default_and_matches_the_other_paths(B):
    from awebox_amd import evaluator as E
    consts, V, P = _inputs(B)
    ev = E.Ap2Evaluator(consts, batch=B)
    assert ev.path == ("soa" if B >= 128 else "colour")   # the default follows the batch size
    out = {"soa_im": _eval(ev, V, P, "soa", True)}
    ms = ev.last_kernel_ms_soa()
    assert ms[1] > 0 and ms[2] > 0 and ms[4] < 0.05          # no output transpose in the solver's layout
    out["soa_aos"] = _eval(ev, V, P, "soa", False)
    out["generated"] = _eval(ev, V, P, "generated", False)
    node_ms, asm_ms = ev.last_kernel_ms_gen()
    assert node_ms > 0 and asm_ms > 0
    out["colour"] = _eval(ev, V, P, "colour", False)
    labels = ("f", "g", "grad_f", "jac")
    diffs = {name: {lab: float(np.max(np.abs(a - b))) for lab, a, b in zip(labels, out[name], out["generated"])}
             for name in ("soa_im", "soa_aos", "colour")}
    print(diffs)
    for name in ("soa_im", "soa_aos"):
        for lab, a, b in zip(labels, out[name], out["generated"]):
            assert np.isfinite(a).all(), (name, lab)
            if lab in ("g", "jac"):
                assert np.array_equal(a, b), (name, lab, diffs[name])
            else:                # the objective's sums run per lane instead of across a wavefront
                for i in range(B):
                    _close(a[i], b[i], rtol=1e-12)
    for a, b in zip(out["generated"], out["colour"]):
        for i in range(B):
            _close(a[i], b[i])


@pytest.mark.parametrize("B", [70, 1])
def test_colour_and_generated_paths_in_the_solvers_layout(B):
    """awe_eval_nlp_im on the colour and the node + gather paths (per-instance evaluation into the
    handle's scratch, then transposed into the instance-minor J_g and grad f the solver allocates)
    equal the same path's per-instance layout bitwise, at a ragged batch and at B = 1."""
    from awebox_amd import evaluator as E
    consts, V, P = _inputs(B)
    ev = E.Ap2Evaluator(consts, batch=B)
    for path in ("colour", "generated"):
        im = _eval(ev, V, P, path, True)
        aos = _eval(ev, V, P, path, False)
        for lab, a, b in zip(("f", "g", "grad_f", "jac"), im, aos):
            assert np.isfinite(a).all(), (path, lab)
            assert np.array_equal(a, b), (path, lab, float(np.max(np.abs(a - b))))


@pytest.mark.parametrize("B", [130, 2])
def test_instance_minor_inputs_give_the_same_bits(B):
    """awe_eval_nlp_imv (V and P handed over instance-minor, Ap2Evaluator.alloc_inputs) against
    awe_eval_nlp_im on the same values in the per-instance layout: the same kernels after the input
    transposition, so f, g, grad f and J_g are bitwise equal (B = 130: two full instance blocks and a
    partial one)."""
    import torch
    from awebox_amd import evaluator as E
    consts, V, P = _inputs(B)
    ev = E.Ap2Evaluator(consts, batch=B)
    ref = _eval(ev, V, P, "soa", True)
    VT, PT = ev.alloc_inputs("cuda")
    VT.copy_(V)
    PT.copy_(P)
    assert VT.stride() == (1, ev.instance_ld) and torch.equal(VT, V)
    got = _eval(ev, VT, PT, "soa", True)
    for a, b in zip(ref, got):
        assert np.array_equal(a, b, equal_nan=True)
    with pytest.raises(RuntimeError):
        _eval(ev, VT, PT, "colour", True)                       # instance-minor inputs: SOA path only
