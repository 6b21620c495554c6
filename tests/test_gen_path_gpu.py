"""The two evaluation paths of awe_eval_nlp on MI355X: the generated path (ap2_node_kernel with
build-time generated node-Jacobian code + ap2_assemble_kernel, the default) and the colour path
(compressed forward mode) return the same f, g, grad f and J_g to rounding, at the bench's shape."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _close(a, b, rtol=1e-9):
    scale = np.max(np.abs(b))
    assert np.all(np.abs(a - b) <= rtol * np.abs(b) + 1e-11 * scale), float(np.max(np.abs(a - b)))


def test_generated_path_is_default_and_matches_colour_path():
    import torch

    from awebox_amd import evaluator as E
    from awebox_amd import problem as pb
    from awebox_amd.initial_guess import batch_member, initial_guess
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    B = 64
    ev = E.Ap2Evaluator(consts, batch=B)
    assert ev.path == "generated"
    V = torch.tensor(np.stack([batch_member(v0, lay, b) for b in range(B)]), device="cuda")
    P = torch.tensor(np.stack([pb.pack_p(lay, consts, v0, u_ref=5.0 + 0.05 * b) for b in range(B)]), device="cuda")
    out = {}
    for path in ("generated", "colour"):
        ev.path = path
        f = torch.empty(B, dtype=torch.float64, device="cuda")
        g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
        gr = torch.empty(B, ev.n_v, dtype=torch.float64, device="cuda")
        jac = torch.empty(B, ev.nnz, dtype=torch.float64, device="cuda")
        ev.eval_nlp_device(V, P, f, g, gr, jac)
        torch.cuda.synchronize()
        out[path] = [x.cpu().numpy() for x in (f, g, gr, jac)]
        if path == "generated":
            node_ms, asm_ms = ev.last_kernel_ms_gen()
            assert node_ms > 0 and asm_ms > 0
    for a, b in zip(out["generated"], out["colour"]):
        for i in range(B):
            _close(a[i], b[i])
    ev.path = "generated"
