"""Short driver for PMC passes over the config-3 and config-5 evaluators (no solver, no sweep):
5 batched evaluations of the dual-kite NLP (B=128) and of the tracking-MPC NLP (B=256), on the
paths and layouts the bench measures (the generated instance-minor paths).

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_cfg_fetch -o run --output-format csv -- python tools/pmc_kernels.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ap2(B=2048):
    """5 batched AP2 N=40 d=4 evaluations at the bench's batch (the headline kernel)."""
    import numpy as np
    import torch

    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.initial_guess import batch_member, initial_guess
    dev = torch.device("cuda:0")
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    V = torch.tensor(np.stack([batch_member(v0, lay, b) for b in range(B)]), device=dev)
    P = torch.tensor(np.stack([pb.pack_p(lay, consts, v0)] * B), device=dev)
    ev = Ap2Evaluator(consts, batch=B)
    if ev.path == "soa":                                    # the bench's call: V and P instance-minor
        VT, PT = ev.alloc_inputs(dev)
        VT.copy_(V)
        PT.copy_(P)
        V, P = VT, PT
    # J_g in the layout the bench and the solver use (instance-minor on the default path)
    out = [torch.empty(B, dtype=torch.float64, device=dev), torch.empty(B, ev.n_g, dtype=torch.float64, device=dev),
           ev.alloc_grad(dev), ev.alloc_jac(dev)]
    for _ in range(5):
        ev.eval_nlp_device(V, P, *out)
    torch.cuda.synchronize()
    print("pmc ap2 done", flush=True)


def hess(B=256):
    """5 batched AP2 N=40 d=4 nlp_hess_l evaluations (sigma = 1, lam ~ N(0,1) seed 7, as the bench)."""
    import numpy as np
    import torch

    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.initial_guess import batch_member, initial_guess
    dev = torch.device("cuda:0")
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    V = torch.tensor(np.stack([batch_member(v0, lay, b) for b in range(B)]), device=dev)
    P = torch.tensor(np.stack([pb.pack_p(lay, consts, v0)] * B), device=dev)
    ev = Ap2Evaluator(consts, batch=B)
    g = torch.Generator().manual_seed(7)
    lam = torch.randn(B, ev.n_g, generator=g, dtype=torch.float64).to(dev)
    sig = torch.ones(B, dtype=torch.float64, device=dev)
    H = torch.empty(B, ev.nnz_h, dtype=torch.float64, device=dev)
    for _ in range(5):
        ev.eval_hess_device(V, P, sig, lam, H)
    torch.cuda.synchronize()
    print("pmc hess done", float(ev.last_hess_ms()), flush=True)


def main():
    import numpy as np
    import torch
    if "--ap2" in sys.argv:
        return ap2()
    if "--hess" in sys.argv:
        return hess()
    # --dual / --mpc: one configuration per process (both generated paths start with the same
    # im::transpose_in_kernel, which the per-kernel summary must not mix)
    want = [w for w in ("dual", "mpc") if "--" + w in sys.argv] or ["dual", "mpc"]

    from awebox_amd import dual as du
    from awebox_amd import kite3 as k3
    from awebox_amd.dual_evaluator import DualEvaluator
    from awebox_amd.mpc import MpcEvaluator

    dev = torch.device("cuda:0")
    c = du.build_constants()
    lay = du.layout_for(c)
    v0 = du.initial_guess(c, lay)
    B = 128
    V = torch.tensor(np.stack([du.batch_member(v0, lay, b) for b in range(B)]), device=dev)
    P = torch.tensor(np.stack([du.pack_p(lay, c, v0)] * B), device=dev)
    ev = DualEvaluator(c, batch=B)
    # the bench's layout: instance-minor J_g / grad f on the generated path when it serves the handle
    gen = ev.generated_available
    out = [torch.empty(B, dtype=torch.float64, device=dev), torch.empty(B, ev.n_g, dtype=torch.float64, device=dev),
           ev.alloc_grad(dev, instance_minor=gen), ev.alloc_jac(dev, instance_minor=gen)]
    for _ in range(5 if "dual" in want else 0):
        ev.eval_nlp_device(V, P, *out)
    torch.cuda.synchronize()
    if "mpc" not in want:
        print("pmc_kernels done", flush=True)
        return
    c3 = k3.build_constants()
    lay3 = k3.MpcLayout(c3.cfg.n_k, c3.cfg.d)
    B = 256
    inst = [k3.batch_instance(c3, lay3, i, B) for i in range(B)]
    V = torch.tensor(np.stack([v for v, _ in inst]), device=dev)
    P = torch.tensor(np.stack([p for _, p in inst]), device=dev)
    ev3 = MpcEvaluator(c3, batch=B)
    out = [torch.empty(B, dtype=torch.float64, device=dev), torch.empty(B, ev3.n_g, dtype=torch.float64, device=dev),
           ev3.alloc_grad(dev), ev3.alloc_jac(dev)]
    for _ in range(5):
        ev3.eval_nlp_device(V, P, *out)
    torch.cuda.synchronize()
    print("pmc_kernels done", flush=True)


if __name__ == "__main__":
    main()
