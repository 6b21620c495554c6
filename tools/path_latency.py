"""Per-call time of the evaluation paths at small and large batches (HIP events; the solver's
shapes: B = 1 single solves, 8-16 sweep shards, and the bench's 2048), J_g and grad f in the
solver's instance-minor layout.

    python tools/path_latency.py [B ...]
"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from awebox_amd import evaluator as E, problem as pb  # noqa: E402
from awebox_amd.initial_guess import batch_member, initial_guess  # noqa: E402


def main():
    Bs = [int(x) for x in sys.argv[1:]] or [1, 8, 16, 32, 64, 128, 256, 2048]
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    for B in Bs:
        V = torch.tensor(np.stack([batch_member(v0, lay, b) for b in range(B)]), device="cuda")
        P = torch.tensor(np.stack([pb.pack_p(lay, consts, v0)] * B), device="cuda")
        ev = E.Ap2Evaluator(consts, batch=B)
        f = torch.empty(B, dtype=torch.float64, device="cuda")
        g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
        gr, jac = ev.alloc_grad("cuda"), ev.alloc_jac("cuda")
        out = {"B": B}
        for path in ("soa", "generated", "colour"):
            ev.path = path
            ms = []
            for i in range(30):
                ev.eval_nlp_device(V, P, f, g, gr, jac)
                a, b_ = ev.last_kernel_ms()
                if i >= 5:
                    ms.append(a + b_)
            torch.cuda.synchronize()
            out[path + "_ms"] = float(np.median(ms))
        print(json.dumps(out), flush=True)
        del ev


if __name__ == "__main__":
    main()
