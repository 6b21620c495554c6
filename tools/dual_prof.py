"""In-process timing of libawedual.so (for rocprofv3 runs: no child processes).

usage: python tools/dual_prof.py [--batch B] [--iters N] [lib.so]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from awebox_amd import dual as du  # noqa: E402
from awebox_amd import dual_evaluator as de  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("lib", nargs="?", default=None)
a = ap.parse_args()
if a.lib:
    de.load_library(a.lib)
c = du.build_constants()
lay = du.layout_for(c)
v0 = du.initial_guess(c, lay)
B = a.batch
ev = de.DualEvaluator(c, batch=B)
V = torch.tensor(np.stack([du.batch_member(v0, lay, b) for b in range(B)]), device="cuda")
P = torch.tensor(np.stack([du.pack_p(lay, c, v0)] * B), device="cuda")
f = torch.empty(B, dtype=torch.float64, device="cuda")
g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
gr = torch.empty(B, ev.n_v, dtype=torch.float64, device="cuda")
jac = torch.empty(B, ev.nnz, dtype=torch.float64, device="cuda")
ks = []
for i in range(a.iters):
    ev.eval_nlp_device(V, P, f, g, gr, jac)
    ks.append(ev.last_kernel_ms()[0])
torch.cuda.synchronize()
print(json.dumps({"lib": a.lib or de._LIB_PATH, "batch": B, "kernel_ms": float(np.median(ks)),
                  "jac_sum": float(jac.sum())}))
