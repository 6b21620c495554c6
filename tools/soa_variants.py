"""Time variants of libawegpu.so on the instance-minor evaluation path, one subprocess each (the
bench's AP2 block: B = 2048 instances of N=40 d=4, J_g instance-minor; HIP-event times of the
input transpose, the node kernels, the interval kernel and the finalize kernel; output checksums so
that variants which change the arithmetic show up).

usage: python tools/soa_variants.py lib1.so lib2.so[:VAR=VAL,VAR2=VAL2] ...
(an optional suffix sets environment variables for that variant's subprocess)
"""
import os
import json
import subprocess
import sys

CHILD = r'''
import sys, json, numpy as np, torch
sys.path.insert(0, ".")
from awebox_amd import evaluator as E, problem as pb
from awebox_amd.initial_guess import batch_member, initial_guess
E._LIB = None
lib = E.load_library(sys.argv[1])
B = 2048
consts = pb.build_constants(); lay = pb.NlpLayout(40, 4); v0 = initial_guess(consts, lay)
V = torch.tensor(np.stack([batch_member(v0, lay, b) for b in range(B)]), device="cuda")
P = torch.tensor(np.stack([pb.pack_p(lay, consts, v0, u_ref=5.0 + 3.0 * b / B) for b in range(B)]), device="cuda")
ev = E.Ap2Evaluator(consts, batch=B)
assert ev._lib is lib, "variant library not in use"
assert ev.path == "soa", ev.path
f = torch.empty(B, dtype=torch.float64, device="cuda"); g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
gr = ev.alloc_grad("cuda"); jac = ev.alloc_jac("cuda")
ks = []
for i in range(25):
    ev.eval_nlp_device(V, P, f, g, gr, jac)
    if i >= 5: ks.append(ev.last_kernel_ms_soa())
torch.cuda.synchronize()
ks = np.median(np.array(ks), axis=0)
tot = float(ks[:4].sum())
print(json.dumps({"lib": sys.argv[1], "total_ms": tot, "evals_per_s": B / tot * 1e3,
                  "in_ms": float(ks[0]), "node_ms": float(ks[1]), "interval_ms": float(ks[2]), "finalize_ms": float(ks[3]),
                  "jac_sum": float(jac.sum()), "g_sum": float(g.sum()), "grad_sum": float(gr.sum()), "f_sum": float(f.sum())}))
'''

if __name__ == "__main__":
    for rep in range(2):
        for spec in sys.argv[1:]:
            lib, _, envs = spec.partition(":")
            env = dict(os.environ)
            for kv in filter(None, envs.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            r = subprocess.run([sys.executable, "-c", CHILD, lib], capture_output=True, text=True, timeout=240, env=env)
            out = r.stdout.strip()
            print((out[:-1] + f', "variant": "{spec}"}}') if out.endswith("}") else
                  json.dumps({"lib": spec, "error": r.stderr[-800:]}), flush=True)
