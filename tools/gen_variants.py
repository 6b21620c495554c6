"""Time the two evaluation paths of libawegpu.so variants on the GPU and check that they agree
(the bench's AP2 block: B = 2048 instances of N=40 d=4; HIP-event kernel times).

usage: python tools/gen_variants.py lib1.so lib2.so ...
"""
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
B = int(sys.argv[2])
consts = pb.build_constants(); lay = pb.NlpLayout(40, 4); v0 = initial_guess(consts, lay)
V = torch.tensor(np.stack([batch_member(v0, lay, b) for b in range(B)]), device="cuda")
P = torch.tensor(np.stack([pb.pack_p(lay, consts, v0)] * B), device="cuda")
ev = E.Ap2Evaluator(consts, batch=B)
assert ev._lib is lib, "variant library not in use"
out = {"lib": sys.argv[1], "B": B}
res = {}
for path in ("colour", "generated"):
    ev.path = path
    f = torch.empty(B, dtype=torch.float64, device="cuda"); g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
    gr = torch.empty(B, ev.n_v, dtype=torch.float64, device="cuda"); jac = torch.empty(B, ev.nnz, dtype=torch.float64, device="cuda")
    ks, kn, ka = [], [], []
    for i in range(20):
        ev.eval_nlp_device(V, P, f, g, gr, jac)
        if i >= 5:
            ks.append(ev.last_kernel_ms()[0])
            if path == "generated":
                a, b = ev.last_kernel_ms_gen(); kn.append(a); ka.append(b)
    torch.cuda.synchronize()
    out[path] = {"main_ms": float(np.median(ks)), "evals_per_s": B / float(np.median(ks)) * 1e3}
    if kn:
        out[path].update(node_ms=float(np.median(kn)), assemble_ms=float(np.median(ka)))
    res[path] = [x.cpu().numpy() for x in (f, g, gr, jac)]
def rel(a, b):
    return float(np.max(np.abs(a - b) / (np.abs(b) + 1e-11 * np.max(np.abs(b)) + 1e-300)))
out["agree"] = {n: rel(res["generated"][i], res["colour"][i]) for i, n in enumerate(("f", "g", "grad", "jac"))}
print(json.dumps(out))
'''

if __name__ == "__main__":
    B = 2048
    for lib in sys.argv[1:]:
        r = subprocess.run([sys.executable, "-c", CHILD, lib, str(B)], capture_output=True, text=True, timeout=300)
        print(r.stdout.strip() or json.dumps({"lib": lib, "error": r.stderr[-1500:]}), flush=True)
