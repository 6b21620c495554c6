"""Time variants of libawedual.so (built with different -D flags) on the GPU, one subprocess each.

usage: python tools/dual_variants.py [--batch B] lib1.so lib2.so ...   (prints one JSON line per lib)
"""
import json
import subprocess
import sys

CHILD = r'''
import sys, time, json, numpy as np, torch
sys.path.insert(0, ".")
from awebox_amd import dual_evaluator as de, dual as du
de.load_library(sys.argv[1])
B = int(sys.argv[2])
c = du.build_constants(); lay = du.layout_for(c); v0 = du.initial_guess(c, lay)
ev = de.DualEvaluator(c, batch=B)
V = torch.tensor(np.stack([du.batch_member(v0, lay, b) for b in range(B)]), device="cuda")
P = torch.tensor(np.stack([du.pack_p(lay, c, v0)] * B), device="cuda")
f = torch.empty(B, dtype=torch.float64, device="cuda"); g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
gr = torch.empty(B, ev.n_v, dtype=torch.float64, device="cuda"); jac = torch.empty(B, ev.nnz, dtype=torch.float64, device="cuda")
ks = []
for i in range(12):
    ev.eval_nlp_device(V, P, f, g, gr, jac); 
    if i >= 2: ks.append(ev.last_kernel_ms()[0])
torch.cuda.synchronize()
print(json.dumps({"lib": sys.argv[1], "kernel_ms": float(np.median(ks)), "evals_per_s": B / (np.median(ks) * 1e-3),
                  "jac_sum": float(jac.sum()), "g_sum": float(g.sum()), "grad_sum": float(gr.sum())}))
'''

if __name__ == "__main__":
    args = sys.argv[1:]
    batch = 128
    if args and args[0] == "--batch":
        batch, args = int(args[1]), args[2:]
    for lib in args:
        r = subprocess.run([sys.executable, "-c", CHILD, lib, str(batch)], capture_output=True, text=True, timeout=240)
        print(r.stdout.strip() or json.dumps({"lib": lib, "error": r.stderr[-800:]}), flush=True)
