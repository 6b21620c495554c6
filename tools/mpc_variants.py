"""Time variants of libawempc.so on the GPU, one subprocess each (config 5 batch: 256 instances).

usage: python tools/mpc_variants.py lib1.so lib2.so ...
"""
import json
import subprocess
import sys

CHILD = r'''
import sys, json, numpy as np, torch
sys.path.insert(0, ".")
from awebox_amd import mpc as mm, kite3 as k3
mm.load_library(sys.argv[1])
B = 256
c = k3.build_constants(); lay = k3.MpcLayout(c.cfg.n_k, c.cfg.d); orbit = k3.CircularOrbit(c.cfg)
inst = [k3.batch_instance(c, lay, i, B, orbit=orbit) for i in range(B)]
V = torch.tensor(np.stack([v for v, _ in inst]), device="cuda"); P = torch.tensor(np.stack([p for _, p in inst]), device="cuda")
ev = mm.MpcEvaluator(c, batch=B)
f = torch.empty(B, dtype=torch.float64, device="cuda"); g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
gr = torch.empty(B, ev.n_v, dtype=torch.float64, device="cuda"); jac = torch.empty(B, ev.nnz, dtype=torch.float64, device="cuda")
ks = []
for i in range(15):
    ev.eval_nlp_device(V, P, f, g, gr, jac)
    if i >= 3: ks.append(ev.last_kernel_ms()[0])
torch.cuda.synchronize()
print(json.dumps({"lib": sys.argv[1], "kernel_ms": float(np.median(ks)), "jac_sum": float(jac.sum()), "g_sum": float(g.sum())}))
'''

if __name__ == "__main__":
    for lib in sys.argv[1:]:
        r = subprocess.run([sys.executable, "-c", CHILD, lib], capture_output=True, text=True, timeout=240)
        print(r.stdout.strip() or json.dumps({"lib": lib, "error": r.stderr[-800:]}), flush=True)
