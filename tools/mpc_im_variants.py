"""Time variants of libawempc.so on the generated instance-minor path (awempc_eval_nlp_im), one
subprocess each, at the config-5 batch (256 instances, N=20 d=4): HIP-event times of the input
transpose, the node kernel(s) and the finalize kernel, wall-clock evaluations/s of a timed loop, and
output checksums so that a variant which changes the arithmetic shows up.

usage: python tools/mpc_im_variants.py lib1.so lib2.so ... [--batch B]
"""
import json
import subprocess
import sys

CHILD = r'''
import sys, json, time, numpy as np, torch
sys.path.insert(0, ".")
from awebox_amd import mpc as mm, kite3 as k3
mm.load_library(sys.argv[1])
B = int(sys.argv[2])
c = k3.build_constants(); lay = k3.MpcLayout(c.cfg.n_k, c.cfg.d); orbit = k3.CircularOrbit(c.cfg)
inst = [k3.batch_instance(c, lay, i, B, orbit=orbit) for i in range(B)]
V = torch.tensor(np.stack([v for v, _ in inst]), device="cuda"); P = torch.tensor(np.stack([p for _, p in inst]), device="cuda")
ev = mm.MpcEvaluator(c, batch=B)
assert ev.generated_available
f = torch.empty(B, dtype=torch.float64, device="cuda"); g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
gr = ev.alloc_grad("cuda", instance_minor=True); jac = ev.alloc_jac("cuda", instance_minor=True)
s = torch.cuda.current_stream().cuda_stream
ks = []
for i in range(25):
    ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
    if i >= 5: ks.append(ev.last_kernel_ms_im())
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(200):
    ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
torch.cuda.synchronize()
el = time.perf_counter() - t0
ks = np.median(np.array(ks), axis=0)
print(json.dumps({"lib": sys.argv[1], "batch": B, "in_ms": float(ks[0]), "node_ms": float(ks[1]), "fin_ms": float(ks[2]),
                  "kernel_ms": float(ks.sum()), "evals_per_s_kernel": B / float(ks.sum()) * 1e3,
                  "evals_per_s_wall": B * 200 / el,
                  "jac_sum": float(jac.sum()), "g_sum": float(g.sum()), "grad_sum": float(gr.sum()), "f_sum": float(f.sum())}))
'''

if __name__ == "__main__":
    args = sys.argv[1:]
    batch = "256"
    if "--batch" in args:
        i = args.index("--batch")
        batch = args[i + 1]
        del args[i:i + 2]
    for rep in range(2):
        for lib in args:
            r = subprocess.run([sys.executable, "-c", CHILD, lib, batch], capture_output=True, text=True, timeout=240)
            print(r.stdout.strip() or json.dumps({"lib": lib, "error": r.stderr[-800:]}), flush=True)
