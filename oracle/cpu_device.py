"""The CPU port behind the evaluator's device-tensor interface (CPU torch tensors) --
TEST INFRASTRUCTURE ONLY: lets the CPU test suite run the GPU solver's algorithm (ipm.py) on
small problems without a GPU.  Never used by the product."""
from __future__ import annotations

import torch

from oracle.cpu_port import CpuPort


class CpuDeviceEvaluator:
    def __init__(self, consts):
        self.port = CpuPort(consts)
        self.port.hess_init()
        self.n_v, self.n_g, self.n_p, self.nnz = self.port.n_v, self.port.n_g, self.port.n_p, self.port.nnz
        self.nnz_h = self.port.hnnz
        from awebox_amd import problem as pb
        self.layout = pb.NlpLayout(consts.cfg.n_k, consts.cfg.d)

    def sparsity_jac(self):
        return self.port.colind.copy(), self.port.row.copy()

    def sparsity_hess(self):
        return self.port.hcolind.copy(), self.port.hrow.copy()

    def eval_nlp_device(self, V, P, f, g, grad_f, jac, stream=None):
        out = self.port.eval_nlp(V.numpy(), P.numpy())
        f.copy_(torch.from_numpy(out["f"]))
        g.copy_(torch.from_numpy(out["g"]))
        grad_f.copy_(torch.from_numpy(out["grad_f"]))
        jac.copy_(torch.from_numpy(out["jac"]))

    def eval_hess_device(self, V, P, sigma, lam_g, H, stream=None):
        H.copy_(torch.from_numpy(self.port.eval_hess(V.numpy(), P.numpy(), sigma.numpy(), lam_g.numpy())))
