"""A CPU stand-in for a libcfx handle, backed by the oracle, used to test host-side drivers (the IPM) on the
CPU.  Test infrastructure only — it is never used by the product."""

import numpy as np

from oracle import fes_collocation as CO
from oracle import fes_oracle as O


def _mod(pb):
    """The oracle module of a problem: collocation or shooting."""
    return CO if isinstance(pb, CO.ColProblem) else O


class OracleHandle:
    def __init__(self, pb: O.Problem, batch: int):
        self.pb, self.batch = pb, batch
        self.nv, self.ng = pb.nv, pb.ng
        M = self.M = _mod(pb)
        r, c = M.jac_structure(pb)
        self._jr, self._jc = r.astype(np.int32), c.astype(np.int32)
        hr, hc = M.hess_structure(pb)
        self._hr, self._hc = hr.astype(np.int32), hc.astype(np.int32)
        self.nnz_jac, self.nnz_hess = r.size, hr.size

    def jac_structure(self):
        return self._jr, self._jc

    def hess_structure(self):
        return self._hr, self._hc

    @staticmethod
    def _np(t):
        return t.detach().cpu().numpy()

    def eval_all(self, v, g=None, jac=None, f=None, grad=None):
        import torch

        vv = self._np(v)
        if g is not None:
            g.copy_(torch.from_numpy(self.M.eval_g(self.pb, vv)))
        if jac is not None:
            jac.copy_(torch.from_numpy(self.M.eval_jac_g(self.pb, vv)))
        if f is not None:
            f.copy_(torch.from_numpy(self.M.eval_f(self.pb, vv)))
        if grad is not None:
            grad.copy_(torch.from_numpy(self.M.eval_grad_f(self.pb, vv)))

    def eval_h(self, v, of, lam, hess):
        import torch

        hess.copy_(torch.from_numpy(self.M.hessian_values(self.pb, self._np(v), self._np(of), self._np(lam))))
        return hess

    def close(self):
        pass


class DenseBandSolver:
    """CPU stand-in for libcfx's batched band LU (GpuBandSolver): expands the band storage to dense matrices
    and solves with torch.linalg.  Test infrastructure only."""

    def factor(self, ab, kl, ku):
        import torch

        B, n, ldab = ab.shape
        kv = kl + ku
        i = torch.arange(n)[:, None]
        j = torch.arange(n)[None, :]
        r = kv + i - j
        inband = (r >= kl) & (r < ldab)
        A = torch.zeros((B, n, n), dtype=ab.dtype)
        jj = j.expand(n, n)[inband]
        A[:, inband] = ab[:, jj, r[inband]]
        return A

    @staticmethod
    def singular(A):
        import torch

        return torch.zeros(A.shape[0], dtype=torch.bool)

    def solve(self, A, rhs):
        import torch

        return torch.linalg.solve(A, rhs)


def oracle_problem_from_ocp(ocp) -> O.Problem:
    """The oracle's description of a product FesOcp (any interval slice included): same model constants,
    stim rows, scheme, objective terms."""
    from cocofest_amd import _cfx

    name = O.MODEL_NAMES[ocp.model.cfx_model_id]
    kw = dict(name=name, c=O.model_constants(name), n_shooting=ocp.n_shooting, final_time=float(ocp.final_time),
              truncation=ocp.truncation, rows=np.asarray(ocp.stim_rows, dtype=float))
    if ocp.degree:
        pb = CO.ColProblem(**kw, degree=ocp.degree, method=ocp.ode_solver.method)
    else:
        scheme = {_cfx.RK1: "RK1", _cfx.RK2: "RK2", _cfx.RK4: "RK4"}[ocp.ode_solver.scheme]
        pb = O.Problem(**kw, scheme=scheme, n_steps=ocp.ode_solver.n_integration_steps)
    if ocp.n_params and ocp.last_stim_idx is not None:
        pb.n_params = ocp.n_params
        pb.last_stim_idx = [int(i) for i in ocp.last_stim_idx]
        pb.intensity_floor = float(ocp.intensity_floor)
    for t in ocp.objectives:
        kind = "lagrange" if t["kind"] == _cfx.OBJ_LAGRANGE else "mayer"
        var = ("x" if t["var_kind"] == _cfx.VAR_STATE else "u", t["var_index"])
        tgt = (np.asarray(t["target"], dtype=float) if t.get("target") is not None
               else np.full(ocp.n_shooting + 1, float(t.get("target_value", 0.0))))
        pb.objectives.append(O.Objective(kind, var, float(t["weight"]), tgt,
                                         list(range(t["node_first"], t["node_last"] + 1))))
    return pb
