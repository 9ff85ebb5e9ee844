"""eval_h throughput (Lagrangian Hessian values) for cfg 2 and cfg 3 at large batch, and a large multi-start
interior-point solve of cfg 3.  Prints one JSON object."""

import json
import pathlib
import sys
import time

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def cfg3():
    from cocofest_amd import ModelMaker, OcpFes, OdeSolver

    ft = json.loads((ROOT / "tests" / "golden" / "ref_formulas.json").read_text())["misc"]["force_tracking"]
    model = ModelMaker.create_model("ding2007", stim_time=[float(v) for v in np.round(np.linspace(0, 1, 31)[:-1], 2)],
                                    sum_stim_truncation=10)
    return OcpFes.prepare_ocp(model=model, final_time=1, pulse_width={"min": model.pd0, "max": 0.0006},
                              objective={"force_tracking": [np.array(ft["time"]), np.array(ft["force"])]},
                              ode_solver=OdeSolver.RK1(n_integration_steps=10))


def hess_rate(ocp, B):
    h = ocp.nlp(batch=B, layout="soa")
    lb, ub = ocp.bounds_vector()
    lo = np.where(np.isfinite(lb), lb, 0.0)
    hi = np.where(np.isfinite(ub), np.minimum(ub, lo + 300.0), lo + 1.0)
    v = (torch.tensor(lo, device="cuda")[:, None] + torch.rand((h.nv, B), dtype=torch.float64, device="cuda")
         * torch.tensor(hi - lo, device="cuda")[:, None]).contiguous()
    lam = torch.randn((h.ng, B), dtype=torch.float64, device="cuda")
    of = torch.ones((B,), dtype=torch.float64, device="cuda")
    H = torch.empty((h.nnz_hess, B), dtype=torch.float64, device="cuda")
    for _ in range(3):
        h.eval_h(v, of, lam, H)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        h.eval_h(v, of, lam, H)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    nbytes = 8 * (h.nv + h.ng + 1 + h.nnz_hess)
    out = {"batch": B, "nnz_hess": h.nnz_hess, "ms": ms, "evals_per_s": B / ms * 1e3,
           "GBps": nbytes * B / ms / 1e6}
    h.close()
    return out


def main():
    from cocofest_amd.solver import BatchedIpm, IpmOptions

    res = {"cfg2_hess": hess_rate(bench.build_problem(), 1 << 18), "cfg3_hess": hess_rate(cfg3(), 1 << 15)}
    ocp = cfg3()
    for B in (1024, 4096):
        rng = np.random.default_rng(0)
        lb, ub = ocp.bounds_vector()
        free = lb != ub
        v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
        v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (B, free.sum())) * np.minimum(ub[free] - lb[free], 10),
                              lb[free], ub[free])
        ipm = BatchedIpm(ocp, batch=B, options=IpmOptions(tol=1e-6, max_iter=300))
        t0 = time.perf_counter()
        r = ipm.solve(v0)
        wall = time.perf_counter() - t0
        ipm.close()
        res[f"cfg3_multistart_{B}"] = {"wall_s": wall, "converged": int(r.converged.sum()),
                                       "iterations_max": int(r.iterations.max()), "solves_per_s": B / wall}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
