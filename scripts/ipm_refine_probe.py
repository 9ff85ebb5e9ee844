"""Interior point with and without iterative refinement of the Newton solves: cfg 5 (RK4 x 5, batch 1, and 64
perturbed starts) and cfg 3 (batch 1 and 256 starts).  Usage: python scripts/ipm_refine_probe.py"""
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from cocofest_amd import ModelMaker, OcpFes, OdeSolver  # noqa: E402
from cocofest_amd.solver import BatchedIpm, IpmOptions  # noqa: E402

ft = json.loads((ROOT / "tests" / "golden" / "ref_formulas.json").read_text())["misc"]["force_tracking"]
model = ModelMaker.create_model("ding2007", stim_time=[float(v) for v in np.round(np.linspace(0, 1, 31)[:-1], 2)],
                                sum_stim_truncation=10)
ocp3 = OcpFes.prepare_ocp(model=model, final_time=1, pulse_width={"min": model.pd0, "max": 0.0006},
                          objective={"force_tracking": [np.array(ft["time"]), np.array(ft["force"])]},
                          ode_solver=OdeSolver.RK1(n_integration_steps=10))
ocp5 = bench.msk_build(5)


def starts(ocp, B, amp, cap):
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    if B > 1:
        rng = np.random.default_rng(0)
        lb, ub = ocp.bounds_vector()
        free = lb != ub
        span = np.minimum(np.where(np.isfinite(ub - lb), ub - lb, cap), cap)[free]
        v0[:, free] = np.clip(v0[:, free] + amp * rng.uniform(0 if amp == 1 else -1, 1, (B, free.sum())) * span,
                              lb[free], ub[free])
    return v0


for refine, max_soc, relax in ((0, 4, 0.0), (0, 4, 0.0)):  # twice: the solve is deterministic
    for name, ocp, B, amp, cap in (("cfg5", ocp5, 1, 0, 10), ("cfg5_ms64", ocp5, 64, 0.1, 10),
                                   ("cfg3", ocp3, 1, 0, 10), ("cfg3_ms256", ocp3, 256, 1, 10)):
        ipm = BatchedIpm(ocp, batch=B, options=IpmOptions(tol=1e-6, max_iter=1000, refine=refine, max_soc=max_soc, bound_relax_factor=relax))
        v0 = starts(ocp, B, amp, cap)
        ipm.solve(v0) if name.startswith("cfg3") else None  # warm-up
        res = ipm.solve(v0)
        ipm.close()
        print(f"refine={refine} max_soc={max_soc} relax={relax} {name}: wall {res.wall_time:.2f} s, converged {int(res.converged.sum())}/{B}, "
              f"iterations median {np.median(res.iterations):.0f} max {res.iterations.max()}, "
              f"f median {np.median(res.f):.6g}", flush=True)
