"""Which restoration variant converges most often: BatchedIpm (the executable specification, torch over libcfx on the
GPU) with the minimum-norm restoration step, Ipopt's restoration phase, and the phase with Ipopt's zero multipliers
after it / with a fresh filter after it.  Problems: the fatigue-family RK4 case of tests/test_ipm_native.py (its
two starts), cfg 5 from 16 perturbed starts.  One JSON line per (problem, variant)."""
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from cocofest_amd.solver import BatchedIpm, IpmOptions  # noqa: E402
from tests import cases  # noqa: E402

VARIANTS = {"step": ("step", {}), "phase": ("phase", {}), "phase_y0": ("phase", {"_resto_y0": True}),
            "phase_fresh": ("phase", {"_resto_fresh_filter": True}),
            "phase_y0_fresh": ("phase", {"_resto_y0": True, "_resto_fresh_filter": True})}


def starts(ocp, B, amp, seed, uniform01=False):
    rng = np.random.default_rng(seed)
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    lb, ub = ocp.bounds_vector()
    free = lb != ub
    if uniform01:
        v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (B, free.sum())) * np.minimum(ub[free] - lb[free], 10.0),
                              lb[free], ub[free])
    else:
        span = np.minimum(np.where(np.isfinite(ub - lb), ub - lb, 10.0), 10.0)[free]
        v0[:, free] = np.clip(v0[:, free] + amp * rng.uniform(-1, 1, (B, free.sum())) * span, lb[free], ub[free])
    return v0


problems = []
t = np.linspace(0, 1, 11)
for name in ("ding2003_with_fatigue", "ding2007_with_fatigue", "hmed2018_with_fatigue"):
    ocp = cases.product_ocp(name=name, stims=[0.0, 0.05, 0.1, 0.15], final_time=0.2, truncation=4, scheme="RK4", m=3,
                            objective={"force_tracking": [t, 40 * t]}, n_shooting=None)
    problems.append((f"{name}_rk4", ocp, starts(ocp, 8, 0, 1, uniform01=True), 1e-8, 300))
ocp5 = bench.msk_build(5)
problems.append(("cfg5_rk4x5", ocp5, starts(ocp5, 16, 0.1, 0), 1e-6, 600))
only = sys.argv[1].split(",") if len(sys.argv) > 1 else list(VARIANTS)
for pname, ocp, v0, tol, mi in problems:
    for vname in only:
        mode, attrs = VARIANTS[vname]
        ipm = BatchedIpm(ocp, batch=len(v0), options=IpmOptions(tol=tol, max_iter=mi, restoration=mode))
        for k, val in attrs.items():
            setattr(ipm, k, val)
        t0 = time.perf_counter()
        r = ipm.solve(v0)
        ipm.close()
        print(json.dumps({"problem": pname, "variant": vname, "batch": len(v0), "converged": int(r.converged.sum()),
                          "iterations": r.iterations.tolist(), "f_min": float(np.min(r.f)),
                          "wall_s": time.perf_counter() - t0}), flush=True)
