"""cfg 5 (RK4 x 5) native interior point from the 64 perturbed starts of scripts/msk_multistart_probe.py (amp 0.1,
seed 0), with the restoration phase, against two Ipopt defaults the native solver's defaults differ from:
bound_relax_factor (Ipopt 1e-8; here 0) and max_iter (Ipopt 3000; the probe's 1000); with --filter-reset, Ipopt's
filter reset heuristic on (the default) and off.  One JSON line per variant."""
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from cocofest_amd.solver import IpmOptions, NativeIpm  # noqa: E402

ocp = bench.msk_build(5)
B, amp = 64, 0.1
rng = np.random.default_rng(0)
v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
lb, ub = ocp.bounds_vector()
free = lb != ub
span = np.minimum(np.where(np.isfinite(ub - lb), ub - lb, 10.0), 10.0)[free]
v0[:, free] = np.clip(v0[:, free] + amp * rng.uniform(-1, 1, (B, free.sum())) * span, lb[free], ub[free])
variants = {"default": {}, "bound_relax_1e-8": {"bound_relax_factor": 1e-8}, "max_iter_3000": {"max_iter": 3000},
            "bound_relax_1e-8_max_iter_3000": {"bound_relax_factor": 1e-8, "max_iter": 3000}}
if len(sys.argv) > 1 and sys.argv[1] == "--filter-reset":  # Ipopt's filter reset heuristic on (default) / off
    variants = {"filter_reset_5": {"max_filter_resets": 5}, "default_no_reset": {},
                "filter_reset_5_max_iter_3000": {"max_filter_resets": 5, "max_iter": 3000}}
for name, kw in variants.items():
    opts = dict(tol=1e-6, max_iter=1000)
    opts.update(kw)
    ipm = NativeIpm(ocp, batch=B, options=IpmOptions(**opts))
    res = ipm.solve(v0)
    st = ipm.last_stats
    ipm.close()
    conv = res.converged.astype(bool)
    print(json.dumps({"variant": name, "options": opts, "converged": int(conv.sum()), "batch": B,
                      "wall_s": res.wall_time, "iterations_median": float(np.median(res.iterations)),
                      "iterations_max": int(res.iterations.max()),
                      "f_converged_median": float(np.median(res.f[conv])) if conv.any() else None,
                      "failed": [int(i) for i in np.where(~conv)[0]],
                      "resto_phases": int(st["resto_phases"]), "resto_iterations": int(st["resto_iterations"])}),
          flush=True)
