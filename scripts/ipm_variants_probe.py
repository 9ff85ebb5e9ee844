"""Iteration / callback counts of the torch-orchestrated interior point (BatchedIpm) with Ipopt's watchdog on and
off, on the bench's convergence problems.  One JSON line per (problem, variant)."""
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from cocofest_amd.solver import BatchedIpm, IpmOptions  # noqa: E402
from scripts.ipm_native_probe import cfg3, starts  # noqa: E402

problems = [("cfg5_rk4x5", bench.msk_build(5), 1), ("cfg3", cfg3(), 1), ("cfg3", cfg3(), 64)]
for name, ocp, B in problems:
    for trig in (10, 0):
        ipm = BatchedIpm(ocp, batch=B, options=IpmOptions(tol=1e-6, max_iter=1000, watchdog_shortened_iter_trigger=trig,
                                                          verbose=len(sys.argv) > 1 and B == 1 and trig == 10))
        res = ipm.solve(starts(ocp, B))
        print(json.dumps({"problem": name, "batch": B, "watchdog": trig, "converged": int(np.sum(res.converged)),
                          "it_max": int(np.max(res.iterations)), "it_median": float(np.median(res.iterations)),
                          "f0": float(res.f[0]), "calls": res.n_callbacks, "wall_s": res.wall_time}), flush=True)
        ipm.close()
