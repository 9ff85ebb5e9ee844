"""Verbose trace of BatchedIpm (the specification; restoration phase) on chosen cfg-5 starts of resto_probe.py
(seed 0, 10 % perturbation).  Usage: python scripts/r3/resto_trace_cfg5.py IDX [IDX ...] > trace.log"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from cocofest_amd.solver import BatchedIpm, IpmOptions  # noqa: E402

ocp = bench.msk_build(5)
B = 64
rng = np.random.default_rng(0)
v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
lb, ub = ocp.bounds_vector()
free = lb != ub
span = np.minimum(np.where(np.isfinite(ub - lb), ub - lb, 10.0), 10.0)[free]
v0[:, free] = np.clip(v0[:, free] + 0.1 * rng.uniform(-1, 1, (B, free.sum())) * span, lb[free], ub[free])
for idx in [int(a) for a in sys.argv[1:]]:
    print(f"==== start {idx}", flush=True)
    ipm = BatchedIpm(ocp, batch=1, options=IpmOptions(tol=1e-6, max_iter=1000, restoration="phase", verbose=True))
    r = ipm.solve(v0[idx:idx + 1])
    ipm.close()
    print(f"==== start {idx}: converged {bool(r.converged[0])} iterations {int(r.iterations[0])} f {float(r.f[0])}",
          flush=True)
