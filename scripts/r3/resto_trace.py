"""Trace of one interior-point solve that enters the restoration phase: BatchedIpm (torch over libcfx, verbose) and
NativeIpm on the same start.  Usage: python scripts/r3/resto_trace.py [phase|step] [max_iter]"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from cocofest_amd.solver import BatchedIpm, IpmOptions, NativeIpm  # noqa: E402
from tests import cases  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "phase"
max_iter = int(sys.argv[2]) if len(sys.argv) > 2 else 300
t = np.linspace(0, 1, 11)
cfg = dict(name="ding2007_with_fatigue", stims=[0.0, 0.05, 0.1, 0.15], final_time=0.2, truncation=4, scheme="RK4", m=3,
           objective={"force_tracking": [t, 40 * t]}, n_shooting=None)
ocp = cases.product_ocp(**cfg)
B = 2
v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
rng = np.random.default_rng(1)
lb, ub = ocp.bounds_vector()
free = lb != ub
v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (B, free.sum())) * np.minimum(ub[free] - lb[free], 10.0),
                      lb[free], ub[free])
v0 = v0[:1]
opts = IpmOptions(tol=1e-8, max_iter=max_iter, restoration=mode, verbose=True)
r = BatchedIpm(ocp, batch=1, options=opts).solve(v0)
print("BatchedIpm", mode, r.converged, r.iterations, r.f, r.kkt_error, flush=True)
opts.verbose = False
nat = NativeIpm(ocp, batch=1, options=opts)
r = nat.solve(v0)
print("NativeIpm", mode, r.converged, r.iterations, r.f, r.kkt_error, nat.last_stats["resto_phases"],
      nat.last_stats["resto_iterations"], flush=True)
