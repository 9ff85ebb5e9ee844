"""cfg 3 multistart under a named solver profile, for a rocprofv3 kernel trace (GPU).
Usage: python scripts/ipm_profile_probe.py --profile ipopt|cfx --batch 4096 [--opt key=value ...]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from cocofest_amd.solver import IpmOptions, NativeIpm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--profile", default="ipopt", choices=["ipopt", "cfx"])
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--opt", action="append", default=[])
ap.add_argument("--guess", action="store_true", help="start every instance at the reference's initial guess")
ap.add_argument("--reps", type=int, default=1, help="timed solves (after one warm-up)")
args = ap.parse_args()
extra = {}
for kv in args.opt:
    k, v = kv.split("=", 1)
    cur = getattr(IpmOptions(), k)
    extra[k] = (v.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(v)
base = dict(tol=1e-6, max_iter=300, **extra)
opts = IpmOptions.ipopt(**base) if args.profile == "ipopt" else IpmOptions(**base)
ocp = bench.build_cfg3()
B = args.batch
rng = np.random.default_rng(0)
v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
lb, ub = ocp.bounds_vector()
free = lb != ub
if not args.guess:
    v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (B, free.sum())) * np.minimum(ub[free] - lb[free], 10),
                          lb[free], ub[free])
ipm = NativeIpm(ocp, batch=B, options=opts)
ipm.solve(v0)
t = time.perf_counter()
for _ in range(args.reps):
    r = ipm.solve(v0)
dt = (time.perf_counter() - t) / args.reps
st = ipm.last_stats
ipm.close()
print({"profile": args.profile, "extra": extra, "batch": B, "wall_s": dt, "iterations_max": int(r.iterations.max()),
       "converged": int(r.converged.sum()), "kkt_factor": st["kkt_factor"], "eval_all": st["eval_all"],
       "eval_g_f": st["eval_g_f"], "host_iterations": st["iterations"], "soft_steps": st["soft_steps"]})
