"""Why cfg-5 (RK4 x 5) solves from perturbed starts stall: solve 64 starts (+-10 % of each range) with the native
interior point, then replay two that did not converge with BatchedIpm (same algorithm) and its per-iteration log.
Usage: python scripts/msk_stuck_probe.py"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from cocofest_amd.solver import BatchedIpm, IpmOptions, NativeIpm  # noqa: E402

ocp = bench.msk_build(5)
B, amp = 64, 0.1
rng = np.random.default_rng(0)
v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
lb, ub = ocp.bounds_vector()
free = lb != ub
span = np.minimum(np.where(np.isfinite(ub - lb), ub - lb, 10.0), 10.0)[free]
v0[:, free] = np.clip(v0[:, free] + amp * rng.uniform(-1, 1, (B, free.sum())) * span, lb[free], ub[free])
ipm = NativeIpm(ocp, batch=B, options=IpmOptions(tol=1e-6, max_iter=1000))
res = ipm.solve(v0)
ipm.close()
bad = np.where(~res.converged)[0]
print(f"converged {int(res.converged.sum())}/{B}; not converged: {bad.tolist()}")
for i in bad:
    print(f"  start {i}: f {res.f[i]:.4e} kkt {res.kkt_error[i]:.3e} its {res.iterations[i]}")
np.save(ROOT / "gpurun_out" / "msk_stuck_v0.npy", v0[bad])
for i in bad[:2]:
    print(f"--- replay of start {i} (BatchedIpm, verbose)", flush=True)
    r = BatchedIpm(ocp, batch=1, options=IpmOptions(tol=1e-6, max_iter=400, verbose=True)).solve(v0[i:i + 1])
    print(f"replay: converged {bool(r.converged[0])} its {int(r.iterations[0])} f {float(r.f[0]):.4e}", flush=True)
