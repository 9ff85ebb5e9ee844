"""Batch-1 native interior point wall-clock (cfg 3 and cfg 2 single solves, best of 5) for the counter-read mode in
the environment (CFX_IPM_PUB=launch: a separate k_ipm_publish launch per read; default: in-kernel publish).  The
in-kernel mode was measured (profiles/round2/ipm_pub/) and not kept; the probe now times the shipped mode either way."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from cocofest_amd.solver import IpmOptions, NativeIpm  # noqa: E402

out = {"CFX_IPM_PUB": os.environ.get("CFX_IPM_PUB")}
for name, ocp in (("cfg3_single", bench.build_cfg3()), ("cfg2_single", bench.build_problem())):
    ipm = NativeIpm(ocp, batch=1, device=0, options=IpmOptions(tol=1e-6, max_iter=300))
    walls, its = [], None
    for _ in range(6):
        res = ipm.solve(None)
        walls.append(res.wall_time)
        its = int(res.iterations.max())
        conv = int(res.converged.sum())
        f = float(res.f[0])
    ipm.close()
    out[name] = {"wall_min_s": min(walls[1:]), "wall_med_s": sorted(walls[1:])[2], "iterations": its,
                 "converged": conv, "f": f}
print(json.dumps(out), flush=True)
