"""cfg 5 (RK4 x 5) batch-1 solve wall-clock with the fused stage/tangent kernel and with the two-kernel path
(CFX_MSK_TANGENTS, read at every launch), alternating.  Usage: python scripts/msk_solve_ab.py [--reps 3]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from cocofest_amd.solver import IpmOptions, NativeIpm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
ocp = bench.msk_build(5)
for r in range(args.reps):
    for mode in ("fused", "split"):
        if mode == "split":
            os.environ["CFX_MSK_TANGENTS"] = "split"
        else:
            os.environ.pop("CFX_MSK_TANGENTS", None)
        ipm = NativeIpm(ocp, batch=1, options=IpmOptions(tol=1e-6, max_iter=1000))
        res = ipm.solve()
        ipm.close()
        print(json.dumps({"mode": mode, "rep": r, "wall_s": res.wall_time, "iterations": int(res.iterations[0]),
                          "f": float(res.f[0])}), flush=True)
