"""Batch-1 solve latency by KKT layout: cfg 3 (Ding2007 pulse widths, N = 100, force tracking)
and cfg 5 (arm26, RK4 x 5) from the reference's initial guess, CFX_IPM_KKT=band (nested dissection, the default at
batch 1) vs chain (block cyclic reduction); several repeats, one JSON line per (problem, layout).

Usage (GPU): python scripts/b1_layout_probe.py [--reps 5]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--out", default=None)
args = ap.parse_args()

from cocofest_amd.solver import IpmOptions, NativeIpm  # noqa: E402

problems = {"cfg3": (bench.build_cfg3(), IpmOptions(tol=1e-6, max_iter=300))}
try:
    problems["cfg5_rk4x5"] = (bench.msk_build(5), IpmOptions(tol=1e-6, max_iter=1000))
except Exception as e:  # noqa: BLE001
    print("cfg5 unavailable:", e)
for name, (ocp, opt) in problems.items():
    for kkt in ("band", "chain"):
        os.environ["CFX_IPM_KKT"] = kkt
        ipm = NativeIpm(ocp, batch=1, options=opt)
        walls, its = [], []
        for r in range(args.reps + 1):
            t0 = time.perf_counter()
            res = ipm.solve()
            if r:
                walls.append(time.perf_counter() - t0)
                its.append(int(res.iterations[0]))
        st = dict(ipm.last_stats)
        ipm.close()
        line = json.dumps({"problem": name, "layout": kkt, "wall_ms": [1e3 * w for w in walls],
                           "median_ms": 1e3 * float(np.median(walls)), "iterations": its, "f": float(res.f[0]),
                           "converged": bool(res.converged[0]), "kkt_blocks": st["kkt_blocks"],
                           "chain_nodes": st["kkt_chain_nodes"], "chain_sp": st["kkt_chain_sp"],
                           "border": st["kkt_border"]})
        print(line, flush=True)
        if args.out:
            with open(args.out, "a") as fh:
                fh.write(line + "\n")
