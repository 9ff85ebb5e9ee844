"""Restoration phase vs restoration step on the native interior point: cfg 5 (RK4 x 5) from perturbed starts (the
multistart of DESIGN.md section 9) and cfg 3 from random starts.  One JSON line per run.
Usage: python scripts/r3/resto_probe.py [--cfg5-batch 64] [--amp 0.1] [--max-iter 1000] [--modes phase,step]"""
import argparse
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from cocofest_amd.solver import IpmOptions, NativeIpm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg5-batch", type=int, default=64)
ap.add_argument("--amp", type=float, default=0.1)
ap.add_argument("--max-iter", type=int, default=1000)
ap.add_argument("--modes", default="phase,step")
ap.add_argument("--cfg3-batch", type=int, default=0)
ap.add_argument("--rir", default="0.9", help="required_infeasibility_reduction values (phase runs), comma-separated")
a = ap.parse_args()


def starts(ocp, B, amp, seed=0):
    rng = np.random.default_rng(seed)
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    lb, ub = ocp.bounds_vector()
    free = lb != ub
    span = np.minimum(np.where(np.isfinite(ub - lb), ub - lb, 10.0), 10.0)[free]
    v0[:, free] = np.clip(v0[:, free] + amp * rng.uniform(-1, 1, (B, free.sum())) * span, lb[free], ub[free])
    return v0


def run(name, ocp, v0, mode, rir=0.9):
    print(f"# {name} {mode} {rir} batch {len(v0)}", file=sys.stderr, flush=True)
    ipm = NativeIpm(ocp, batch=len(v0), options=IpmOptions(tol=1e-6, max_iter=a.max_iter, restoration=mode,
                                                            required_infeasibility_reduction=rir))
    res = ipm.solve(v0)
    st = ipm.last_stats
    ipm.close()
    conv = res.converged.astype(bool)
    print(json.dumps({"problem": name, "restoration": mode, "required_infeasibility_reduction": rir, "batch": len(v0), "converged": int(conv.sum()),
                      "wall_s": res.wall_time, "iterations_median": float(np.median(res.iterations)),
                      "iterations_max": int(res.iterations.max()),
                      "f_converged_min": float(res.f[conv].min()) if conv.any() else None,
                      "f_converged_median": float(np.median(res.f[conv])) if conv.any() else None,
                      "resto_phases": int(st["resto_phases"]), "resto_iterations": int(st["resto_iterations"]),
                      "eval_all": int(st["eval_all"]), "kkt_factor": int(st["kkt_factor"]),
                      "failed": np.where(~conv)[0].tolist(), "iterations": res.iterations.tolist()}), flush=True)


modes = a.modes.split(",")
if a.cfg5_batch:
    ocp = bench.msk_build(5)
    v0 = starts(ocp, a.cfg5_batch, a.amp)
    for mode in modes:
        for rir in ([float(r) for r in a.rir.split(",")] if mode == "phase" else [0.9]):
            run(f"cfg5_rk4x5_amp{a.amp}", ocp, v0, mode, rir)
if a.cfg3_batch:  # bench.convergence's random starts
    ocp3 = bench.build_cfg3()
    rng = np.random.default_rng(0)
    v0 = np.tile(ocp3.initial_guess_vector(), (a.cfg3_batch, 1))
    lb, ub = ocp3.bounds_vector()
    free = lb != ub
    v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (a.cfg3_batch, free.sum())) *
                          np.minimum(ub[free] - lb[free], 10), lb[free], ub[free])
    for mode in modes:
        run("cfg3_random_starts", ocp3, v0, mode)
