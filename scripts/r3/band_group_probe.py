"""Grouped register band LU (4 instances per wave) against one instance per wave and the lane placement: factor +
solve of cfg-3-shaped KKT bands (n = 500, kl = ku = 6) at several batches, HIP events; then the cfg-3 native
interior point from bench.py's random starts with each placement.  One JSON line per measurement."""
import json
import os
import pathlib
import sys
import time

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from cocofest_amd import _cfx  # noqa: E402

n, kl, ku = 500, 6, 6
ldab = 2 * kl + ku + 1
for B in (256, 1024, 4096, 16384):
    g = torch.Generator(device="cuda").manual_seed(B)
    ab0 = torch.randn((B, n, ldab), dtype=torch.float64, device="cuda", generator=g)
    ab0[:, :, kl + ku] += 8.0  # diagonally dominant enough to stay regular
    rhs0 = torch.randn((B, 1, n), dtype=torch.float64, device="cuda", generator=g)
    for label, env in (("group", {"CFX_BAND_PLACEMENT": "3", "CFX_BAND_GROUP": "1"}),
                       ("wave", {"CFX_BAND_PLACEMENT": "3", "CFX_BAND_GROUP": "0"}),
                       ("lane", {"CFX_BAND_PLACEMENT": "4", "CFX_BAND_GROUP": "0"})):
        os.environ.update(env)
        ipiv = torch.empty((B, n), dtype=torch.int32, device="cuda")
        info = torch.empty((B,), dtype=torch.int32, device="cuda")
        ts = []
        for rep in range(4):
            ab = ab0.clone()
            x = rhs0.clone()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _cfx.band_lu(ab, ipiv, info, kl, ku, rhs=x)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                ts.append(e0.elapsed_time(e1))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        x = rhs0.clone()
        e0.record()
        _cfx.band_lu_solve(ab, ipiv, kl, ku, x)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"batch": B, "placement": label, "factor_solve_ms": float(np.median(ts)),
                          "solve_ms": e0.elapsed_time(e1)}), flush=True)
for k in ("CFX_BAND_PLACEMENT", "CFX_BAND_GROUP"):
    os.environ.pop(k, None)

import bench  # noqa: E402
from cocofest_amd.solver import IpmOptions, NativeIpm  # noqa: E402

ocp = bench.build_cfg3()
for B in (256, 1024, 4096):
    rng = np.random.default_rng(0)
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    lb, ub = ocp.bounds_vector()
    free = lb != ub
    v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (B, free.sum())) * np.minimum(ub[free] - lb[free], 10),
                          lb[free], ub[free])
    for grp in ("1", "0"):
        os.environ["CFX_BAND_GROUP"] = grp
        ipm = NativeIpm(ocp, batch=B, options=IpmOptions(tol=1e-6, max_iter=300))
        ipm.solve(v0)
        walls = []
        for _ in range(3):
            t = time.perf_counter()
            r = ipm.solve(v0)
            walls.append(time.perf_counter() - t)
        ipm.close()
        print(json.dumps({"cfg3_batch": B, "group": grp, "wall_s": float(np.median(walls)),
                          "converged": int(r.converged.sum()), "iterations_max": int(r.iterations.max())}), flush=True)
