"""A/B of the native interior point with and without CFX_KEEP_CONSTANT_JAC on its callbacks (CFX_IPM_KEEPJ=1 / 0),
alternating on one box: cfg 3 from 4,096 random starts (bench.convergence's start set), from 256, and from the
reference's initial guess at batch 1; plus the cfg-2 headline launch with and without the flag.
Each measurement runs in a child process (one HIP runtime per process).  Usage: python scripts/r3/keepj_ab.py [rounds]"""
import json
import os
import subprocess
import sys

CHILD = r"""
import json, sys, time
import numpy as np
sys.path.insert(0, '.')
import bench
from cocofest_amd.solver import IpmOptions, NativeIpm
ocp = bench.build_cfg3()
out = {}
for B in (4096, 256, 1):
    rng = np.random.default_rng(0)
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    if B > 1:
        lb, ub = ocp.bounds_vector()
        free = lb != ub
        v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (B, free.sum())) * np.minimum(ub[free] - lb[free], 10),
                              lb[free], ub[free])
    ipm = NativeIpm(ocp, batch=B, options=IpmOptions(tol=1e-6, max_iter=300))
    ipm.solve(v0 if B > 1 else None)
    w = []
    for _ in range(5 if B > 1 else 15):
        t = time.perf_counter(); r = ipm.solve(v0 if B > 1 else None); w.append(time.perf_counter() - t)
    ipm.close()
    out[f"cfg3_b{B}_ms_median"] = 1e3 * float(np.median(w))
    out[f"cfg3_b{B}_converged"] = int(r.converged.sum())
    out[f"cfg3_b{B}_iterations_max"] = int(r.iterations.max())
import torch
h = bench.build_problem().nlp(batch=1 << 20, layout="tiled64", device=0)
B = 1 << 20
v = bench.to_tiled(bench.synthetic_soa(bench.build_problem(), B, seed=1234, device="cuda:0"))
g = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device="cuda")
j = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device="cuda")
for keep in (False, True, False, True):
    for _ in range(20): h.eval_all(v, g=g, jac=j, keep_constant_jac=keep)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200): h.eval_all(v, g=g, jac=j, keep_constant_jac=keep)
    e1.record(); torch.cuda.synchronize()
    out.setdefault("cfg2_launch_ms_keep" if keep else "cfg2_launch_ms_full", []).append(e0.elapsed_time(e1) / 200)
print(json.dumps(out))
"""

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for _ in range(rounds):
    for keep in ("1", "0"):
        out = subprocess.run([sys.executable, "-c", CHILD], env=dict(os.environ, CFX_IPM_KEEPJ=keep),
                             capture_output=True, text=True, timeout=500)
        line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-400:]
        print(json.dumps({"CFX_IPM_KEEPJ": keep, **(json.loads(line) if line.startswith("{") else {"error": line})}),
              flush=True)
