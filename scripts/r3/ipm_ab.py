"""A/B of two libcfx builds on one box: the cfg-3 native interior point at batch 1 (the reference's initial guess)
and the cfg-2 headline launch, alternating builds.  Usage: python scripts/r3/ipm_ab.py LIB_A LIB_B [rounds]
Each measurement runs in a child process with CFX_LIB set (one HIP runtime per process)."""
import json
import os
import subprocess
import sys

CHILD = r"""
import json, sys, time, pathlib
import numpy as np
sys.path.insert(0, '.')
import bench
from cocofest_amd.solver import IpmOptions, NativeIpm
ocp = bench.build_cfg3()
ipm = NativeIpm(ocp, batch=1, options=IpmOptions(tol=1e-6, max_iter=300))
ipm.solve()
w = []
for _ in range(15):
    t = time.perf_counter(); r = ipm.solve(); w.append(time.perf_counter() - t)
ipm.close()
import torch
from cocofest_amd import _cfx
h = bench.build_problem().nlp(batch=1 << 20, layout="tiled64", device=0)
B = 1 << 20
v = torch.rand((B // 64, h.nv, 64), dtype=torch.float64, device="cuda")
g = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device="cuda")
j = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device="cuda")
for _ in range(10): h.eval_all(v, g=g, jac=j)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200): h.eval_all(v, g=g, jac=j)
e1.record(); torch.cuda.synchronize()
print(json.dumps({"cfg3_b1_ms_median": 1e3 * float(np.median(w)), "cfg3_b1_ms_min": 1e3 * min(w),
                  "iterations": int(r.iterations[0]), "cfg2_launch_ms": e0.elapsed_time(e1) / 200}))
"""

libs = sys.argv[1:3]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
for _ in range(rounds):
    for lib in libs:
        out = subprocess.run([sys.executable, "-c", CHILD], env=dict(os.environ, CFX_LIB=lib), capture_output=True,
                             text=True, timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-400:]
        print(json.dumps({"lib": lib, **(json.loads(line) if line.startswith("{") else {"error": line})}), flush=True)
