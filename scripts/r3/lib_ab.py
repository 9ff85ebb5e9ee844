"""A/B of libcfx builds on the shooting launches the bench times: cfg 2 headline (B = 2^20, tiles) and cfg 3 callbacks
(B = 2^18, tiles), 200 / 100 back-to-back launches after a 2 s settle, alternating child processes (CFX_LIB).
Usage: python scripts/r3/lib_ab.py LIB_A LIB_B [rounds]"""
import json
import os
import subprocess
import sys

CHILD = r"""
import json, sys, time
sys.path.insert(0, '.')
import numpy as np
import torch
import bench
out = {}
for name, ocp, B, steps in (("cfg2", bench.build_problem(), 1 << 20, 200), ("cfg3", bench.build_cfg3(), 1 << 18, 100)):
    h = ocp.nlp(batch=B, layout="tiled64", device=0)
    if name == "cfg2":
        v = bench.to_tiled(bench.synthetic_soa(ocp, B, seed=1234, device="cuda:0"))
    else:
        v = bench.to_tiled(torch.from_numpy(np.ascontiguousarray(bench.cfg3_synthetic(ocp, B, seed=0).T)).cuda())
    g = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device="cuda")
    j = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        for _ in range(10): h.eval_all(v, g=g, jac=j)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps): h.eval_all(v, g=g, jac=j)
    e1.record(); torch.cuda.synchronize()
    out[name + "_ms"] = e0.elapsed_time(e1) / steps
    out[name + "_sample"] = [float(g[3, 2, 5]), float(j[7, 11, 13])]
    h.close()
print(json.dumps(out))
"""

libs = sys.argv[1:3]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
for _ in range(rounds):
    for lib in libs:
        out = subprocess.run([sys.executable, "-c", CHILD], env=dict(os.environ, CFX_LIB=lib), capture_output=True,
                             text=True, timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-400:]
        print(json.dumps({"lib": lib, **(json.loads(line) if line.startswith("{") else {"error": line})}), flush=True)
