"""Store policy of the headline launch (cfg 2, B = 2^20, 64-instance tiles): CFX_STPOL = 0 (global nt stores), 1 (buffer
sc1: write-through), 2 (buffer sc1 nt), alternating child processes.  Per policy: 200 back-to-back launches timed with HIP
events (kernel + boundary, as bench.py), and 30 launches timed one by one with the stream drained in between.
Usage: python scripts/r3/stpol_ab.py [rounds]"""
import json
import os
import subprocess
import sys

CHILD = r"""
import json, sys, time
sys.path.insert(0, '.')
import torch
import bench
ocp = bench.build_problem()
B = 1 << 20
h = ocp.nlp(batch=B, layout="tiled64", device=0)
v = bench.to_tiled(bench.synthetic_soa(ocp, B, seed=1234, device="cuda:0"))
g = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device="cuda")
j = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device="cuda")
t0 = time.perf_counter()
while time.perf_counter() - t0 < 2.0:
    for _ in range(10): h.eval_all(v, g=g, jac=j)
    torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200): h.eval_all(v, g=g, jac=j)
e1.record(); torch.cuda.synchronize()
b2b = e0.elapsed_time(e1) / 200
one = []
for _ in range(30):
    torch.cuda.synchronize()
    e0.record(); h.eval_all(v, g=g, jac=j); e1.record(); torch.cuda.synchronize()
    one.append(e0.elapsed_time(e1))
gs = float(g[5, 3, 7]); js = float(j[100, 17, 9])
print(json.dumps({"b2b_ms": b2b, "one_by_one_ms": sum(one) / len(one), "sample": [gs, js]}))
"""

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for _ in range(rounds):
    for pol in ("0", "1", "2"):
        out = subprocess.run([sys.executable, "-c", CHILD], env=dict(os.environ, CFX_STPOL=pol), capture_output=True,
                             text=True, timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-400:]
        print(json.dumps({"CFX_STPOL": pol, **(json.loads(line) if line.startswith("{") else {"error": line})}),
              flush=True)
