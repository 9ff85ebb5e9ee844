"""A/B probe of libcfx builds on the headline launch (cfg 2, B = 2^20, tiled64): each build runs in its own child
process (CFX_LIB selects the library), settles for 0.3 s, then times three K = 200 loops (HIP events).  Builds are
alternated over several rounds so box state (clocks, temperature) affects them alike.

usage: python scripts/ab_probe.py name=path [name=path ...]   (path "" = the in-tree libcfx.so)
"""

import json
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]

CHILD = r"""
import json, sys, time, torch
sys.path.insert(0, %r)
import bench
ocp = bench.build_problem()
B = 1 << 20
h = ocp.nlp(batch=B, layout="tiled64")
v = bench.to_tiled(bench.synthetic_soa(ocp, B, 1234, "cuda:0"))
g = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device="cuda")
j = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device="cuda")
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    for _ in range(10):
        h.eval_all(v, g=g, jac=j)
    torch.cuda.synchronize()
out = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        h.eval_all(v, g=g, jac=j)
    e1.record()
    torch.cuda.synchronize()
    out.append(round(e0.elapsed_time(e1) / 200, 4))
print(json.dumps(out))
"""


def main():
    builds = dict(a.split("=", 1) for a in sys.argv[1:])
    res = {k: [] for k in builds}
    for _ in range(2):
        for name, path in builds.items():
            env = dict(os.environ)
            if path:
                env["CFX_LIB"] = str(ROOT / path)
            r = subprocess.run([sys.executable, "-c", CHILD % str(ROOT)], env=env, capture_output=True, text=True,
                               timeout=120)
            if r.returncode != 0:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(r.returncode)
            res[name] += json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps({k: {"ms": v, "min": min(v)} for k, v in res.items()}))


if __name__ == "__main__":
    main()
