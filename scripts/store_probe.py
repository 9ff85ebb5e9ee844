"""Time the cfg-2 headline launch (tiled64, g + J_g, B = 2^20) in one process; the library and the launch shape come
from the environment (CFX_LIB, CFX_KPT, CFX_IFAST, CFX_NI), so variants built with other flags can be compared by
running this once per variant.  Prints one JSON line.  Usage: python scripts/store_probe.py [label]"""
import json
import os
import pathlib
import sys

import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

B = 1 << 20
ocp = bench.build_problem()
h = ocp.nlp(batch=B, layout="tiled64")
v = bench.synthetic_soa(ocp, B, 1, "cuda:0")
vt = v.T.reshape(B // 64, 64, -1).transpose(1, 2).contiguous()
gt = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device="cuda")
jt = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device="cuda")
res = []
for _ in range(5):
    for _ in range(20):
        h.eval_all(v=vt, g=gt, jac=jt)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        h.eval_all(v=vt, g=gt, jac=jt)
    e1.record()
    torch.cuda.synchronize()
    res.append(e0.elapsed_time(e1) / 200)
ms = sorted(res)[2]
print(json.dumps({"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": os.environ.get("CFX_LIB", "default"),
                  "kpt": os.environ.get("CFX_KPT"), "ifast": os.environ.get("CFX_IFAST"), "ms_median": ms,
                  "ms_all": res, "TBps": 1456 * B / ms / 1e9}), flush=True)
