"""Band LU placements at large batches (cfg-3 KKT shape n = 502, kl = ku = 6): factor (+ one solve) and solve-only
times per placement (CFX_BAND_PLACEMENT 3 register / 4 lane, coalesced through instance-minor copies / 4d lane
on the caller's instance-major arrays / 0 windowed).  Prints one JSON line per case."""
import json
import os
import pathlib
import sys

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from cocofest_amd import _cfx  # noqa: E402

n, kl, ku = 502, 6, 6
ldab = 2 * kl + ku + 1
for B in (1024, 4096, 16384):
    rng = np.random.default_rng(0)
    ab0 = torch.tensor(rng.standard_normal((B, n, ldab)), device="cuda")
    ab0[:, :, :kl] = 0.0
    rhs0 = torch.tensor(rng.standard_normal((B, 1, n)), device="cuda")
    for pl in ("3", "4", "4d", "0"):
        os.environ["CFX_BAND_PLACEMENT"] = pl[0]
        if pl == "4d":
            os.environ["CFX_BAND_LANE_DIRECT"] = "1"
        else:
            os.environ.pop("CFX_BAND_LANE_DIRECT", None)
        ab = ab0.clone()
        ipiv = torch.empty((B, n), dtype=torch.int32, device="cuda")
        info = torch.empty((B,), dtype=torch.int32, device="cuda")
        x = rhs0.clone()
        ts = []
        for r in range(4):
            ab.copy_(ab0)
            x.copy_(rhs0)
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
            _cfx.band_lu(ab, ipiv, info, kl, ku, rhs=x)
            e1.record()
            _cfx.band_lu_solve(ab, ipiv, kl, ku, x)
            e2.record()
            torch.cuda.synchronize()
            ts.append((e0.elapsed_time(e1), e1.elapsed_time(e2)))
        f, s = sorted(ts)[len(ts) // 2]
        print(json.dumps({"B": B, "placement": pl, "factor_solve_ms": f, "solve_ms": s}), flush=True)
