"""Profile target: BASELINE config 5 at RK4 x 5 solved by the native interior point (NativeIpm), batch 1 and 64
(run plain or under rocprofv3 --kernel-trace --stats)."""
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

import bench  # noqa: E402
from cocofest_amd.solver import IpmOptions, NativeIpm  # noqa: E402

ocp = bench.msk_build(5)
for B in [int(a) for a in (sys.argv[1:] or ["1"])]:
    ipm = NativeIpm(ocp, batch=B, options=IpmOptions(tol=1e-6, max_iter=1000))
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    res = ipm.solve(v0)  # warm-up (handle, code objects)
    t = time.perf_counter()
    res = ipm.solve(v0)
    wall = time.perf_counter() - t
    st = ipm.last_stats
    print(json.dumps({"batch": B, "wall_s": wall, "iterations": np.asarray(res.iterations).tolist()[:4],
                      "converged": int(np.sum(res.converged)), "f": float(np.asarray(res.f)[0]),
                      "stats": {k: (float(v) if isinstance(v, (float, np.floating)) else v) for k, v in st.items()}
                      if isinstance(st, dict) else str(st)}), flush=True)
    ipm.close()
