"""Native interior point at batch 1 from the reference's initial guess, solved `reps` times after a warm-up, for a
rocprofv3 kernel trace: python scripts/r3/profile_native_b1.py {cfg2|cfg3} [reps].  Prints wall-clock, iterations and
the solver's counters (callbacks, factorisations, host reads, restoration phases)."""
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from cocofest_amd.solver import IpmOptions, NativeIpm  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ocp = bench.build_problem() if name == "cfg2" else bench.build_cfg3()
ipm = NativeIpm(ocp, batch=1, options=IpmOptions(tol=1e-6, max_iter=300))
ipm.solve()
walls = []
for _ in range(reps):
    t = time.perf_counter()
    r = ipm.solve()
    walls.append(time.perf_counter() - t)
st = ipm.last_stats
ipm.close()
print(json.dumps({"problem": name, "wall_ms_median": 1e3 * float(np.median(walls)), "wall_ms_min": 1e3 * min(walls),
                  "iterations": int(r.iterations[0]), "converged": int(r.converged[0]),
                  "stats_last_solve": {k: (v if isinstance(v, (int, float)) else str(v)) for k, v in st.items()}}))
