"""Filter reset heuristic diagnostics: the fatigue-family RK4 case of tests/test_ipm_native.py (Ding2007 with fatigue,
two starts) with BatchedIpm and NativeIpm, heuristic on (Ipopt's default) and off."""
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from cocofest_amd.solver import BatchedIpm, IpmOptions, NativeIpm  # noqa: E402
from tests import cases  # noqa: E402
from tests.test_ipm_native import _starts  # noqa: E402

t = np.linspace(0, 1, 11)
for name in ("ding2003_with_fatigue", "ding2007_with_fatigue", "hmed2018_with_fatigue"):
    cfg = dict(name=name, stims=[0.0, 0.05, 0.1, 0.15], final_time=0.2, truncation=4, scheme="RK4", m=3,
               objective={"force_tracking": [t, 40 * t]}, n_shooting=None)
    ocp = cases.product_ocp(**cfg)
    v0 = _starts(ocp, 2, 1)
    for resets in (5, 0):
        for cls in (BatchedIpm, NativeIpm):
            ipm = cls(ocp, batch=2, options=IpmOptions(tol=1e-8, max_iter=300, restoration="phase",
                                                       max_filter_resets=resets))
            r = ipm.solve(v0)
            ipm.close()
            print(json.dumps({"problem": name, "solver": cls.__name__, "max_filter_resets": resets,
                              "converged": r.converged.tolist(), "iterations": r.iterations.tolist(),
                              "f": r.f.tolist()}), flush=True)
