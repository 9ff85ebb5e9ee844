"""cfg 3 multi-start (4,096 starts) wall-clock under each band-LU placement (CFX_BAND_PLACEMENT, set per run)."""
import os
import sys
import time
import pathlib

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))

from ipm_native_probe import cfg3, starts  # noqa: E402
from cocofest_amd.solver import IpmOptions, NativeIpm  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ocp = cfg3()
ipm = NativeIpm(ocp, batch=B, options=IpmOptions(tol=1e-6, max_iter=300))
v0 = starts(ocp, B)
ipm.solve(v0)
t0 = time.perf_counter()
r = ipm.solve(v0)
print(os.environ.get("CFX_BAND_PLACEMENT", "auto"), B, round(time.perf_counter() - t0, 4), int(r.converged.sum()),
      int(r.iterations.max()), flush=True)
ipm.close()
