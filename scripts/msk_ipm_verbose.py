"""Per-iteration log of the torch-orchestrated interior point on BASELINE config 5 at RK4 x 5 (GPU callbacks)."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from cocofest_amd.solver import BatchedIpm, IpmOptions  # noqa: E402

ipm = BatchedIpm(bench.msk_build(5), batch=1, options=IpmOptions(tol=1e-6, max_iter=1000, verbose=True))
res = ipm.solve()
print(res.iterations, res.f, res.wall_time, res.n_callbacks)
