import pathlib, sys
ROOT = pathlib.Path("/root/repo"); sys.path.insert(0, str(ROOT))
import bench
from cocofest_amd.solver import BatchedIpm, IpmOptions
ipm = BatchedIpm(bench.msk_build(5), batch=1, options=IpmOptions(tol=1e-6, max_iter=1000, verbose=True))
res = ipm.solve()
print(res.iterations, res.f, res.wall_time)
