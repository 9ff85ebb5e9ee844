"""Which variables cut the primal steps of the reaching-task solve from the reference start (BatchedIpm, the
specification, verbose: the blocking variable of the fraction to the boundary per iteration).  GPU; slow (band LU
panel placement, ~1 s per iteration): a few dozen iterations.  Usage: python scripts/reaching_blocking_probe.py [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_reference_solution as R  # noqa: E402
from cocofest_amd.solver import BatchedIpm, IpmOptions  # noqa: E402

ocp = R.legacy_product("fatigue")
nz = ocp.nx + ocp.nu
names = [f"x{k}" for k in range(ocp.nx)] + [f"u{k}" for k in range(ocp.nu)]
ipm = BatchedIpm(ocp, batch=1, options=IpmOptions(tol=1e-6, max_iter=int(sys.argv[1]) if len(sys.argv) > 1 else 30,
                                                   bound_relax_factor=1e-8, restoration="phase", verbose=True))
print("node layout: nz", nz, "nx", ocp.nx, "(muscle m: Cn F A Tau1 Km at 5m..5m+4; q at 30, 31; qdot at 32, 33)")
ipm.solve()
