"""One batched interior-point solve of cfg 3 (B from argv, default 4096) for a rocprofv3 kernel trace."""

import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from scripts.probe_hessian import cfg3  # noqa: E402


def main():
    from cocofest_amd.solver import BatchedIpm, IpmOptions

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    ocp = cfg3()
    rng = np.random.default_rng(0)
    lb, ub = ocp.bounds_vector()
    free = lb != ub
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (B, free.sum())) * np.minimum(ub[free] - lb[free], 10),
                          lb[free], ub[free])
    ipm = BatchedIpm(ocp, batch=B, options=IpmOptions(tol=1e-6, max_iter=300))
    r = ipm.solve(v0)
    print("wall", r.wall_time, "iters", int(r.iterations.max()), r.n_callbacks)
    ipm.close()


if __name__ == "__main__":
    main()
