"""Wall-clock to convergence: libcfx's native interior point (NativeIpm) vs the torch-orchestrated BatchedIpm on
the bench's convergence problems.  One JSON line per problem."""
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from cocofest_amd import ModelMaker, OcpFes, OdeSolver  # noqa: E402
from cocofest_amd.solver import BatchedIpm, IpmOptions, NativeIpm  # noqa: E402


def cfg3():
    ft = json.loads((ROOT / "tests" / "golden" / "ref_formulas.json").read_text())["misc"]["force_tracking"]
    model = ModelMaker.create_model("ding2007", stim_time=[float(v) for v in np.round(np.linspace(0, 1, 31)[:-1], 2)],
                                    sum_stim_truncation=10)
    return OcpFes.prepare_ocp(model=model, final_time=1, pulse_width={"min": model.pd0, "max": 0.0006},
                              objective={"force_tracking": [np.array(ft["time"]), np.array(ft["force"])]},
                              ode_solver=OdeSolver.RK1(n_integration_steps=10))


def starts(ocp, B):
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    if B > 1:
        rng = np.random.default_rng(0)
        lb, ub = ocp.bounds_vector()
        free = lb != ub
        v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (B, free.sum())) * np.minimum(ub[free] - lb[free], 10),
                              lb[free], ub[free])
    return v0


def run(name, ocp, B, max_iter=300, which=("torch", "native")):
    out = {"problem": name, "batch": B}
    for kind in which:
        cls = BatchedIpm if kind == "torch" else NativeIpm
        ipm = cls(ocp, batch=B, options=IpmOptions(tol=1e-6, max_iter=max_iter))
        v0 = starts(ocp, B)
        ipm.solve(v0)  # warm-up
        t0 = time.perf_counter()
        res = ipm.solve(v0)
        wall = time.perf_counter() - t0
        out[kind] = {"wall_s": wall, "converged": int(res.converged.sum()), "it_max": int(res.iterations.max()),
                     "it_median": float(np.median(res.iterations)), "f0": float(res.f[0]), "calls": res.n_callbacks}
        if kind == "native":
            out[kind]["stats"] = ipm.last_stats
        ipm.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    which = tuple(sys.argv[1].split(",")) if len(sys.argv) > 1 else ("torch", "native")
    o3 = cfg3()
    run("cfg3", o3, 1, which=which)
    run("cfg2", bench.build_problem(), 1, which=which)
    run("cfg3", o3, 256, which=which)
    run("cfg3", o3, 4096, which=which)
    run("cfg5_rk4x5", bench.msk_build(5), 1, max_iter=1000, which=which)
