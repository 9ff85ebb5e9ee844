"""Host-side profile of one interior-point solve (cfg 3, batch 1 and 256): cProfile top entries."""

import cProfile
import json
import pathlib
import pstats
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from cocofest_amd import ModelMaker, OcpFes, OdeSolver
    from cocofest_amd.solver import BatchedIpm, IpmOptions

    ft = json.loads((ROOT / "tests" / "golden" / "ref_formulas.json").read_text())["misc"]["force_tracking"]
    model = ModelMaker.create_model("ding2007", stim_time=[float(v) for v in np.round(np.linspace(0, 1, 31)[:-1], 2)],
                                    sum_stim_truncation=10)
    ocp = OcpFes.prepare_ocp(model=model, final_time=1, pulse_width={"min": model.pd0, "max": 0.0006},
                             objective={"force_tracking": [np.array(ft["time"]), np.array(ft["force"])]},
                             ode_solver=OdeSolver.RK1(n_integration_steps=10))
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    ipm = BatchedIpm(ocp, batch=B, options=IpmOptions(tol=1e-6))
    ipm.solve()
    pr = cProfile.Profile()
    pr.enable()
    res = ipm.solve()
    pr.disable()
    print("wall", res.wall_time, "iters", res.iterations.max(), res.n_callbacks)
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
