"""cfg 4 NMPC timing breakdown: per-window wall vs interior-point wall, iterations, callback counts."""
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from cocofest_amd import DingModelPulseIntensityFrequency, OdeSolver  # noqa: E402
from cocofest_amd.nmpc import FesNmpc  # noqa: E402


def main(n_windows=30, batch=64):
    ft = json.loads((ROOT / "tests" / "golden" / "ref_formulas.json").read_text())["misc"]["force_tracking"]
    model = DingModelPulseIntensityFrequency(stim_time=[round(0.1 * i, 1) for i in range(10)], sum_stim_truncation=10)
    nmpc = FesNmpc(model, cycle_duration=1.0, n_cycles_simultaneous=1, n_cycles_to_advance=1,
                   objective={"force_tracking": [np.array(ft["time"]), np.array(ft["force"])]},
                   pulse_intensity={"max": 130}, ode_solver=OdeSolver.RK1(n_integration_steps=10), batch=batch)
    rng = np.random.default_rng(0)
    x0 = np.stack([rng.uniform(0, 0.5, batch), rng.uniform(0, 50, batch)], axis=1)
    res = nmpc.solve(n_cycles=n_windows, x0=x0)
    its = np.stack(res.iterations)
    print(json.dumps({"windows": n_windows, "batch": batch, "window_ms": [round(1e3 * w, 2) for w in res.window_wall],
                      "solve_ms": [round(1e3 * w, 2) for w in res.solve_wall],
                      "it_max": its.max(1).tolist(), "it_median": np.median(its, 1).tolist()}))


if __name__ == "__main__":
    main()
