"""Profile target: one batched interior-point solve of BASELINE config 5 at RK4 x 5 (run under rocprofv3)."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

import cocofest_amd as C  # noqa: E402
from cocofest_amd.solver import BatchedIpm, IpmOptions  # noqa: E402

mm = C.FesMskModel(biorbd_path=str(ROOT / "tests/golden/biomod_arm26_biceps_triceps.json"),
                   muscles_model=[C.DingModelPulseWidthFrequencyWithFatigue(muscle_name=n, sum_stim_truncation=10)
                                  for n in ("BIClong", "TRIlong")],
                   stim_time=[0.1 * i for i in range(10)], activate_force_length_relationship=True,
                   activate_force_velocity_relationship=True)
ol = C.ObjectiveList()
ol.add(C.ObjectiveFcn.Mayer.MINIMIZE_STATE, key="qdot", index=[0, 1], node=C.Node.END, target=np.zeros((2, 1)), weight=100)
ocp = C.OcpFesMsk.prepare_ocp(model=mm, final_time=1, objective={"custom": ol, "minimize_muscle_fatigue": True},
                              msk_info={"bound_type": "start_end", "bound_data": [[0, 5], [0, 90]]},
                              ode_solver=C.OdeSolver.RK4(n_integration_steps=5))
ipm = BatchedIpm(ocp, batch=1, options=IpmOptions(tol=1e-6, max_iter=1000))
t = time.perf_counter()
res = ipm.solve()
print("wall", time.perf_counter() - t, "iterations", res.iterations, "calls", res.n_callbacks, flush=True)
