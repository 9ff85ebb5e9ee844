"""Optimiser parity on the reference's one stored optimum with degrees of freedom: the
1,500-interval reaching task (examples/dynamics/reaching_task/reaching_task_pulse_duration_optimization.py:80-118,
stored revision's conventions: tests/test_reference_solution.py::legacy_product) started as a true Ipopt warm start at
the stored fatigue optimum.

The warm start: the stored states and pulse widths; multipliers from the product's own J_g and grad f at that point
(tests/reaching_kkt.py::adjoint_multipliers: discrete adjoint of the RK4 x 1 transcription, least squares for the
marker / end-state multipliers and the per-pulse bound multipliers); Ipopt's warm_start_init_point with mu_init =
warm_start_bound_push = warm_start_mult_bound_push = 1e-9; each pulse's width bounds on its first interval, as on the
stored revision's per-pulse parameter (FesMskOcp.bounds_vector, per_pulse_bounds "first").

The solver holds the stored point: every state within 1e-6 of its range, every width within 1e-6 of the width range,
f equal to 1e-8.  It does not certify it: the point is not a KKT point of the NLP to Ipopt's tolerance — 49 of the 353
bound-active pulses have wrong-signed multipliers (reduced dual infeasibility 5.4e-4 of the largest reduced-gradient
term, tests/reaching_kkt.py), so the iteration stalls there (a restoration phase called at an almost-feasible point)
instead of converging.  DESIGN.md section 9 records the numbers and the solves from the reference's own start."""

import numpy as np
import pytest

from tests import reaching_kkt as K
from tests import test_reference_solution as R

pytestmark = pytest.mark.gpu


def test_warm_start_holds_the_stored_fatigue_optimum():
    from cocofest_amd.solver import IpmOptions, NativeIpm

    ocp = R.legacy_product("fatigue", pulse_bounds="first")
    X, U = R.trajectory(R.load("fatigue"))
    nz = ocp.nx + ocp.nu
    vs = R.decision_vector(X, U[: len(R.MUSCLES)], nz)
    lb, ub = ocp.bounds_vector()
    y, zl, zu, rep = K.adjoint_multipliers(ocp, vs, lb, ub, pulse_bounds="first")
    assert rep["pulses_at_bounds"] == 353 and rep["pulses_sign_kept"] < rep["pulses_at_bounds"], rep
    assert rep["reduced_dual_inf_rel"] < 1e-3, rep
    ipm = NativeIpm(ocp, batch=1, options=IpmOptions(tol=1e-6, max_iter=40, bound_relax_factor=1e-8,
                                                      warm_start_init_point=True, mu_init=1e-9,
                                                      warm_start_bound_push=1e-9, warm_start_mult_bound_push=1e-9))
    r = ipm.solve(vs[None], warm_start=(y[None], zl[None], zu[None]))
    ipm.close()
    v = r.v[0]
    span = np.where(np.isfinite(ub - lb) & (ub > lb), ub - lb, np.maximum(1.0, np.abs(vs)))
    body0, body = vs[: R.N * nz].reshape(R.N, nz), v[: R.N * nz].reshape(R.N, nz)
    dx = np.abs(body[:, : ocp.nx] - body0[:, : ocp.nx]) / span[: R.N * nz].reshape(R.N, nz)[:, : ocp.nx]
    dx_end = np.abs(v[R.N * nz:] - vs[R.N * nz:]) / span[R.N * nz:]
    w = ub[ocp.nx] - lb[ocp.nx]  # the width range (first interval)
    dpw = np.abs(body[:, ocp.nx:] - body0[:, ocp.nx:]).max() / w
    print({"iterations": int(r.iterations[0]), "status": int(r.status[0]), "dx": float(max(dx.max(), dx_end.max())),
           "dpw": float(dpw), "f": float(r.f[0])})
    assert max(dx.max(), dx_end.max()) < 1e-6 and dpw < 1e-6
    np.testing.assert_allclose(r.f[0], 7.841959196, rtol=1e-8)
