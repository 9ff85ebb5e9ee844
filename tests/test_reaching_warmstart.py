"""The native interior point's solve of the reference's reaching task from the reference script's own initial guess,
checked by the oracle.

scripts/reaching_warmstart.py --start reference (GPU, `profiles/round5/reaching/`) solves the product's 1,500-interval
reaching task under the stored revision's conventions (tests/test_reference_solution.py::legacy_product) with cfx_ipm
from the product's default initial guess (the reference's own start; Ipopt's defaults mu_init 0.1, bound_push 0.01;
bound_relax_factor 1e-8 as the stored solve).  With the stage-chain KKT layout (block cyclic reduction, 20-35 ms per
iteration) it converges under Ipopt's full termination tests in 818 iterations / 28.5 s to a KKT point 0.65 % below
the stored Ipopt optimum on the fatigue objective (the reference's own solve: 17,973 s, unknown hardware).  The
returned point is the iterate itself (honor_original_bounds off, Ipopt 3.14's default: the widths may sit up to
bound_relax_factor = 1e-8 outside [pd0, 0.6 ms], as the stored widths do); it is committed
(tests/golden/reaching_solve_fatigue.npz) and checked here by the oracle's plain-C port, independently of the GPU
kernels: every continuity row of the 1,500 intervals within Ipopt's constr_viol_tol, the marker rows, the postures,
the bounds and both objectives."""

import pathlib

import numpy as np

from oracle import fes_msk as M
from oracle import fes_oracle as O
from tests import reaching_kkt as K
from tests import test_reference_solution as R

GOLDEN = pathlib.Path(__file__).parent / "golden"


def _objectives(X, model):
    dt = R.FINAL_TIME / R.N
    return (sum((mus.a_rest / X[5 * m + 2, R.N]) ** 2 for m, mus in enumerate(model.muscles_dynamics_model)),
            dt * sum(float((X[5 * m + 1] ** 2).sum()) for m in range(len(R.MUSCLES))))


def test_solve_from_the_reference_start_is_a_feasible_point_with_a_lower_fatigue_objective():
    v = np.load(GOLDEN / "reaching_solve_fatigue.npz")["v"]
    pb = R.oracle_problem(legacy=True)  # its residual torque controls are zero here (the script has none)
    nm, nx = len(R.MUSCLES), pb.nx
    nzp = nx + nm
    assert v.size == R.N * nzp + nx
    body = v[: R.N * nzp].reshape(R.N, nzp)
    X = np.concatenate([body[:, :nx].T, v[R.N * nzp:][:, None]], axis=1)
    U = np.concatenate([body[:, nx:].T, np.zeros((pb.nu - nm, R.N))])
    res = R.all_residuals(pb, X, U)
    nxm = pb.nxm
    # continuity: the returned iterate meets Ipopt's constr_viol_tol (1e-4) with room to spare
    assert np.abs(res).max() < 1e-6, np.abs(res).max()
    assert np.abs(res[:, nxm:]).max() < 1e-6  # q, qdot rows
    vo = R.decision_vector(X, U, pb.nz)
    assert np.abs(M.marker_rows(pb, vo)).max() < 1e-6
    np.testing.assert_allclose(X[nxm: nxm + 2, 0], [0.0, 5 * 3.14 / 180], atol=1e-12)
    np.testing.assert_allclose(X[nxm: nxm + 2, R.N], [0.0, 5 * 3.14 / 180], atol=1e-6)
    pw = U[:nm]  # inside [pd0, 0.6 ms] up to bound_relax_factor (1e-8 absolute for bounds below 1)
    assert pw.min() >= O.model_constants("ding2007")["pd0"] - 1e-8 and pw.max() <= 6e-4 + 1e-8
    idx = R.pulse_index()  # one width per pulse (the per-pulse rows)
    assert max(float(np.ptp(pw[:, idx == i], axis=1).max()) for i in range(int(idx.max()) + 1)) < 1e-8
    # the objectives: a lower fatigue objective than the stored Ipopt optimum (7.8420), at a higher force cost
    _, _, _, _, model = K.product_bounds("fatigue")
    f_fat, f_force = _objectives(X, model)
    Xs, _ = R.trajectory(R.load("fatigue"))
    s_fat, s_force = _objectives(Xs, model)
    np.testing.assert_allclose(s_fat, 7.841959196, rtol=1e-8)
    np.testing.assert_allclose(f_fat, 7.7912473, rtol=1e-6)
    assert f_fat < s_fat * (1 - 6e-3), (f_fat, s_fat)
    print({"f_fatigue": f_fat, "stored": s_fat, "f_force": f_force, "stored_force": s_force,
           "continuity": float(np.abs(res).max())})
