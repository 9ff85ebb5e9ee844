"""The CPU restatement of the direct-collocation transcription (oracle/fes_collocation.py): coefficients,
consistency of g / J_g / H with each other, and convergence of the collocation solution to the ODE solution."""

import numpy as np
import pytest
from scipy.optimize import fsolve

from oracle import fes_collocation as CO
from oracle import fes_oracle as O
from tests import cases


def test_collocation_points_match_the_published_values():
    # Gauss-Legendre and Radau IIA points on (0, 1] (the values casadi.collocation_points returns)
    np.testing.assert_allclose(CO.collocation_points(4, "legendre"),
                               [0.0694318442029737, 0.3300094782075719, 0.6699905217924281, 0.9305681557970263],
                               rtol=1e-13)
    np.testing.assert_allclose(CO.collocation_points(3, "radau"), [0.1550510257216822, 0.6449489742783178, 1.0],
                               rtol=1e-13)
    np.testing.assert_allclose(CO.collocation_points(1, "radau"), [1.0])
    np.testing.assert_allclose(CO.collocation_points(1, "legendre"), [0.5])


@pytest.mark.parametrize("method", ["legendre", "radau"])
@pytest.mark.parametrize("d", [1, 2, 3, 4, 5])
def test_coefficients_differentiate_and_extrapolate_polynomials_exactly(d, method):
    tau, C, D = CO.coefficients(d, method)
    rng = np.random.default_rng(d)
    p = np.poly1d(rng.standard_normal(d + 1))  # degree d
    vals = p(tau)
    np.testing.assert_allclose(vals @ C, p.deriv()(tau), rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(vals @ D, p(1.0), rtol=1e-12)


def _col_problem(name, d=3, method="legendre", N=None, objective=None):
    stims = [0.0, 0.1, 0.2, 0.3, 0.4]
    base = cases.oracle_problem(name, stims, 0.5, 4, scheme="RK1", m=1, n_shooting=N, objective=objective)
    return CO.ColProblem(**{f: getattr(base, f) for f in base.__dataclass_fields__}, degree=d, method=method)


def _random_v(pb, B, seed):
    base = cases.random_decision(O.Problem(**{f: getattr(pb, f) for f in O.Problem.__dataclass_fields__}), B, seed)
    X, U, P = O.Problem.unpack(O.Problem(**{f: getattr(pb, f) for f in O.Problem.__dataclass_fields__}), base)
    rng = np.random.default_rng(seed + 1)
    XC = np.repeat(X[:, :-1, None, :], pb.degree + 1, axis=2) * rng.uniform(0.8, 1.2, (B, pb.n_shooting,
                                                                                          pb.degree + 1, pb.nx))
    return pb.pack(XC, X[:, -1], U if pb.nu else None, P if pb.n_params else None)


@pytest.mark.parametrize("name", O.MODEL_NAMES)
def test_jacobian_structure_and_values_match_complex_step_of_g(name):
    pb = _col_problem(name, d=3)
    v = _random_v(pb, 2, seed=4)
    rows, cols = CO.jac_structure(pb)
    vals = CO.eval_jac_g(pb, v)
    dense = np.zeros((2, pb.ng, pb.nv))
    for b in range(2):
        dense[b, rows, cols] = vals[b]
    h = 1e-30
    for c in range(pb.nv):
        vc = v.astype(np.complex128)
        vc[:, c] += 1j * h
        col = CO.eval_g(pb, vc).imag / h
        np.testing.assert_allclose(dense[:, :, c], col, rtol=1e-12, atol=1e-12 * (1 + np.abs(col).max()))
    assert len(set(zip(rows.tolist(), cols.tolist()))) == len(rows)


@pytest.mark.parametrize("name", ["ding2003", "ding2007_with_fatigue", "hmed2018"])
def test_hessian_matches_differences_of_the_jacobian(name):
    pb = _col_problem(name, d=2, objective={"end_node_tracking": 50.0})
    v = _random_v(pb, 1, seed=8)
    rng = np.random.default_rng(2)
    lam = rng.standard_normal((1, pb.ng))
    of = np.array([0.7])
    rows, cols = CO.hess_structure(pb)
    vals = CO.hessian_values(pb, v, of, lam)
    H = np.zeros((pb.nv, pb.nv))
    H[rows, cols] = vals[0]
    H = H + np.tril(H, -1).T
    jr, jc = CO.jac_structure(pb)

    def lag_grad(vv):
        J = np.zeros((pb.ng, pb.nv))
        J[jr, jc] = CO.eval_jac_g(pb, vv)[0]
        return of[0] * CO.eval_grad_f(pb, vv)[0] + lam[0] @ J

    ref = np.zeros_like(H)
    for c in range(pb.nv):
        s = 1e-6 * max(1e-3, abs(v[0, c]))
        vp, vm = v.copy(), v.copy()
        vp[0, c] += s
        vm[0, c] -= s
        ref[:, c] = (lag_grad(vp) - lag_grad(vm)) / (2 * s)
    scale = np.abs(ref).max()
    assert np.abs(H - ref).max() <= 1e-5 * scale
    # every non-zero of the reference Hessian is in the structure
    mask = np.zeros_like(H, dtype=bool)
    mask[rows, cols] = True
    mask = mask | mask.T
    assert np.abs(ref[~mask]).max(initial=0.0) <= 1e-6 * scale


@pytest.mark.parametrize("method", ["legendre", "radau"])
def test_collocation_solution_converges_to_the_ode_solution(method):
    """Solve the collocation equations interval by interval from the rest state (0 DOF Ding2003 IVP) and
    compare the node states with a fine RK4 integration: the error falls with the degree."""
    pb0 = _col_problem("ding2003", d=1, method=method, N=20)
    ref = O.ivp_integrate("ding2003", pb0.c, pb0.rows, np.zeros((pb0.n_shooting, 0)), pb0.final_time, "RK4", 200)
    ref_nodes = ref[:, ::200]
    errs = []
    for d in (1, 2, 3, 4, 5):
        pb = _col_problem("ding2003", d=d, method=method, N=20)
        tau, C, D = CO.coefficients(d, method)
        x = np.zeros(2)
        nodes = [x]
        for k in range(pb.n_shooting):
            def residual(z, k=k, x=x):
                XC = np.concatenate([x, z]).reshape(d + 1, 2)
                out = []
                for j in range(1, d + 1):
                    t = k * pb.dt + tau[j] * pb.dt
                    f = O.rhs("ding2003", pb.c, t, XC[j][:, None], None, pb.rows[k][:, None])[:, 0]
                    out.append(C[:, j] @ XC - pb.dt * f)
                return np.concatenate(out)

            z = fsolve(residual, np.tile(x, d), xtol=1e-14)
            XC = np.concatenate([x, z]).reshape(d + 1, 2)
            x = D @ XC
            nodes.append(x)
        errs.append(np.abs(np.array(nodes).T - ref_nodes).max())
    assert all(b < a for a, b in zip(errs, errs[1:])) and errs[-1] < errs[0] / 20, errs
