"""The batched interior-point driver (cocofest_amd/solver.py) on the CPU, with the oracle as evaluator."""

import numpy as np
import pytest

from oracle import fes_oracle as O
from tests import cases
from tests.oracle_handle import DenseBandSolver, OracleHandle


def _ipm(cfg, batch, **opts):
    from cocofest_amd.solver import BatchedIpm, IpmOptions

    ocp = cases.product_ocp(**cfg)
    pb = cases.oracle_problem(**cfg)
    ipm = BatchedIpm(ocp, batch=batch, options=IpmOptions(**opts), handle=OracleHandle(pb, batch), torch_device="cpu",
                     band=DenseBandSolver())
    return ocp, pb, ipm


def test_zero_dof_problem_converges_to_forward_integration():
    """cfg 2 (reference N = 10): 0 DOF, so the optimum is the RK1 x 10 forward integration from rest."""
    cfg = cases.cfg2(n_shooting=None)
    ocp, pb, ipm = _ipm(cfg, batch=2, tol=1e-8)
    rng = np.random.default_rng(0)
    v0 = np.tile(ocp.initial_guess_vector(), (2, 1))
    v0[1] += rng.uniform(0, 5, pb.nv)  # a second, perturbed start
    res = ipm.solve(v0)
    assert res.converged.all(), res.kkt_error
    c = O.model_constants("ding2003")
    traj = O.ivp_integrate("ding2003", c, pb.rows, np.zeros((pb.n_shooting, 0)), 1.0, "RK1", 10)
    X, _, _ = pb.unpack(res.v)
    for b in range(2):
        np.testing.assert_allclose(X[b].T, traj[:, ::10], rtol=1e-7, atol=1e-8)


def test_pulse_width_problem_reaches_a_kkt_point():
    """A small Ding2007 pulse-width problem with an end-force target: converged, feasible, bounds respected."""
    cfg = dict(name="ding2007", stims=[0.0, 0.05, 0.1, 0.15], final_time=0.2, truncation=4, scheme="RK1", m=5,
               objective={"end_node_tracking": 30}, n_shooting=None)
    ocp, pb, ipm = _ipm(cfg, batch=1)
    res = ipm.solve()
    assert res.converged.all(), res.kkt_error
    assert np.max(np.abs(O.eval_g(pb, res.v))) < 1e-6
    lb, ub = ocp.bounds_vector()
    assert np.all(res.v >= lb - 1e-9) and np.all(res.v <= ub + 1e-9)
    X, U, _ = pb.unpack(res.v)
    assert abs(X[0, -1, 1] - 30) < 1.0  # reachable target: the end force is driven to it


def test_zero_initial_guess_needs_multiplier_init_and_restoration():
    """cfg 2 from the reference's default initial guess (all states 0, on their lower bounds): converges to the
    forward integration (least-squares multipliers + restoration steps when the filter search fails)."""
    cfg = cases.cfg2()
    ocp, pb, ipm = _ipm(cfg, batch=1)
    res = ipm.solve()
    assert res.converged.all(), (res.kkt_error, res.iterations)
    c = O.model_constants("ding2003")
    traj = O.ivp_integrate("ding2003", c, pb.rows, np.zeros((pb.n_shooting, 0)), 1.0, "RK1", 10)
    X, _, _ = pb.unpack(res.v)
    np.testing.assert_allclose(X[0].T, traj[:, ::10], rtol=1e-6, atol=1e-6)


def _scipy_reference(ocp, pb):
    """The same NLP solved by an independent solver (scipy trust-constr, exact g / J_g / f / grad f from the
    oracle): the Ipopt stand-in for 'Ipopt-equivalent' optima (Ipopt / CasADi are not installable here)."""
    from scipy.optimize import Bounds, NonlinearConstraint, minimize

    lb, ub = ocp.bounds_vector()
    free = lb != ub
    sc = np.where(ub[free] - lb[free] < 1, ub[free] - lb[free], 1.0)
    jr, jc = O.jac_structure(pb)

    def full(y):
        v = lb.copy()
        v[free] = y * sc
        return v[None]

    def dG(y):
        J = np.zeros((pb.ng, pb.nv))
        J[jr, jc] = O.eval_jac_g(pb, full(y))[0]
        return J[:, free] * sc

    x0 = np.clip(ocp.initial_guess_vector()[free], lb[free], ub[free]) / sc
    r = minimize(lambda y: O.eval_f(pb, full(y))[0], x0, jac=lambda y: O.eval_grad_f(pb, full(y))[0][free] * sc,
                 method="trust-constr", constraints=[NonlinearConstraint(lambda y: O.eval_g(pb, full(y))[0], 0, 0,
                                                                         jac=dG)],
                 bounds=Bounds(lb[free] / sc, ub[free] / sc), options=dict(gtol=1e-12, xtol=1e-14, maxiter=5000))
    return full(r.x)[0], r


@pytest.mark.parametrize("name", ["ding2007", "hmed2018"])
def test_interior_point_matches_an_independent_nlp_solver(name):
    """Force tracking with 4 pulses (pulse widths / intensities free): the batched interior point and scipy's
    trust-constr reach the same KKT point (decision vectors within 1e-8 relative, same objective)."""
    import warnings

    t = np.linspace(0, 1, 11)
    cfg = dict(name=name, stims=[0.0, 0.05, 0.1, 0.15], final_time=0.2, truncation=4, scheme="RK1", m=5,
               objective={"force_tracking": [t, 40 * t]}, n_shooting=None)
    ocp, pb, ipm = _ipm(cfg, batch=1, tol=1e-10)
    res = ipm.solve()
    assert res.converged.all()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ref, r = _scipy_reference(ocp, pb)
    np.testing.assert_allclose(res.f[0], r.fun, rtol=1e-9)
    scale = np.maximum(np.abs(ref), 1e-3 * np.abs(ref).max())
    scale = np.where(np.abs(ref) < 1e-2, np.abs(ref) + 1e-6, scale)  # pulse widths ~1e-4 s
    assert np.max(np.abs(res.v[0] - ref) / scale) < 1e-6


def test_segment_sum_matches_index_add():
    """The KKT assembly's fixed gather-sum (no atomics) adds every source into its position like index_add_,
    duplicates included, and is bitwise reproducible."""
    import torch

    from cocofest_amd.solver import _SegmentSum

    rng = np.random.default_rng(0)
    idx = rng.integers(0, 40, 300)
    src = torch.as_tensor(rng.standard_normal((5, 300)))
    seg = _SegmentSum(torch, idx, torch.device("cpu"))
    got = seg.add_(torch.ones((5, 50), dtype=torch.float64), src)
    ref = torch.ones((5, 50), dtype=torch.float64).index_add_(1, torch.as_tensor(idx), src)
    torch.testing.assert_close(got, ref, rtol=1e-13, atol=1e-13)
    again = seg.add_(torch.ones((5, 50), dtype=torch.float64), src)
    assert torch.equal(got, again)


def test_safe_slacks_and_watchdog_keep_the_end_game_short():
    """Near the optimum of the Hmed force-tracking case (tol 1e-10, mu -> 1e-11) the fraction-to-the-boundary step
    lands intensities exactly on I_min in floating point: without Ipopt's safe slacks (slack_move bound moves) the
    barrier is +inf there and every iteration halves its step (159 iterations); with them, and the watchdog for
    the shortened-step streaks that remain, the solve ends in a few dozen."""
    t = np.linspace(0, 1, 11)
    cfg = dict(name="hmed2018", stims=[0.0, 0.05, 0.1, 0.15], final_time=0.2, truncation=4, scheme="RK1", m=5,
               objective={"force_tracking": [t, 40 * t]}, n_shooting=None)
    ocp, pb, ipm = _ipm(cfg, batch=1, tol=1e-10)
    res = ipm.solve()
    assert res.converged.all() and res.iterations[0] <= 60, res.iterations
    lb, ub = ocp.bounds_vector()
    # the iterate is returned as it is (honor_original_bounds off, Ipopt 3.14's default): within the bounds up to the
    # safe slacks' move eps^(3/4) max(1, |bound|)
    mv = 2e-12 * np.maximum(1.0, np.abs(np.where(np.isfinite(lb), lb, 0.0)))
    mvu = 2e-12 * np.maximum(1.0, np.abs(np.where(np.isfinite(ub), ub, 0.0)))
    assert np.all(res.v[0] >= lb - mv) and np.all(res.v[0] <= ub + mvu)


def test_restoration_phase_reduces_the_infeasibility():
    """Ipopt's restoration phase (BatchedIpm._restoration_phase, the specification of cfx_ipm's k_rs_* kernels) run
    directly from badly infeasible points of a Ding2007 pulse-width problem: each instance leaves it successfully with
    ||c||_1 <= required_infeasibility_reduction * ||c||_1 at the start, inside the bounds, with positive bound
    multipliers; the closed-form p, n of its start satisfy c - p + n = 0 and 2 rho = mu / p + mu / n."""
    import torch

    cfg = dict(name="ding2007", stims=[0.0, 0.05, 0.1, 0.15], final_time=0.2, truncation=4, scheme="RK1", m=5,
               objective={"end_node_tracking": 30}, n_shooting=None)
    B = 3
    ocp, pb, ipm = _ipm(cfg, batch=B, tol=1e-8, restoration="phase")
    rng = np.random.default_rng(4)
    lb, ub = ocp.bounds_vector()
    v = np.tile(ocp.initial_guess_vector(), (B, 1))
    free = lb != ub
    v[:, free] = np.clip(v[:, free] + rng.uniform(0, 1, (B, free.sum())) * np.minimum(ub[free] - lb[free], 50.0),
                         lb[free], ub[free])
    # the solver's state at such a point, as solve() sets it up
    vt = torch.as_tensor(v)
    ipm._set_function_scaling(vt)
    ipm._v_template = vt.clone()
    x = vt[:, ipm.freeT] / ipm.d
    lbF, ubF = ipm.lbF.expand(B, -1).clone(), ipm.ubF.expand(B, -1).clone()
    ipm._lbI, ipm._ubI = lbF, ubF
    x = torch.where(ipm.hasL, torch.maximum(x, lbF + 1e-2), x)
    x = torch.where(ipm.hasU, torch.minimum(x, ubF - 1e-2), x)
    mu = torch.full((B,), 0.1, dtype=torch.float64)
    zl = torch.where(ipm.hasL, mu[:, None] / (x - lbF), torch.zeros_like(x))
    zu = torch.where(ipm.hasU, mu[:, None] / (ubF - x), torch.zeros_like(x))
    g, _, f, _ = ipm._scaled_all(ipm._full(x))
    theta = g.abs().sum(1)
    phi = ipm._barrier_obj(f, x, mu)
    filt = torch.full((B, 64, 2), np.inf, dtype=torch.float64)
    filt[:, :, 1] = -np.inf
    on = torch.ones((B,), dtype=torch.bool)
    xr, zl2, zu2, filt2, fpos2, its, rexit = ipm._restoration_phase(on, x, zl, zu, g, theta, phi, mu,
                                                                    torch.full((B,), 0.99, dtype=torch.float64), filt,
                                                                    torch.zeros((B,), dtype=torch.int64),
                                                                    torch.zeros((B,), dtype=torch.int64))
    gr, _ = ipm._scaled_gf(ipm._full(xr))
    assert torch.all(its >= 1)
    assert torch.all(rexit == ipm.RS_OK)
    assert torch.all(gr.abs().sum(1) <= 0.9 * theta), (gr.abs().sum(1), theta)
    assert torch.all(xr[:, ipm.hasL] > lbF[:, ipm.hasL]) and torch.all(xr[:, ipm.hasU] < ubF[:, ipm.hasU])
    assert torch.all(zl2[:, ipm.hasL] > 0) and torch.all(zu2[:, ipm.hasU] > 0)
    assert torch.all(fpos2 == 1)  # the starting point entered the original filter
    # Ipopt's closed-form relaxation of the start (restated in k_rs_init / rs_pn)
    c = g
    muR = torch.maximum(mu, c.abs().amax(1))[:, None]
    rho = ipm.opt.resto_penalty
    s = torch.hypot(muR, rho * c)
    n = torch.where(c > 0, (muR + muR * muR / (s + rho * c)) / (2 * rho), (muR - rho * c + s) / (2 * rho))
    p = torch.where(c < 0, (muR + muR * muR / (s - rho * c)) / (2 * rho), (muR + rho * c + s) / (2 * rho))
    assert torch.all(p > 0) and torch.all(n > 0)
    np.testing.assert_allclose((c - p + n).numpy(), 0.0, atol=1e-12 * float(c.abs().max()))
    np.testing.assert_allclose((muR / p + muR / n).numpy(), 2 * rho, rtol=1e-10)
    ipm.close()


def test_filter_reset_heuristic():
    """Ipopt's filter reset heuristic (off by default here): with a trigger of one iteration the filter is cleared
    whenever the line search's last rejection was the filter's, at most max_filter_resets times; cfg 2 from the zero
    initial guess (a long backtracking line search) still reaches the forward integration.  Solver.IPOPT maps
    bioptim-style option names onto it."""
    from cocofest_amd.solver import IpmOptions, Solver

    cfg = cases.cfg2()
    _, pb, ipm = _ipm(cfg, batch=1, filter_reset_trigger=1, max_filter_resets=3)
    res = ipm.solve()
    assert res.converged.all(), (res.kkt_error, res.iterations)
    assert 1 <= int(ipm.filter_resets[0]) <= 3, ipm.filter_resets
    c = O.model_constants("ding2003")
    traj = O.ivp_integrate("ding2003", c, pb.rows, np.zeros((pb.n_shooting, 0)), 1.0, "RK1", 10)
    X, _, _ = pb.unpack(res.v)
    np.testing.assert_allclose(X[0].T, traj[:, ::10], rtol=1e-6, atol=1e-6)
    _, _, off = _ipm(cfg, batch=1)
    off.solve()
    assert int(off.filter_resets[0]) == 0  # the default: off
    o = Solver.IPOPT(_filter_reset_trigger=2, _max_filter_resets=5).apply(IpmOptions())
    assert (o.filter_reset_trigger, o.max_filter_resets) == (2, 5)


def test_soft_restoration_steps():
    """Ipopt's soft restoration (IpmOptions.soft_resto_pderror_reduction_factor, Ipopt's TrySoftRestoStep) on cfg 2 from
    the zero guess and 7 starts perturbed by 30 % of each range: failed line searches take soft steps (primal and dual
    at the fraction to the boundary, accepted by the filter or by a primal-dual error decrease), and every start still
    reaches the forward integration, as without them."""
    cfg = cases.cfg2()
    out = {}
    for fac in (0.0, 0.9999):
        ocp, pb, ipm = _ipm(cfg, batch=8, soft_resto_pderror_reduction_factor=fac, max_iter=300)
        rng = np.random.default_rng(1)
        v0 = np.tile(ocp.initial_guess_vector(), (8, 1))
        lb, ub = ocp.bounds_vector()
        free = lb != ub
        span = np.minimum(np.where(np.isfinite(ub - lb), ub - lb, 10.0), 10.0)[free]
        v0[1:, free] = np.clip(v0[1:, free] + 0.3 * rng.uniform(-1, 1, (7, free.sum())) * span, lb[free], ub[free])
        out[fac] = (ipm.solve(v0), ipm.soft_steps)
    (r0, n0), (r1, n1) = out[0.0], out[0.9999]
    assert n0 == 0 and n1 > 0, (n0, n1)
    assert r0.converged.all() and r1.converged.all()
    np.testing.assert_allclose(r1.f, r0.f, rtol=1e-8)
    np.testing.assert_allclose(r1.v, r0.v, rtol=1e-6, atol=1e-6)


def test_soft_restoration_options_are_validated():
    from cocofest_amd.solver import IpmOptions, Solver, apply_solver

    with pytest.raises(ValueError):
        IpmOptions(soft_resto_pderror_reduction_factor=-1.0)
    with pytest.raises(ValueError):
        IpmOptions(max_soft_resto_iters=-1)
    o = apply_solver(IpmOptions(), Solver.IPOPT(_soft_resto_pderror_reduction_factor=0.9999, _max_soft_resto_iters=3))
    assert (o.soft_resto_pderror_reduction_factor, o.max_soft_resto_iters) == (0.9999, 3)


@pytest.mark.parametrize("restart", [False, True])
def test_failed_restoration_stops_or_restarts(restart):
    """An infeasible instance (cfg 2 with its fixed initial force at 5,000 N: every later force exceeds its 1,000 N
    bound) beside a feasible one.  With Ipopt's exits its restoration phase ends it (Infeasible_Problem_Detected or
    Restoration_Failed); with the resto_failure_restart extension a failed phase sends it back to the main iteration
    instead, so it never ends with Restoration_Failed.  The feasible instance converges to the same point either way."""
    cfg = cases.cfg2()
    ocp, pb, ipm = _ipm(cfg, batch=2, tol=1e-8, max_iter=120, resto_failure_restart=restart)
    lb, ub = ocp.bounds_vector()
    fixed = np.tile(lb[lb == ub], (2, 1))
    fixed[1, 1] = 5000.0
    res = ipm.solve(np.tile(ocp.initial_guess_vector(), (2, 1)), fixed_values=fixed)
    assert res.converged[0] and not res.converged[1], (res.status, res.iterations)
    assert res.status[0] == 0
    if restart:
        assert res.status[1] in (2, -1), res.status
    else:
        assert res.status[1] in (2, -2), res.status
    c = O.model_constants("ding2003")
    traj = O.ivp_integrate("ding2003", c, pb.rows, np.zeros((pb.n_shooting, 0)), 1.0, "RK1", 10)
    X, _, _ = pb.unpack(res.v)
    np.testing.assert_allclose(X[0].T, traj[:, ::10], rtol=1e-6, atol=1e-6)


def test_unscaled_termination_tests():
    """Ipopt's termination also checks the UNSCALED problem (IpOptErrorConv: constr_viol_tol, dual_inf_tol,
    compl_inf_tol beside tol on the scaled error).  A complementarity tolerance below anything an interior point
    reaches (its s z stay positive) keeps the solver iterating past its scaled convergence, here until max_iter, at
    the same point; Solver.IPOPT maps the options and IpmOptions validates them."""
    from cocofest_amd.solver import IpmOptions, Solver, apply_solver

    cfg = cases.cfg2(n_shooting=None)
    ocp, pb, ipm = _ipm(cfg, batch=1, tol=1e-6)
    base = ipm.solve()
    assert base.converged.all() and base.status[0] == 0
    it0 = int(base.iterations[0])
    ocp, pb, tight = _ipm(cfg, batch=1, tol=1e-6, compl_inf_tol=1e-300, acceptable_compl_inf_tol=1e-300,
                          max_iter=it0 + 5)
    res = tight.solve()
    assert not res.converged[0] and res.status[0] == -1 and int(res.iterations[0]) == it0 + 5, (res.status,
                                                                                                  res.iterations)
    np.testing.assert_allclose(res.v, base.v, rtol=1e-6, atol=1e-6)  # it stays at the optimum meanwhile
    for k in ("constr_viol_tol", "dual_inf_tol", "compl_inf_tol", "acceptable_constr_viol_tol",
              "acceptable_dual_inf_tol", "acceptable_compl_inf_tol"):
        with pytest.raises(ValueError):
            IpmOptions(**{k: 0.0})
    o = apply_solver(IpmOptions(), Solver.IPOPT(_constr_viol_tol=1e-6, _dual_inf_tol=0.5, _compl_inf_tol=1e-5))
    assert (o.constr_viol_tol, o.dual_inf_tol, o.compl_inf_tol) == (1e-6, 0.5, 1e-5)


# ---- Ipopt's adaptive barrier update and the Ipopt / bioptim solver profile (round 6) -------------------------------
# The documented facade defaults (DESIGN.md "Solver profiles"): Ipopt 3.14's defaults where bioptim's Solver.IPOPT leaves
# them, bioptim's values where it sets them (recalled: external/bioptim is empty in the reference tree).
SOLVER_IPOPT_DEFAULTS = dict(
    tol=1e-6, max_iter=1000, acceptable_tol=1e-6, acceptable_iter=15, mu_init=0.1, mu_strategy="adaptive",
    mu_oracle="quality-function", adaptive_mu_globalization="obj-constr-filter", mu_max_fact=1000.0, mu_min=1e-11,
    adaptive_mu_monotone_init_factor=0.8, sigma_max=100.0, sigma_min=1e-6, quality_function_max_section_steps=8,
    quality_function_section_sigma_tol=1e-2, quality_function_section_qf_tol=0.0, filter_margin_fact=1e-5,
    filter_max_margin=1.0, mu_change_resets_filter=True, monotone_mu_floor="ipopt", kappa_eps=10.0, kappa_mu=0.2,
    theta_mu=1.5, tau_min=0.99, bound_relax_factor=1e-8, bound_push=1e-2, bound_frac=1e-2,
    bound_mult_init_method="constant", bound_mult_init_val=1.0, honor_original_bounds=False, range_scaling=False,
    nlp_scaling_method="gradient-based", nlp_scaling_max_gradient=100.0, nlp_scaling_min_value=1e-8,
    hessian_approximation="exact", limited_memory_max_history=50, max_soc=4, kappa_soc=0.99,
    watchdog_shortened_iter_trigger=10, watchdog_trial_iter_max=3, max_resto_iter=3_000_000, resto_penalty=1000.0,
    required_infeasibility_reduction=0.9, filter_reset_trigger=5, max_filter_resets=5,
    soft_resto_pderror_reduction_factor=0.9999, max_soft_resto_iters=10, resto_failure_restart=False,
    constr_viol_tol=1e-4, dual_inf_tol=1.0, compl_inf_tol=1e-4, acceptable_constr_viol_tol=1e-2,
    acceptable_dual_inf_tol=1e10, acceptable_compl_inf_tol=1e-2, warm_start_init_point=False,
    warm_start_bound_push=1e-3, warm_start_bound_frac=1e-3, warm_start_mult_bound_push=1e-3, inertia_test=True)


def test_solver_ipopt_defaults_are_ipopts_and_bioptims():
    """Solver.IPOPT() maps onto Ipopt's / bioptim's settings (the table above, DESIGN.md "Solver profiles"); the
    library's tuned set is the opt-in profile "cfx"; bioptim's option names and Ipopt's yes / no strings map; choices
    Ipopt has but this library does not restate raise instead of being ignored."""
    from cocofest_amd.solver import IpmOptions, Solver, native_options

    o = Solver.IPOPT().options()
    for k, v in SOLVER_IPOPT_DEFAULTS.items():
        assert getattr(o, k) == v, (k, getattr(o, k), v)
    lib = Solver.IPOPT(profile="cfx").options()
    ref = IpmOptions(max_iter=1000)  # bioptim's _max_iter in either profile
    assert {k: getattr(lib, k) for k in SOLVER_IPOPT_DEFAULTS} == {k: getattr(ref, k) for k in SOLVER_IPOPT_DEFAULTS}
    assert lib.mu_strategy == "monotone" and lib.range_scaling and lib.bound_relax_factor == 0.0
    o = Solver.IPOPT(_mu_strategy="monotone", _nlp_scaling_method="none", _honor_original_bounds="yes").options()
    assert (o.mu_strategy, o.nlp_scaling_method, o.honor_original_bounds) == ("monotone", "none", True)
    n = native_options(Solver.IPOPT().options())
    assert (n["mu_strategy"], n["nlp_scaling_method"], n["bound_mult_init_method"], n["range_scaling"]) == (1, 1, 0, 0)
    for bad in (dict(_nlp_scaling_method="equilibration-based"), dict(_mu_strategy="probing"),
                dict(_mu_oracle="loqo"), dict(_adaptive_mu_globalization="kkt-error")):
        with pytest.raises(ValueError):
            Solver.IPOPT(**bad)
    with pytest.raises(ValueError):
        IpmOptions(bound_mult_init_method="mu_based")
    with pytest.raises(ValueError):
        Solver.IPOPT(profile="fast")


T11 = np.linspace(0, 1, 11)
SMALL = {
    "d07_track": dict(name="ding2007", stims=[0.0, 0.05, 0.1, 0.15], final_time=0.2, truncation=4, scheme="RK1", m=5,
                      objective={"force_tracking": [T11, 40 * T11]}, n_shooting=None),
    "hmed_track": dict(name="hmed2018", stims=[0.0, 0.05, 0.1, 0.15], final_time=0.2, truncation=4, scheme="RK1", m=5,
                       objective={"force_tracking": [T11, 40 * T11]}, n_shooting=None),
    "d07_end": dict(name="ding2007", stims=[0.0, 0.05, 0.1, 0.15], final_time=0.2, truncation=4, scheme="RK1", m=5,
                    objective={"end_node_tracking": 30}, n_shooting=None),
}


@pytest.mark.parametrize("name,glob", [(n, "obj-constr-filter") for n in sorted(SMALL)] +
                         [("d07_track", "never-monotone-mode"), ("d07_end", "never-monotone-mode")])
def test_adaptive_mu_reaches_the_monotone_optimum(name, glob):
    """The adaptive strategy (quality-function oracle) reaches the monotone strategy's KKT point (same f to 1e-8,
    decision vectors within 1e-6 of their range) on force tracking with free pulse widths / intensities and on an
    end-force target, with Ipopt's default globalisation.  Without one ("never-monotone-mode", which Ipopt offers as
    unsafe) the Hmed case stalls at a scaled error of 2.9e-8 with mu at mu_min, its steps rejected and the watchdog
    returning to the same iterate — so it is run only where it converges here."""
    cfg = SMALL[name]
    _, _, mono = _ipm(cfg, batch=1, tol=1e-8)
    r_m = mono.solve()
    ocp, pb, ad = _ipm(cfg, batch=1, tol=1e-8, mu_strategy="adaptive", adaptive_mu_globalization=glob)
    r_a = ad.solve()
    assert r_m.converged.all() and r_a.converged.all(), (r_a.status, r_a.iterations)
    np.testing.assert_allclose(r_a.f, r_m.f, rtol=1e-8, atol=1e-12)
    lb, ub = ocp.bounds_vector()
    span = np.where(np.isfinite(ub - lb), ub - lb, np.maximum(np.abs(r_m.v).max(0), 1.0))
    if name != "d07_end":  # (an end-force target leaves a flat valley of optimal widths)
        assert np.max(np.abs(r_a.v - r_m.v) / np.maximum(span, 1e-12)) < 1e-6
    assert np.max(np.abs(O.eval_g(pb, r_a.v))) < 1e-6


def test_mu_oracle_minimises_the_quality_function():
    """The oracle's sigma against a dense scan of Ipopt's quality function at a real iterate (the d07_track problem
    after 3 iterations): its value is within 1 % of the scan's minimum over [sigma_min, sigma_max] (golden section on
    a unimodal-enough function), and mu = sigma * average complementarity."""
    import torch

    cfg = SMALL["d07_track"]
    ocp, pb, ipm = _ipm(cfg, batch=1, tol=1e-8, mu_strategy="adaptive", max_iter=3)
    seen = {}
    orig = ipm._mu_oracle

    def spy(sel, sl, su, zl, zu, dxa, dxc, rd2, c2, avg, mu_max):
        mu = orig(sel, sl, su, zl, zu, dxa, dxc, rd2, c2, avg, mu_max)
        seen.update(args=(sel, sl, su, zl, zu, dxa, dxc, rd2, c2, avg, mu_max), mu=mu)
        return mu

    ipm._mu_oracle = spy
    ipm.solve()
    sel, sl, su, zl, zu, dxa, dxc, rd2, c2, avg, mu_max = seen["args"]
    opt = ipm.opt
    hasL, hasU = ipm.hasL, ipm.hasU
    nc = int(hasL.sum()) + int(hasU.sum())

    def q(mu):
        mu = torch.as_tensor([mu], dtype=torch.float64)
        dx = dxa + mu[:, None] * dxc
        z = torch.zeros_like(sl)
        dzl = torch.where(hasL, mu[:, None] / sl - zl - zl / sl * dx, z)
        dzu = torch.where(hasU, mu[:, None] / su - zu + zu / su * dx, z)
        tau = torch.clamp(1.0 - mu, min=opt.tau_min)
        ap = torch.minimum(ipm._max_step(sl, dx, hasL, tau), ipm._max_step(su, -dx, hasU, tau))
        ad = torch.minimum(ipm._max_step(zl, dzl, hasL, tau), ipm._max_step(zu, dzu, hasU, tau))
        cl = torch.where(hasL, (sl + ap[:, None] * dx) * (zl + ad[:, None] * dzl), z)
        cu = torch.where(hasU, (su - ap[:, None] * dx) * (zu + ad[:, None] * dzu), z)
        return float((1 - ad) ** 2 * rd2 / sl.shape[1] + (1 - ap) ** 2 * c2 / ipm.m +
                     ((cl * cl).sum(1) + (cu * cu).sum(1)) / nc)

    a = float(avg[0])
    sig = np.exp(np.linspace(np.log(opt.sigma_min), np.log(min(opt.sigma_max, float(mu_max[0]) / a)), 2000))
    qs = np.array([q(s_ * a) for s_ in sig])
    mu = float(seen["mu"][0])
    assert opt.mu_min <= mu <= float(mu_max[0])
    assert q(mu) <= qs.min() * 1.01 + 1e-300, (q(mu), qs.min(), mu / a, sig[qs.argmin()])


def test_nlp_scaling_method_none_and_filter_reset_on_mu_change():
    """Ipopt's nlp_scaling_method "none" leaves f and g unscaled (s_f = s_g = 1) and reaches the gradient-based run's
    optimum; Ipopt's filter reset whenever mu changes (mu_change_resets_filter, on in the Ipopt profile) also does."""
    cfg = SMALL["d07_track"]
    _, _, base = _ipm(cfg, batch=1, tol=1e-8)
    r0 = base.solve()
    _, _, none = _ipm(cfg, batch=1, tol=1e-8, nlp_scaling_method="none")
    r1 = none.solve()
    assert float(none.sf[0]) == 1.0 and bool((none.sg == 1.0).all())
    assert float(base.sf[0]) < 1.0  # the force-tracking objective's gradient exceeds 100 at the start
    _, _, rst = _ipm(cfg, batch=1, tol=1e-8, mu_change_resets_filter=True, monotone_mu_floor="ipopt")
    r2 = rst.solve()
    for r in (r0, r1, r2):
        assert r.converged.all(), (r.status, r.iterations)
    np.testing.assert_allclose(r1.f, r0.f, rtol=1e-8)
    np.testing.assert_allclose(r2.f, r0.f, rtol=1e-8)
