"""Receding-horizon control (cocofest_amd/nmpc.py) on the CPU with the oracle as evaluator: window shifting,
stimulation history and the Hmed history intensities are checked against single forward integrations of the
whole committed horizon."""

import numpy as np
import pytest

from oracle import fes_oracle as O
from tests.oracle_handle import DenseBandSolver, OracleHandle, oracle_problem_from_ocp

CYCLE = [0.0, 0.1, 0.2]  # three pulses per 0.5 s cycle


def _nmpc(model, **kw):
    from cocofest_amd import OdeSolver
    from cocofest_amd.nmpc import FesNmpc
    from cocofest_amd.solver import IpmOptions

    return FesNmpc(model, cycle_duration=0.5, n_cycles_simultaneous=2, n_cycles_to_advance=1,
                   ode_solver=OdeSolver.RK4(n_integration_steps=5), options=IpmOptions(tol=1e-9),
                   evaluator=lambda ocp, B: OracleHandle(oracle_problem_from_ocp(ocp), B), band=DenseBandSolver(),
                   torch_device="cpu", **kw)


def _forward(name, stims, n_cycles, T, controls=None, x0=None):
    c = O.model_constants(name)
    N = 10 * n_cycles // 2
    tab = O.stim_table(stims, N, 0.5 * n_cycles, T)
    u = np.zeros((N, 0)) if controls is None else controls(tab, N)
    return O.ivp_integrate(name, c, tab.rows, u, 0.5 * n_cycles, "RK4", 5, x0=x0)[:, ::5]


def test_zero_dof_nmpc_equals_one_long_integration():
    """Ding2003 (no controls): every window's optimum is the forward integration from its start state with its
    stimulation history, so the committed horizon is one long integration with every pulse."""
    from cocofest_amd import DingModelFrequency

    model = DingModelFrequency(stim_time=CYCLE, sum_stim_truncation=4)
    res = _nmpc(model, objective={"end_node_tracking": 50.0}, batch=1).solve(n_cycles=3)
    assert all(c.all() for c in res.converged)
    stims = [t + 0.5 * c for c in range(3) for t in CYCLE]
    np.testing.assert_allclose(res.stim_time, stims)
    ref = _forward("ding2003", stims, 3, 4)
    got = np.stack([res.states["Cn"][0], res.states["F"][0]])
    np.testing.assert_allclose(res.time, np.linspace(0, 1.5, 16), atol=1e-12)
    np.testing.assert_allclose(got, ref, rtol=1e-7, atol=1e-7)


def test_hmed_fixed_intensities_with_history_equal_one_long_integration():
    """Hmed2018 with every intensity fixed (0 DOF): the history intensities carried from window to window must
    reproduce the long integration in which every pulse has that intensity."""
    from cocofest_amd import DingModelPulseIntensityFrequency

    model = DingModelPulseIntensityFrequency(stim_time=CYCLE, sum_stim_truncation=4)
    res = _nmpc(model, pulse_intensity={"fixed": 80.0}, objective={"end_node_tracking": 50.0}, batch=2).solve(
        n_cycles=3)
    assert all(c.all() for c in res.converged)
    stims = [t + 0.5 * c for c in range(3) for t in CYCLE]
    ref = _forward("hmed2018", stims, 3, 4, controls=lambda tab, N: np.full((N, 4), 80.0))
    for b in range(2):
        got = np.stack([res.states["Cn"][b], res.states["F"][b]])
        np.testing.assert_allclose(got, ref, rtol=1e-7, atol=1e-7)
    np.testing.assert_allclose(res.pulse_intensity, 80.0)


@pytest.mark.parametrize("fatigue", [False])  # the fatigue variant runs on the GPU (test_gpu_parity.py)
def test_hmed_free_intensities_are_self_consistent(fatigue, batch=1, nmpc_factory=None):
    """Hmed2018 intensities optimised per window (end-force tracking): every window converges, intensities stay
    in their bounds, and integrating the committed intensities from rest reproduces the committed states."""
    from cocofest_amd import DingModelPulseIntensityFrequency, DingModelPulseIntensityFrequencyWithFatigue

    cls = DingModelPulseIntensityFrequencyWithFatigue if fatigue else DingModelPulseIntensityFrequency
    name = "hmed2018_with_fatigue" if fatigue else "hmed2018"
    model = cls(stim_time=CYCLE, sum_stim_truncation=4)
    res = (nmpc_factory or _nmpc)(model, pulse_intensity={"max": 130}, objective={"end_node_tracking": 40.0},
                                  batch=batch).solve(n_cycles=3)
    assert all(c.all() for c in res.converged), res.iterations
    imin = O.min_pulse_intensity(O.model_constants(name))
    assert res.pulse_intensity.min() >= imin - 1e-8 and res.pulse_intensity.max() <= 130 + 1e-8
    stims = [t + 0.5 * c for c in range(3) for t in CYCLE]
    for b in range(batch):
        I = res.pulse_intensity[b]

        def controls(tab, N, I=I):
            # row k holds the last T pulses <= t_k; placeholder slots contribute nothing (any value)
            out = np.empty((N, 4))
            for k in range(N):
                idx = [i for i, t in enumerate(stims) if t <= k * 0.1 + 1e-12][-4:]
                vals = [I[i] for i in idx]
                out[k] = [50.0] * (4 - len(vals)) + vals
            return out

        ref = _forward(name, stims, 3, 4, controls=controls)
        got = np.stack([res.states[k][b] for k in model.name_dof])
        np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6)


def test_msk_nmpc_window_history_matches_one_long_transcription():
    """NmpcFesMsk's window stimulation tables (update_stim, fes_ocp_dynamics_nmpc_cyclic.py:34-46): a window that
    starts after k committed cycles sees, interval for interval, the stim rows of one long transcription shifted by k
    cycles, and every state of its node 0 is fixed (the per-scenario start values go in at solve time)."""
    import cocofest_amd as C
    from tests import msk_cases as MC

    mm = C.FesMskModel(biorbd_path=MC.biomod_path("arm26_biceps_triceps"),
                       muscles_model=[C.DingModelPulseWidthFrequencyWithFatigue(muscle_name=n, sum_stim_truncation=4)
                                      for n in ("BIClong", "TRIlong")],
                       stim_time=[0.0, 0.1, 0.2, 0.3, 0.4], activate_force_length_relationship=True,
                       activate_force_velocity_relationship=True)
    nm = C.NmpcFesMsk.prepare_nmpc(model=mm, cycle_duration=0.5, n_cycles_simultaneous=2, n_cycles_to_advance=1,
                                   msk_info={"bound_type": "start", "bound_data": [0, 5]},
                                   objective={"minimize_muscle_fatigue": True})
    assert nm.n_shooting == 10 and nm.cycle_len == 5
    long_m = C.FesMskModel(biorbd_path=MC.biomod_path("arm26_biceps_triceps"),
                           muscles_model=[C.DingModelPulseWidthFrequencyWithFatigue(muscle_name=n,
                                                                                     sum_stim_truncation=4)
                                          for n in ("BIClong", "TRIlong")],
                           stim_time=[round(0.1 * i, 1) for i in range(20)])
    long = C.OcpFesMsk.prepare_ocp(model=long_m, final_time=2.0, n_shooting=20,
                                   msk_info={"bound_type": "start", "bound_data": [0, 5]})
    for k in range(3):  # history after k committed cycles (relative to the window start)
        past = [round(0.1 * i - 0.5 * k, 10) for i in range(5 * k)][-4:]
        hist = [-1e7] * (4 - len(past)) + past
        w = nm._window_ocp(hist)
        rows = np.asarray(w.stim_rows)[:10]  # the intervals' rows (node N's row drives no interval)
        ref = np.asarray(long.stim_rows)[5 * k: 5 * k + 10] - 0.5 * k
        pad = ref < -1e6
        assert np.allclose(rows[~pad], ref[~pad], atol=1e-12, rtol=0), k
        assert np.all(rows[pad] < -1e6)
        lo, hi = w.x_bounds
        assert np.array_equal(lo[:, 0], hi[:, 0])
    assert nm.model.muscles_dynamics_model[0].stim_time == [0.0, 0.1, 0.2, 0.3, 0.4]  # the caller's model untouched
    with pytest.raises(NotImplementedError):
        C.NmpcFesMsk.prepare_nmpc(model=mm, cycle_duration=0.5, n_cycles_simultaneous=2, n_cycles_to_advance=1,
                                  pulse_intensity={"min": 20})
    with pytest.raises(ValueError):
        C.NmpcFesMsk(mm, cycle_duration=0.3)


def test_solve_fes_nmpc_driver_entry_and_update_functions():
    """FesNmpc.solve_fes_nmpc (fes_nmpc.py:150-192): the update function decides when to stop (bioptim's
    `update_functions(nmpc, cycle_idx, sol)`), the Solver.IPOPT options reach every window's interior point."""
    from cocofest_amd import DingModelFrequency, Solver

    model = DingModelFrequency(stim_time=CYCLE, sum_stim_truncation=4)
    calls = []

    def update_functions(nmpc, cycle_idx, sol):
        calls.append(cycle_idx)
        return cycle_idx < 2

    res = _nmpc(model, objective={"end_node_tracking": 50.0}, batch=1).solve_fes_nmpc(
        update_functions, solver=Solver.IPOPT(_max_iter=40, _tol=1e-9), total_cycles=10)
    assert calls == [1, 2] and len(res.converged) == 2 and all(c.all() for c in res.converged)
    assert max(int(i.max()) for i in res.iterations) <= 40
    assert res.states["F"].shape == (1, 2 * 5 + 1) and not np.isnan(res.states["F"]).any()
    assert list(res.stopped_at) == [-1]
    ref = _forward("ding2003", [t + 0.5 * c for c in range(2) for t in CYCLE], 2, 4)
    np.testing.assert_allclose(res.states["F"][0], ref[1], rtol=1e-7, atol=1e-7)


def test_max_consecutive_failing_stops_each_scenario():
    """max_consecutive_failing = 3 (the reference's default, fes_nmpc.py:158): with an interior point capped at one
    iteration every window fails, so each scenario stops at its third window, which is not committed (NaN), and
    the loop ends there instead of running the 6 requested cycles."""
    from cocofest_amd import DingModelPulseIntensityFrequency, Solver

    model = DingModelPulseIntensityFrequency(stim_time=CYCLE, sum_stim_truncation=4)
    res = _nmpc(model, pulse_intensity={"max": 130}, objective={"end_node_tracking": 40.0}, batch=2).solve_fes_nmpc(
        lambda nmpc, k, sol: True, solver=Solver.IPOPT(_max_iter=1), total_cycles=6, max_consecutive_failing=3)
    assert len(res.converged) == 3 and not any(c.any() for c in res.converged)
    assert list(res.stopped_at) == [2, 2]
    F = res.states["F"]
    assert F.shape == (2, 3 * 5 + 1)
    assert not np.isnan(F[:, : 2 * 5 + 1]).any() and np.isnan(F[:, 2 * 5 + 1:]).all()
    assert np.isnan(res.pulse_intensity[:, 2 * len(CYCLE):]).all()


def test_solver_ipopt_facade():
    """Solver.IPOPT keeps bioptim's private option names and setters; unknown options are refused."""
    from cocofest_amd import IpmOptions, Solver
    from cocofest_amd.solver import apply_solver

    s = Solver.IPOPT(show_online_optim=False, _max_iter=77, _tol=1e-8, _hessian_approximation="limited-memory",
                     _print_level=0, _linear_solver="ma57")
    s.set_limited_memory_max_history(9)
    o = apply_solver(IpmOptions(), s)
    assert (o.max_iter, o.tol, o.hessian_approximation, o.limited_memory_max_history) == (77, 1e-8, "limited-memory", 9)
    s.set_maximum_iterations(5)
    s.set_tol(1e-4)
    assert (s.max_iter, s.tol) == (5, 1e-4)
    with pytest.raises(TypeError):
        Solver.IPOPT(_max_itr=3)
    with pytest.raises(ValueError):
        Solver.IPOPT(_hessian_approximation="bfgs")
