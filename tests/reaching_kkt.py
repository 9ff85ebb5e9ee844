"""First-order optimality of the reference's stored reaching-task optima (test infrastructure).

The two stored solutions of examples/dynamics/reaching_task/reaching_task_pulse_duration_optimization.py:80-118
(result_file/pulse_duration_minimize_muscle_{fatigue,force}.pkl: bioptim + Ipopt + biorbd, an older revision of the
script; extracted as numbers by tests/golden/extract_reaching_solution.py) are Ipopt KKT points.  Feasibility is checked
in tests/test_reference_solution.py; this module checks STATIONARITY in the stored revision's decision space: per-pulse
pulse-width PARAMETERS p_{m,i} (6 muscles x 60 pulses) — interval k's `last_pulse_width` is the parameter of the pulse
it follows, i.e. tie rows last_pulse_width_k - p_{m,i(k)} = 0 eliminated — no residual torque (`with_residual_torque:
False`, as the script sets it), node states given by the dynamics.  Objectives:

* CustomObjective.minimize_overall_muscle_fatigue (cocofest/custom_objectives.py:77-97) as a Mayer term at Node.END
  (fes_ocp_dynamics.py:675-683): sum_m (a_rest_m / A_m(T))^2, quadratic, weight 1;
* CustomObjective.minimize_overall_muscle_force_production (custom_objectives.py:100-117) as a Lagrange term at
  Node.ALL (fes_ocp_dynamics.py:685-693): sum_k w_k sum_m F_{m,k}^2 — w_k = dt for k < N and ``w_end`` * dt at node N
  (the convention the product recalls includes node N with the same weight: w_end = 1).

Bounds are the reference's (fes_ocp_dynamics.py:453-546, as cocofest_amd.msk builds them); the stored pulse widths sit
at pd0 - 1e-8 and 6e-4 + 1e-8 (Ipopt's bound_relax_factor).  The interval Jacobians come from the plain-C port of the
oracle (oracle/c/fes_msk.c, complex step; numerically the numpy oracle's, test_msk_cpu.py), run with the stored
revision's muscle conventions (``legacy``: fatigue rates x10, calcium sum without a window's first pulse, r0 from Km;
test_reference_solution.py) or the current ones."""

from __future__ import annotations

import numpy as np

from tests import test_reference_solution as R

MUSCLES = R.MUSCLES


def problem(legacy=True):
    pb = R.oracle_problem(legacy=legacy)
    pb.residual = False
    return pb


def product_bounds(objective="fatigue"):
    """Node-state bounds (nx, N+1) and the pulse-width range of the reference's OcpFesMsk for this task (built by
    cocofest_amd.msk on the host; no device needed)."""
    import cocofest_amd as C
    from oracle import fes_oracle as O

    models = []
    for n, c in zip(MUSCLES, R.muscle_constants()):
        mm = C.DingModelPulseWidthFrequencyWithFatigue(muscle_name=n, sum_stim_truncation=R.T)
        for k in ("alpha_a", "alpha_tau1", "alpha_km", "a_scale"):
            setattr(mm, k, c[k])
        models.append(mm)
    model = C.FesMskModel(biorbd_path=str(R.GOLDEN / "biomod_arm26.json"), muscles_model=models, stim_time=R.STIMS,
                          activate_force_length_relationship=True, activate_force_velocity_relationship=True,
                          activate_residual_torque=False)
    ocp = C.OcpFesMsk.prepare_ocp(model=model, final_time=R.FINAL_TIME, n_shooting=R.N,
                                  pulse_width={"min": O.model_constants("ding2007")["pd0"], "max": 0.0006},
                                  objective={f"minimize_muscle_{objective}": True},
                                  msk_info={"with_residual_torque": False, "bound_type": "start_end",
                                            "bound_data": [[0, 5], [0, 5]]},
                                  ode_solver=C.OdeSolver.RK4(n_integration_steps=1))
    xlo, xhi = (np.asarray(b, dtype=float) for b in ocp.x_bounds)
    ulo, uhi = (np.asarray(b, dtype=float) for b in ocp.u_bounds)
    return xlo, xhi, float(ulo.min()), float(uhi.max()), model


def _marker_jacobian(pb, X):
    """d(marker rows) / d q at the marker node, by complex step on the oracle's forward kinematics."""
    from oracle import fes_msk as M

    c = pb.marker_pairs[0]
    q = X[pb.nxm: pb.nxm + pb.nq, c["node"]]
    out = np.empty((len(c["axes"]), pb.nq))
    for j in range(pb.nq):
        qq = q.astype(complex)
        qq[j] += 1e-30j
        d = M.marker_position(pb.bm, c["second"], qq) - M.marker_position(pb.bm, c["first"], qq)
        out[:, j] = np.imag([d[a] for a in c["axes"]]) / 1e-30
    return out


def reduced_stationarity(objective="fatigue", data=None, legacy=True, w_end=1.0, threads=8):
    """First-order optimality in the space of the decisions that remain once the dynamics are solved: the 360
    per-pulse pulse widths p.  The stored states are the forward integration of p (their continuity rows hold to
    1e-12 / 1e-9), so the stored point is a KKT point of the reference's NLP iff

        grad_p f + sum_i nu_i grad_p c_i = z,   z_{m,i} >= 0 at p = pd0, <= 0 at p = 0.6 ms, 0 elsewhere,

    with c the equality rows the dynamics do not satisfy by themselves: the marker superimposition at node 1000 (2)
    and the end posture q_N (2).  The state bounds do not bind in this space (F >= 0 holds along the dynamics).
    Reduced gradients by the discrete adjoint of the RK4 x 1 transcription (lambda_k = dPhi_k/dx^T lambda_{k+1} +
    df/dx_k), the Jacobians from the C port; nu and z by least squares (z signs enforced).  Returns the residual of the
    pulses off their bounds relative to the largest reduced-gradient term."""
    from oracle import c_msk

    d = R.load(data or objective)
    X, U = R.trajectory(d)
    U = U[: len(MUSCLES)]
    pb = problem(legacy)
    N, nx, nxm, nq = R.N, pb.nx, pb.nxm, pb.nq
    v = R.decision_vector(X, U, pb.nz)
    _, J = c_msk.shooting(pb, v[None], want_g=False, threads=threads)
    J = J[0]
    xlo, xhi, pwlo, pwhi, model = product_bounds(objective)
    dt = R.FINAL_TIME / N
    # seeds d(function)/dx_k for the objective and the 4 equality rows
    seeds = np.zeros((N + 1, nx, 5))
    for m, mus in enumerate(model.muscles_dynamics_model):
        if objective == "fatigue":
            seeds[N, 5 * m + 2, 0] = -2.0 * mus.a_rest ** 2 / X[5 * m + 2, N] ** 3
        else:
            w = np.full(N + 1, dt)
            w[N] = w_end * dt
            seeds[:, 5 * m + 1, 0] = 2.0 * w * X[5 * m + 1]
    mk = _marker_jacobian(pb, X)
    seeds[pb.marker_pairs[0]["node"], nxm: nxm + nq, 1:3] = mk.T
    for j in range(nq):
        seeds[N, nxm + j, 3 + j] = 1.0
    lam = seeds[N].copy()
    grad_pw = np.zeros((N, len(MUSCLES), 5))
    for k in range(N - 1, -1, -1):
        grad_pw[k] = J[k][:, nx:].T @ lam
        lam = J[k][:, :nx].T @ lam + seeds[k]
    pidx = R.pulse_index()
    G = np.zeros((len(MUSCLES), int(pidx.max()) + 1, 5))
    for k in range(N):
        G[:, pidx[k]] += grad_pw[k]
    G = G.reshape(-1, 5) * (pwhi - pwlo)  # per unit of the pulse-width range
    P = np.stack([d[f"pulse_duration_{n}"] for n in MUSCLES]).ravel()
    at_lo = P <= pwlo + 1e-12
    at_hi = P >= pwhi - 1e-12
    sign = np.where(at_lo, 1.0, np.where(at_hi, -1.0, 0.0))
    keep = sign != 0
    for _ in range(20):  # least squares for nu (4) and z, wrong-signed z dropped
        idx = np.nonzero(keep)[0]
        A = np.concatenate([G[:, 1:], -np.eye(len(P))[:, idx]], axis=1)
        sol, *_ = np.linalg.lstsq(A, -G[:, 0], rcond=None)
        z = np.zeros(len(P))
        z[idx] = sol[4:]
        wrong = keep & (z * sign < 0)
        if not wrong.any():
            break
        keep &= ~wrong
    res = G[:, 0] + G[:, 1:] @ sol[:4] - z
    free = sign == 0
    scale = np.abs(G[:, 0]).max()
    return {"objective": objective, "data": data or objective, "legacy": legacy, "w_end": w_end,
            "pulses": len(P), "at_bounds": int((~free).sum()), "active_kept": int(keep.sum()),
            "grad_f_max": float(scale), "nu": [float(x) for x in sol[:4]],
            "dual_inf_rel": float(np.abs(res).max() / scale),
            "dual_inf_rel_free": float(np.abs(res[free]).max() / scale) if free.any() else 0.0,
            "dual_inf_rel_free_median": float(np.median(np.abs(res[free])) / scale) if free.any() else 0.0}
