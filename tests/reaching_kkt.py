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


def reduced_stationarity(objective="fatigue", data=None, legacy=True, w_end=1.0, threads=8, _keep=None):
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
    G_seconds = G.reshape(-1, 5).copy()  # per second of pulse width (the stored revision's parameter unit)
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
    if _keep is not None:  # (ipopt_termination_audit's inputs)
        _keep.update(G_seconds=G_seconds, sign=sign, nu_ls=sol[:4].copy(), z_ls=z / (pwhi - pwlo), J=J, X=X, v=v,
                     seeds=seeds, pb=pb, pwlo=pwlo, pwhi=pwhi, P=P, xlo=xlo, xhi=xhi)
    return {"objective": objective, "data": data or objective, "legacy": legacy, "w_end": w_end,
            "pulses": len(P), "at_bounds": int((~free).sum()), "active_kept": int(keep.sum()),
            "grad_f_max": float(scale), "nu": [float(x) for x in sol[:4]],
            "dual_inf_rel": float(np.abs(res).max() / scale),
            "dual_inf_rel_free": float(np.abs(res[free]).max() / scale) if free.any() else 0.0,
            "dual_inf_rel_free_median": float(np.median(np.abs(res[free])) / scale) if free.any() else 0.0}


def adjoint_multipliers(ocp, v, lb, ub, pulse_bounds="all"):
    """Ipopt warm-start multipliers (y, z_l, z_u, report) of the legacy product's NLP at the point v, from the PRODUCT's
    J_g and grad f (libcfx, GPU): the continuity-row multipliers by the discrete adjoint of the RK4 x 1 transcription
    (y_{c_{k-1}} = df/dx_k + A_k^T y_{c_k} + marker terms; free at the fixed end states), the marker and end-state
    multipliers and the per-pulse bound multipliers by least squares over the 360 pulse-width sums with their signs
    enforced (reduced_stationarity's problem), the bound multiplier of each pulse on its first interval
    (pulse_bounds "first", FesMskOcp.bounds_vector) or spread over its copies ("all"), the tie-row multipliers by the
    recursion along each pulse.  NLP rows [N nx continuity | 2 marker rows | tie rows], decision [x_k, u_k]_k, x_N."""
    N, nx, nu = R.N, ocp.nx, ocp.nu
    nz = nx + nu
    h = ocp.nlp(batch=1, layout="aos")
    jr, jc = h.jac_structure()
    jv = h.eval_jac_g(v[None])[0]
    gf = h.eval_grad_f(v[None])[0]
    ng = h.ng
    h.close()
    fixed = lb == ub
    # interval blocks A_k = dPhi_k/dx_k, B_k = dPhi_k/du_k
    cont = jr < N * nx
    k = jr[cont] // nx
    loc = jc[cont] - k * nz
    inb = (loc >= 0) & (loc < nz)
    J = np.zeros((N, nx, nz))
    np.add.at(J, (k[inb], jr[cont][inb] - k[inb] * nx, loc[inb]), jv[cont][inb])
    A, Bu = J[:, :, :nx], J[:, :, nx:]
    # marker rows (N nx, N nx + 1): entries on node MARKER_NODE's states
    mrow = [N * nx, N * nx + 1]
    seeds = []  # (N + 1, nx) seeds of the adjoint recursion
    s0 = np.zeros((N + 1, nx))
    s0[:N] = gf[: N * nz].reshape(N, nz)[:, :nx]
    s0[N] = gf[N * nz: N * nz + nx]
    xN_fixed = fixed[N * nz: N * nz + nx]
    s0[N][xN_fixed] = 0.0
    seeds.append(s0)
    for r in mrow:
        s = np.zeros((N + 1, nx))
        sel = jr == r
        node = jc[sel] // nz
        assert np.all(node == R.MARKER_NODE)
        s[R.MARKER_NODE, jc[sel] - R.MARKER_NODE * nz] = jv[sel]
        seeds.append(s)
    end_idx = np.nonzero(xN_fixed)[0]
    for i in end_idx:
        s = np.zeros((N + 1, nx))
        s[N, i] = 1.0
        seeds.append(s)
    S = np.stack(seeds, axis=-1)  # (N + 1, nx, ns)
    lam = np.zeros((N + 1, nx, S.shape[-1]))  # lam[k] = multiplier of the continuity row into x_k (k >= 1)
    lam[N] = S[N]
    for kk in range(N - 1, 0, -1):
        lam[kk] = S[kk] + A[kk].T @ lam[kk + 1]
    gu = gf[: N * nz].reshape(N, nz)[:, nx:]
    G = np.einsum("kxu,kxs->kus", Bu, lam[1:])  # (N, nu, ns): d/du_k of (f, marker rows, end states) via x
    G[:, :, 0] += gu
    pidx = R.pulse_index()
    npulse = int(pidx.max()) + 1
    Gp = np.zeros((npulse, nu, G.shape[-1]))
    np.add.at(Gp, pidx, G)
    Gp = Gp.reshape(npulse * nu, -1)
    u = v[: N * nz].reshape(N, nz)[:, nx:]
    ulo = lb[: N * nz].reshape(N, nz)[:, nx:]
    uhi = ub[: N * nz].reshape(N, nz)[:, nx:]
    first = np.array([np.nonzero(pidx == p)[0][0] for p in range(npulse)])
    P = u[first].reshape(-1)
    rng_u = (uhi - ulo)[first].reshape(-1)
    tolb = 1e-6 * rng_u
    at_lo = P <= ulo[first].reshape(-1) + tolb
    at_hi = P >= uhi[first].reshape(-1) - tolb
    sign = np.where(at_lo, 1.0, np.where(at_hi, -1.0, 0.0))
    keep = sign != 0
    for _ in range(50):  # least squares for nu and the pulse totals Z, wrong-signed Z dropped (reaching_kkt.py)
        idx = np.nonzero(keep)[0]
        Am = np.concatenate([Gp[:, 1:], -np.eye(len(P))[:, idx]], axis=1)
        sol, *_ = np.linalg.lstsq(Am, -Gp[:, 0], rcond=None)
        Z = np.zeros(len(P))
        Z[idx] = sol[Gp.shape[1] - 1:]
        wrong = keep & (Z * sign < 0)
        if not wrong.any():
            break
        keep &= ~wrong
    nu_ = sol[: Gp.shape[1] - 1]
    resid = Gp[:, 0] + Gp[:, 1:] @ nu_ - Z
    coef = np.concatenate([[1.0], nu_])
    lamc = lam @ coef  # (N + 1, nx)
    y = np.zeros(ng)
    y[: N * nx] = lamc[1:].reshape(-1)
    y[mrow] = nu_[:2]
    # per-interval width multipliers: the pulse total on its first interval (the only one whose bounds bind,
    # FesMskOcp.bounds_vector); tie rows by the recursion along the pulse
    g = (G @ coef)  # (N, nu): stationarity of u_k without the tie rows and bounds
    Zp = Z.reshape(npulse, nu)
    zk = np.zeros((N, nu))
    for p in range(npulse):
        ks = np.nonzero(pidx == p)[0]
        if pulse_bounds == "first":
            zk[ks[0]] = Zp[p]
        else:  # every copy's bound binds: the total spread evenly
            zk[ks] = Zp[p] / len(ks)
    tie = jr >= N * nx + 2
    tie_rows = np.unique(jr[tie])
    # tie row -> (later interval k, muscle m, sign of its entry on u_k)
    kpos = {}
    for r, c, val in zip(jr[tie], jc[tie], jv[tie]):
        kpos.setdefault(int(r), []).append((int(c // nz), int(c % nz - nx), float(val)))
    tval = np.zeros((N + 1, nu))  # multiplier of the tie row written +u_k - u_{k-1}
    for kk in range(N):
        if kk + 1 < N and pidx[kk + 1] == pidx[kk]:
            tval[kk + 1] = g[kk] + tval[kk] - zk[kk]
    for r in tie_rows:
        (ka, ma, va), (kb, mb, vb) = kpos[int(r)]
        kl, ml, vl = (ka, ma, va) if ka > kb else (kb, mb, vb)
        y[r] = tval[kl, ml] * vl
    zl = np.zeros(v.size)
    zu = np.zeros(v.size)
    ucols = (np.arange(N)[:, None] * nz + nx + np.arange(nu)[None, :])
    zl[ucols] = np.maximum(zk, 0.0)
    zu[ucols] = np.maximum(-zk, 0.0)
    scale = np.abs(Gp[:, 0]).max()
    rep = {"nu_marker": [float(a) for a in nu_[:2]], "nu_end": [float(a) for a in nu_[2:]],
           "pulses_at_bounds": int((sign != 0).sum()), "pulses_sign_kept": int(keep.sum()),
           "reduced_dual_inf_rel": float(np.abs(resid).max() / scale)}
    return y, zl, zu, rep


def ipopt_termination_audit(objective="fatigue", legacy=True, threads=8):
    """Ipopt's termination tests (IpOptErrorConv: CurrentIsOptimal / CurrentIsAcceptable) at a stored optimum, in the
    stored revision's NLP — per-pulse pulse-width parameters in SECONDS (VariableScaling 1, fes_ocp_dynamics.py:373),
    the script's Solver.IPOPT(_max_iter=10000) (reaching_task_pulse_duration_optimization.py:117) with bioptim's tol =
    acceptable_tol = 1e-6 (recalled).  In the reduced space of reduced_stationarity every multiplier is fixed by the 4
    equality multipliers nu (the continuity multipliers are their adjoint) and the 360 per-pulse bound multipliers z, so
    the best achievable dual infeasibility is a small problem:
      * least squares with the signs of z enforced (reduced_stationarity's multipliers), and
      * the linear program  min_{nu, z} max_j |g_j + G_j nu - z_j|  (z_j >= 0 at the lower bound, <= 0 at the upper,
        0 off the bounds): d*, the smallest max-norm unscaled dual infeasibility ANY multipliers give.
    Ipopt's scaled error uses its gradient-based NLP scaling (s_f = 1 at the script's initial guess: the objective's
    gradient there is far below nlp_scaling_max_gradient 100 — 2 / a_rest for the fatigue Mayer term at A = a_rest, 0 for
    the force term at F = 0; the continuity rows' factors s_g from the interval Jacobians at that guess) and the
    multiplier scaling s_d = max(s_max, (|y_s|_1 + |z_s|_1) / (m + n_z)) / s_max, s_max = 100.  Returns the numbers."""
    from scipy.optimize import linprog

    from oracle import c_msk

    keep = {}
    base = reduced_stationarity(objective, legacy=legacy, threads=threads, _keep=keep)
    G, sign = keep["G_seconds"], keep["sign"]
    pb, X, seeds, J = keep["pb"], keep["X"], keep["seeds"], keep["J"]
    n_p = G.shape[0]
    # least squares (signs enforced), converted to seconds
    nu_ls, z_ls = keep["nu_ls"], keep["z_ls"]
    r_ls = G[:, 0] + G[:, 1:] @ nu_ls - z_ls
    # the linear program over (nu, z, t)
    nv = 4 + n_p + 1
    c = np.zeros(nv)
    c[-1] = 1.0
    A = np.zeros((2 * n_p, nv))
    A[:n_p, :4], A[:n_p, 4:4 + n_p], A[:n_p, -1] = G[:, 1:], -np.eye(n_p), -1.0
    A[n_p:, :4], A[n_p:, 4:4 + n_p], A[n_p:, -1] = -G[:, 1:], np.eye(n_p), -1.0
    b = np.concatenate([-G[:, 0], G[:, 0]])
    bounds = [(None, None)] * 4 + [((0, None) if s_ > 0 else ((None, 0) if s_ < 0 else (0, 0))) for s_ in sign] + \
        [(0, None)]
    lp = linprog(c, A_ub=A, b_ub=b, bounds=bounds, method="highs")
    nu_lp, z_lp, dstar = lp.x[:4], lp.x[4:4 + n_p], float(lp.x[-1])
    # Ipopt's constraint scaling of the continuity rows at the script's initial guess (states at rest, widths at their
    # initial value: the product's initial guess for this problem)
    ocp = R.legacy_product(objective)
    v0 = ocp.initial_guess_vector()
    _, J0 = c_msk.shooting(pb, v0[None], want_g=False, threads=threads)
    J0 = J0[0]  # (N, nx, nz): dPhi_k/d(x_k, u_k); the -1 on x_{k+1} as well
    sg = np.minimum(1.0, 100.0 / np.maximum(np.maximum(np.abs(J0).max(2), 1.0), 1e-300)).reshape(-1)
    sg = np.maximum(sg, 1e-8)
    N, nx = R.N, pb.nx

    def scaled_error(nu, z, dinf):
        coef = np.concatenate([[1.0], nu])
        lam = seeds[R.N] @ coef
        ys = [lam]
        for k in range(N - 1, 0, -1):  # continuity multipliers: the adjoint (the row into x_k)
            lam = J[k][:, :nx].T @ lam + seeds[k] @ coef
            ys.append(lam)
        y = np.concatenate(ys[::-1])  # rows 1..N-1, N (N - 1 + 1 blocks of nx)
        y_s = np.abs(y) / sg          # scaled problem's multipliers (s_f = 1): y / s_g (row k: into x_{k+1})
        n_rows = y.size + 2
        lo, hi = keep["xlo"], keep["xhi"]
        n_z = int(np.isfinite(lo[:, 1:]).sum() + np.isfinite(hi[:, 1:]).sum()) + 2 * n_p
        s_d = max(100.0, (y_s.sum() + np.abs(nu[:2]).sum() + np.abs(z).sum()) / (n_rows + n_z)) / 100.0
        return dinf / s_d, s_d

    err_ls, sd_ls = scaled_error(nu_ls, z_ls, float(np.abs(r_ls).max()))
    err_lp, sd_lp = scaled_error(nu_lp, z_lp, dstar)
    return {**base, "dual_inf_unscaled_ls": float(np.abs(r_ls).max()), "dual_inf_unscaled_min_lp": dstar,
            "lp_status": int(lp.status), "s_d_ls": sd_ls, "s_d_lp": sd_lp, "scaled_error_ls": err_ls,
            "scaled_error_lp": err_lp, "s_g_min": float(sg.min()), "s_g_median": float(np.median(sg)),
            "wrong_signed_or_free_pulses_ls": int((np.abs(r_ls) > 1e-6 * np.abs(G[:, 0]).max()).sum()),
            "tol": 1e-6, "acceptable_tol": 1e-6, "dual_inf_tol": 1.0}
