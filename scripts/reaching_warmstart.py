"""The native solver on the reference's reaching task: a true Ipopt warm start at the
stored optimum, and solves from the reference script's own initial guess, timed.

The product's OcpFesMsk for examples/dynamics/reaching_task/reaching_task_pulse_duration_optimization.py:80-118 (six
Ding2007-with-fatigue muscles at the stored revision's fatigue rates, 60 pulses at 40 Hz, N = 1,500, RK4 x 1, the hand on
the target at node 1000, no residual torque; tests/test_reference_solution.py::legacy_product: the stored revision's
calcium convention and per-pulse widths, where the stored point is feasible) is solved by cfx_ipm.

--start stored (default): the stored states and pulse widths (tests/golden/reaching_pulse_duration_*.npz).
  --multipliers adjoint (default): Ipopt's warm start (warm_start_init_point) with multipliers computed at the stored
  point from the PRODUCT's J_g and grad f: the continuity-row multipliers by the discrete adjoint of the RK4 x 1
  transcription (y_{c_{k-1}} = df/dx_k + A_k^T y_{c_k} + marker terms; at the fixed end states y is free), the marker
  and end-state multipliers and the per-pulse bound multipliers by least squares over the 360 pulse-width sums with
  their signs enforced (tests/reaching_kkt.py's reduced problem), the per-interval bound multipliers as the pulse's
  total spread evenly and the tie-row multipliers by the recursion along each pulse.  Options mu_init /
  warm_start_bound_push / warm_start_mult_bound_push (default 1e-9 each).
  --multipliers none: Ipopt's cold start from the stored point (round 4).
--start reference: the product's default initial guess for the script's problem (the reference's own start).

Reports start and end objective, the constraint violation, the change of every state and pulse width relative to its
range (the distance to the stored optimum), wall-clock and iterations beside the stored solve's time_to_optimize
(pickle.py:32; unknown hardware, an older revision).  One JSON line per objective.

Usage (GPU): python scripts/reaching_warmstart.py [--objectives fatigue,force] [--start stored|reference]
             [--multipliers adjoint|none] [--max-iter 3000] [--wall 600] [--current]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests import test_reference_solution as R  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--objectives", default="fatigue,force")
ap.add_argument("--start", default="stored", choices=["stored", "reference"])
ap.add_argument("--multipliers", default="adjoint", choices=["adjoint", "none"])
ap.add_argument("--max-iter", type=int, default=3000)
ap.add_argument("--wall", type=float, default=600.0)
ap.add_argument("--out", default=None, help="append the JSON lines to this file")
ap.add_argument("--mu-init", type=float, default=None, help="Ipopt mu_init (warm start 1e-9, else 0.1)")
ap.add_argument("--bound-push", type=float, default=1e-9, help="warm start: warm_start_bound_push")
ap.add_argument("--mult-push", type=float, default=1e-9, help="warm start: warm_start_mult_bound_push")
ap.add_argument("--bound-relax", type=float, default=1e-8,
                help="Ipopt's bound_relax_factor (its default 1e-8, as the stored solve used)")
ap.add_argument("--tol", type=float, default=1e-6)
ap.add_argument("--curv-min", type=float, default=None, help="the inertia-free curvature test's threshold")
ap.add_argument("--range-scaling", type=int, default=1,
                help="1: the product's variable scaling by the bound range (default); 0: none, as Ipopt")
ap.add_argument("--current", action="store_true",
                help="today's calcium conventions and per-interval widths instead of the stored revision's")
args = ap.parse_args()


def build(objective):
    import cocofest_amd as C

    models = []
    for n, c in zip(R.MUSCLES, R.muscle_constants(legacy_rates=True)):
        mm = C.DingModelPulseWidthFrequencyWithFatigue(muscle_name=n, sum_stim_truncation=R.T)
        for k in ("alpha_a", "alpha_tau1", "alpha_km", "a_scale"):
            setattr(mm, k, c[k])
        models.append(mm)
    model = C.FesMskModel(biorbd_path=str(R.GOLDEN / "biomod_arm26.json"), muscles_model=models, stim_time=R.STIMS,
                          activate_force_length_relationship=True, activate_force_velocity_relationship=True,
                          activate_residual_torque=False)
    cl = C.ConstraintList()
    cl.add(C.ConstraintFcn.SUPERIMPOSE_MARKERS, first_marker="COM_hand", second_marker="reaching_target", phase=0,
           node=R.MARKER_NODE, axes=[C.Axis.X, C.Axis.Y])
    return C.OcpFesMsk.prepare_ocp(model=model, final_time=R.FINAL_TIME, n_shooting=R.N,
                                   pulse_width={"min": C.DingModelPulseWidthFrequency().pd0, "max": 0.0006},
                                   objective={f"minimize_muscle_{objective}": True},
                                   msk_info={"with_residual_torque": False, "bound_type": "start_end",
                                             "bound_data": [[0, 5], [0, 5]], "custom_constraint": cl},
                                   ode_solver=C.OdeSolver.RK4(n_integration_steps=1),
                                   apply_custom_constraint=True)


def adjoint_multipliers(ocp, v, lb, ub):
    """(y, z_l, z_u, report) at v from the product's callbacks (see the module docstring).  Structure of the legacy
    product's NLP: rows [N nx continuity | 2 marker rows | tie rows u_k - u_{k-1}], decision [x_k, u_k]_k, x_N."""
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
    # per-interval width multipliers: the pulse total spread evenly; tie rows by the recursion along the pulse
    g = (G @ coef)  # (N, nu): stationarity of u_k without the tie rows and bounds
    Zp = Z.reshape(npulse, nu)
    zk = np.zeros((N, nu))
    for p in range(npulse):
        ks = np.nonzero(pidx == p)[0]
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


def run(objective):
    from cocofest_amd.solver import IpmOptions, NativeIpm

    ocp = build(objective) if args.current else R.legacy_product(objective)
    d = R.load(objective)
    X, U = R.trajectory(d)
    nm = len(R.MUSCLES)
    nx, nz = ocp.nx, ocp.nx + ocp.nu
    assert ocp.nu == nm, ocp.nu
    vs = R.decision_vector(X, U[:nm], nz)  # the stored optimum
    lb, ub = ocp.bounds_vector()
    v0 = vs if args.start == "stored" else ocp.initial_guess_vector()
    h = ocp.nlp(batch=1, layout="aos")
    g0 = h.eval_g(v0[None])[0]
    f0 = float(h.eval_f(v0[None])[0])
    fs = float(h.eval_f(vs[None])[0])
    h.close()
    warm = args.start == "stored" and args.multipliers == "adjoint"
    rep = {}
    t0 = time.perf_counter()
    kw = dict(tol=args.tol, max_iter=args.max_iter, max_wall_time=args.wall, print_frequency_time=30.0,
              bound_relax_factor=args.bound_relax, range_scaling=bool(args.range_scaling))
    if args.curv_min is not None:
        kw["curv_min"] = args.curv_min
    if warm:
        y, zl, zu, rep = adjoint_multipliers(ocp, vs, lb, ub)
        kw.update(warm_start_init_point=True, mu_init=args.mu_init or 1e-9, warm_start_bound_push=args.bound_push,
                  warm_start_mult_bound_push=args.mult_push)
    elif args.mu_init:
        kw["mu_init"] = args.mu_init
    t_mult = time.perf_counter() - t0
    ipm = NativeIpm(ocp, batch=1, options=IpmOptions(**kw))
    t1 = time.perf_counter()
    res = ipm.solve(v0[None], warm_start=(y[None], zl[None], zu[None]) if warm else None)
    t2 = time.perf_counter()
    st = dict(ipm.last_stats)
    ipm.close()
    v = res.v[0]
    h = ocp.nlp(batch=1, layout="aos")
    g1 = h.eval_g(v[None])[0]
    h.close()
    nrow = R.N * ocp.nx
    span = np.where(np.isfinite(ub - lb) & (ub > lb), ub - lb, np.maximum(1.0, np.abs(vs)))
    body0, body = vs[: R.N * nz].reshape(R.N, nz), v[: R.N * nz].reshape(R.N, nz)
    dstate = np.abs(body[:, :nx] - body0[:, :nx]) / span[: R.N * nz].reshape(R.N, nz)[:, :nx]
    dstate_end = np.abs(v[R.N * nz:] - vs[R.N * nz:]) / span[R.N * nz:]
    pw0, pw = body0[:, nx:], body[:, nx:]
    pwlo, pwhi = lb[nx], ub[nx]
    out = {"objective": objective, "start": args.start, "warm_start": warm,
           "conventions": "current" if args.current else "stored revision (legacy, per pulse)",
           "status": int(res.status[0]), "converged": bool(res.converged[0]),
           "iterations": int(res.iterations[0]), "solve_wall_s": t2 - t1, "create_s": t1 - t0 - t_mult,
           "multipliers_s": t_mult, "kkt_error": float(res.kkt_error[0]),
           "f_start": f0, "f_stored": fs, "f_end": float(res.f[0]), "f_end_rel_to_stored": float(res.f[0]) / fs - 1,
           "g_start_max": float(np.abs(g0).max()),
           "g_end_max_continuity": float(np.abs(g1[:nrow]).max()), "g_end_max_other": float(np.abs(g1[nrow:]).max()),
           "dist_to_stored_state_rel_max": float(max(dstate.max(), dstate_end.max())),
           "dist_to_stored_state_rel_median": float(np.median(dstate)),
           "dist_to_stored_pw_rel_max": float(np.abs(pw - pw0).max() / (pwhi - pwlo)),
           "dist_to_stored_pw_rel_median": float(np.median(np.abs(pw - pw0)) / (pwhi - pwlo)),
           "pw_at_bounds_stored": int(((pw0 <= pwlo + 1e-9) | (pw0 >= pwhi - 1e-9)).sum()),
           "pw_at_bounds_end": int(((pw <= pwlo + 1e-9) | (pw >= pwhi - 1e-9)).sum()), "pw_total": int(pw.size),
           "resto_phases": int(st.get("resto_phases", 0)), "kkt_chain_nodes": st.get("kkt_chain_nodes"),
           "kkt_n": st.get("kkt_n"), "s_per_iteration": (t2 - t1) / max(1, int(res.iterations[0])),
           "reference_time_to_optimize_s": float(d["time_to_optimize"]), **{k: kw[k] for k in kw if k != "tol"},
           **rep}
    if args.out:  # the end point, for a later look
        np.savez(os.path.splitext(args.out)[0] + f"_{objective}_{args.start}.npz", v=res.v[0], g=g1)
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "a") as fh:
            fh.write(line + "\n")


for obj in args.objectives.replace("+", ",").split(","):
    run(obj)
