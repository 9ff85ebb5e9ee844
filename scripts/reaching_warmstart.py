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
  their signs enforced (tests/reaching_kkt.py's reduced problem), the bound multiplier of each pulse on its first
  interval (the copies' bounds never bind, FesMskOcp.bounds_vector) and the tie-row multipliers by the recursion along
  each pulse.  Options mu_init /
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

from tests import reaching_kkt as K  # noqa: E402
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
ap.add_argument("--inertia-test", type=int, default=0, help="1: Ipopt's inertia correction (chain pivot-block inertias)")
ap.add_argument("--bound-mult-init", default="mu-based", choices=["mu-based", "constant"],
                help="Ipopt's bound_mult_init_method (its default: constant 1)")
ap.add_argument("--ipopt-defaults", action="store_true",
                help="Ipopt's defaults where this library's differ: soft restoration (factor 0.9999), filter resets "
                     "(5), constant bound-multiplier initialisation (1)")
ap.add_argument("--pulse-bounds", default="all", choices=["all", "first"],
                help="per-pulse widths: bounds on every interval's copy (all) or on the pulse's first interval (first)")
ap.add_argument("--range-scaling", type=int, default=1,
                help="1: the product's variable scaling by the bound range (default); 0: none, as Ipopt")
ap.add_argument("--profile", default="script", choices=["script", "ipopt", "cfx"],
                help="ipopt: Solver.IPOPT()'s Ipopt / bioptim profile (IpmOptions.ipopt: adaptive mu, Ipopt's bound push, "
                     "constant bound multipliers, no range scaling, ...) with only tol / max_iter / wall and the warm "
                     "start taken from this script; cfx: the library profile (IpmOptions()) likewise; script: this "
                     "script's own flags")
ap.add_argument("--mu-strategy", default=None, choices=["monotone", "adaptive"], help="override Ipopt's mu_strategy")
ap.add_argument("--trace", action="store_true", help="CFX_IPM_TRACE=1 (one stderr line per iteration)")
ap.add_argument("--hessian", default=None, choices=["exact", "limited-memory"], help="Ipopt's hessian_approximation")
ap.add_argument("--lm-history", type=int, default=None, help="limited_memory_max_history")
ap.add_argument("--n-shooting", type=int, default=None,
                help="a coarser grid of the same task (a multiple of 60; from the reference start only, no comparison "
                     "with the stored optimum)")
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


def run(objective):
    from cocofest_amd.solver import IpmOptions, NativeIpm

    ocp = build(objective) if args.current else R.legacy_product(objective, pulse_bounds=args.pulse_bounds)
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
    kw["bound_mult_init_method"] = args.bound_mult_init
    if args.ipopt_defaults:
        kw.update(bound_mult_init_method="constant", soft_resto_pderror_reduction_factor=0.9999, max_filter_resets=5)
    if args.inertia_test:
        kw["inertia_test"] = True
    if args.curv_min is not None:
        kw["curv_min"] = args.curv_min
    if warm:
        y, zl, zu, rep = K.adjoint_multipliers(ocp, vs, lb, ub, pulse_bounds=args.pulse_bounds)
        kw.update(warm_start_init_point=True, mu_init=args.mu_init or 1e-9, warm_start_bound_push=args.bound_push,
                  warm_start_mult_bound_push=args.mult_push)
    elif args.mu_init:
        kw["mu_init"] = args.mu_init
    t_mult = time.perf_counter() - t0
    if args.profile != "script":  # a named profile: only the solve's budget and the warm start from this script
        keep = {k: kw[k] for k in ("tol", "max_iter", "max_wall_time", "print_frequency_time", "warm_start_init_point",
                                   "mu_init", "warm_start_bound_push", "warm_start_mult_bound_push") if k in kw}
        kw = {**(IpmOptions.IPOPT_PROFILE if args.profile == "ipopt" else {}), **keep}
    if args.mu_strategy:
        kw["mu_strategy"] = args.mu_strategy
    if args.hessian:
        kw["hessian_approximation"] = args.hessian
    if args.lm_history:
        kw["limited_memory_max_history"] = args.lm_history
    if args.trace:
        os.environ["CFX_IPM_TRACE"] = "1"
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
           "reference_time_to_optimize_s": float(d["time_to_optimize"]), "pulse_bounds": args.pulse_bounds,
           "profile": args.profile, "mu_mode_switches": int(st.get("mu_mode_switches", 0)), "lib": os.environ.get("CFX_LIB", "libcfx.so"),
           **{k: kw[k] for k in kw if k != "tol"},
           **rep}
    if args.out:  # the end point, for a later look
        np.savez(os.path.splitext(args.out)[0] + f"_{objective}_{args.start}.npz", v=res.v[0], g=g1)
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "a") as fh:
            fh.write(line + "\n")


def run_coarse(objective):
    """The task on a coarser grid (legacy conventions), from the product's initial guess."""
    from cocofest_amd.solver import IpmOptions, NativeIpm

    ocp = R.legacy_product(objective, n_shooting=args.n_shooting)
    base = dict(tol=args.tol, max_iter=args.max_iter, max_wall_time=args.wall, print_frequency_time=30.0)
    kw = {**(IpmOptions.IPOPT_PROFILE if args.profile == "ipopt" else {}), **base}
    if args.mu_strategy:
        kw["mu_strategy"] = args.mu_strategy
    if args.hessian:
        kw["hessian_approximation"] = args.hessian
    ipm = NativeIpm(ocp, batch=1, options=IpmOptions(**kw))
    t1 = time.perf_counter()
    res = ipm.solve()
    t2 = time.perf_counter()
    st = dict(ipm.last_stats)
    ipm.close()
    h = ocp.nlp(batch=1, layout="aos")
    g1 = h.eval_g(res.v)[0]
    h.close()
    out = {"objective": objective, "n_shooting": args.n_shooting, "profile": args.profile,
           "mu_strategy": kw.get("mu_strategy", "monotone"), "status": int(res.status[0]),
           "iterations": int(res.iterations[0]), "solve_wall_s": t2 - t1, "f_end": float(res.f[0]),
           "g_end_max": float(np.abs(g1).max()), "resto_phases": int(st.get("resto_phases", 0)),
           "mu_mode_switches": int(st.get("mu_mode_switches", 0)), "kkt_chain_nodes": st.get("kkt_chain_nodes")}
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "a") as fh:
            fh.write(line + "\n")


for obj in args.objectives.replace("+", ",").split(","):
    run_coarse(obj) if args.n_shooting else run(obj)
