"""Warm-started native solve of the reference's reaching task from its stored optimum.

The product's OcpFesMsk for examples/dynamics/reaching_task/reaching_task_pulse_duration_optimization.py:80-118 (six
Ding2007-with-fatigue muscles at the stored revision's fatigue rates, 60 pulses at 40 Hz, N = 1,500, RK4 x 1, the hand on
the target at node 1000, no residual torque) is solved by cfx_ipm starting at the stored states and pulse widths
(tests/golden/reaching_pulse_duration_*.npz).  The stored point solves the stored revision's NLP (tests/
test_reference_solution.py); the product states today's reference, whose calcium sum keeps every pulse of the window
(the stored Cn rows miss by 8.6e-3 after the second pulse under it) and whose pulse width is a control per interval,
not a parameter per pulse.  By default the product runs the stored revision's conventions (FesMskModel(
legacy_calcium=True), pulse_width["per_pulse"]: tests/test_reference_solution.py::legacy_product), where the stored
point is feasible; --current runs today's.  The script measures how far the solve moves: start and end objective,
the largest constraint row at the start, the change of every state and pulse width relative to its range, and how
many pulse widths sit on a bound.  One JSON line per objective.

Usage (GPU): python scripts/reaching_warmstart.py [--objectives fatigue,force] [--max-iter 3000] [--wall 400]
             [--current]"""
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
ap.add_argument("--max-iter", type=int, default=3000)
ap.add_argument("--wall", type=float, default=400.0)
ap.add_argument("--out", default=None, help="append the JSON lines to this file")
ap.add_argument("--mu-init", type=float, default=1e-9, help="warm start: Ipopt's mu_init (default 1e-9)")
ap.add_argument("--bound-push", type=float, default=1e-9, help="warm start: Ipopt's bound_push (default 1e-9)")
ap.add_argument("--bound-relax", type=float, default=1e-8,
                help="Ipopt's bound_relax_factor (its default 1e-8, as the stored solve used)")
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

    ocp = build(objective) if args.current else R.legacy_product(objective)
    X, U = R.trajectory(R.load(objective))
    nm = len(R.MUSCLES)
    nx, nz = ocp.nx, ocp.nx + ocp.nu
    assert ocp.nu == nm, ocp.nu
    v0 = R.decision_vector(X, U[:nm], nz)
    lb, ub = ocp.bounds_vector()
    h = ocp.nlp(batch=1, layout="aos")
    g0 = h.eval_g(v0[None])[0]  # the stored point as it is (its widths sit 1e-8 outside: Ipopt's bound_relax_factor)
    f0 = float(h.eval_f(v0[None])[0])
    h.close()
    t0 = time.perf_counter()
    # Ipopt-style warm start: a small barrier and bound push, the relaxed bounds of the stored solve
    ipm = NativeIpm(ocp, batch=1, options=IpmOptions(tol=1e-6, max_iter=args.max_iter, max_wall_time=args.wall,
                                                      print_frequency_time=30.0, mu_init=args.mu_init,
                                                      bound_push=args.bound_push,
                                                      bound_relax_factor=args.bound_relax))
    res = ipm.solve(v0[None])
    st = dict(ipm.last_stats)
    g_solver = ipm.h.eval_g(res.v)[0]  # the solver's own handle, at the returned point
    ipm.close()
    wall = time.perf_counter() - t0
    v = res.v[0]
    h = ocp.nlp(batch=1, layout="aos")
    g1 = h.eval_g(v[None])[0]
    h.close()
    nrow = R.N * ocp.nx
    span = np.where(np.isfinite(ub - lb) & (ub > lb), ub - lb, np.maximum(1.0, np.abs(v0)))
    body0, body = v0[: R.N * nz].reshape(R.N, nz), v[: R.N * nz].reshape(R.N, nz)
    dstate = np.abs(body[:, :nx] - body0[:, :nx]) / span[: R.N * nz].reshape(R.N, nz)[:, :nx]
    pw0, pw = body0[:, nx:], body[:, nx:]
    pwlo, pwhi = lb[nx], ub[nx]
    pidx = R.pulse_index()
    spread = max(float(np.ptp(pw[pidx == i], axis=0).max()) for i in range(int(pidx.max()) + 1))
    out = {"objective": objective, "conventions": "current" if args.current else "stored revision (legacy, per pulse)",
           "status": int(res.status[0]), "converged": bool(res.converged[0]),
           "iterations": int(res.iterations[0]), "wall_s": wall, "kkt_error": float(res.kkt_error[0]),
           "f_start": f0, "f_end": float(res.f[0]), "g_start_max": float(np.abs(g0).max()),
           "g_end_max_continuity": float(np.abs(g1[:nrow]).max()), "g_end_max_other": float(np.abs(g1[nrow:]).max()),
           "g_end_max_solver_handle": float(np.abs(g_solver).max()),
           "g_end_argmax_row": int(np.abs(g1).argmax()), "ng": int(g1.size),
           "g_start_rows_over_1e-6": int((np.abs(g0) > 1e-6).sum()),
           "dstate_rel_max": float(dstate.max()), "dstate_rel_median": float(np.median(dstate)),
           "dpw_rel_max": float(np.abs(pw - pw0).max() / (pwhi - pwlo)),
           "dpw_rel_median": float(np.median(np.abs(pw - pw0)) / (pwhi - pwlo)),
           "pw_at_bounds_start": int(((pw0 <= pwlo + 1e-9) | (pw0 >= pwhi - 1e-9)).sum()),
           "pw_at_bounds_end": int(((pw <= pwlo + 1e-9) | (pw >= pwhi - 1e-9)).sum()), "pw_total": int(pw.size),
           "pw_spread_within_pulse_max_rel": spread / (pwhi - pwlo),
           "resto_phases": int(st.get("resto_phases", 0)), "kkt_n": st.get("kkt_n"), "kkt_kl": st.get("kkt_kl"),
           "kkt_blocks": st.get("kkt_blocks"), "mu_init": args.mu_init, "bound_push": args.bound_push,
           "bound_relax_factor": args.bound_relax, "s_per_iteration": wall / max(1, int(res.iterations[0]))}
    if args.out:  # the end point, for a later look
        np.savez(os.path.splitext(args.out)[0] + f"_{objective}.npz", v=res.v[0], g=g1)
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "a") as fh:
            fh.write(line + "\n")


for obj in args.objectives.replace("+", ",").split(","):
    run(obj)
