"""The product's Lagrangian Hessian against central differences of its own first derivatives (GPU).

At a point v with multipliers lam and objective factor sigma: H(v) d (the lower-triangle triplets of cfx_eval_h, made
symmetric) against [sigma grad f(v + e d) + J(v + e d)^T lam - (v - e d)] / (2 e), the first derivatives from
cfx_eval_jac_g / cfx_eval_grad_f (exact, analytic tangents).  Directions scaled by each variable's bound range (pulse
widths ~1e-4 s).  Reports the relative error of the whole product and per variable group (muscle states, q, qdot,
widths), for the reaching task (legacy conventions) and cfg 5.

Usage (GPU): python scripts/hessian_check.py [--problem reaching|cfg5] [--objective fatigue|force] [--point stored|guess]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--problem", default="reaching", choices=["reaching", "cfg5", "reaching_current"])
ap.add_argument("--objective", default="force")
ap.add_argument("--point", default="stored", choices=["stored", "guess"])
ap.add_argument("--eps", type=float, default=1e-6)
ap.add_argument("--seed", type=int, default=0)
ap.add_argument("--sigma", type=float, default=1.0)
args = ap.parse_args()

from tests import test_reference_solution as R  # noqa: E402

if args.problem == "cfg5":
    import bench

    ocp = bench.msk_build(5)
    v = ocp.initial_guess_vector()
else:
    ocp = R.legacy_product(args.objective) if args.problem == "reaching" else None
    X, U = R.trajectory(R.load(args.objective))
    nz = ocp.nx + ocp.nu
    v = R.decision_vector(X, U[: len(R.MUSCLES)], nz) if args.point == "stored" else ocp.initial_guess_vector()
lb, ub = ocp.bounds_vector()
rng = np.random.default_rng(args.seed)
h = ocp.nlp(batch=1, layout="aos")
jr, jc = h.jac_structure()
hr, hc = h.hess_structure()
lam = rng.normal(size=h.ng)
span = np.where(np.isfinite(ub - lb) & (ub > lb), np.minimum(ub - lb, 1.0), 1.0)
d = rng.normal(size=h.nv) * span
d[lb == ub] = 0.0


def grad_l(x):
    jv = h.eval_jac_g(x[None])[0]
    g = args.sigma * h.eval_grad_f(x[None])[0]
    np.add.at(g, jc, jv * lam[jr])
    return g


hv = h.eval_h(v[None], np.array([args.sigma]), lam[None])[0]
Hd = np.zeros(h.nv)
np.add.at(Hd, hr, hv * d[hc])
off = hr != hc
np.add.at(Hd, hc[off], hv[off] * d[hr[off]])
out = {"problem": args.problem, "objective": args.objective, "point": args.point, "nv": h.nv, "nnz_h": len(hr)}
for eps in (args.eps, args.eps * 10, args.eps / 10):
    fd = (grad_l(v + eps * d) - grad_l(v - eps * d)) / (2 * eps)
    err = np.abs(Hd - fd)
    scale = np.abs(fd).max()
    out[f"eps{eps:g}"] = {"rel_err_max": float(err.max() / scale), "scale": float(scale),
                          "worst_var": int(err.argmax()), "worst_rel_local": float(err.max() / max(abs(fd[err.argmax()]), 1e-300))}
# per group at the first eps
fd = (grad_l(v + args.eps * d) - grad_l(v - args.eps * d)) / (2 * args.eps)
if args.problem != "cfg5":
    nx, nu = ocp.nx, ocp.nu
    N = R.N
    idx = np.arange(h.nv)
    node_off = idx % (nx + nu)
    body = idx < N * (nx + nu)
    groups = {"muscle_states": body & (node_off < 30), "q_qdot": body & (node_off >= 30) & (node_off < nx),
              "widths": body & (node_off >= nx)}
    for g, m in groups.items():
        e = np.abs(Hd[m] - fd[m])
        out[g] = {"rel_err_max": float(e.max() / max(np.abs(fd[m]).max(), 1e-300)), "scale": float(np.abs(fd[m]).max())}
h.close()
print(json.dumps(out))
