"""Per-iteration cost of the reaching task's native interior point with the stage-chain KKT layout (block cyclic
reduction) against the round-4 panel band factorisation: a few iterations from the stored fatigue optimum in each
layout, wall time per iteration and the layout statistics, one JSON line per layout.

Usage (GPU): python scripts/chain_probe.py [--iters 5] [--layouts chain,band] [--out file.jsonl]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests import test_reference_solution as R  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--layouts", default="chain,band")
ap.add_argument("--objective", default="fatigue")
ap.add_argument("--out", default=None)
args = ap.parse_args()

from cocofest_amd.solver import IpmOptions, NativeIpm  # noqa: E402

ocp = R.legacy_product(args.objective)
X, U = R.trajectory(R.load(args.objective))
v0 = R.decision_vector(X, U[: len(R.MUSCLES)], ocp.nx + ocp.nu)[None]
for kkt in args.layouts.split(","):
    os.environ["CFX_IPM_KKT"] = kkt
    t0 = time.perf_counter()
    ipm = NativeIpm(ocp, batch=1, options=IpmOptions(tol=1e-6, max_iter=args.iters, bound_relax_factor=1e-8))
    t1 = time.perf_counter()
    r = ipm.solve(v0)
    t2 = time.perf_counter()
    st = dict(ipm.last_stats)
    ipm.close()
    out = {"layout": kkt, "create_s": t1 - t0, "solve_s": t2 - t1, "iterations": int(r.iterations[0]),
           "s_per_iteration": (t2 - t1) / max(1, int(r.iterations[0])), "f": float(r.f[0]),
           **{k: st[k] for k in ("kkt_n", "kkt_kl", "kkt_border", "kkt_chain_nodes", "kkt_chain_sp", "kkt_factor",
                                 "eval_all", "eval_g_f")}}
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "a") as fh:
            fh.write(line + "\n")
