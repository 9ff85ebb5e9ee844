"""cfg-5 (RK4 x 5) batched interior point from perturbed starts, and the stage-wise Hessian's throughput at batch
65,536 (RK4 x 1).

Usage: python scripts/msk_multistart_probe.py [--native] [--hess-only] [--runs B:amp,B:amp,...] [--max-iter N]
                                              [--wall SECONDS] [--soft FACTOR] [--restart] [--jsonl FILE]
Each run prints one line (converged count, Ipopt status histogram, restoration phases / iterations, wall time); the
native solver prints a progress line on stderr every 20 s (print_frequency_time)."""
import argparse
import collections
import json
import pathlib
import re
import sys
import time

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from cocofest_amd._cfx import IPM_STATUS  # noqa: E402
from cocofest_amd.solver import BatchedIpm, IpmOptions, NativeIpm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--native", action="store_true")
ap.add_argument("--hess-only", action="store_true")
ap.add_argument("--runs", default="64:0.1,64:0.3,512:0.1")
ap.add_argument("--max-iter", type=int, default=1000)
ap.add_argument("--wall", type=float, default=1e20)
ap.add_argument("--jsonl", default=None)
ap.add_argument("--soft", type=float, default=None, help="soft_resto_pderror_reduction_factor (default: the option's)")
ap.add_argument("--restart", action="store_true", help="resto_failure_restart (extension: a failed phase restarts)")
ap.add_argument("--opt", action="append", default=[], help="extra IpmOptions key=value (repeatable)")
ap.add_argument("--label", default="")
ap.add_argument("--dump", default=None, help="save every start's status / iterations / f of the last run here (.npz)")
ap.add_argument("--first", type=int, default=None,
                help="swap start FIRST with start 0 (CFX_IPM_TRACE=1 traces instance 0; the batch, and so the KKT "
                     "layout and every instance's path, is otherwise unchanged)")
ap.add_argument("--profile", default="cfx", choices=["cfx", "ipopt"],
                help="ipopt: the facade's Ipopt / bioptim profile (IpmOptions.ipopt) under the options above")
args = ap.parse_args()

ocp = bench.msk_build(5)
runs = [] if args.hess_only else [(int(r.split(":")[0]), float(r.split(":")[1])) for r in re.split(r"[,+]", args.runs)]
for B, amp in runs:
    rng = np.random.default_rng(0)
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    lb, ub = ocp.bounds_vector()
    free = lb != ub
    span = np.minimum(np.where(np.isfinite(ub - lb), ub - lb, 10.0), 10.0)[free]
    v0[:, free] = np.clip(v0[:, free] + amp * rng.uniform(-1, 1, (B, free.sum())) * span, lb[free], ub[free])
    if args.first is not None:
        v0[[0, args.first]] = v0[[args.first, 0]]
    cls = NativeIpm if args.native else BatchedIpm
    extra = {} if args.soft is None else {"soft_resto_pderror_reduction_factor": args.soft}
    if args.restart:
        extra["resto_failure_restart"] = True
    for kv in args.opt:
        k, val = kv.split("=", 1)
        cur = getattr(IpmOptions, k)
        extra[k] = type(cur)(val) if not isinstance(cur, bool) else val.lower() in ("1", "true", "yes")
    base = dict(tol=1e-6, max_iter=args.max_iter, max_wall_time=args.wall, print_frequency_time=20.0, **extra)
    opts = IpmOptions.ipopt(**base) if args.profile == "ipopt" else IpmOptions(**base)
    ipm = cls(ocp, batch=B, options=opts)
    res = ipm.solve(v0)
    st = dict(getattr(ipm, "last_stats", {}) or {})
    ipm.close()
    hist = collections.Counter(IPM_STATUS.get(int(s), str(s)) for s in res.status)
    conv = res.converged.astype(bool)
    rec = dict(label=args.label, profile=args.profile, mu_strategy=opts.mu_strategy,
               mu_mode_switches=st.get("mu_mode_switches"),
               options={k: v for k, v in extra.items()}, solver=cls.__name__, batch=B, amp=amp, max_iter=args.max_iter, wall_s=round(res.wall_time, 3),
               converged=int(conv.sum()), status=dict(hist), iterations_median=float(np.median(res.iterations)),
               iterations_max=int(res.iterations.max()), f_converged_min=float(res.f[conv].min()) if conv.any() else None,
               f_converged_max=float(res.f[conv].max()) if conv.any() else None,
               resto_phases=st.get("resto_phases"), resto_iterations=st.get("resto_iterations"),
               host_iterations=st.get("iterations"), soft=opts.soft_resto_pderror_reduction_factor,
               restart=opts.resto_failure_restart,
               soft_steps=getattr(ipm, "soft_steps", st.get("soft_steps")))
    print(json.dumps(rec), flush=True)
    if args.dump:
        np.savez(args.dump, status=res.status, iterations=res.iterations, f=res.f, converged=res.converged,
                 kkt_error=res.kkt_error)
    if args.jsonl:
        with open(args.jsonl, "a") as fh:
            fh.write(json.dumps(rec) + "\n")

ocp1 = bench.msk_build(1)
for B in ((4096,) if args.hess_only else (() if args.runs else (1, 4096, 65536))):
    h = ocp1.nlp(batch=B, layout="soa", device=0)
    r = torch.rand((h.nv, B), dtype=torch.float64, device="cuda:0", generator=torch.Generator("cuda:0").manual_seed(1))
    lo, hi = ocp1.bounds_vector()
    lo = np.where(np.isfinite(lo), lo, -2.0)
    hi = np.minimum(np.where(np.isfinite(hi), hi, 2.0), lo + 100.0)
    v = (torch.as_tensor(lo, device="cuda:0")[:, None] + torch.as_tensor(hi - lo, device="cuda:0")[:, None] * (0.2 + 0.6 * r)).contiguous()
    lam = torch.randn((h.ng, B), dtype=torch.float64, device="cuda:0")
    of = torch.ones((B,), dtype=torch.float64, device="cuda:0")
    H = torch.empty((h.nnz_hess, B), dtype=torch.float64, device="cuda:0")
    for _ in range(2):
        h.eval_h(v, of, lam, H)
    torch.cuda.synchronize()
    t = time.perf_counter()
    n = 5
    for _ in range(n):
        h.eval_h(v, of, lam, H)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / n * 1e3
    print(f"eval_h B={B}: {ms:.3f} ms, {B / ms * 1e3:.3e} instance-Hessians/s, nnz_hess {h.nnz_hess}", flush=True)
    h.close()
