"""cfg-5 (RK4 x 5) batched interior point from perturbed starts, and the stage-wise Hessian's throughput at batch
65,536 (RK4 x 1).  Usage: python scripts/msk_multistart_probe.py [--hess-only]"""
import pathlib
import sys
import time

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from cocofest_amd.solver import BatchedIpm, IpmOptions, NativeIpm  # noqa: E402

ocp = bench.msk_build(5)
for B, amp in (() if "--hess-only" in sys.argv else ((64, 0.1), (64, 0.3), (512, 0.1))):
    rng = np.random.default_rng(0)
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    lb, ub = ocp.bounds_vector()
    free = lb != ub
    span = np.minimum(np.where(np.isfinite(ub - lb), ub - lb, 10.0), 10.0)[free]
    v0[:, free] = np.clip(v0[:, free] + amp * rng.uniform(-1, 1, (B, free.sum())) * span, lb[free], ub[free])
    cls = NativeIpm if "--native" in sys.argv else BatchedIpm
    ipm = cls(ocp, batch=B, options=IpmOptions(tol=1e-6, max_iter=1000))
    res = ipm.solve(v0)
    ipm.close()
    print(f"{cls.__name__} B={B} amp={amp}: wall {res.wall_time:.2f} s, converged {int(res.converged.sum())}/{B}, iterations "
          f"median {np.median(res.iterations):.0f} max {res.iterations.max()}, f median {np.median(res.f):.4f} "
          f"min {res.f.min():.4f}", flush=True)

ocp1 = bench.msk_build(1)
for B in ((4096,) if "--hess-only" in sys.argv else (1, 4096, 65536)):
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
