"""MSK kernel probe: time g + J_g, g, the Hessian and the IVP of BASELINE config 5 (arm26 biceps/triceps +
Ding2007 with fatigue, RK4 x 1, N = 10) on device-resident SoA batches.  Variant libraries (built with another
CFX_MSK_DIRS) are compared with ``--libs a.so b.so``.  Usage: python scripts/msk_probe.py [--batch B ...]"""

import argparse
import json
import os
import pathlib
import sys

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def build(m=1):
    import cocofest_amd as C

    mm = C.FesMskModel(biorbd_path=str(ROOT / "tests/golden/biomod_arm26_biceps_triceps.json"),
                       muscles_model=[C.DingModelPulseWidthFrequencyWithFatigue(muscle_name=n, sum_stim_truncation=10)
                                      for n in ("BIClong", "TRIlong")],
                       stim_time=[0.1 * i for i in range(10)], activate_force_length_relationship=True,
                       activate_force_velocity_relationship=True)
    ol = C.ObjectiveList()
    ol.add(C.ObjectiveFcn.Mayer.MINIMIZE_STATE, key="qdot", index=[0, 1], node=C.Node.END, target=np.zeros((2, 1)),
           weight=100)
    return C.OcpFesMsk.prepare_ocp(model=mm, final_time=1, objective={"custom": ol, "minimize_muscle_fatigue": True},
                                   msk_info={"bound_type": "start_end", "bound_data": [[0, 5], [0, 90]]},
                                   ode_solver=C.OdeSolver.RK4(n_integration_steps=m))


def synthetic(ocp, B, seed=0):
    """(nv, B) decisions: midpoints of finite bounds +- 20 %, angles in range, velocities within +-2 rad/s."""
    lo, hi = ocp.bounds_vector()
    r = np.random.default_rng(seed)
    lo = np.where(np.isfinite(lo), lo, -2.0)
    hi = np.where(np.isfinite(hi), hi, 2.0)
    hi = np.where(hi - lo > 100, lo + 100, hi)  # forces up to 100 N
    v = lo[:, None] + (hi - lo)[:, None] * r.uniform(0.2, 0.8, size=(len(lo), B))
    return torch.as_tensor(v, device="cuda")


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[4096, 65536])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--libs", nargs="*", default=[])
    ap.add_argument("--reaching", action="store_true",
                    help="the 1,500-interval reaching task (6 muscles, tests/test_reference_solution.py) instead of cfg 5")
    ap.add_argument("--dump", default=None, help="save g and J_g of the first batch's first 256 instances here (.npz), for A/B comparisons")
    a = ap.parse_args()
    from cocofest_amd import _cfx

    out = []
    for lib in a.libs or [None]:
        if lib:
            _cfx._lib = None
            os.environ["CFX_LIB"] = lib
        if a.reaching:
            sys.path.insert(0, str(ROOT))
            from tests import test_reference_solution as R

            ocp = R.legacy_product("fatigue")
        else:
            ocp = build()
        for B in a.batch:
            h = ocp.nlp(batch=B, layout="soa")
            v = synthetic(ocp, B)
            g = torch.empty((h.ng, B), dtype=torch.float64, device="cuda")
            j = torch.empty((h.nnz_jac, B), dtype=torch.float64, device="cuda")
            t_gj = timeit(lambda: h.eval_all(v, g=g, jac=j), a.reps)
            if a.dump and B == a.batch[0]:
                np.savez(a.dump, g=g[:, :256].cpu().numpy(), j=j[:, :256].cpu().numpy())
            t_g = timeit(lambda: h.eval_all(v, g=g), a.reps)
            row = dict(lib=lib or "default", geom_lds=os.environ.get("CFX_MSK_GEOM_LDS", ""), batch=B, nnz_jac=h.nnz_jac, ms_g_jac=t_gj, ms_g=t_g,
                       evals_per_s=B / t_gj * 1e3, GBps=B * 8 * (h.nv + h.ng + h.nnz_jac) / t_gj / 1e6)
            if B <= 4096:
                lam = torch.randn((h.ng, B), dtype=torch.float64, device="cuda")
                of = torch.ones(B, dtype=torch.float64, device="cuda")
                hv = torch.empty((h.nnz_hess, B), dtype=torch.float64, device="cuda")
                row["ms_hess"] = timeit(lambda: h.eval_h(v, of, lam, hess=hv), max(2, a.reps // 4))
            x0 = v[: h.nx].contiguous()
            u = torch.full((ocp.n_shooting * h.nu, B), 3e-4, dtype=torch.float64, device="cuda")
            tr = torch.empty(((ocp.n_shooting + 1) * h.nx, B), dtype=torch.float64, device="cuda")
            row["ms_ivp"] = timeit(lambda: h.integrate(x0=x0, u=u, traj=tr), a.reps)
            h.close()
            print(json.dumps(row), flush=True)
            out.append(row)
    return out


if __name__ == "__main__":
    main()
