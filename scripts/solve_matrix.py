"""Interior-point robustness matrix on the GPU: each model family x transcription from the default initial
guess (the reference's x_init / u_init), force tracking or end-force objectives.  Prints one JSON object."""

import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def cases():
    from cocofest_amd import ModelMaker, OcpFes, OdeSolver

    ft = json.loads((ROOT / "tests" / "golden" / "ref_formulas.json").read_text())["misc"]["force_tracking"]
    track = {"force_tracking": [np.array(ft["time"]), np.array(ft["force"])]}
    st30 = [float(t) for t in np.round(np.linspace(0, 1, 31)[:-1], 2)]
    st10 = [round(0.1 * i, 1) for i in range(10)]
    solvers = {"RK1x10": OdeSolver.RK1(n_integration_steps=10), "RK4x5": OdeSolver.RK4(n_integration_steps=5),
               "COL4": OdeSolver.COLLOCATION(4, "legendre"), "RADAU3": OdeSolver.COLLOCATION(3, "radau")}
    out = {}
    for sname, solver in solvers.items():
        for name in ("ding2007", "ding2007_with_fatigue"):
            m = ModelMaker.create_model(name, stim_time=st30, sum_stim_truncation=10)
            out[f"{name} N=100 {sname} track"] = OcpFes.prepare_ocp(
                model=m, final_time=1, pulse_width={"min": m.pd0, "max": 6e-4}, objective=track, ode_solver=solver)
        for name in ("hmed2018", "hmed2018_with_fatigue"):
            m = ModelMaker.create_model(name, stim_time=st10, sum_stim_truncation=10)
            out[f"{name} N=10 {sname} track"] = OcpFes.prepare_ocp(
                model=m, final_time=1, pulse_intensity={"max": 130}, objective=track, ode_solver=solver)
        for name in ("ding2003", "ding2003_with_fatigue"):
            m = ModelMaker.create_model(name, stim_time=st10, sum_stim_truncation=10)
            out[f"{name} N=10 {sname} end"] = OcpFes.prepare_ocp(
                model=m, final_time=1, objective={"end_node_tracking": 100}, ode_solver=solver)
    return out


def main():
    """usage: solve_matrix.py [--native] [name filters...]; --native: the native interior point (cfx_ipm, the product
    path of OcpFes.solve) instead of the torch-orchestrated BatchedIpm of round 1."""
    from cocofest_amd.solver import BatchedIpm, IpmOptions, NativeIpm

    res = {}
    native = "--native" in sys.argv[1:]
    only = [a for a in sys.argv[1:] if a != "--native"]
    for name, ocp in cases().items():
        if only and not any(o in name for o in only):
            continue
        t0 = time.perf_counter()
        try:
            opts = IpmOptions(tol=1e-6, max_iter=300)
            ipm = NativeIpm(ocp, batch=1, device=0, options=opts) if native else BatchedIpm(ocp, batch=1, options=opts)
            r = ipm.solve()
            ipm.close()
            res[name] = {"converged": bool(r.converged[0]), "iters": int(r.iterations[0]), "f": float(r.f[0]),
                         "kkt": float(r.kkt_error[0]), "wall": round(time.perf_counter() - t0, 3)}
            if not native:
                res[name].update(nK=ipm.nK, kl=ipm.kl)
        except Exception as e:  # report, keep going
            res[name] = {"error": repr(e)[:200]}
        print(name, res[name], flush=True, file=sys.stderr)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
