"""g + J_g throughput of the shooting kernel across the model families (SoA, device-resident, sustained loops):
cfg 3 (Ding2007 pulse width, N = 100, RK1 x 10, with and without fatigue), cfg 4 (Hmed2018 intensities, N = 10,
T = 10, with the sliding-window rows), Ding2003 with fatigue.  Prints one JSON object."""

import json
import pathlib
import sys

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def problems():
    from cocofest_amd import ModelMaker, OcpFes, OdeSolver

    st30 = [float(t) for t in np.round(np.linspace(0, 1, 31)[:-1], 2)]
    st10 = [round(0.1 * i, 1) for i in range(10)]
    out = {}
    for name in ("ding2007", "ding2007_with_fatigue"):
        m = ModelMaker.create_model(name, stim_time=st30, sum_stim_truncation=10)
        out[f"cfg3 {name}"] = OcpFes.prepare_ocp(model=m, final_time=1, pulse_width={"min": m.pd0, "max": 6e-4},
                                                 objective={"end_node_tracking": 100},
                                                 ode_solver=OdeSolver.RK1(n_integration_steps=10))
    m = ModelMaker.create_model("hmed2018", stim_time=st10, sum_stim_truncation=10)
    out["cfg4 hmed2018"] = OcpFes.prepare_ocp(model=m, final_time=1, pulse_intensity={"max": 130},
                                              objective={"end_node_tracking": 100},
                                              ode_solver=OdeSolver.RK1(n_integration_steps=10))
    m = ModelMaker.create_model("ding2003_with_fatigue", stim_time=st10, sum_stim_truncation=10)
    out["ding2003_with_fatigue N=20"] = OcpFes.prepare_ocp(model=m, final_time=1, objective={"end_node_tracking": 100},
                                                           ode_solver=OdeSolver.RK1(n_integration_steps=10),
                                                           n_shooting=20)
    return out


def main():
    B = 1 << 18
    res = {}
    only = sys.argv[1] if len(sys.argv) > 1 else None
    for name, ocp in problems().items():
        if only and only not in name:
            continue
        h = ocp.nlp(batch=B, layout="soa")
        lb, ub = ocp.bounds_vector()
        lo = np.where(np.isfinite(lb), lb, 0.0)
        hi = np.where(np.isfinite(ub), np.minimum(ub, lo + 300.0), lo + 1.0)
        gen = torch.Generator(device="cuda")
        gen.manual_seed(3)
        r = torch.rand((h.nv, B), generator=gen, dtype=torch.float64, device="cuda")
        v = (torch.tensor(lo, device="cuda")[:, None] + r * torch.tensor(hi - lo, device="cuda")[:, None]).contiguous()
        g = torch.empty((h.ng, B), dtype=torch.float64, device="cuda")
        j = torch.empty((h.nnz_jac, B), dtype=torch.float64, device="cuda")
        for _ in range(10):
            h.eval_all(v, g=g, jac=j)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(100):
            h.eval_all(v, g=g, jac=j)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 100
        nbytes = 8 * (h.nv + h.ng + h.nnz_jac)
        res[name] = {"ms": round(ms, 4), "GBps": round(nbytes * B / ms / 1e6, 1), "bytes_per_instance": nbytes,
                     "evals_per_s": B / ms * 1e3}
        h.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
