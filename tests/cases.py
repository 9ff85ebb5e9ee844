"""Problem builders shared by the parity tests, smoke() and bench.py.

Each case is built twice from the same inputs: once through the product API (cocofest_amd.OcpFes) and
once, independently, through the oracle (oracle.fes_oracle), so the comparison checks the product's
table building, layout, objective assembly and kernels together.
"""

from __future__ import annotations

import numpy as np

from oracle import fes_oracle as O

SCHEMES = {"RK1": 1, "RK2": 2, "RK4": 4}


def product_ocp(name, stims, final_time, truncation, scheme="RK4", m=3, objective=None, n_shooting=None,
                intensity_params=True):
    from cocofest_amd import ModelMaker, OcpFes, OdeSolver

    model = ModelMaker.create_model(name, stim_time=list(stims), sum_stim_truncation=truncation)
    kw = {}
    if name.startswith("ding2007"):
        kw["pulse_width"] = {"min": model.pd0, "max": 0.0006}
    if name.startswith("hmed2018") and intensity_params:
        kw["pulse_intensity"] = {"max": 130}
    solver = {"RK1": OdeSolver.RK1, "RK2": OdeSolver.RK2, "RK4": OdeSolver.RK4}[scheme](n_integration_steps=m)
    return OcpFes.prepare_ocp(model=model, final_time=final_time, objective=objective or {}, ode_solver=solver,
                              n_shooting=n_shooting, **kw)


def oracle_problem(name, stims, final_time, truncation, scheme="RK4", m=3, objective=None, n_shooting=None,
                   intensity_params=True):
    c = O.model_constants(name)
    n = O.prepare_n_shooting(stims, final_time) if n_shooting is None else n_shooting
    tab = O.stim_table(stims, n, final_time, truncation)
    pb = O.Problem(name=name, c=c, n_shooting=n, final_time=final_time, truncation=truncation, rows=tab.rows,
                   scheme=scheme, n_steps=m)
    if name.startswith("hmed2018") and intensity_params:
        pb.n_params = len(stims)
        pb.last_stim_idx = [s[-1] for s in tab.stim_idx_at_node[:n]]
        pb.intensity_floor = O.min_pulse_intensity(c)
    objective = objective or {}
    if objective.get("force_tracking") is not None:
        t, f = objective["force_tracking"]
        pb.objectives.append(O.Objective("lagrange", ("x", 1), 100.0, O.fourier_target(t, f, n), list(range(n + 1))))
    if objective.get("end_node_tracking") is not None:
        pb.objectives.append(O.Objective("mayer", ("x", 1), 1.0, np.full(n + 1, float(objective["end_node_tracking"])),
                                         [n]))
    return pb


def random_decision(pb, B, seed=0):
    """Decision vectors (B, nv) around physiological values (states inside the OCP bounds)."""
    r = np.random.default_rng(seed)
    X = np.empty((B, pb.n_shooting + 1, pb.nx))
    X[..., 0] = r.uniform(0.0, 1.5, X.shape[:2])
    X[..., 1] = r.uniform(0.0, 250.0, X.shape[:2])
    if pb.nx == 5:
        a0 = pb.c["a_scale"] if pb.name.startswith("ding2007") else pb.c["a_rest"]
        X[..., 2] = a0 * r.uniform(0.7, 1.0, X.shape[:2])
        X[..., 3] = r.uniform(pb.c["tau1_rest"], 0.1, X.shape[:2])
        X[..., 4] = r.uniform(pb.c["km_rest"], 0.3, X.shape[:2])
    U = np.empty((B, pb.n_shooting, pb.nu))
    if O.control_kind(pb.name) == "pulse_width":
        U[...] = r.uniform(pb.c["pd0"], 6e-4, U.shape)
    elif pb.nu:
        U[...] = r.uniform(17.1, 130.0, U.shape)
    P = r.uniform(17.1, 130.0, (B, pb.n_params))
    body = np.concatenate([X[:, :-1, :], U], axis=2).reshape(B, -1)
    return np.concatenate([body, X[:, -1, :], P], axis=1)


# BASELINE.json configs
TEN_PULSES = [round(0.1 * i, 1) for i in range(10)]


def cfg2(n_shooting=20):
    """OcpFes DingModelFrequency, 10 pulses @ 10 Hz, T = 1 s, end force 100 N, RK1 x 10 (reference default)."""
    return dict(name="ding2003", stims=TEN_PULSES, final_time=1.0, truncation=20, scheme="RK1", m=10,
                objective={"end_node_tracking": 100}, n_shooting=n_shooting)


def cfg3(fatigue=False):
    """OcpFes Ding2007 pulse width, 30 pulses at round(linspace(0,1,31)[:-1], 2), truncation 10, force tracking."""
    stims = [float(v) for v in np.round(np.linspace(0, 1, 31)[:-1], 2)]
    return dict(name="ding2007_with_fatigue" if fatigue else "ding2007", stims=stims, final_time=1.0, truncation=10,
                scheme="RK1", m=10, objective=None, n_shooting=None)


def random_collocation_decision(pb, B, seed=0):
    """Decision vectors (B, nv) of a collocation problem (oracle ColProblem): node states / controls / parameters
    as random_decision, collocation states within +-20 % of their interval's start state."""
    from oracle import fes_oracle as O

    base_pb = O.Problem(**{f: getattr(pb, f) for f in O.Problem.__dataclass_fields__})
    base = random_decision(base_pb, B, seed)
    X, U, P = base_pb.unpack(base)
    rng = np.random.default_rng(seed + 1)
    XC = np.repeat(X[:, :-1, None, :], pb.degree + 1, axis=2)
    XC[:, :, 1:, :] *= rng.uniform(0.8, 1.2, (B, pb.n_shooting, pb.degree, pb.nx))
    return pb.pack(XC, X[:, -1], U if pb.nu else None, P if pb.n_params else None)


def product_collocation_ocp(name, stims, final_time, truncation, degree=3, method="legendre", objective=None,
                            n_shooting=None, intensity_params=True):
    from cocofest_amd import ModelMaker, OcpFes, OdeSolver

    model = ModelMaker.create_model(name, stim_time=list(stims), sum_stim_truncation=truncation)
    kw = {}
    if name.startswith("ding2007"):
        kw["pulse_width"] = {"min": model.pd0, "max": 0.0006}
    if name.startswith("hmed2018") and intensity_params:
        kw["pulse_intensity"] = {"max": 130}
    return OcpFes.prepare_ocp(model=model, final_time=final_time, objective=objective or {},
                              ode_solver=OdeSolver.COLLOCATION(degree, method), n_shooting=n_shooting, **kw)
