"""Musculoskeletal problem builders shared by the MSK parity tests, smoke() and bench.py.

Every case is built twice from the same inputs: through the product API (cocofest_amd.FesMskModel /
OcpFesMsk, fed the parsed bioMod fixture) and independently through the oracle (oracle.fes_msk, which walks the
full segment tree of the same fixture), so the comparison covers the product's chain reduction, stim tables,
layout, objective assembly and kernels together.
"""

from __future__ import annotations

import json
import pathlib

import numpy as np

from oracle import fes_msk as M
from oracle import fes_oracle as O

GOLDEN = pathlib.Path(__file__).with_name("golden")
STIMS = [round(0.1 * i, 10) for i in range(10)]  # 10 pulses @ 10 Hz (BASELINE config 5)
FAMILY = {"ding2003": "DingModelFrequency", "ding2003_with_fatigue": "DingModelFrequencyWithFatigue",
          "ding2007": "DingModelPulseWidthFrequency", "ding2007_with_fatigue": "DingModelPulseWidthFrequencyWithFatigue",
          "hmed2018": "DingModelPulseIntensityFrequency",
          "hmed2018_with_fatigue": "DingModelPulseIntensityFrequencyWithFatigue"}
I_MAX = 130.0  # the reference's Hmed MSK intensity bounds (tests/shard2/test_fes_dynamics.py:120-125)


def _hmed(model):
    return model.startswith("hmed2018")


def biomod_path(name="arm26_biceps_triceps") -> str:
    """A fixture name, or the path of a parsed bioMod written by a test (ends in .json)."""
    return name if name.endswith(".json") else str(GOLDEN / f"biomod_{name}.json")


_ROTATED = {}


def rotated_biomod(axes=("x", "y"), base="arm26_biceps_triceps") -> str:
    """The arm26 fixture with its two joints turned to rotate about other axes (shoulder ``axes[0]``, elbow
    ``axes[1]``; the reference model has z for both), written once to a temporary .json: exercises the kernels'
    z-axis canonical frames (cfx_msk_create) against the oracle, which walks the tree with the axes as given."""
    key = (tuple(axes), base)
    if key not in _ROTATED:
        import tempfile

        d = json.loads((GOLDEN / f"biomod_{base}.json").read_text())
        it = iter(axes)
        for seg in d["segments"]:
            if seg.get("rotations") == "z":
                seg["rotations"] = next(it)
        path = pathlib.Path(tempfile.mkdtemp(prefix="cfx_biomod_")) / f"biomod_{base}_{''.join(axes)}.json"
        path.write_text(json.dumps(d))
        _ROTATED[key] = str(path)
    return _ROTATED[key]


def cfg5(**kw):
    """BASELINE config 5: arm26 biceps/triceps + Ding2007 with fatigue, 10 pulses @ 10 Hz, 1 s, elbow 5 -> 90 deg,
    FL/FV on, no residual torque, qdot(end) = 0 (weight 100) and minimize_muscle_fatigue, RK4 x 1
    (examples/dynamics/minimize_fatigue/pulse_duration_optimization_minimize_fatigue.py:15-55)."""
    d = dict(model="ding2007_with_fatigue", biomod="arm26_biceps_triceps", muscles=("BIClong", "TRIlong"),
             scheme="RK4", m=1, fv=True, residual=False, fatigue=True, qdot_end=True, truncation=10)
    d.update(kw)
    return d


def product_ocp(model, biomod, muscles, scheme, m, fv, residual, fatigue, qdot_end, truncation, bound=(5, 90),
                passive=False, markers=(), bound_type="start_end", legacy=False):
    """``markers``: SUPERIMPOSE_MARKERS constraints as dicts first, second, node (int or "end"), axes (indices),
    passed through msk_info["custom_constraint"] with apply_custom_constraint=True.  ``legacy``: the stored
    reaching-task revision's calcium sum (FesMskModel(legacy_calcium=True), CFX_MSK_LEGACY_CALCIUM)."""
    import cocofest_amd as C

    pint = None
    if _hmed(model):  # intensities bounded by [I_min, 130] (the reference's Hmed MSK test)
        pint = {"min": float(O.min_pulse_intensity(O.model_constants(model))), "max": I_MAX}
    cls = getattr(C, FAMILY[model])
    mm = C.FesMskModel(biorbd_path=biomod_path(biomod),
                       muscles_model=[cls(muscle_name=n, sum_stim_truncation=truncation) for n in muscles],
                       stim_time=list(STIMS), activate_force_length_relationship=fv,
                       activate_force_velocity_relationship=fv, activate_residual_torque=residual,
                       legacy_calcium=legacy)
    obj = {}
    if qdot_end:
        ol = C.ObjectiveList()
        ol.add(C.ObjectiveFcn.Mayer.MINIMIZE_STATE, key="qdot", index=list(range(mm.nb_q)), node=C.Node.END,
               target=np.zeros((mm.nb_q, 1)), weight=100, quadratic=True, phase=0)
        obj["custom"] = ol
    if fatigue:
        obj["minimize_muscle_fatigue"] = True
    if residual:
        obj["minimize_residual_torque"] = True
    solver = {"RK1": C.OdeSolver.RK1, "RK2": C.OdeSolver.RK2, "RK4": C.OdeSolver.RK4}[scheme](n_integration_steps=m)
    nq = mm.nb_q
    start, end = [0] * (nq - 1) + [bound[0]], [0] * (nq - 1) + [bound[1]]
    info = {"bound_type": bound_type, "bound_data": {"start_end": [start, end], "start": start, "end": end}[bound_type],
            "with_residual_torque": residual}
    if markers:
        cl = C.ConstraintList()
        for mk in markers:
            cl.add(C.ConstraintFcn.SUPERIMPOSE_MARKERS, first_marker=mk["first"], second_marker=mk["second"],
                   node=C.Node.END if mk["node"] == "end" else mk["node"], axes=[C.Axis(a) for a in mk["axes"]],
                   phase=0)
        info["custom_constraint"] = cl
    ocp = C.OcpFesMsk.prepare_ocp(model=mm, final_time=1, objective=obj, msk_info=info, ode_solver=solver,
                                  pulse_intensity=pint, apply_custom_constraint=bool(markers))
    if passive:  # OcpFesMsk drops the flag as the reference does; set it back to exercise the kernels' FP term
        ocp.model.activate_passive_force_relationship = True
    return ocp


def oracle_problem(model, biomod, muscles, scheme, m, fv, residual, fatigue, qdot_end, truncation, bound=(5, 90),
                   passive=False, markers=(), bound_type="start_end", legacy=False):
    bm = json.loads(pathlib.Path(biomod_path(biomod)).read_text())
    n = O.prepare_n_shooting(STIMS, 1)
    tab = O.stim_table(STIMS, n, 1, truncation)
    mus = [M.MskMuscle(model=model, name=nm, c=O.model_constants(model)) for nm in muscles]
    pb = M.MskProblem(bm=bm, muscles=mus, rows=tab.rows, n_shooting=n, final_time=1.0, scheme=scheme, m=m, fv_on=fv,
                      fp_on=passive, residual=residual, legacy=legacy)
    if _hmed(model):  # one block of n_stim intensity parameters per muscle; node k's window ends at its last pulse
        pb.n_params = len(STIMS) * len(muscles)
        pb.param_offset = [i * len(STIMS) for i in range(len(muscles))]
        dt = 1.0 / n
        pb.last_stim_idx = [sum(1 for t in STIMS if t <= k * dt + 1e-12) - 1 for k in range(n)]
    nq, nxm = pb.nq, pb.nxm
    if qdot_end:
        for j in range(nq):
            pb.objectives.append(dict(kind=1, var_kind=0, var_index=nxm + nq + j, node_first=n, node_last=n,
                                      weight=100.0, target_value=0.0))
    if residual:
        for j in range(nq):
            pb.objectives.append(dict(kind=0, var_kind=1, var_index=pb.n_pw + pb.n_int + j, node_first=0,
                                      node_last=n - 1, weight=10000.0, target_value=0.0))
    if fatigue:
        pb.fatigue_weight = 1.0
    for mk in markers:
        pb.marker_pairs.append(dict(node=n if mk["node"] == "end" else mk["node"], first=mk["first"],
                                    second=mk["second"], axes=sorted(set(mk["axes"]))))
    return pb


def random_decision(pb, B, seed=0):
    """(B, nv) decision vectors inside the physiological envelope: calcium / force / fatigue states around their
    rest values, elbow angle in (0.1, 2.5) rad, shoulder in (-0.5, 0.5), joint velocities within +-2 rad/s,
    pulse widths in [pd0, 0.6 ms], residual torques within +-5 N m."""
    r = np.random.default_rng(seed)
    N, nx, nq = pb.n_shooting, pb.nx, pb.nq
    X = np.empty((B, N + 1, nx))
    off = 0
    for mus in pb.muscles:
        c = mus.c
        X[..., off] = r.uniform(0.0, 1.5, X.shape[:2])
        X[..., off + 1] = r.uniform(0.0, 150.0, X.shape[:2])
        if O.n_states(mus.model) == 5:
            a0 = c["a_scale"] if mus.model.startswith("ding2007") else c["a_rest"]
            X[..., off + 2] = a0 * r.uniform(0.8, 1.0, X.shape[:2])
            X[..., off + 3] = c["tau1_rest"] * r.uniform(1.0, 1.2, X.shape[:2])
            X[..., off + 4] = c["km_rest"] * r.uniform(1.0, 1.2, X.shape[:2])
        off += O.n_states(mus.model)
    for j in range(nq):
        last = j == nq - 1
        X[..., off + j] = r.uniform(0.1, 2.5, X.shape[:2]) if last else r.uniform(-0.5, 0.5, X.shape[:2])
        X[..., off + nq + j] = r.uniform(-2.0, 2.0, X.shape[:2])
    U = np.empty((B, N, pb.nu))
    for i in range(pb.n_pw):
        U[..., i] = r.uniform(1.4e-4, 6e-4, U.shape[:2])
    imin = [O.min_pulse_intensity(m.c) for m in pb.muscles if O.control_kind(m.model) == "pulse_intensity"]
    for i in range(pb.n_int):  # intensities in [I_min, 130]
        U[..., pb.n_pw + i] = r.uniform(imin[i // pb.T], I_MAX, U.shape[:2])
    for j in range(nq if pb.residual else 0):
        U[..., pb.n_pw + pb.n_int + j] = r.uniform(-5.0, 5.0, U.shape[:2])
    V = np.empty((B, pb.nv))
    body = V[:, : N * pb.nz].reshape(B, N, pb.nz)
    body[..., :nx] = X[:, :N]
    body[..., nx:] = U
    V[:, N * pb.nz: N * pb.nz + nx] = X[:, N]
    if pb.n_params:
        V[:, N * pb.nz + nx:] = r.uniform(imin[0], I_MAX, (B, pb.n_params))
    return V
