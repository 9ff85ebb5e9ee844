"""Musculoskeletal FES problems: ``FesMskModel`` and ``OcpFesMsk`` (reference: cocofest/models/dynamical_model.py,
cocofest/optimization/fes_ocp_dynamics.py).

The reference couples its FES muscle models to a biorbd rigid-body model through bioptim; neither library is
part of this build.  Here the bioMod file is read on the host (the subset of the format the reference's
``examples/msk_models/*.bioMod`` use), reduced to a serial chain of revolute dofs — constant segment
transforms between two dofs are composed, segments that move with the same dof are merged into one composite
rigid body, muscle path points are re-expressed in the frame of the dof they move with — and handed to libcfx
(``cfx_msk_create``), whose gfx950 kernels evaluate the coupled right-hand side (muscle ODEs, De Groote force
coefficients, muscle-tendon lengths and their Jacobian, joint torques, forward dynamics) inside the RK
transcription, with its Jacobian and Lagrangian Hessian.  No part of the evaluation runs on the CPU.
"""

from __future__ import annotations

import json
import math
import pathlib
import re
import warnings

import numpy as np

from . import _cfx
from .fes_models import DingModelPulseIntensityFrequency, DingModelPulseWidthFrequency, FesModel
from .fourier import FourierSeries
from .ocp import Constraint, ConstraintFcn, Node, Objective, ObjectiveFcn, ObjectiveList, OcpFes
from .ode_solver import ControlType, OdeSolver

# ---------------------------------------------------------------------------------------------------------------
# bioMod reading (biorbd text format)
# ---------------------------------------------------------------------------------------------------------------

_NUM = re.compile(r"^[-+]?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?$")


def _value(tok: str) -> float:
    """A number, or a product / quotient of numbers and ``pi`` (``-2*pi``, ``pi/2``)."""
    if _NUM.match(tok):
        return float(tok)
    sign = -1.0 if tok.startswith("-") else 1.0
    tok = tok.lstrip("+-")
    out, op = 1.0, "*"
    for part in re.split(r"([*/])", tok):
        if part in ("*", "/"):
            op = part
            continue
        v = math.pi if part == "pi" else float(part)
        out = out * v if op == "*" else out / v
    return sign * out


_SKIP = {"meshfile": 1, "meshscale": 3, "meshcolor": 3, "mesh": 3}


def parse_biomod(text: str) -> dict:
    """bioMod text -> {"gravity", "segments", "markers", "muscles"} (segments in file order, each with parent, 4x4
    RT, rotation axes, mass, com, inertia, q ranges; markers with their parent segment and position; muscles with
    their path and characteristics)."""
    words = " ".join(line.split("//", 1)[0] for line in text.splitlines()).split()
    it = iter(words)
    model = {"gravity": [0.0, 0.0, -9.81], "segments": [], "markers": [], "muscles": []}
    groups, vias = {}, []

    def take(n):
        return [_value(next(it)) for _ in range(n)]

    for word in it:
        key = word.lower()
        if key == "version":
            next(it)
        elif key == "gravity":
            model["gravity"] = take(3)
        elif key == "segment":
            seg = {"name": next(it), "parent": None, "RT": np.eye(4).tolist(), "rotations": "", "mass": 0.0,
                   "com": [0.0, 0.0, 0.0], "inertia": [[0.0] * 3 for _ in range(3)], "rangesQ": []}
            matrix = False
            for w in it:
                k = w.lower()
                if k == "endsegment":
                    break
                if k == "parent":
                    seg["parent"] = next(it)
                elif k == "rtinmatrix":
                    matrix = _value(next(it)) != 0
                elif k == "rt":
                    if not matrix:
                        raise NotImplementedError("bioMod: only RTinMatrix 1 segment transforms are supported")
                    seg["RT"] = np.array(take(16)).reshape(4, 4).tolist()
                elif k == "rotations":
                    seg["rotations"] = next(it).lower()
                elif k == "translations":
                    raise NotImplementedError("bioMod: translational dofs are not supported")
                elif k == "mass":
                    seg["mass"] = _value(next(it))
                elif k == "com":
                    seg["com"] = take(3)
                elif k == "inertia":
                    seg["inertia"] = np.array(take(9)).reshape(3, 3).tolist()
                elif k == "rangesq":
                    seg["rangesQ"] = np.array(take(2 * len(seg["rotations"]))).reshape(-1, 2).tolist()
                elif k in _SKIP:
                    for _ in range(_SKIP[k]):
                        next(it)
                else:
                    raise NotImplementedError(f"bioMod: segment keyword {w!r} is not supported")
            model["segments"].append(seg)
        elif key == "marker":  # a point fixed in its parent segment: parent, position
            mk = {"name": next(it), "parent": None, "position": [0.0, 0.0, 0.0]}
            for w in it:
                k = w.lower()
                if k == "endmarker":
                    break
                if k == "parent":
                    mk["parent"] = next(it)
                elif k == "position":
                    mk["position"] = take(3)
                elif k in ("technical", "anatomical", "axestoremove"):
                    next(it)
                else:
                    raise NotImplementedError(f"bioMod: marker keyword {w!r} is not supported")
            model["markers"].append(mk)
        elif key == "musclegroup":
            name, grp = next(it), {}
            for w in it:
                if w.lower() == "endmusclegroup":
                    break
                grp[w.lower()] = next(it)
            groups[name] = grp
        elif key == "muscle":
            mus = {"name": next(it)}
            for w in it:
                k = w.lower()
                if k == "endmuscle":
                    break
                if k in ("type", "statetype", "musclegroup"):
                    mus[k] = next(it)
                elif k in ("originposition", "insertionposition"):
                    mus[k.replace("position", "")] = take(3)
                elif k == "fatigueparameters":
                    for w2 in it:
                        if w2.lower() == "endfatigueparameters":
                            break
                else:
                    mus[k] = _value(next(it))
            model["muscles"].append(mus)
        elif key == "viapoint":
            via = {"name": next(it)}
            for w in it:
                k = w.lower()
                if k == "endviapoint":
                    break
                via[k] = take(3) if k == "position" else next(it)
            vias.append(via)
        else:
            raise NotImplementedError(f"bioMod: {word!r} is not supported")
    for mus in model["muscles"]:
        grp = groups[mus["musclegroup"]]
        mus["origin_parent"], mus["insertion_parent"] = grp["originparent"], grp["insertionparent"]
        mus["via"] = [{"parent": v["parent"], "position": v["position"]} for v in vias if v["muscle"] == mus["name"]]
    return model


def load_biomod(path) -> dict:
    """Read a ``.bioMod`` file, or the same content already parsed and saved as ``.json``."""
    p = pathlib.Path(path)
    text = p.read_text()
    return json.loads(text) if p.suffix.lower() == ".json" else parse_biomod(text)


_AXIS = {"x": 0, "y": 1, "z": 2}


def reduce_to_chain(bm: dict) -> dict:
    """Serial chain of revolute dofs: per dof the constant joint frame relative to the previous dof's frame, one
    composite body per dof frame, and every muscle path point and marker in the frame of the dof it moves with."""
    frame_of, K_of = {}, {}  # segment -> (dof frame index or -1, constant 4x4 from that frame to the segment)
    axes, frames, names, ranges = [], [], [], []
    for seg in bm["segments"]:
        f, K = (frame_of[seg["parent"]], K_of[seg["parent"]]) if seg["parent"] else (-1, np.eye(4))
        T = K @ np.asarray(seg["RT"], dtype=float)
        for i, ax in enumerate(seg["rotations"]):
            if f != len(axes) - 1:
                raise NotImplementedError("bioMod: branched kinematic trees are not supported (serial chains only)")
            frames.append(np.concatenate([T[:3, :3].reshape(-1), T[:3, 3]]))
            axes.append(_AXIS[ax])
            names.append(f"{seg['name']}_Rot{ax.upper()}")
            ranges.append(seg["rangesQ"][i] if seg["rangesQ"] else [-np.pi, np.pi])
            f, T = len(axes) - 1, np.eye(4)
        frame_of[seg["name"]], K_of[seg["name"]] = f, T
    nq = len(axes)
    if nq == 0:
        raise ValueError("bioMod: the model has no degree of freedom")
    mass = np.zeros(nq)
    msum = np.zeros((nq, 3))
    parts = [[] for _ in range(nq)]
    for seg in bm["segments"]:
        f = frame_of[seg["name"]]
        if f < 0 or seg["mass"] == 0:
            continue
        K = K_of[seg["name"]]
        c = K[:3, :3] @ np.asarray(seg["com"], dtype=float) + K[:3, 3]
        I = K[:3, :3] @ np.asarray(seg["inertia"], dtype=float) @ K[:3, :3].T
        mass[f] += seg["mass"]
        msum[f] += seg["mass"] * c
        parts[f].append((seg["mass"], c, I))
    com = np.where(mass[:, None] > 0, msum / np.maximum(mass, 1e-300)[:, None], 0.0)
    inertia = np.zeros((nq, 3, 3))
    for f in range(nq):
        for m, c, I in parts[f]:
            d = c - com[f]
            inertia[f] += I + m * (d @ d * np.eye(3) - np.outer(d, d))
    muscles = {}
    for mus in bm["muscles"]:
        path = ([(mus["origin_parent"], mus["origin"])] + [(v["parent"], v["position"]) for v in mus["via"]]
                + [(mus["insertion_parent"], mus["insertion"])])
        pf, pp = [], []
        for seg, p in path:
            K = K_of[seg]
            pf.append(frame_of[seg])
            pp.append(K[:3, :3] @ np.asarray(p, dtype=float) + K[:3, 3])
        muscles[mus["name"]] = {"point_frame": np.array(pf, dtype=np.int32), "point_pos": np.array(pp),
                                "optimal_length": float(mus["optimallength"]),
                                "tendon_slack_length": float(mus["tendonslacklength"]),
                                "pennation_angle": float(mus.get("pennationangle", 0.0))}
    markers = {}
    for mk in bm.get("markers", []):
        K = K_of[mk["parent"]]
        markers[mk["name"]] = {"frame": int(frame_of[mk["parent"]]),
                               "pos": K[:3, :3] @ np.asarray(mk["position"], dtype=float) + K[:3, 3]}
    return {"axis": np.array(axes, dtype=np.int32), "frame": np.array(frames), "gravity": np.array(bm["gravity"]),
            "mass": mass, "com": com, "inertia": inertia.reshape(nq, 9), "q_names": names,
            "q_ranges": np.array(ranges, dtype=float), "muscles": muscles,
            "muscle_order": [m["name"] for m in bm["muscles"]], "markers": markers}


# ---------------------------------------------------------------------------------------------------------------
# FesMskModel (cocofest/models/dynamical_model.py:28-495)
# ---------------------------------------------------------------------------------------------------------------


class FesMskModel:
    """FES muscles driving a biorbd skeleton (reference: ``FesMskModel``, dynamical_model.py:28-125).

    ``biorbd_path`` names a ``.bioMod`` (or its parsed ``.json``); ``muscles_model`` lists one FES model per
    driven muscle, matched to the bioMod muscles by ``muscle_name``."""

    def __init__(self, name: str = None, biorbd_path: str = None, muscles_model: list = None,
                 stim_time: list = None, previous_stim: dict = None,
                 activate_force_length_relationship: bool = False, activate_force_velocity_relationship: bool = False,
                 activate_passive_force_relationship: bool = False, activate_residual_torque: bool = False,
                 parameters=None, external_force_set=None, legacy_calcium: bool = False):
        if parameters is not None or external_force_set is not None:
            raise NotImplementedError("FesMskModel: parameters / external forces are not supported")
        self._model_sanity(muscles_model, activate_force_length_relationship, activate_force_velocity_relationship)
        self._name = name
        self.biorbd_path = biorbd_path
        self.bio_model = load_biomod(biorbd_path)
        self.chain = reduce_to_chain(self.bio_model)
        self.muscles_dynamics_model = muscles_model
        for m in self.muscles_dynamics_model:
            if m.muscle_name not in self.chain["muscles"]:
                raise ValueError(f"muscle {m.muscle_name!r} is not in {biorbd_path}")
            m.stim_time = stim_time if stim_time else m.stim_time
            m.previous_stim = previous_stim if previous_stim else m.previous_stim
            m.all_stim = list(m.previous_stim["time"]) + list(m.stim_time or [])
        self.bio_stim_model = [self.bio_model] + self.muscles_dynamics_model
        self.activate_force_length_relationship = activate_force_length_relationship
        self.activate_force_velocity_relationship = activate_force_velocity_relationship
        self.activate_passive_force_relationship = activate_passive_force_relationship
        self.activate_residual_torque = activate_residual_torque
        self.parameters_list = parameters
        self.external_forces_set = external_force_set
        # extension: the calcium-sum conventions of the revision that stored the reaching-task solutions (a window's
        # first pulse left out once it holds several; the fatigue models' r0 from the Km state), CFX_MSK_LEGACY_CALCIUM
        self.legacy_calcium = bool(legacy_calcium)

    @staticmethod
    def _model_sanity(muscles_model, activate_force_length_relationship, activate_force_velocity_relationship):
        """dynamical_model.py:455-479."""
        if not isinstance(muscles_model, list):
            raise TypeError("The given muscles_model must be a list of FesModel")
        for muscle_model in muscles_model:
            if not isinstance(muscle_model, FesModel):
                raise TypeError(
                    f"The current model type used is {type(muscles_model)}, it must be a FesModel type."
                    f"Current available models are: DingModelFrequency, DingModelFrequencyWithFatigue,"
                    f"DingModelPulseWidthFrequency, DingModelPulseWidthFrequencyWithFatigue,"
                    f"DingModelPulseIntensityFrequency, DingModelPulseIntensityFrequencyWithFatigue")
        if not isinstance(activate_force_length_relationship, bool):
            raise TypeError("The activate_force_length_relationship must be a boolean")
        if not isinstance(activate_force_velocity_relationship, bool):
            raise TypeError("The activate_force_velocity_relationship must be a boolean")

    @property
    def name(self):
        return self._name

    @property
    def name_dof(self) -> tuple:
        return tuple(self.chain["q_names"])

    @property
    def nb_q(self) -> int:
        return len(self.chain["axis"])

    nb_qdot = nb_q
    nb_tau = nb_q

    @property
    def muscle_names(self) -> list:
        return [m.muscle_name for m in self.muscles_dynamics_model]

    def muscle_name_dof(self, index: int = 0) -> list:
        m = self.muscles_dynamics_model[index]
        return [f"{n}_{m.muscle_name}" for n in m.name_dof]

    @property
    def nb_state(self) -> int:
        return sum(m.nb_state for m in self.muscles_dynamics_model) + self.nb_q

    def state_names(self) -> list:
        """Decision-state order: muscle blocks (state_configure.py:294-307), q, qdot (dynamical_model.py:429-433)."""
        out = []
        for i in range(len(self.muscles_dynamics_model)):
            out += self.muscle_name_dof(i)
        return out + [f"q_{n}" for n in self.name_dof] + [f"qdot_{n}" for n in self.name_dof]

    def bounds_from_ranges(self, key: str) -> np.ndarray:
        """(nq, 2) bounds from the bioMod ranges: rangesQ for q, biorbd's default +-10 pi for qdot."""
        if key == "q":
            return self.chain["q_ranges"].copy()
        if key == "qdot":
            return np.tile([-10 * np.pi, 10 * np.pi], (self.nb_q, 1))
        raise ValueError(f"unknown key {key}")

    def cfx_chain(self) -> dict:
        return {k: self.chain[k] for k in ("axis", "frame", "gravity", "mass", "com", "inertia")}

    def cfx_muscles(self) -> list:
        out = []
        for m in self.muscles_dynamics_model:
            g = self.chain["muscles"][m.muscle_name]
            out.append({"model_id": m.cfx_model_id, "constants": m.cfx_constants(), **g})
        return out

    def cfx_flags(self) -> int:
        """Force-coefficient flags as the reference applies them: the force-length coefficient is computed only
        when ``activate_force_velocity_relationship`` is set (dynamical_model.py:259-269)."""
        f = 0
        if self.activate_force_velocity_relationship:
            f |= _cfx.MSK_FORCE_LENGTH | _cfx.MSK_FORCE_VELOCITY
        if self.activate_passive_force_relationship:
            f |= _cfx.MSK_PASSIVE_FORCE
        if self.activate_residual_torque:
            f |= _cfx.MSK_RESIDUAL_TORQUE
        if getattr(self, "legacy_calcium", False):
            f |= _cfx.MSK_LEGACY_CALCIUM
        return f


# ---------------------------------------------------------------------------------------------------------------
# OcpFesMsk (cocofest/optimization/fes_ocp_dynamics.py:33-801)
# ---------------------------------------------------------------------------------------------------------------


class FesMskOcp:
    """Transcribed musculoskeletal FES OCP: layout, bounds, initial guess, objective and GPU callbacks.

    Decision vector per instance [x_0, u_0, ..., x_{N-1}, u_{N-1}, x_N (, p)]; states [muscle blocks, q, qdot],
    controls [pulse width per muscle (Ding2007) | T pulse intensities per muscle (Hmed2018)] then [tau] (residual
    torque); Hmed2018: the trailing parameters p are the pulses' intensities (per muscle, or shared), tied to the
    intensity controls by the sliding-window rows (fes_ocp_dynamics.py:343-438)."""

    def __init__(self, model: FesMskModel, n_shooting, final_time, ode_solver, rows, objectives, x_bounds, x_init,
                 u_bounds, u_init, state_names, control_names, n_threads=1, use_sx=True, n_params=0, p_bounds=None,
                 p_init=None, param_names=(), last_stim_idx=None, param_offset=None, marker_pairs=(), per_pulse=False,
                 per_pulse_bounds="all"):
        self.model = model
        self.n_shooting = n_shooting
        self.final_time = final_time
        self.ode_solver = ode_solver
        self.stim_rows = rows
        self.objectives = objectives
        self.x_bounds, self.x_init = x_bounds, x_init
        self.u_bounds, self.u_init = u_bounds, u_init
        self.state_names, self.control_names = state_names, control_names
        self.nx, self.nu = len(state_names), len(control_names)
        self.n_threads, self.use_sx = n_threads, use_sx
        self.truncation = model.muscles_dynamics_model[0]._sum_stim_truncation
        self.n_params = int(n_params)
        self.p_bounds = p_bounds if p_bounds is not None else (np.zeros(0), np.zeros(0))
        self.p_init = p_init if p_init is not None else np.zeros(0)
        self.param_names = list(param_names)  # one name per parameter block, e.g. pulse_intensity_BIClong
        self.last_stim_idx = last_stim_idx
        self.param_offset = param_offset
        # SUPERIMPOSE_MARKERS rows after every interval's rows (cfx_msk_marker_pair dicts + marker names)
        self.marker_pairs = list(marker_pairs)
        # pulse_width["per_pulse"]: the intervals that follow one pulse share its widths (rows after the marker rows);
        # per_pulse_bounds: "all" (every interval's copy bounded) or "first" (the pulse's first interval; bounds_vector)
        self.per_pulse = bool(per_pulse)
        self.per_pulse_bounds = per_pulse_bounds

    @property
    def n_marker_rows(self) -> int:
        return sum(bin(c["axes"]).count("1") for c in self.marker_pairs)

    @property
    def nzb(self):
        return self.nx + self.nu

    @property
    def nv(self):
        return self.n_shooting * self.nzb + self.nx + self.n_params

    def pack(self, x, u=None, p=None):
        N, nx = self.n_shooting, self.nx
        v = np.empty(self.nv)
        body = v[: N * self.nzb].reshape(N, self.nzb)
        body[:, :nx] = np.asarray(x, dtype=float)[:, :N].T
        if self.nu:
            body[:, nx:] = np.asarray(u, dtype=float).T
        v[N * self.nzb: N * self.nzb + nx] = np.asarray(x, dtype=float)[:, N]
        if self.n_params:
            v[N * self.nzb + nx:] = np.asarray(p, dtype=float)
        return v

    def unpack(self, v):
        """(states, controls, parameters) dicts, each value (1, n) — parameters by block name."""
        N, nx = self.n_shooting, self.nx
        v = np.asarray(v)
        body = v[: N * self.nzb].reshape(N, self.nzb)
        x = np.concatenate([body[:, :nx].T, v[N * self.nzb: N * self.nzb + nx, None]], axis=1)
        states = {n: x[i][None, :] for i, n in enumerate(self.state_names)}
        controls = {n: body[:, nx + i][None, :] for i, n in enumerate(self.control_names)}
        params = {}
        if self.n_params:
            p = v[N * self.nzb + nx:]
            bounds = list(self.param_offset_blocks()) + [self.n_params]
            for i, name in enumerate(self.param_names):
                params[name] = p[bounds[i]: bounds[i + 1]][None, :]
        return states, controls, params

    def param_offset_blocks(self):
        return sorted(set(int(o) for o in self.param_offset)) if self.n_params else []

    def tied_intervals(self):
        """pulse_width["per_pulse"]: the intervals k >= 1 that follow the same pulse as k - 1 (same last stimulation
        time in the window: the tie rows u_k - u_{k-1} = 0 of CFX_MSK_PULSE_WIDTH_PER_PULSE, cfx_api.hip)."""
        if not self.per_pulse:
            return np.zeros(self.n_shooting, dtype=bool)
        last = np.asarray(self.stim_rows, dtype=float).reshape(self.n_shooting + 1, -1)[:, -1]
        return np.concatenate([[False], last[1: self.n_shooting] == last[: self.n_shooting - 1]])

    def bounds_vector(self):
        """(lb, ub) over the decision vector.  pulse_width["per_pulse"] with per_pulse_bounds "first": the bounds of a
        pulse's width bind on the pulse's first interval only, as on the stored revision's per-pulse PARAMETER (one
        bound per pulse; the tie-row statement otherwise has a copy per interval, 25 copies of one active bound tied by
        24 rows: degenerate multipliers); the copies' bounds are moved one range outwards (never active while the tie
        rows hold; finite, so the range scaling of the variable is unchanged).  "all" (default) bounds every copy —
        the iterates then stay inside the range even where the tie rows do not yet hold (DESIGN.md section 9 has the
        solves of both)."""
        lb = self.pack(self.x_bounds[0], self.u_bounds[0], self.p_bounds[0])
        ub = self.pack(self.x_bounds[1], self.u_bounds[1], self.p_bounds[1])
        tied = self.tied_intervals()
        if tied.any() and self.per_pulse_bounds == "first":
            nm = len(self.model.muscles_dynamics_model)
            cols = (np.nonzero(tied)[0][:, None] * self.nzb + self.nx + np.arange(nm)[None, :]).ravel()
            w = ub[cols] - lb[cols]
            lb[cols] -= w
            ub[cols] += w
        return lb, ub

    def initial_guess_vector(self):
        return self.pack(self.x_init, self.u_init, self.p_init)

    def nlp(self, batch: int = 1, layout: str = "aos", device: int = 0) -> _cfx.MskHandle:
        """Open a libcfx handle evaluating ``batch`` instances of this problem on GPU ``device``."""
        return _cfx.MskHandle(
            chain=self.model.cfx_chain(), muscles=self.model.cfx_muscles(), scheme=self.ode_solver.scheme,
            n_steps=self.ode_solver.n_integration_steps, n_shooting=self.n_shooting, truncation=self.truncation,
            final_time=float(self.final_time), stim_rows=self.stim_rows, batch=batch,
            flags=self.model.cfx_flags() | (_cfx.MSK_PULSE_WIDTH_PER_PULSE if self.per_pulse else 0),
            layout={"aos": _cfx.LAYOUT_AOS, "soa": _cfx.LAYOUT_SOA}[layout], objectives=self.objectives,
            device=device, n_params=self.n_params, last_stim_idx=self.last_stim_idx, param_offset=self.param_offset,
            marker_pairs=self.marker_pairs)

    def solve(self, solver=None, **kwargs):
        from .solver import solve_ocp

        return solve_ocp(self, solver=solver, **kwargs)


class OcpFesMsk:
    """Prepares the musculoskeletal FES OCP (reference: cocofest/optimization/fes_ocp_dynamics.py:33-801)."""

    @staticmethod
    def prepare_ocp(model: FesMskModel = None, final_time: int | float = None, pulse_width: dict = None,
                    pulse_intensity: dict = None, objective: dict = None, msk_info: dict = None, use_sx: bool = True,
                    initial_guess_warm_start: bool = False, ode_solver=OdeSolver.RK4(n_integration_steps=1),
                    control_type: ControlType = ControlType.CONSTANT, n_threads: int = 1, external_forces: dict = None,
                    n_shooting: int | None = None, apply_custom_constraint: bool = False) -> FesMskOcp:
        """Same arguments as the reference (fes_ocp_dynamics.py:158-251).  Extensions: ``n_shooting`` overrides the
        LCM node count of ``OcpFes.prepare_n_shooting``; ``pulse_width["per_pulse"]`` makes the intervals that follow
        one pulse share its widths (the per-pulse parameters of the revision that stored the reaching-task solutions,
        as band-local equality rows); ``apply_custom_constraint`` enforces
        ``msk_info["custom_constraint"]``.  The reference accepts that constraint list but never applies it: its
        ``_prepare_optimization_problem`` calls ``_build_constraints`` without it (fes_ocp_dynamics.py:107; the
        parameter is read at 424-450), so by default it is ignored here too, with a warning."""
        if external_forces:
            raise NotImplementedError("OcpFesMsk: external forces are not supported")
        if initial_guess_warm_start:
            raise NotImplementedError("OcpFesMsk: initial_guess_warm_start is not supported")
        muscles = model.muscles_dynamics_model
        n = OcpFes.prepare_n_shooting(muscles[0].stim_time, final_time) if n_shooting is None else n_shooting
        pulse_width, pulse_intensity, objective = OcpFes._fill_dict(pulse_width, pulse_intensity, objective)
        pulse_width, pulse_intensity, objective, msk_info = OcpFesMsk._fill_msk_dict(pulse_width, pulse_intensity,
                                                                                     objective, msk_info)
        OcpFes._sanity_check(model=model, n_shooting=n, final_time=final_time, objective=objective, use_sx=use_sx,
                             ode_solver=ode_solver, n_threads=n_threads)
        OcpFesMsk._sanity_check_msk_inputs(model, msk_info, objective)
        if isinstance(ode_solver, OdeSolver.COLLOCATION):
            raise NotImplementedError("OcpFesMsk: direct collocation is not available for musculoskeletal models")
        if len({type(m) for m in muscles}) != 1 or len({m._sum_stim_truncation for m in muscles}) != 1:
            raise ValueError("OcpFesMsk: every muscle must use the same model class and truncation")
        if bool(msk_info["with_residual_torque"]) != bool(model.activate_residual_torque):
            raise ValueError("msk_info['with_residual_torque'] must match the model's activate_residual_torque")
        # the OCP's model is rebuilt without the passive-force flag (fes_ocp_dynamics.py:120-131)
        model.activate_passive_force_relationship = False
        table, stim_idx_at_node_list = muscles[0].get_numerical_data_time_series(n, final_time)
        rows = table["stim_time"][:, 0, :].T.copy()
        state_names = model.state_names()
        hmed = isinstance(muscles[0], DingModelPulseIntensityFrequency)
        T = muscles[0]._sum_stim_truncation
        if isinstance(muscles[0], DingModelPulseWidthFrequency):
            control_names = [f"last_pulse_width_{m.muscle_name}" for m in muscles]
        elif hmed:  # configure_pulse_intensity: T intensities per muscle (dynamical_model.py:437-440)
            control_names = [f"pulse_intensity_{m.muscle_name}_{j}" for m in muscles for j in range(T)]
        else:
            control_names = []
        control_names += [f"tau_{q}" for q in model.name_dof] if model.activate_residual_torque else []
        x_bounds, x_init = OcpFesMsk._set_bounds(model, n, msk_info)
        u_bounds, u_init = OcpFesMsk._set_u_bounds(model, n)
        terms = OcpFesMsk._set_objective(model, n, objective, state_names, control_names)
        par = {}
        if hmed:
            n_params, p_bounds, p_init, names, offsets = OcpFesMsk._build_parameters(model, pulse_intensity)
            # _build_constraints (fes_ocp_dynamics.py:413-438): the window of node k ends at its last pulse
            last = np.array([stim_idx_at_node_list[k][-1] for k in range(n)], dtype=np.int32)
            par = dict(n_params=n_params, p_bounds=p_bounds, p_init=p_init, param_names=names, last_stim_idx=last,
                       param_offset=offsets)
        pairs = []
        if msk_info["custom_constraint"]:
            if apply_custom_constraint:
                pairs = OcpFesMsk._build_constraints(model, n, msk_info["custom_constraint"])
            else:
                warnings.warn("msk_info['custom_constraint'] is not applied, as in the reference "
                              "(fes_ocp_dynamics.py:107 builds the constraints without it); pass "
                              "apply_custom_constraint=True to enforce it", stacklevel=2)
        per_pulse = bool(pulse_width.get("per_pulse"))
        if per_pulse and not isinstance(muscles[0], DingModelPulseWidthFrequency):
            raise ValueError("pulse_width['per_pulse'] needs pulse-width (Ding2007) muscles")
        ppb = pulse_width.get("per_pulse_bounds", "all")
        if ppb not in ("all", "first"):
            raise ValueError("pulse_width['per_pulse_bounds'] must be 'all' or 'first'")
        return FesMskOcp(model, n, final_time, ode_solver, rows, terms, x_bounds, x_init, u_bounds, u_init,
                         state_names, control_names, n_threads, use_sx, marker_pairs=pairs, per_pulse=per_pulse,
                         per_pulse_bounds=ppb, **par)

    @staticmethod
    def _build_constraints(model, n, custom_constraint) -> list:
        """The custom constraints of ``_build_constraints`` (fes_ocp_dynamics.py:444-448) as marker pairs: every
        ``ConstraintFcn.SUPERIMPOSE_MARKERS`` of phase 0, one pair per node, markers re-expressed in the frame of
        the dof they move with (``reduce_to_chain``)."""
        markers = model.chain["markers"]
        pairs = []
        for i in range(len(custom_constraint)):
            if not custom_constraint[i]:
                continue
            for c in custom_constraint[i]:
                if not isinstance(c, Constraint) or c.constraint is not ConstraintFcn.SUPERIMPOSE_MARKERS:
                    raise NotImplementedError("custom_constraint: only ConstraintFcn.SUPERIMPOSE_MARKERS is supported")
                for name in (c.first_marker, c.second_marker):
                    if name not in markers:
                        raise ValueError(f"marker {name!r} is not in {model.biorbd_path}")
                m1, m2 = markers[c.first_marker], markers[c.second_marker]
                if m1["frame"] < 0 and m2["frame"] < 0:
                    raise ValueError("SUPERIMPOSE_MARKERS: both markers are fixed to the ground")
                axes = sum(1 << int(a) for a in set(c.axes))
                for k in c.nodes(n):
                    pairs.append({"node": k, "axes": axes, "frame": [m1["frame"], m2["frame"]],
                                  "pos": [list(m1["pos"]), list(m2["pos"])], "first": c.first_marker,
                                  "second": c.second_marker})
        return pairs

    @staticmethod
    def _build_parameters(model, pulse_intensity):
        """Hmed2018 pulse-intensity parameters (fes_ocp_dynamics.py:343-411): one block of n_stim intensities per
        muscle (one shared block with same_for_all_muscles), fixed or bounded by [min, max] with the mid-point as
        initial guess.  Returns (n_params, (lb, ub), init, block names, per-muscle block offsets)."""
        muscles = model.muscles_dynamics_model
        n_stim = len(muscles[0].stim_time)
        if pulse_intensity["bimapping"]:
            raise NotImplementedError("bimapped pulse intensities are not supported (the reference's sliding-window "
                                      "constraint indexes past a size-1 parameter)")
        fixed, lo, hi = pulse_intensity["fixed"], pulse_intensity["min"], pulse_intensity["max"]
        if fixed:
            vals = np.array(fixed if isinstance(fixed, list) else [fixed] * n_stim, dtype=float)
            if vals.size != n_stim:
                raise ValueError("pulse_intensity['fixed'] must hold one value per pulse")
            blo, bhi, binit = vals, vals, vals
        elif lo and hi:
            blo, bhi = np.full(n_stim, float(lo)), np.full(n_stim, float(hi))
            binit = np.full(n_stim, (float(lo) + float(hi)) / 2)
        else:
            raise ValueError("Hmed2018 muscles need pulse_intensity 'fixed', or 'min' and 'max'")
        shared = bool(pulse_intensity["same_for_all_muscles"])
        nblocks = 1 if shared else len(muscles)
        names = (["pulse_intensity"] if shared else [f"pulse_intensity_{m.muscle_name}" for m in muscles])
        offsets = np.array([0 if shared else i * n_stim for i in range(len(muscles))], dtype=np.int32)
        return (nblocks * n_stim, (np.tile(blo, nblocks), np.tile(bhi, nblocks)), np.tile(binit, nblocks), names,
                offsets)

    @staticmethod
    def _fill_msk_dict(pulse_width, pulse_intensity, objective, msk_info):
        """fes_ocp_dynamics.py:253-301."""
        dpw = {"fixed": None, "min": None, "max": None, "bimapping": False, "same_for_all_muscles": False,
               "per_pulse": False}
        dobj = {"force_tracking": None, "end_node_tracking": None, "custom": None, "q_tracking": None,
                "minimize_muscle_fatigue": False, "minimize_muscle_force": False, "minimize_residual_torque": False}
        dmsk = {"bound_type": None, "bound_data": None, "with_residual_torque": False, "custom_constraint": None}
        return ({**dpw, **(pulse_width or {})}, {**dpw, **(pulse_intensity or {})}, {**dobj, **(objective or {})},
                {**dmsk, **(msk_info or {})})

    @staticmethod
    def _sanity_check_msk_inputs(model, msk_info, objective):
        """fes_ocp_dynamics.py:682-801 (same messages)."""
        if msk_info["bound_type"]:
            if not isinstance(msk_info["bound_type"], str) or msk_info["bound_type"] not in ["start", "end",
                                                                                          "start_end"]:
                raise ValueError("bound_type should be a string and should be equal to start, end or start_end")
            if not isinstance(msk_info["bound_data"], list):
                raise TypeError("bound_data should be a list")
            if msk_info["bound_type"] == "start_end":
                bd = msk_info["bound_data"]
                if len(bd) != 2 or not isinstance(bd[0], list) or not isinstance(bd[1], list):
                    raise TypeError("bound_data should be a list of two list")
                if len(bd[0]) != model.nb_q or len(bd[1]) != model.nb_q:
                    raise ValueError(f"bound_data should be a list of {model.nb_q} elements")
                for i in range(len(bd[0])):
                    if not isinstance(bd[0][i], int | float) or not isinstance(bd[1][i], int | float):
                        raise TypeError(f"bound data index {i}: {bd[0][i]} and {bd[1][i]} should be an int or float")
            if msk_info["bound_type"] in ("start", "end"):
                if len(msk_info["bound_data"]) != model.nb_q:
                    raise ValueError(f"bound_data should be a list of {model.nb_q} element")
                for i in range(len(msk_info["bound_data"])):
                    if not isinstance(msk_info["bound_data"][i], int | float):
                        raise TypeError(f"bound data index {i}: {msk_info['bound_data'][i]} should be an int or float")
        ft = objective["force_tracking"]
        if ft:
            if not isinstance(ft, list):
                raise TypeError(f"force_tracking: {ft} must be list type")
            if len(ft) != 2:
                raise ValueError("force_tracking must of size 2")
            if not isinstance(ft[0], np.ndarray):
                raise TypeError(f"force_tracking index 0: {ft[0]} must be np.ndarray type")
            if not isinstance(ft[1], list):
                raise TypeError(f"force_tracking index 1: {ft[1]} must be list type")
            if len(ft[1]) != len(model.muscles_dynamics_model):
                raise ValueError("force_tracking index 1 list must have the same size as the number of muscles in "
                                 "model.muscles_dynamics_model")
            for i in range(len(ft[1])):
                if len(ft[0]) != len(ft[1][i]):
                    raise ValueError("force_tracking time and force argument must be the same length")
        et = objective["end_node_tracking"]
        if et:
            if not isinstance(et, list):
                raise TypeError(f"force_tracking: {et} must be list type")
            if len(et) != len(model.muscles_dynamics_model):
                raise ValueError("end_node_tracking list must have the same size as the number of muscles in "
                                 "fes_muscle_models")
            for i in range(len(et)):
                if not isinstance(et[i], int | float):
                    raise TypeError(f"end_node_tracking index {i}: {et[i]} must be int or float type")
        qt = objective["q_tracking"]
        if qt:
            if not isinstance(qt, list) and len(qt) != 2:
                raise TypeError("q_tracking should be a list of size 2")
            if not isinstance(qt[0], list | np.ndarray):
                raise ValueError("q_tracking[0] should be a list or array type")
            if len(qt[1]) != model.nb_q:
                raise ValueError("q_tracking[1] should have the same size as the number of generalized coordinates")
            for i in range(model.nb_q):
                if len(qt[0]) != len(qt[1][i]):
                    raise ValueError("q_tracking[0] and q_tracking[1] should have the same size")
        for name in ("minimize_muscle_fatigue", "minimize_muscle_force"):
            if objective[name] and not isinstance(objective[name], bool):
                raise TypeError(f"{name} should be a boolean")
        if msk_info["with_residual_torque"] and not isinstance(msk_info["with_residual_torque"], bool):
            raise TypeError("with_residual_torque should be a boolean")

    @staticmethod
    def _set_bounds(model, n, msk_info):
        """_set_bounds_fes (fes_ocp_dynamics.py:453-497) + _set_bounds_msk (499-540): muscle states fixed at rest
        at node 0, then Cn in [0, 10], F in [0, 1000], A in [0, rest], Tau1 / Km in [rest, 1]; q from the bioMod
        ranges with the start / end angles (degrees x 3.14 / 180, as the reference converts), qdot from the
        ranges and 0 at node 0.  Initial guess: rest states, q = qdot = 0."""
        lo_cols, hi_cols, init = [], [], []
        for m in model.muscles_dynamics_model:
            rest = m.standard_rest_values().astype(float)[:, 0]
            lo, hi = rest.copy(), rest.copy()
            for i, s in enumerate(m.name_dof):
                if s == "Cn":
                    hi[i] = 10
                elif s == "F":
                    hi[i] = 1000
                elif s in ("Tau1", "Km"):
                    hi[i] = 1
                elif s == "A":
                    lo[i] = 0
            lo_cols.append(np.stack([rest, lo, lo], axis=1))
            hi_cols.append(np.stack([rest, hi, hi], axis=1))
            init.append(rest)
        nq = model.nb_q
        deg = lambda d: 3.14 / (180 / d) if d != 0 else 0  # noqa: E731  (fes_ocp_dynamics.py:501-521)
        qb = model.bounds_from_ranges("q")
        qlo = np.repeat(qb[:, :1], 3, axis=1)
        qhi = np.repeat(qb[:, 1:], 3, axis=1)
        bt, bd = msk_info["bound_type"], msk_info["bound_data"]
        for j in range(nq):
            if bt in ("start_end", "start"):
                v = deg((bd[0] if bt == "start_end" else bd)[j])
                qlo[j, 0] = qhi[j, 0] = v
            if bt in ("start_end", "end"):
                v = deg((bd[1] if bt == "start_end" else bd)[j])
                qlo[j, 2] = qhi[j, 2] = v
        qd = model.bounds_from_ranges("qdot")
        qdlo = np.repeat(qd[:, :1], 3, axis=1)
        qdhi = np.repeat(qd[:, 1:], 3, axis=1)
        qdlo[:, 0] = qdhi[:, 0] = 0
        lo3 = np.concatenate(lo_cols + [qlo, qdlo])
        hi3 = np.concatenate(hi_cols + [qhi, qdhi])
        # CONSTANT_WITH_FIRST_AND_LAST_DIFFERENT: column 0 at node 0, column 1 in between, column 2 at node N
        cols = np.r_[0, np.ones(n - 1, dtype=int), 2]
        x_init = np.repeat(np.concatenate(init + [np.zeros(2 * nq)])[:, None], n + 1, axis=1)
        return (lo3[:, cols], hi3[:, cols]), x_init

    @staticmethod
    def _set_u_bounds(model, n):
        """_set_u_bounds_fes / _set_u_bounds_msk (fes_ocp_dynamics.py:542-589): pulse width in [pd0, 0.0006],
        pulse intensities in [I_min, 130] (initial guess 0), residual torque in [-200, 200] (initial guess 0)."""
        lo, hi = [], []
        if isinstance(model.muscles_dynamics_model[0], DingModelPulseWidthFrequency):
            for m in model.muscles_dynamics_model:
                lo.append(m.pd0)
                hi.append(0.0006)
        if isinstance(model.muscles_dynamics_model[0], DingModelPulseIntensityFrequency):
            for m in model.muscles_dynamics_model:
                lo += [float(m.min_pulse_intensity())] * m._sum_stim_truncation
                hi += [130.0] * m._sum_stim_truncation
        if model.activate_residual_torque:
            lo += [-200.0] * model.nb_q
            hi += [200.0] * model.nb_q
        nu = len(lo)
        lb = np.repeat(np.asarray(lo, dtype=float).reshape(nu, 1), n, axis=1)
        ub = np.repeat(np.asarray(hi, dtype=float).reshape(nu, 1), n, axis=1)
        return (lb, ub), np.zeros((nu, n))

    @staticmethod
    def _set_objective(model, n, objective, state_names, control_names):
        """fes_ocp_dynamics.py:591-680 as libcfx terms."""
        terms = []
        sidx = {s: i for i, s in enumerate(state_names)}
        cidx = {s: i for i, s in enumerate(control_names)}
        ranges = {Node.START: (0, 0), Node.ALL: (0, n), Node.ALL_SHOOTING: (0, n - 1)}

        def term(kind, var_kind, index, first, last, weight, target=None, target_value=0.0):
            t = dict(kind=kind, var_kind=var_kind, var_index=index, node_first=first, node_last=last,
                     weight=float(weight), target_value=float(target_value))
            if target is not None:
                t["target"] = np.asarray(target, dtype=float)
            terms.append(t)

        if objective["custom"]:
            for ob in objective["custom"][0]:
                OcpFesMsk._custom_term(ob, n, model, sidx, cidx, term)
        muscles = model.muscles_dynamics_model
        if objective["force_tracking"]:
            for j, m in enumerate(muscles):
                coeffs = FourierSeries().compute_real_fourier_coeffs(objective["force_tracking"][0],
                                                                     objective["force_tracking"][1][j], 50)
                tgt = FourierSeries().fit_func_by_fourier_series_with_real_coeffs(np.linspace(0, 1, n + 1), coeffs)
                term(_cfx.OBJ_LAGRANGE, _cfx.VAR_STATE, sidx[f"F_{m.muscle_name}"], 0, n, 100.0, target=tgt)
        if objective["end_node_tracking"] is not None:
            for j, m in enumerate(muscles):
                term(_cfx.OBJ_MAYER, _cfx.VAR_STATE, sidx[f"F_{m.muscle_name}"], n, n, 1.0,
                     target_value=objective["end_node_tracking"][j])
        if objective["q_tracking"]:
            for j in range(model.nb_q):
                coeffs = FourierSeries().compute_real_fourier_coeffs(np.asarray(objective["q_tracking"][0]),
                                                                     np.asarray(objective["q_tracking"][1][j]), 50)
                tgt = FourierSeries().fit_func_by_fourier_series_with_real_coeffs(np.linspace(0, 1, n + 1), coeffs)
                term(_cfx.OBJ_LAGRANGE, _cfx.VAR_STATE, sidx[f"q_{model.name_dof[j]}"], 0, n, 100.0, target=tgt)
        if objective["minimize_muscle_fatigue"]:
            # CustomObjective.minimize_overall_muscle_fatigue (custom_objectives.py:80-101): sum (a_rest / A)^2 at
            # node N, weight 1
            for m in muscles:
                if "A" not in m.name_dof:
                    raise ValueError("minimize_muscle_fatigue needs muscle models with fatigue")
                term(_cfx.OBJ_MAYER_INV, _cfx.VAR_STATE, sidx[f"A_{m.muscle_name}"], n, n, 1.0,
                     target_value=m.a_rest)
        if objective["minimize_muscle_force"]:
            for m in muscles:  # custom_objectives.py:103-117: Lagrange, every node, weight 1
                term(_cfx.OBJ_LAGRANGE, _cfx.VAR_STATE, sidx[f"F_{m.muscle_name}"], 0, n, 1.0)
        if objective["minimize_residual_torque"]:
            for q in model.name_dof:  # MINIMIZE_CONTROL tau, weight 10000
                term(_cfx.OBJ_LAGRANGE, _cfx.VAR_CONTROL, cidx[f"tau_{q}"], 0, n - 1, 10000.0)
        return terms

    @staticmethod
    def _custom_term(ob: Objective, n, model, sidx, cidx, term):
        """A bioptim-style custom objective on q / qdot / tau / muscle states / pulse widths (with ``index``)."""
        state = ob.objective in (ObjectiveFcn.Lagrange.MINIMIZE_STATE, ObjectiveFcn.Lagrange.TRACK_STATE,
                                 ObjectiveFcn.Mayer.MINIMIZE_STATE, ObjectiveFcn.Mayer.TRACK_STATE)
        names = sidx if state else cidx
        if ob.key in ("q", "qdot", "tau"):
            keys = [f"{ob.key}_{q}" for q in model.name_dof]
        else:
            keys = [ob.key]
        idx = ob.index if ob.index is not None else list(range(len(keys)))
        idx = [idx] if isinstance(idx, int) else list(idx)
        last = n if state else n - 1
        first, end = {Node.START: (0, 0), Node.END: (last, last), Node.ALL: (0, last),
                      Node.ALL_SHOOTING: (0, n - 1)}[ob.node]
        tgt = None if ob.target is None else np.asarray(ob.target, dtype=float).reshape(len(idx), -1)
        for r, i in enumerate(idx):
            if keys[i] not in names:
                raise ValueError(f"unknown {'state' if state else 'control'} key {keys[i]}")
            kind = _cfx.OBJ_LAGRANGE if ob.lagrange else _cfx.OBJ_MAYER
            if tgt is None:
                term(kind, _cfx.VAR_STATE if state else _cfx.VAR_CONTROL, names[keys[i]], first, end, ob.weight)
            elif tgt.shape[1] == 1:
                term(kind, _cfx.VAR_STATE if state else _cfx.VAR_CONTROL, names[keys[i]], first, end, ob.weight,
                     target_value=tgt[r, 0])
            else:
                full = np.zeros(n + 1)
                full[first: first + tgt.shape[1]] = tgt[r]
                term(kind, _cfx.VAR_STATE if state else _cfx.VAR_CONTROL, names[keys[i]], first, end, ob.weight,
                     target=full)
