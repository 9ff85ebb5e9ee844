"""OcpFes: build the transcribed FES optimal-control problem (reference: cocofest/optimization/fes_ocp.py).

``OcpFes.prepare_ocp`` keeps the reference's signature and validation messages.  Instead of a bioptim
``OptimalControlProgram`` it returns a :class:`FesOcp`, which owns the NLP layout, bounds, initial
guess and objective, and opens libcfx handles that evaluate g, J_g, f, grad f and the Lagrangian
Hessian for batches of instances on the GPU (``FesOcp.nlp``), plus a host interior-point driver
(``FesOcp.solve``).

Transcription: bioptim multiple shooting with explicit RK sub-steps (``OdeSolver.RK1/RK2/RK4``);
decision vector per instance [x_0, u_0, ..., x_{N-1}, u_{N-1}, x_N, p]; constraints per interval:
Phi(x_k, u_k) - x_{k+1}, then (Hmed with intensity parameters) u_k - window_k(p).
"""

from __future__ import annotations

from enum import Enum, IntEnum
from fractions import Fraction
from math import gcd

import numpy as np

from . import _cfx
from .fes_models import (
    DingModelPulseIntensityFrequency,
    DingModelPulseWidthFrequency,
    FesModel,
)
from .fourier import FourierSeries
from .ode_solver import ControlType, OdeSolver


class Node(Enum):
    START = "start"
    END = "end"
    ALL = "all"
    ALL_SHOOTING = "all_shooting"


class Axis(IntEnum):
    """bioptim ``Axis`` (world axes of marker constraints)."""
    X = 0
    Y = 1
    Z = 2


class ConstraintFcn(Enum):
    """The bioptim constraint the reference's OcpFesMsk examples pass as ``msk_info["custom_constraint"]``
    (examples/dynamics/reaching_task/*.py)."""
    SUPERIMPOSE_MARKERS = "superimpose_markers"


class Constraint:
    """One ``ConstraintFcn.SUPERIMPOSE_MARKERS`` equality: marker(second) - marker(first) = 0 on ``axes`` (all three
    by default) at ``node`` (an int, ``Node.START`` / ``Node.END`` / ``Node.ALL`` / ``Node.ALL_SHOOTING``)."""

    def __init__(self, constraint, node=None, first_marker: str = None, second_marker: str = None, axes=None,
                 phase: int = 0, **extra):
        if not isinstance(constraint, ConstraintFcn):
            raise NotImplementedError(f"constraint {constraint!r} is not supported (SUPERIMPOSE_MARKERS only)")
        if extra:
            raise NotImplementedError(f"SUPERIMPOSE_MARKERS: unsupported arguments {sorted(extra)}")
        if phase != 0:
            raise NotImplementedError("single-phase problems only")
        if node is None:
            raise ValueError("SUPERIMPOSE_MARKERS: give the node (an int or a Node)")
        if not first_marker or not second_marker:
            raise ValueError("SUPERIMPOSE_MARKERS needs first_marker and second_marker")
        self.constraint = constraint
        self.node = node
        self.first_marker, self.second_marker = first_marker, second_marker
        self.axes = [Axis(a) for a in (axes if axes is not None else (Axis.X, Axis.Y, Axis.Z))]
        self.phase = phase

    def nodes(self, n_shooting: int) -> list:
        if isinstance(self.node, Node):
            return {Node.START: [0], Node.END: [n_shooting], Node.ALL: list(range(n_shooting + 1)),
                    Node.ALL_SHOOTING: list(range(n_shooting))}[self.node]
        nodes = [int(k) for k in (self.node if isinstance(self.node, (list, tuple, range)) else [self.node])]
        for k in nodes:
            if not 0 <= k <= n_shooting:
                raise ValueError(f"SUPERIMPOSE_MARKERS: node {k} is outside [0, {n_shooting}]")
        return nodes


class ConstraintList:
    """bioptim ``ConstraintList`` for one phase: ``custom_constraint[0]`` is the phase's list (the reference walks
    it as ``custom_constraint[i][j]``, fes_ocp_dynamics.py:444-448)."""

    def __init__(self):
        self._items = []

    def add(self, constraint, **kwargs):
        self._items.append(constraint if isinstance(constraint, Constraint) else Constraint(constraint, **kwargs))

    def __getitem__(self, i):
        if i != 0:
            raise IndexError("single-phase ConstraintList")
        return self._items

    def __len__(self):
        return 1 if self._items else 0

    def __iter__(self):
        return iter(self._items)


class ObjectiveFcn:
    class Lagrange(Enum):
        MINIMIZE_STATE = "minimize_state"
        TRACK_STATE = "track_state"
        MINIMIZE_CONTROL = "minimize_control"
        TRACK_CONTROL = "track_control"

    class Mayer(Enum):
        MINIMIZE_STATE = "minimize_state"
        TRACK_STATE = "track_state"


class Objective:
    """One quadratic objective term (the subset of bioptim ObjectiveFcn the reference's FES OCPs use)."""

    def __init__(self, objective, key: str, weight: float = 1, target=None, node: Node = None, quadratic: bool = True,
                 index=None, phase: int = 0):
        if not quadratic:
            raise NotImplementedError("only quadratic objective terms are supported")
        if phase != 0:
            raise NotImplementedError("single-phase problems only")
        self.objective = objective
        self.key = key
        self.index = index
        self.weight = float(weight)
        self.target = target
        lagrange = isinstance(objective, ObjectiveFcn.Lagrange)
        self.node = node if node is not None else (Node.ALL_SHOOTING if lagrange else Node.END)
        self.lagrange = lagrange


class ObjectiveList:
    def __init__(self):
        self._items = []

    def add(self, objective, **kwargs):
        self._items.append(objective if isinstance(objective, Objective) else Objective(objective, **kwargs))

    def __getitem__(self, i):
        # the reference indexes ObjectiveList as objective["custom"][0][i] (fes_ocp.py:331,537)
        return self._items if i == 0 else self._items[i]

    def __len__(self):
        return len(self._items)

    def __iter__(self):
        return iter(self._items)


class FesOcp:
    """The transcribed OCP: layout, bounds, initial guess, objective and GPU callbacks."""

    def __init__(self, model, n_shooting, final_time, ode_solver, rows, stim_idx_at_node_list, objectives,
                 x_bounds, x_init, u_bounds, u_init, p_bounds, p_init, n_params, last_stim_idx, intensity_floor,
                 n_threads=1, use_sx=True):
        self.model = model
        self.n_shooting = n_shooting
        self.final_time = final_time
        self.ode_solver = ode_solver
        self.stim_rows = rows
        self.stim_idx_at_node_list = stim_idx_at_node_list
        self.objectives = objectives
        self.x_bounds, self.x_init = x_bounds, x_init
        self.u_bounds, self.u_init = u_bounds, u_init
        self.p_bounds, self.p_init = p_bounds, p_init
        self.n_params = n_params
        self.last_stim_idx = last_stim_idx
        self.intensity_floor = intensity_floor
        self.n_threads, self.use_sx = n_threads, use_sx
        self.nx = model.nb_state
        self.nu = u_init.shape[0]
        self.truncation = model._sum_stim_truncation

    # ---- layout -------------------------------------------------------------------------------------
    # Decision vector per instance: per interval k the block [x_k, u_k] (multiple shooting) or
    # [x_k^0, x_k^1..x_k^d, u_k] (direct collocation, degree d), then x_N, then the parameters.
    @property
    def degree(self):
        return self.ode_solver.polynomial_degree if isinstance(self.ode_solver, OdeSolver.COLLOCATION) else 0

    @property
    def uoff(self):
        return (self.degree + 1) * self.nx if self.degree else self.nx

    @property
    def nzb(self):
        """Size of one interval's decision block."""
        return self.uoff + self.nu

    @property
    def ngk(self):
        """Constraint rows per interval (dynamics rows, then the Hmed sliding-window rows)."""
        n_slide = self.nu if (self.n_params and self.last_stim_idx is not None) else 0
        return (self.degree + 1) * self.nx + n_slide if self.degree else self.nx + n_slide

    @property
    def nv(self):
        return self.n_shooting * self.nzb + self.nx + self.n_params

    def pack(self, x, u=None, p=None, x_points=None):
        """(nx, N+1) node states, (nu, N) controls, (n_params,) parameters -> decision vector (nv,).
        Collocation states: ``x_points`` (nx, N, d), by default each interval's start node state."""
        N, nx, nu, d, nzb = self.n_shooting, self.nx, self.nu, self.degree, self.nzb
        x = np.asarray(x, dtype=float)
        v = np.empty(self.nv)
        body = v[: N * nzb].reshape(N, nzb)
        body[:, :nx] = x[:, :N].T
        if d:
            xp = np.repeat(x[:, :N, None], d, axis=2) if x_points is None else np.asarray(x_points, dtype=float)
            body[:, nx: (d + 1) * nx] = xp.transpose(1, 2, 0).reshape(N, d * nx)
        if nu:
            body[:, self.uoff:] = np.asarray(u).T
        v[N * nzb: N * nzb + nx] = x[:, N]
        if self.n_params:
            v[N * nzb + nx:] = p
        return v

    def unpack(self, v):
        N, nx, nu, nzb = self.n_shooting, self.nx, self.nu, self.nzb
        v = np.asarray(v)
        body = v[: N * nzb].reshape(N, nzb)
        x = np.concatenate([body[:, :nx].T, v[N * nzb: N * nzb + nx, None]], axis=1)
        states = {name: x[i][np.newaxis, :] for i, name in enumerate(self.model.name_dof)}
        controls = {}
        if nu:
            key = "last_pulse_width" if isinstance(self.model, DingModelPulseWidthFrequency) else "pulse_intensity"
            controls[key] = body[:, self.uoff:].T
        params = {"pulse_intensity": v[N * nzb + nx:]} if self.n_params else {}
        return states, controls, params

    def bounds_vector(self):
        """Collocation points of interval k take the bounds of the intermediate nodes (column max(k, 1)), so the
        fixed initial node does not pin the first interval's interior states."""
        pts = None
        if self.degree:
            cols = np.minimum(np.maximum(np.arange(self.n_shooting), 1), self.n_shooting)
            pts = [np.repeat(np.asarray(b, dtype=float)[:, cols, None], self.degree, axis=2) for b in self.x_bounds]
        lo = self.pack(self.x_bounds[0], self.u_bounds[0] if self.nu else None, self.p_bounds[0],
                       x_points=None if pts is None else pts[0])
        hi = self.pack(self.x_bounds[1], self.u_bounds[1] if self.nu else None, self.p_bounds[1],
                       x_points=None if pts is None else pts[1])
        return lo, hi

    def initial_guess_vector(self):
        return self.pack(self.x_init, self.u_init if self.nu else None, self.p_init)

    # ---- GPU callbacks ------------------------------------------------------------------------------
    def nlp(self, batch: int = 1, layout: str = "aos", device: int = 0) -> _cfx.Handle:
        """Open a libcfx handle evaluating ``batch`` instances of this problem on GPU ``device``."""
        return _cfx.Handle(
            model_id=self.model.cfx_model_id, constants=self.model.cfx_constants(), scheme=self.ode_solver.scheme,
            n_steps=self.ode_solver.n_integration_steps, n_shooting=self.n_shooting,
            truncation=self.truncation, final_time=float(self.final_time), stim_rows=self.stim_rows, batch=batch,
            layout={"aos": _cfx.LAYOUT_AOS, "soa": _cfx.LAYOUT_SOA, "tiled64": _cfx.LAYOUT_TILED64}[layout],
            n_params=self.n_params,
            last_stim_idx=self.last_stim_idx, intensity_floor=self.intensity_floor,
            objectives=self.objectives, device=device)

    def interval_slice(self, k0: int, k1: int) -> "FesOcp":
        """The callbacks of intervals [k0, k1) as a problem of their own (multi-GPU interval sharding).

        Its decision vector is ``[x_k0, u_k0, ..., x_k1, p]`` — the global slice ``v[k0 nz : k1 nz + nx]`` plus
        every parameter — and its constraints are the global rows of those intervals.  Stim times are shifted
        by k0 dt (only the differences t - t_i enter the model).  Objective terms keep the nodes this slice
        owns: k0 .. k1 - 1, and node N on the slice that ends at N, so summing the slices' f gives f."""
        N = self.n_shooting
        if not (0 <= k0 < k1 <= N):
            raise ValueError(f"interval slice [{k0}, {k1}) outside [0, {N})")
        dt = self.final_time / N
        shift = k0 * dt
        rows = np.where(self.stim_rows > -1e6, self.stim_rows - shift, self.stim_rows)[k0: k1 + 1].copy()
        own_last = k1 if k1 == N else k1 - 1
        terms = []
        for t in self.objectives:
            last = min(t["node_last"], own_last if t["var_kind"] == _cfx.VAR_STATE else k1 - 1)
            first = max(t["node_first"], k0)
            if first > last:
                continue
            nt = dict(t, node_first=first - k0, node_last=last - k0)
            if t.get("target") is not None:
                nt["target"] = np.asarray(t["target"], dtype=float)[k0: k1 + 1].copy()
            terms.append(nt)
        sl = lambda a: None if a is None else np.asarray(a)[..., k0: k1 + 1]  # noqa: E731
        su = lambda a: None if a is None else np.asarray(a)[..., k0: k1]  # noqa: E731
        x_bounds = (sl(self.x_bounds[0]), sl(self.x_bounds[1]))
        u_bounds = (su(self.u_bounds[0]), su(self.u_bounds[1])) if self.nu else self.u_bounds
        last_idx = None if self.last_stim_idx is None else np.asarray(self.last_stim_idx)[k0:k1].copy()
        sub = FesOcp(self.model, k1 - k0, (k1 - k0) * dt, self.ode_solver, rows,
                     self.stim_idx_at_node_list[k0: k1 + 1], terms, x_bounds, sl(self.x_init), u_bounds,
                     su(self.u_init) if self.nu else self.u_init, self.p_bounds, self.p_init, self.n_params, last_idx,
                     self.intensity_floor, self.n_threads, self.use_sx)
        sub.global_slice = (k0, k1)
        return sub

    def solve(self, solver=None, **kwargs):
        from .solver import solve_ocp

        return solve_ocp(self, solver=solver, **kwargs)


class OcpFes:
    """Prepares the FES OCP (reference: cocofest/optimization/fes_ocp.py:32-577)."""

    @staticmethod
    def prepare_ocp(model: FesModel = None, final_time: int | float = None, pulse_width: dict = None,
                    pulse_intensity: dict = None, objective: dict = None, use_sx: bool = True,
                    ode_solver=OdeSolver.RK1(n_integration_steps=10), control_type: ControlType = ControlType.CONSTANT,
                    n_threads: int = 1, n_shooting: int | None = None) -> FesOcp:
        """Same arguments as the reference (fes_ocp.py:112-190).  ``n_shooting`` (extension) overrides the
        LCM node count of ``prepare_n_shooting``; the default keeps the reference's rule."""
        n = OcpFes.prepare_n_shooting(model.stim_time, final_time) if n_shooting is None else n_shooting
        pulse_width, pulse_intensity, objective = OcpFes._fill_dict(pulse_width, pulse_intensity, objective)
        OcpFes._sanity_check(model=model, n_shooting=n, final_time=final_time, objective=objective, use_sx=use_sx,
                             ode_solver=ode_solver, n_threads=n_threads)
        n_params, p_bounds, p_init = OcpFes._build_parameters(model, pulse_intensity)
        table, stim_idx_at_node_list = model.get_numerical_data_time_series(n, final_time)
        rows = table["stim_time"][:, 0, :].T.copy()
        x_bounds, x_init = OcpFes._set_bounds(model, n)
        max_bound = (pulse_width["max"] if isinstance(model, DingModelPulseWidthFrequency)
                     else pulse_intensity["max"] if isinstance(model, DingModelPulseIntensityFrequency) else None)
        u_bounds, u_init = OcpFes._set_u_bounds(model, n, max_bound=max_bound)
        objectives = OcpFes._set_objective(model, n, objective)
        last_stim_idx, floor = None, 0.0
        if isinstance(model, DingModelPulseIntensityFrequency):
            floor = float(model.min_pulse_intensity())
            if n_params:
                last_stim_idx = OcpFes._build_constraints(model, n, stim_idx_at_node_list)
        return FesOcp(model, n, final_time, ode_solver, rows, stim_idx_at_node_list, objectives, x_bounds, x_init,
                      u_bounds, u_init, p_bounds, p_init, n_params, last_stim_idx, floor, n_threads, use_sx)

    @staticmethod
    def prepare_n_shooting(stim_time, final_time):
        """Number of shooting nodes so that every stimulation falls on a node: the LCM of the reduced
        denominators of t_i / final_time (fes_ocp.py:192-222)."""
        t_final = Fraction(final_time).limit_denominator()
        n_shooting = 1
        for t in stim_time:
            d = (Fraction(t).limit_denominator() / t_final).denominator
            n_shooting = n_shooting * d // gcd(n_shooting, d)
        if n_shooting >= 1000:
            print(f"Warning: The number of shooting nodes is very high n = {n_shooting}.\n"
                  "The optimization might be long, consider using stimulation time with even spacing (common frequency).")
        return n_shooting

    @staticmethod
    def _fill_dict(pulse_width, pulse_intensity, objective):
        default_pulse = {"fixed": None, "min": None, "max": None, "bimapping": False}
        default_objective = {"force_tracking": None, "end_node_tracking": None, "cycling": None, "custom": None}
        return ({**default_pulse, **(pulse_width or {})}, {**default_pulse, **(pulse_intensity or {})},
                {**default_objective, **(objective or {})})

    @staticmethod
    def _sanity_check(model=None, n_shooting=None, final_time=None, objective=None, use_sx=None, ode_solver=None,
                      n_threads=None):
        """Input validation with the reference's messages (fes_ocp.py:279-344).  A FesMskModel passes the model
        check (fes_ocp.py:289-291); every other check applies to it unchanged."""
        if not isinstance(model, FesModel) and not hasattr(model, "muscles_dynamics_model"):
            raise TypeError(
                f"The current model type used is {type(model)}, it must be a FesModel type."
                f"Current available models are: DingModelFrequency, DingModelFrequencyWithFatigue,"
                f"DingModelPulseWidthFrequency, DingModelPulseWidthFrequencyWithFatigue,"
                f"DingModelPulseIntensityFrequency, DingModelPulseIntensityFrequencyWithFatigue")
        if not isinstance(n_shooting, int) or n_shooting < 0:
            raise TypeError("n_shooting must be a positive int type")
        if not isinstance(final_time, int | float) or final_time < 0:
            raise TypeError("final_time must be a positive int or float type")
        ft = objective["force_tracking"]
        if ft is not None:
            if isinstance(ft, list):
                if isinstance(ft[0], np.ndarray) and isinstance(ft[1], np.ndarray):
                    if len(ft[0]) != len(ft[1]) or len(ft) != 2:
                        raise ValueError("force_tracking time and force argument must be same length and force_tracking "
                                         "list size 2")
                else:
                    raise TypeError("force_tracking argument must be np.ndarray type")
            else:
                raise TypeError("force_tracking must be list type")
        if objective["end_node_tracking"] is not None:
            if not isinstance(objective["end_node_tracking"], int | float):
                raise TypeError("end_node_tracking must be int or float type")
        if objective["custom"] is not None:
            if not isinstance(objective["custom"], ObjectiveList):
                raise TypeError("custom_objective must be a ObjectiveList type")
            if not all(isinstance(x, Objective) for x in objective["custom"][0]):
                raise TypeError("All elements in ObjectiveList must be an Objective type")
        if not isinstance(ode_solver, (OdeSolver.RK1, OdeSolver.RK2, OdeSolver.RK4, OdeSolver.COLLOCATION)):
            raise TypeError("ode_solver must be a OdeSolver type")
        if not isinstance(use_sx, bool):
            raise TypeError("use_sx must be a bool type")
        if not isinstance(n_threads, int):
            raise TypeError("n_thread must be a int type")

    @staticmethod
    def _build_parameters(model, pulse_intensity):
        """Hmed pulse-intensity parameters (fes_ocp.py:350-411) -> (n_params, (lb, ub), init)."""
        empty = (0, (np.zeros(0), np.zeros(0)), np.zeros(0))
        if not isinstance(model, DingModelPulseIntensityFrequency):
            return empty
        n_stim = len(model.stim_time)
        if pulse_intensity["bimapping"]:
            raise NotImplementedError("bimapped pulse intensities are not supported (the reference's sliding-window "
                                      "constraint indexes past a size-1 parameter)")
        fixed = pulse_intensity["fixed"]
        if fixed:
            vals = np.array(fixed if isinstance(fixed, list) else [fixed] * n_stim, dtype=float)
            return n_stim, (vals.copy(), vals.copy()), vals.copy()
        if pulse_intensity["max"]:
            lo = float(model.min_pulse_intensity())
            hi = float(pulse_intensity["max"])
            return n_stim, (np.full(n_stim, lo), np.full(n_stim, hi)), np.full(n_stim, (lo + hi) / 2)
        return empty

    @staticmethod
    def _build_constraints(model, n_shooting, stim_idx_at_node_list):
        """Sliding-window rows, one per node (fes_ocp.py:413-438): index of the last parameter of node k."""
        return np.array([stim_idx_at_node_list[i][-1] for i in range(n_shooting)], dtype=np.int32)

    @staticmethod
    def _set_bounds(model, n_shooting):
        """State bounds (fes_ocp.py:452-499): node 0 fixed at rest; after it Cn in [0, 2], F in [0, 1000],
        A in [0, A_rest], Tau1 / Km in [rest, 1].  Returns ((lb, ub) each (nx, N+1), x_init (nx, N+1))."""
        rest = model.standard_rest_values().astype(float)[:, 0]
        lo, hi = rest.copy(), rest.copy()
        for i, name in enumerate(model.name_dof):
            if name == "Cn":
                hi[i] = 2
            if name == "F":
                hi[i] = 1000
            elif name in ("Tau1", "Km"):
                hi[i] = 1
            elif name == "A":
                lo[i] = 0
        lb = np.repeat(lo[:, None], n_shooting + 1, axis=1)
        ub = np.repeat(hi[:, None], n_shooting + 1, axis=1)
        lb[:, 0] = rest
        ub[:, 0] = rest
        x_init = np.repeat(rest[:, None], n_shooting + 1, axis=1)
        return (lb, ub), x_init

    @staticmethod
    def _set_u_bounds(model, n_shooting, max_bound):
        """Control bounds and initial guess (fes_ocp.py:501-529) -> ((lb, ub) each (nu, N), u_init (nu, N))."""
        hi = np.inf if max_bound is None else float(max_bound)
        if isinstance(model, DingModelPulseWidthFrequency):
            lo = float(model.pd0)
            return (np.full((1, n_shooting), lo), np.full((1, n_shooting), hi)), np.zeros((1, n_shooting))
        if isinstance(model, DingModelPulseIntensityFrequency):
            T = model._sum_stim_truncation
            lo = float(model.min_pulse_intensity())
            return (np.full((T, n_shooting), lo), np.full((T, n_shooting), hi)), np.zeros((T, n_shooting))
        return (np.zeros((0, n_shooting)), np.zeros((0, n_shooting))), np.zeros((0, n_shooting))

    @staticmethod
    def _set_objective(model, n_shooting, objective):
        """Objective terms (fes_ocp.py:531-569) as libcfx term descriptors."""
        terms = []
        if objective["custom"]:
            for ob in objective["custom"][0]:
                terms.append(OcpFes._term_from_objective(model, n_shooting, ob))
        if objective["force_tracking"]:
            coeffs = FourierSeries().compute_real_fourier_coeffs(objective["force_tracking"][0],
                                                                 objective["force_tracking"][1], 50)
            target = FourierSeries().fit_func_by_fourier_series_with_real_coeffs(np.linspace(0, 1, n_shooting + 1),
                                                                                 coeffs)
            terms.append(dict(kind=_cfx.OBJ_LAGRANGE, var_kind=_cfx.VAR_STATE, var_index=model.name_dof.index("F"),
                              node_first=0, node_last=n_shooting, weight=100.0, target=np.asarray(target, float)))
        if objective["end_node_tracking"]:
            terms.append(dict(kind=_cfx.OBJ_MAYER, var_kind=_cfx.VAR_STATE, var_index=model.name_dof.index("F"),
                              node_first=n_shooting, node_last=n_shooting, weight=1.0,
                              target_value=float(objective["end_node_tracking"])))
        return terms

    @staticmethod
    def _term_from_objective(model, n_shooting, ob: Objective):
        state = ob.objective in (ObjectiveFcn.Lagrange.MINIMIZE_STATE, ObjectiveFcn.Lagrange.TRACK_STATE,
                                 ObjectiveFcn.Mayer.MINIMIZE_STATE, ObjectiveFcn.Mayer.TRACK_STATE)
        if state:
            idx = model.name_dof.index(ob.key)
        else:
            if ob.key not in ("last_pulse_width", "pulse_intensity"):
                raise ValueError(f"unknown control key {ob.key}")
            idx = 0
        last = n_shooting if state else n_shooting - 1
        first, end = {Node.START: (0, 0), Node.END: (last, last), Node.ALL: (0, last),
                      Node.ALL_SHOOTING: (0, n_shooting - 1)}[ob.node]
        term = dict(kind=_cfx.OBJ_LAGRANGE if ob.lagrange else _cfx.OBJ_MAYER,
                    var_kind=_cfx.VAR_STATE if state else _cfx.VAR_CONTROL, var_index=idx, node_first=first,
                    node_last=end, weight=ob.weight)
        if ob.target is None:
            term["target_value"] = 0.0
        elif np.ndim(ob.target) == 0:
            term["target_value"] = float(ob.target)
        else:
            tgt = np.zeros(n_shooting + 1)
            arr = np.asarray(ob.target, dtype=float).ravel()
            tgt[first: first + arr.size] = arr
            term["target"] = tgt
        return term
