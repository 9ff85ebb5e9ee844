"""Receding-horizon (NMPC) FES control over the GPU callbacks.

Reference: ``FesNmpc`` (cocofest/optimization/fes_nmpc.py:20-192), a bioptim
``MultiCyclicNonlinearModelPredictiveControl`` hard-coded to Ding2007-with-fatigue (fes_nmpc.py:74, 145).
Here every model family is supported, including Hmed2018 pulse intensities:

* a window covers ``n_cycles_simultaneous`` cycles of ``cycle_duration`` seconds; each cycle repeats the
  model's ``stim_time`` (the pulses of one cycle, relative to its start);
* after solving a window, the first ``n_cycles_to_advance`` cycles are committed, the next window starts
  from the committed end state, and the solution is shifted as its warm start (bioptim's
  advance_window_* methods, fes_nmpc.py:44-79);
* the stimulation history of a window — the last T pulses before its start, at negative times — enters its
  stim table exactly as ``previous_stim`` does in the reference (fes_nmpc.py:69-85); for Hmed the history
  intensities enter as fixed leading parameters, so the sliding-window rows of the first nodes see the
  intensities actually applied, not the padding value.

B independent scenarios (initial states, targets) advance in lockstep in one batched interior-point solve per
window; scenarios shard across GPUs like any independent instances (distributed.shard_instances).  Windows of
one trajectory are sequential.
"""

from __future__ import annotations

import copy
import time
from dataclasses import dataclass, field

import numpy as np

from .fes_models import (DingModelPulseIntensityFrequency, DingModelPulseWidthFrequency, FesModel,
                         PLACEHOLDER_TIME)
from .ocp import FesOcp, OcpFes
from .ode_solver import OdeSolver


@dataclass
class NmpcResult:
    time: np.ndarray                 # committed node times (n_nodes,)
    states: dict                     # name -> (B, n_nodes)
    controls: dict                   # name -> (B, n_nodes - 1)
    pulse_intensity: np.ndarray | None  # Hmed: (B, committed pulses)
    stim_time: list                  # committed pulse times
    iterations: list = field(default_factory=list)   # per window: (B,) IPM iterations
    converged: list = field(default_factory=list)    # per window: (B,) bool
    window_wall: list = field(default_factory=list)  # per window: seconds
    solve_wall: list = field(default_factory=list)   # per window: seconds inside the interior point
    # max_consecutive_failing: per scenario, the window whose failure made it the limit-th in a row (-1: never); that
    # window and everything after it are not committed (NaN), as bioptim's loop stops before storing it
    stopped_at: np.ndarray | None = None


class _Failing:
    """bioptim's ``max_consecutive_failing`` (MultiCyclicNonlinearModelPredictiveControl.solve, passed by
    fes_nmpc.py:158,168) per scenario of a lockstep batch: a scenario stops after that many consecutive windows whose
    interior point did not converge; the loop ends when every scenario has stopped (or the cycles / the update
    function say so)."""

    def __init__(self, B: int, limit: int | None):
        self.limit = int(limit) if limit else 0
        self.count = np.zeros(B, dtype=int)
        self.stopped_at = np.full(B, -1, dtype=int)

    def update(self, converged, w: int):
        converged = np.asarray(converged, dtype=bool)
        self.count = np.where(converged, 0, self.count + 1)
        if self.limit:
            newly = (self.stopped_at < 0) & (self.count >= self.limit)
            self.stopped_at[newly] = w

    def mask(self):
        """Scenarios whose commits from the current window on are void."""
        return self.stopped_at >= 0

    def all_stopped(self) -> bool:
        return bool(self.limit) and bool(np.all(self.stopped_at >= 0))


class FesNmpc:
    def __init__(self, model: FesModel, cycle_duration: float, n_cycles_simultaneous: int = 3,
                 n_cycles_to_advance: int = 1, objective: dict | None = None, pulse_width: dict | None = None,
                 pulse_intensity: dict | None = None, ode_solver=OdeSolver.RK4(n_integration_steps=10),
                 n_shooting_per_cycle: int | None = None, batch: int = 1, device: int = 0, options=None,
                 evaluator=None, band=None, torch_device=None):
        if not isinstance(model, FesModel):
            raise TypeError("model must be a FesModel type")
        if n_cycles_to_advance < 1 or n_cycles_simultaneous < n_cycles_to_advance:
            raise ValueError("need 1 <= n_cycles_to_advance <= n_cycles_simultaneous")
        st = list(model.stim_time)
        if not st or min(st) < 0 or max(st) >= cycle_duration:
            raise ValueError("model.stim_time must hold one cycle's pulses in [0, cycle_duration)")
        self.model, self.cycle_duration = model, float(cycle_duration)
        self.n_sim, self.n_adv = n_cycles_simultaneous, n_cycles_to_advance
        self.cycle_stims = st
        self.objective = dict(objective or {})
        self.pulse_width, self.pulse_intensity = pulse_width, pulse_intensity
        self.ode_solver = ode_solver
        self.B, self.device, self.options = batch, device, options
        self.evaluator, self.band, self.torch_device = evaluator, band, torch_device
        self.T = model._sum_stim_truncation
        self.hmed = isinstance(model, DingModelPulseIntensityFrequency)
        window_stims = self._window_stims()
        n = OcpFes.prepare_n_shooting(window_stims, self.cycle_duration * self.n_sim)
        if n_shooting_per_cycle is not None:
            n = n_shooting_per_cycle * self.n_sim
        if n % self.n_sim:
            raise ValueError("the window's node count must split evenly into cycles")
        self.n_shooting, self.cycle_len = n, n // self.n_sim

    # ---- window construction ------------------------------------------------------------------------
    def _window_stims(self):
        return [round(t + c * self.cycle_duration, 10) for c in range(self.n_sim) for t in self.cycle_stims]

    def _window_model(self, hist_times, hist_int):
        kw = dict(stim_time=self._window_stims(), sum_stim_truncation=self.T)
        prev = {"time": list(hist_times)}
        if self.hmed:
            prev["pulse_intensity"] = list(hist_int)
        return type(self.model)(previous_stim=prev, **kw)

    def _objective(self):
        obj = dict(self.objective)
        ft = obj.get("force_tracking")
        if ft is not None:  # one cycle's target curve, repeated over the window's cycles
            t, f = np.asarray(ft[0], dtype=float), np.asarray(ft[1], dtype=float)
            tt = np.concatenate([t / t.max() * self.cycle_duration + c * self.cycle_duration
                                 for c in range(self.n_sim)]) / (self.cycle_duration * self.n_sim)
            obj["force_tracking"] = [tt, np.tile(f, self.n_sim)]
        return obj

    def _window_ocp(self, hist_times, hist_int) -> FesOcp:
        model = self._window_model(hist_times, hist_int)
        ocp = OcpFes.prepare_ocp(model=model, final_time=self.cycle_duration * self.n_sim,
                                 pulse_width=self.pulse_width, pulse_intensity=self.pulse_intensity,
                                 objective=self._objective(), ode_solver=self.ode_solver, n_shooting=self.n_shooting)
        if self.hmed and ocp.n_params:
            # the T history intensities become fixed leading parameters; node k's window ends at the last pulse
            # <= t_k counted in [history, window pulses]
            nw = ocp.n_params
            dt = ocp.final_time / ocp.n_shooting
            stims = np.asarray(self._window_stims())
            last = np.array([self.T + int(np.sum(stims <= k * dt + 1e-12)) - 1 for k in range(ocp.n_shooting)],
                            dtype=np.int32)
            lo, hi = ocp.p_bounds
            h = np.asarray(hist_int, dtype=float)
            ocp.p_bounds = (np.concatenate([h, lo]), np.concatenate([h, hi]))
            ocp.p_init = np.concatenate([h, ocp.p_init])
            ocp.n_params = self.T + nw
            ocp.last_stim_idx = last
        return ocp

    # ---- the receding-horizon loop --------------------------------------------------------------------
    def solve(self, n_cycles: int | None = None, x0=None, hist=None, update_functions=None, solver=None,
              max_consecutive_failing: int | None = None):
        """Advance until ``n_cycles`` cycles are committed, or — bioptim style — while
        ``update_functions(self, cycle_idx, result)`` returns True (cycle_idx = windows solved so far).  x0: (B, nx)
        initial states (default rest); solver: a Solver.IPOPT (options of every window's interior point);
        max_consecutive_failing: stop a scenario after that many consecutive non-converged windows (NmpcResult.
        stopped_at).  Returns an NmpcResult with the committed trajectory of every scenario."""
        from .solver import BatchedIpm, IpmOptions, NativeIpm, apply_solver

        if n_cycles is None and update_functions is None:
            raise ValueError("give n_cycles or update_functions")
        options = self.options if solver is None else apply_solver(copy.copy(self.options or IpmOptions()), solver)

        B, T = self.B, self.T
        nx = self.model.nb_state
        rest = self.model.standard_rest_values().astype(float)[:, 0]
        x_start = np.tile(rest, (B, 1)) if x0 is None else np.asarray(x0, dtype=float).reshape(B, nx)
        hist_t = [PLACEHOLDER_TIME] * T if hist is None else list(hist[0])
        hist_i = np.full((B, T), float(self.model.min_pulse_intensity())) if self.hmed else None
        committed_stims, committed_int = [], []
        t_nodes = [0.0]
        states = [x_start[:, :, None]]
        ctrl_parts = []
        result = NmpcResult(time=None, states={}, controls={}, pulse_intensity=None, stim_time=[])
        warm = None
        n_windows = int(np.ceil(n_cycles / self.n_adv)) if n_cycles is not None else None
        t_off = 0.0
        failing = _Failing(B, max_consecutive_failing)
        # windows whose stimulation history has the same times share one transcription (stim table, handle,
        # KKT maps): with identical cycles that is every window after the first T pulses
        cache = {}
        w = 0
        while n_windows is None or w < n_windows:
            t0 = time.perf_counter()
            key = tuple(np.round(hist_t, 9))
            if key not in cache:
                ocp = self._window_ocp(hist_t, hist_i[0] if self.hmed else None)
                if self.evaluator is not None:
                    ipm = BatchedIpm(ocp, batch=B, options=options, handle=self.evaluator(ocp, B),
                                     torch_device=self.torch_device, band=self.band)
                else:
                    ipm = NativeIpm(ocp, batch=B, device=self.device, options=options)
                cache[key] = (ocp, ipm)
            ocp, ipm = cache[key]
            v0 = np.tile(ocp.initial_guess_vector(), (B, 1)) if warm is None else warm
            fixed = np.tile(ocp.bounds_vector()[0][ipm.fixed], (B, 1))
            # node-0 states are this window's start state per scenario; Hmed history intensities per scenario
            nzb = ocp.nzb
            fidx = {int(j): i for i, j in enumerate(ipm.fixed)}
            for r in range(nx):
                if r in fidx:
                    fixed[:, fidx[r]] = x_start[:, r]
            if self.hmed and ocp.n_params:
                p0 = ocp.nv - ocp.n_params
                for j in range(T):
                    if p0 + j in fidx:
                        fixed[:, fidx[p0 + j]] = hist_i[:, j]
            v0 = v0.copy()
            v0[:, ipm.fixed] = fixed
            ts = time.perf_counter()
            res = ipm.solve(v0, fixed_values=fixed)
            result.solve_wall.append(time.perf_counter() - ts)
            result.iterations.append(res.iterations)
            result.converged.append(res.converged)
            failing.update(res.converged, w)
            void = failing.mask()
            # commit the first n_adv cycles
            adv_nodes = self.n_adv * self.cycle_len
            V = res.v
            body = V[:, : ocp.n_shooting * nzb].reshape(B, ocp.n_shooting, nzb)
            xs = np.concatenate([body[:, :, :nx], V[:, None, ocp.n_shooting * nzb: ocp.n_shooting * nzb + nx]], 1)
            dt = ocp.final_time / ocp.n_shooting
            states.append(np.where(void[:, None, None], np.nan, np.transpose(xs[:, 1: adv_nodes + 1, :], (0, 2, 1))))
            t_nodes += [t_off + (k + 1) * dt for k in range(adv_nodes)]
            if ocp.nu:
                ctrl_parts.append(np.where(void[:, None, None], np.nan,
                                           np.transpose(body[:, :adv_nodes, ocp.uoff:], (0, 2, 1))))
            x_start = xs[:, adv_nodes, :]
            # pulses of the committed cycles and the new history (relative to the next window's start)
            adv_time = self.n_adv * self.cycle_duration
            win_stims = self._window_stims()
            new = [t for t in win_stims if t < adv_time - 1e-12]
            committed_stims += [t + t_off for t in new]
            all_hist = [t for t in hist_t] + new
            if self.hmed:
                P = V[:, ocp.nv - ocp.n_params:]
                new_int = P[:, T: T + len(new)]
                committed_int.append(np.where(void[:, None], np.nan, new_int))
                all_int = np.concatenate([hist_i, new_int], axis=1)
                hist_i = all_int[:, -T:]
            hist_t = [t - adv_time for t in all_hist[-T:]]
            hist_t = [PLACEHOLDER_TIME if t < PLACEHOLDER_TIME / 2 else t for t in hist_t]
            t_off += adv_time
            # warm start: shift by the committed nodes, repeat the last cycle
            warm = self._shift(ocp, V, adv_nodes)
            result.window_wall.append(time.perf_counter() - t0)
            w += 1
            if failing.all_stopped() or (update_functions is not None and not update_functions(self, w, result)):
                break
        for _, ipm in cache.values():
            ipm.close()
        result.stopped_at = failing.stopped_at
        if n_cycles is None or w * self.n_adv < n_cycles:
            n_cycles = w * self.n_adv
        X = np.concatenate(states, axis=2)
        n_keep = n_cycles * self.cycle_len
        result.time = np.asarray(t_nodes[: n_keep + 1])
        result.states = {name: X[:, i, : n_keep + 1] for i, name in enumerate(self.model.name_dof)}
        if ctrl_parts:
            key = "last_pulse_width" if isinstance(self.model, DingModelPulseWidthFrequency) else "pulse_intensity"
            result.controls = {key: np.concatenate(ctrl_parts, axis=2)[:, :, :n_keep]}
        n_pulses = n_cycles * len(self.cycle_stims)
        result.stim_time = committed_stims[:n_pulses]
        if self.hmed:
            result.pulse_intensity = np.concatenate(committed_int, axis=1)[:, :n_pulses]
        return result

    def solve_fes_nmpc(self, update_functions, solver=None, total_cycles: int | None = None, cycle_solutions=None,
                       get_all_iterations: bool = True, cyclic_options: dict | None = None,
                       max_consecutive_failing: int = 3, x0=None):
        """The reference's driver entry (fes_nmpc.py:150-192): run the receding horizon while ``update_functions``
        allows it (at most ``total_cycles`` cycles), each window solved with ``solver``'s options, stopping a scenario
        after ``max_consecutive_failing`` consecutive non-converged windows.  ``cycle_solutions`` /
        ``get_all_iterations`` / ``cyclic_options`` select which bioptim Solution objects are built; every window's
        convergence, iterations and the committed trajectory are always in the returned NmpcResult."""
        del cycle_solutions, get_all_iterations, cyclic_options
        return self.solve(n_cycles=total_cycles, x0=x0, update_functions=update_functions, solver=solver,
                          max_consecutive_failing=max_consecutive_failing)

    def _shift(self, ocp, V, adv_nodes):
        """Warm start of the next window: the solution shifted by ``adv_nodes`` intervals, the freed tail filled
        with the last cycle again (and, for Hmed, the parameters shifted by the committed pulses)."""
        N, nzb, nx = ocp.n_shooting, ocp.nzb, ocp.nx
        B = V.shape[0]
        body = V[:, : N * nzb].reshape(B, N, nzb)
        tail = V[:, N * nzb: N * nzb + nx]
        blocks = np.concatenate([body[:, adv_nodes:], body[:, N - adv_nodes:]], axis=1)
        out = V.copy()
        out[:, : N * nzb] = blocks.reshape(B, -1)
        out[:, N * nzb: N * nzb + nx] = tail
        if self.hmed and ocp.n_params:
            T = self.T
            P = V[:, N * nzb + nx:]
            w = P[:, T:]
            n_new = int(round(self.n_adv * len(self.cycle_stims)))
            out[:, N * nzb + nx + T:] = np.concatenate([w[:, n_new:], w[:, w.shape[1] - n_new:]], axis=1)
        return out


class NmpcFesMsk:
    """Receding horizon over musculoskeletal windows (reference: ``NmpcFesMsk``,
    cocofest/optimization/fes_ocp_dynamics_nmpc_cyclic.py:16-102, a bioptim
    ``MultiCyclicNonlinearModelPredictiveControl`` over ``OcpFesMsk._prepare_optimization_problem``).

    A window is ``n_cycles_simultaneous`` cycles of the muscles' ``stim_time`` (one cycle's pulses), transcribed
    by :class:`OcpFesMsk` with the window's stimulation history (the last T pulses, ``update_stim``,
    fes_ocp_dynamics_nmpc_cyclic.py:34-46) as ``previous_stim`` of every muscle.  After each window the first
    ``n_cycles_to_advance`` cycles are committed; the next window starts from the committed state (every state of
    its node 0 fixed to it, per scenario: bioptim's advance_window_bounds_states) and the shifted solution is its
    warm start (advance_window_initial_guess_states).  B scenarios advance in lockstep in one native interior-point
    solve per window.  The cycling-specific parts (wheel angle, ``prepare_nmpc_for_cycling``, which calls a
    method the reference does not define) and external forces are not covered."""

    def __init__(self, model, cycle_duration: float, n_cycles_simultaneous: int = 3, n_cycles_to_advance: int = 1,
                 pulse_width: dict | None = None, objective: dict | None = None, msk_info: dict | None = None,
                 ode_solver=OdeSolver.RK4(n_integration_steps=1), n_shooting_per_cycle: int | None = None,
                 n_total_cycles: int | None = None, batch: int = 1, device: int = 0, options=None):
        from .msk import FesMskModel

        if not isinstance(model, FesMskModel):
            raise TypeError("model must be a FesMskModel")
        if n_cycles_to_advance < 1 or n_cycles_simultaneous < n_cycles_to_advance:
            raise ValueError("need 1 <= n_cycles_to_advance <= n_cycles_simultaneous")
        muscles = model.muscles_dynamics_model
        st = list(muscles[0].stim_time)
        if not st or min(st) < 0 or max(st) >= cycle_duration:
            raise ValueError("the muscles' stim_time must hold one cycle's pulses in [0, cycle_duration)")
        self.model, self.cycle_duration = model, float(cycle_duration)
        self.n_sim, self.n_adv, self.n_total = n_cycles_simultaneous, n_cycles_to_advance, n_total_cycles
        self.cycle_stims = st
        self.pulse_width, self.objective, self.msk_info = pulse_width, dict(objective or {}), dict(msk_info or {})
        self.ode_solver = ode_solver
        self.B, self.device, self.options = batch, device, options
        self.T = muscles[0]._sum_stim_truncation
        n = OcpFes.prepare_n_shooting(self._window_stims(), self.cycle_duration * self.n_sim)
        if n_shooting_per_cycle is not None:
            n = n_shooting_per_cycle * self.n_sim
        if n % self.n_sim:
            raise ValueError("the window's node count must split evenly into cycles")
        self.n_shooting, self.cycle_len = n, n // self.n_sim

    @staticmethod
    def prepare_nmpc(model=None, cycle_duration=None, n_cycles_simultaneous: int = None, n_cycles_to_advance: int = None,
                     n_total_cycles: int = None, pulse_width: dict = None, pulse_intensity: dict = None,
                     objective: dict = None, msk_info: dict = None, external_forces: dict = None,
                     initial_guess_warm_start: bool = False, use_sx: bool = True,
                     ode_solver=OdeSolver.RK4(n_integration_steps=1), n_threads: int = 1, control_type=None,
                     n_shooting_per_cycle: int | None = None, batch: int = 1, device: int = 0, options=None):
        """Same arguments as the reference's ``NmpcFesMsk.prepare_nmpc`` (fes_ocp_dynamics_nmpc_cyclic.py:49-102),
        plus the batch / device of the native solver."""
        if external_forces:
            raise NotImplementedError("NmpcFesMsk: external forces are not supported")
        if pulse_intensity:
            raise NotImplementedError("NmpcFesMsk: Hmed2018 pulse-intensity muscles are not supported")
        return NmpcFesMsk(model, cycle_duration, n_cycles_simultaneous, n_cycles_to_advance, pulse_width=pulse_width,
                          objective=objective, msk_info=msk_info, ode_solver=ode_solver,
                          n_shooting_per_cycle=n_shooting_per_cycle, n_total_cycles=n_total_cycles, batch=batch,
                          device=device, options=options)

    def _window_stims(self):
        return [round(t + c * self.cycle_duration, 10) for c in range(self.n_sim) for t in self.cycle_stims]

    def _window_ocp(self, hist_times):
        from .msk import FesMskModel, OcpFesMsk

        base = self.model
        muscles = []
        for m in base.muscles_dynamics_model:  # copies keep any constants the caller set on the muscles
            c = copy.deepcopy(m)
            c.stim_time, c.previous_stim = self._window_stims(), {"time": list(hist_times)}
            c._last_table_src = None
            muscles.append(c)
        model = FesMskModel(name=base.name, biorbd_path=base.biorbd_path, muscles_model=muscles,
                            activate_force_length_relationship=base.activate_force_length_relationship,
                            activate_force_velocity_relationship=base.activate_force_velocity_relationship,
                            activate_passive_force_relationship=base.activate_passive_force_relationship,
                            activate_residual_torque=base.activate_residual_torque)
        ocp = OcpFesMsk.prepare_ocp(model=model, final_time=self.cycle_duration * self.n_sim,
                                    pulse_width=self.pulse_width, objective=self.objective, msk_info=self.msk_info,
                                    ode_solver=self.ode_solver, n_shooting=self.n_shooting)
        # node 0 of every state is the window's start state (the values are set per scenario at each solve)
        lo, hi = ocp.x_bounds
        start = np.where(lo[:, 0] == hi[:, 0], lo[:, 0], ocp.x_init[:, 0])
        lo[:, 0] = hi[:, 0] = start
        return ocp

    def solve(self, update_functions=None, solver=None, n_cycles: int | None = None, x0=None,
              max_consecutive_failing: int | None = None):
        """Advance until ``n_cycles`` cycles are committed (default ``n_total_cycles``), or — bioptim style — while
        ``update_functions(self, cycle_idx, result)`` returns True.  x0: (B, nx) start states (default: the first
        window's node-0 bounds / initial guess); solver: a Solver.IPOPT; max_consecutive_failing: stop a scenario
        after that many consecutive non-converged windows (NmpcResult.stopped_at).  Returns an NmpcResult."""
        from .solver import IpmOptions, NativeIpm, apply_solver

        if n_cycles is None:
            n_cycles = self.n_total
        if n_cycles is None and update_functions is None:
            raise ValueError("give n_cycles (or n_total_cycles) or update_functions")
        opts = apply_solver(copy.copy(self.options or IpmOptions()), solver)
        failing = _Failing(self.B, max_consecutive_failing)
        B, T = self.B, self.T
        hist_t = [PLACEHOLDER_TIME] * T
        cache = {}
        result = NmpcResult(time=None, states={}, controls={}, pulse_intensity=None, stim_time=[])
        states, ctrl_parts, committed = [], [], []
        t_nodes, t_off, warm, x_start = [0.0], 0.0, None, None
        adv_nodes, adv_time = self.n_adv * self.cycle_len, self.n_adv * self.cycle_duration
        ocp = None
        w = 0
        while True:
            if n_cycles is not None and w * self.n_adv >= n_cycles:
                break
            t0 = time.perf_counter()
            key = tuple(np.round(hist_t, 9))
            if key not in cache:
                o = self._window_ocp(hist_t)
                cache[key] = (o, NativeIpm(o, batch=B, device=self.device, options=opts))
            ocp, ipm = cache[key]
            nx = ocp.nx
            if x_start is None:
                x_start = np.tile(ocp.x_bounds[0][:, 0], (B, 1)) if x0 is None else \
                    np.asarray(x0, dtype=float).reshape(B, nx)
                states.append(x_start[:, :, None])
            lb, _ = ocp.bounds_vector()
            fixed = np.tile(lb[ipm.fixed], (B, 1))
            fidx = {int(j): i for i, j in enumerate(ipm.fixed)}
            for r in range(nx):
                fixed[:, fidx[r]] = x_start[:, r]
            v0 = np.tile(ocp.initial_guess_vector(), (B, 1)) if warm is None else warm.copy()
            v0[:, ipm.fixed] = fixed
            ts = time.perf_counter()
            res = ipm.solve(v0, fixed_values=fixed)
            result.solve_wall.append(time.perf_counter() - ts)
            result.iterations.append(res.iterations)
            result.converged.append(res.converged)
            failing.update(res.converged, w)
            void = failing.mask()
            N, nzb = ocp.n_shooting, ocp.nzb
            body = res.v[:, : N * nzb].reshape(B, N, nzb)
            xs = np.concatenate([body[:, :, :nx], res.v[:, None, N * nzb: N * nzb + nx]], 1)
            states.append(np.where(void[:, None, None], np.nan, np.transpose(xs[:, 1: adv_nodes + 1, :], (0, 2, 1))))
            dt = ocp.final_time / N
            t_nodes += [t_off + (k + 1) * dt for k in range(adv_nodes)]
            if ocp.nu:
                ctrl_parts.append(np.where(void[:, None, None], np.nan, np.transpose(body[:, :adv_nodes, nx:], (0, 2, 1))))
            x_start = xs[:, adv_nodes, :]
            new = [t for t in self._window_stims() if t < adv_time - 1e-12]
            committed += [t + t_off for t in new]
            hist_t = [t - adv_time for t in (list(hist_t) + new)[-T:]]
            hist_t = [PLACEHOLDER_TIME if t < PLACEHOLDER_TIME / 2 else t for t in hist_t]
            t_off += adv_time
            blocks = np.concatenate([body[:, adv_nodes:], body[:, N - adv_nodes:]], axis=1)
            warm = res.v.copy()
            warm[:, : N * nzb] = blocks.reshape(B, -1)
            result.window_wall.append(time.perf_counter() - t0)
            w += 1
            if failing.all_stopped() or (update_functions is not None and not update_functions(self, w, result)):
                break
        for _, ipm in cache.values():
            ipm.close()
        result.stopped_at = failing.stopped_at
        X = np.concatenate(states, axis=2)
        n_keep = min(w * self.n_adv, n_cycles if n_cycles is not None else w * self.n_adv) * self.cycle_len
        result.time = np.asarray(t_nodes[: n_keep + 1])
        result.states = {name: X[:, i, : n_keep + 1] for i, name in enumerate(ocp.state_names)}
        if ctrl_parts:
            C = np.concatenate(ctrl_parts, axis=2)[:, :, :n_keep]
            result.controls = {name: C[:, i] for i, name in enumerate(ocp.control_names)}
        result.stim_time = committed[: (n_keep // self.cycle_len) * len(self.cycle_stims)]
        return result
