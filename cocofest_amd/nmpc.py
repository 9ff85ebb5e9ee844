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
    def solve(self, n_cycles: int, x0=None, hist=None):
        """Advance until ``n_cycles`` cycles are committed.  x0: (B, nx) initial states (default rest).
        Returns an NmpcResult with the committed trajectory of every scenario."""
        from .solver import BatchedIpm, NativeIpm

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
        n_windows = int(np.ceil(n_cycles / self.n_adv))
        t_off = 0.0
        # windows whose stimulation history has the same times share one transcription (stim table, handle,
        # KKT maps): with identical cycles that is every window after the first T pulses
        cache = {}
        for w in range(n_windows):
            t0 = time.perf_counter()
            key = tuple(np.round(hist_t, 9))
            if key not in cache:
                ocp = self._window_ocp(hist_t, hist_i[0] if self.hmed else None)
                if self.evaluator is not None:
                    ipm = BatchedIpm(ocp, batch=B, options=self.options, handle=self.evaluator(ocp, B),
                                     torch_device=self.torch_device, band=self.band)
                else:
                    ipm = NativeIpm(ocp, batch=B, device=self.device, options=self.options)
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
            # commit the first n_adv cycles
            adv_nodes = self.n_adv * self.cycle_len
            V = res.v
            body = V[:, : ocp.n_shooting * nzb].reshape(B, ocp.n_shooting, nzb)
            xs = np.concatenate([body[:, :, :nx], V[:, None, ocp.n_shooting * nzb: ocp.n_shooting * nzb + nx]], 1)
            dt = ocp.final_time / ocp.n_shooting
            states.append(np.transpose(xs[:, 1: adv_nodes + 1, :], (0, 2, 1)))
            t_nodes += [t_off + (k + 1) * dt for k in range(adv_nodes)]
            if ocp.nu:
                ctrl_parts.append(np.transpose(body[:, :adv_nodes, ocp.uoff:], (0, 2, 1)))
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
                committed_int.append(new_int)
                all_int = np.concatenate([hist_i, new_int], axis=1)
                hist_i = all_int[:, -T:]
            hist_t = [t - adv_time for t in all_hist[-T:]]
            hist_t = [PLACEHOLDER_TIME if t < PLACEHOLDER_TIME / 2 else t for t in hist_t]
            t_off += adv_time
            # warm start: shift by the committed nodes, repeat the last cycle
            warm = self._shift(ocp, V, adv_nodes)
            result.window_wall.append(time.perf_counter() - t0)
        for _, ipm in cache.values():
            ipm.close()
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
