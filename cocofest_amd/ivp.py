"""IvpFes: forward simulation of an FES model (reference: cocofest/integration/ivp_fes.py).

Same constructor dictionaries, defaults, pulse modes and validation messages as the reference.  The
integration itself (single shooting, every RK sub-step returned) runs on the GPU through
``cfx_integrate``; batches of independent instances use :meth:`IvpFes.handle`.
"""

from __future__ import annotations

import numpy as np

from . import _cfx
from .fes_models import (
    DingModelPulseIntensityFrequency,
    DingModelPulseIntensityFrequencyWithFatigue,
    DingModelPulseWidthFrequency,
    DingModelPulseWidthFrequencyWithFatigue,
    FesModel,
    PLACEHOLDER_INTENSITY,
)
from .ocp import OcpFes
from .ode_solver import OdeSolver


class IvpFes:
    def __init__(self, fes_parameters: dict = None, ivp_parameters: dict = None):
        self._fill_fes_dict(fes_parameters)
        self._fill_ivp_dict(ivp_parameters)
        self.dictionaries_check()

        self.model = self.fes_parameters["model"]
        self.stim_time = self.model.stim_time
        self.n_stim = len(self.stim_time)
        self.pulse_width = self.fes_parameters["pulse_width"]
        self.pulse_intensity = self.fes_parameters["pulse_intensity"]
        self.final_time = self.ivp_parameters["final_time"]
        # extension: ivp_parameters["n_shooting"] sets the node count (the reference always takes the LCM rule of
        # OcpFes.prepare_n_shooting, ivp_fes.py:73), e.g. BASELINE configs[0]'s n_shooting = 20 for 10 pulses
        self._n_shooting_given = self.ivp_parameters["n_shooting"]
        self.n_shooting = self._n_shooting_given or OcpFes.prepare_n_shooting(self.stim_time, self.final_time)
        self.pulse_mode = self.fes_parameters["pulse_mode"]
        self._pulse_mode_settings()
        self.dt = np.array([self.final_time / self.n_shooting])

        self.controls_keys = None
        if isinstance(self.model, DingModelPulseWidthFrequency):
            self.controls_keys = ["last_pulse_width"]
        if isinstance(self.model, DingModelPulseIntensityFrequency):
            self.controls_keys = ["pulse_intensity"]

        table, self.stim_idx_at_node_list = self.model.get_numerical_data_time_series(self.n_shooting,
                                                                                      self.final_time)
        self.stim_rows = table["stim_time"][:, 0, :].T.copy()
        self.controls = self._build_controls()
        self.ode_solver = self.ivp_parameters["ode_solver"]
        self.n_threads = self.ivp_parameters["n_threads"]

    # ---- dictionaries (ivp_fes.py:113-230) ----------------------------------------------------------
    def _fill_fes_dict(self, fes_parameters):
        default = {"model": FesModel, "stim_time": None, "pulse_width": 0.0003, "pulse_intensity": 50,
                   "pulse_mode": "single"}
        fes_parameters = {} if fes_parameters is None else fes_parameters
        for key in default:
            if key not in fes_parameters:
                fes_parameters[key] = default[key]
        self.fes_parameters = fes_parameters

    def _fill_ivp_dict(self, ivp_parameters):
        default = {"final_time": None, "ode_solver": OdeSolver.RK4(n_integration_steps=10), "n_threads": 1,
                   "n_shooting": None}
        ivp_parameters = {} if ivp_parameters is None else ivp_parameters
        for key in default:
            if key not in ivp_parameters:
                ivp_parameters[key] = default[key]
        self.ivp_parameters = ivp_parameters

    def dictionaries_check(self):
        fes, ivp = self.fes_parameters, self.ivp_parameters
        if not isinstance(fes, dict):
            raise ValueError("fes_parameters must be a dictionary")
        if not isinstance(ivp, dict):
            raise ValueError("ivp_parameters must be a dictionary")
        if not isinstance(fes["model"], FesModel):
            raise TypeError("model must be a FesModel type")
        model = fes["model"]
        if isinstance(model, DingModelPulseWidthFrequency | DingModelPulseWidthFrequencyWithFatigue):
            pw = fes["pulse_width"]
            if isinstance(pw, bool) or not isinstance(pw, int | float | list):
                raise TypeError("pulse_width must be int, float or list type")
            ok = all(p >= model.pd0 for p in pw) if isinstance(pw, list) else pw >= model.pd0
            if not ok:
                raise ValueError("pulse width must be greater than minimum pulse width")
        if isinstance(model, DingModelPulseIntensityFrequency | DingModelPulseIntensityFrequencyWithFatigue):
            pi = fes["pulse_intensity"]
            if isinstance(pi, bool) or not isinstance(pi, int | float | list):
                raise TypeError("pulse_intensity must be int, float or list type")
            imin = model.min_pulse_intensity()
            ok = all(p >= imin for p in pi) if isinstance(pi, list) else bool(pi >= imin)
            if not ok:
                raise ValueError("Pulse intensity must be greater than minimum pulse intensity")
        if not isinstance(fes["pulse_mode"], str):
            raise ValueError("pulse_mode must be a string type")
        if not isinstance(ivp["final_time"], int | float):
            raise ValueError("final_time must be an int or float type")
        if not isinstance(ivp["ode_solver"], (OdeSolver.RK1, OdeSolver.RK2, OdeSolver.RK4, OdeSolver.COLLOCATION)):
            raise ValueError("ode_solver must be a OdeSolver type")
        if not isinstance(ivp["n_threads"], int):
            raise ValueError("n_thread must be a int type")
        ns = ivp["n_shooting"]
        if ns is not None and (isinstance(ns, bool) or not isinstance(ns, int) or ns < 1):
            raise ValueError("n_shooting must be a positive int (or None for the stimulation-time LCM rule)")

    def _pulse_mode_settings(self):
        """Doublets / triplets add pulses 5 and 10 ms after each one and write the list back into the model
        (ivp_fes.py:232-256; the write-back is the reference's behaviour)."""
        if self.pulse_mode == "single":
            return
        if self.pulse_mode == "doublet":
            extra = [[round(t + 0.005, 3) for t in self.stim_time]]
        elif self.pulse_mode == "triplet":
            extra = [[round(t + 0.005, 3) for t in self.stim_time], [round(t + 0.01, 3) for t in self.stim_time]]
        else:
            raise ValueError("Pulse mode not yet implemented")
        self.stim_time = self.stim_time + [t for e in extra for t in e]
        self.stim_time.sort()
        self.model.stim_time = self.stim_time
        self.n_stim = len(self.stim_time)
        if self._n_shooting_given is None:
            self.n_shooting = OcpFes.prepare_n_shooting(self.stim_time, self.final_time)

    def _build_controls(self):
        """Per-interval controls, (nu, N).  Ding2007: width of the last pulse at or before the node
        (ivp_fes.py:344-351).  Hmed2018: the T intensities aligned with the node's stim row, history
        placeholders at 50 mA (equal to ivp_fes.py:324-342 whenever N == n_stim)."""
        N = self.n_shooting
        if isinstance(self.model, DingModelPulseWidthFrequency):
            pw = self.pulse_width
            if isinstance(pw, list) and len(pw) != 1:
                vals = [pw[self.stim_idx_at_node_list[k][-1]] for k in range(N)]
            else:
                vals = [pw[0] if isinstance(pw, list) else pw] * N
            return np.array([vals], dtype=float)
        if isinstance(self.model, DingModelPulseIntensityFrequency):
            T = self.model._sum_stim_truncation
            src = self.model._last_table_src
            n_prefix = len(self.model.previous_stim["time"])
            pi = self.pulse_intensity
            out = np.empty((T, N))
            for k in range(N):
                for j in range(T):
                    s = src[k, j] - n_prefix
                    if s < 0:
                        out[j, k] = PLACEHOLDER_INTENSITY
                    elif isinstance(pi, list):
                        out[j, k] = pi[s] if len(pi) != 1 else pi[0]
                    else:
                        out[j, k] = pi
            return out
        return np.zeros((0, N))

    # ---- integration ---------------------------------------------------------------------------------
    def handle(self, batch: int = 1, layout: str = "aos", device: int = 0) -> _cfx.Handle:
        if isinstance(self.ode_solver, OdeSolver.COLLOCATION):
            raise NotImplementedError("COLLOCATION integration is not available in libcfx yet")
        return _cfx.Handle(model_id=self.model.cfx_model_id, constants=self.model.cfx_constants(),
                           scheme=self.ode_solver.scheme, n_steps=self.ode_solver.n_integration_steps,
                           n_shooting=self.n_shooting, truncation=self.model._sum_stim_truncation,
                           final_time=float(self.final_time), stim_rows=self.stim_rows, batch=batch,
                           layout=_cfx.LAYOUT_AOS if layout == "aos" else _cfx.LAYOUT_SOA, device=device)

    def integrate(self, shooting_type=None, integrator=None, to_merge=None, return_time=True,
                  duplicated_times=False):
        """Single-shooting integration from the rest state; returns {state: (1, N*m+1)} (and the time)."""
        if getattr(self, "_h1", None) is None:  # the handle (tables, buffers) is built once per IvpFes
            self._h1 = self.handle(batch=1)
            self._u1 = self.controls.T.reshape(1, -1).copy() if self.controls.shape[0] else None
        traj = self._h1.integrate(u=self._u1)
        m = self.ode_solver.n_integration_steps
        nx = self.model.nb_state
        traj = traj.reshape(self.n_shooting * m + 1, nx)
        result = {name: traj[:, i][np.newaxis, :] for i, name in enumerate(self.model.name_dof)}
        if not return_time:
            return result
        hstep = self.final_time / self.n_shooting / m
        time = np.array([k * (self.final_time / self.n_shooting) + j * hstep for k in range(self.n_shooting)
                         for j in range(m)] + [float(self.final_time)])
        return result, time

    def close(self):
        if getattr(self, "_h1", None) is not None:
            self._h1.close()
            self._h1 = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @classmethod
    def from_frequency_and_final_time(cls, fes_parameters: dict = None, ivp_parameters: dict = None):
        """ivp_fes.py:359-405."""
        frequency = fes_parameters["frequency"]
        if not isinstance(frequency, int):
            raise ValueError("Frequency must be an int")
        round_down = fes_parameters["round_down"]
        if not isinstance(round_down, bool):
            raise ValueError("Round down must be a bool")
        final_time = ivp_parameters["final_time"]
        if not isinstance(final_time, int | float):
            raise ValueError("Final time must be an int or float")
        fes_parameters["n_stim"] = final_time * frequency
        if round_down or float(fes_parameters["n_stim"]).is_integer():
            fes_parameters["n_stim"] = int(fes_parameters["n_stim"])
        else:
            raise ValueError("The number of stimulation needs to be integer within the final time t, set round down "
                             "to True or set final_time * frequency to make the result an integer.")
        fes_parameters["stim_time"] = list(np.round([i * 1 / frequency for i in range(fes_parameters["n_stim"])], 3))
        return cls(fes_parameters, ivp_parameters)

    @classmethod
    def from_frequency_and_n_stim(cls, fes_parameters: dict = None, ivp_parameters: dict = None):
        """ivp_fes.py:407-443."""
        n_stim = fes_parameters["n_stim"]
        if not isinstance(n_stim, int):
            raise ValueError("n_stim must be an int")
        frequency = fes_parameters["frequency"]
        if not isinstance(frequency, int):
            raise ValueError("Frequency must be an int")
        ivp_parameters["final_time"] = n_stim / frequency
        fes_parameters["stim_time"] = list(np.round([i * 1 / frequency for i in range(n_stim)], 3))
        return cls(fes_parameters, ivp_parameters)
