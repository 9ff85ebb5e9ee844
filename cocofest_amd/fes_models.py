"""FES muscle models: constants, state layout and the stimulation table (host side).

Mirrors the public surface of the reference model plugins (cocofest/models/*.py): same class names,
constructor arguments, default constants, ``name_dof`` / ``nb_state`` / ``standard_rest_values`` /
``get_numerical_data_time_series`` / ``min_pulse_intensity``.  The right-hand sides themselves are not
evaluated here: they are compiled into the gfx950 kernels of libcfx (``csrc/cfx_kernels.h``), which
these classes parameterise through ``cfx_model_id`` and ``cfx_constants()``.
"""

from __future__ import annotations

from fractions import Fraction

import numpy as np

from ._cfx import MODEL_IDS

PLACEHOLDER_TIME = -10000000  # ding2003.py:396
PLACEHOLDER_INTENSITY = 50  # hmed2018.py:315


class FesModel:
    """Base of every FES model (reference: cocofest/models/fes_model.py:8-225)."""

    _with_fatigue = False

    @property
    def with_fatigue(self):
        return self._with_fatigue

    @property
    def model_name(self):
        return self._model_name

    @property
    def muscle_name(self):
        return self._muscle_name

    @property
    def cfx_model_id(self) -> int:
        raise NotImplementedError

    def cfx_constants(self) -> dict:
        return {k: float(getattr(self, k, 0.0)) for k in (
            "tauc", "r0_km_relationship", "a_rest", "tau1_rest", "tau2", "km_rest", "a_scale", "pd0", "pdt",
            "ar", "bs", "Is", "cr", "alpha_a", "alpha_tau1", "alpha_km", "tau_fat")} | {"fl": 1.0, "fv": 1.0, "fp": 0.0}


class DingModelFrequency(FesModel):
    """Ding 2003 calcium / force model, stimulation frequency as input (cocofest/models/ding2003.py:17-429)."""

    def __init__(self, model_name: str = "ding2003", muscle_name: str = None, stim_time: list = None,
                 previous_stim: dict = None, sum_stim_truncation: int = 20):
        self._model_name = model_name
        self._muscle_name = muscle_name
        self._sum_stim_truncation = sum_stim_truncation
        self._with_fatigue = False
        self.pulse_apparition_time = None
        self.stim_time = stim_time if stim_time else []
        self.previous_stim = previous_stim if previous_stim else {"time": []}
        self.all_stim = self.previous_stim["time"] + self.stim_time
        # ding2003.py:51-66
        self.tauc = 0.020
        self.r0_km_relationship = 1.04
        self.a_rest = 3009
        self.tau1_rest = 0.050957
        self.tau2 = 0.060
        self.km_rest = 0.103
        self._last_table_src = None

    # setters kept for API parity (ding2003.py:68-79)
    def set_a_rest(self, model, a_rest):
        self.a_rest = a_rest

    def set_km_rest(self, model, km_rest):
        self.km_rest = km_rest

    def set_tau1_rest(self, model, tau1_rest):
        self.tau1_rest = tau1_rest

    def set_tau2(self, model, tau2):
        self.tau2 = tau2

    def standard_rest_values(self) -> np.ndarray:
        return np.array([[0], [0]])

    def serialize(self):
        return type(self), {k: getattr(self, k) for k in ("tauc", "a_rest", "tau1_rest", "km_rest", "tau2")}

    @property
    def name_dof(self) -> list:
        return ["Cn", "F"]

    @property
    def nb_state(self) -> int:
        return 2

    @property
    def identifiable_parameters(self):
        return {"a_rest": self.a_rest, "tau1_rest": self.tau1_rest, "km_rest": self.km_rest, "tau2": self.tau2}

    @property
    def km_name(self) -> str:
        return "Km" + ("_" + self.muscle_name if self.muscle_name else "")

    @property
    def cn_sum_name(self):
        return "Cn_sum" + ("_" + self.muscle_name if self.muscle_name else "")

    def get_r0(self, km):
        return km + self.r0_km_relationship

    @property
    def cfx_model_id(self) -> int:
        return MODEL_IDS["ding2003_with_fatigue" if self._with_fatigue else "ding2003"]

    # ---- stimulation table (ding2003.py:394-429) ----
    def _get_additional_previous_stim_time(self):
        while len(self.previous_stim["time"]) < self._sum_stim_truncation:
            self.previous_stim["time"].insert(0, PLACEHOLDER_TIME)
        return self.previous_stim

    def get_numerical_data_time_series(self, n_shooting, final_time, all_stim_time=None):
        """Stimulation table of the reference: for node k the last T stim times <= k*final_time/n_shooting.

        The node lookup uses exact rational arithmetic; the reference's float ``<=`` (ding2003.py:411)
        drops pulses that fall on a node whose float time rounds below it (e.g. T=0.3 s, n=3), which the
        reference's own golden vectors do not reproduce.
        Returns ({"stim_time": (T, 1, n_shooting+1)}, stim_idx_at_node_list).
        """
        truncation = self._sum_stim_truncation
        if truncation is None:
            raise ValueError(f"sum_stim_truncation must be set for {type(self).__name__} "
                             "(the reference's default None is not a usable truncation)")
        self.previous_stim = self._get_additional_previous_stim_time()
        stim_time = all_stim_time if all_stim_time else self.stim_time
        self.all_stim = self.previous_stim["time"] + list(stim_time)
        exact = [Fraction(s).limit_denominator() for s in self.all_stim]
        tf = Fraction(final_time).limit_denominator()
        node_idx = []
        for k in range(n_shooting + 1):
            tk = tf * k / n_shooting
            node_idx.append(max(i for i, s in enumerate(exact) if s <= tk))
        arr = np.asarray(self.all_stim, dtype=np.float64)
        rows = np.empty((n_shooting + 1, truncation))
        src = np.empty((n_shooting + 1, truncation), dtype=np.int64)
        for k, idx in enumerate(node_idx):
            lo = idx + 1 - truncation
            if lo < 0:
                raise ValueError("stimulation history shorter than the truncation")
            rows[k] = arr[lo: idx + 1]
            src[k] = np.arange(lo, idx + 1)
        node_list = list(range(n_shooting + 1))
        stim_idx_at_node_list = [node_list[: idx - truncation + 1][-truncation:] for idx in node_idx]
        self._last_table_src = src
        return {"stim_time": rows.T[:, np.newaxis, :].copy()}, stim_idx_at_node_list


class DingModelFrequencyWithFatigue(DingModelFrequency):
    """Ding 2003 with fatigue states A, Tau1, Km (cocofest/models/ding2003_with_fatigue.py:20-325)."""

    def __init__(self, model_name: str = "ding2003_with_fatigue", muscle_name: str = None, stim_time: list = None,
                 previous_stim: dict = None, sum_stim_truncation: int = 20, is_approximated: bool = False):
        super().__init__(model_name=model_name, muscle_name=muscle_name, stim_time=stim_time,
                         previous_stim=previous_stim, sum_stim_truncation=sum_stim_truncation)
        self._with_fatigue = True
        self.is_approximated = is_approximated
        _set_fatigue_defaults(self)

    def standard_rest_values(self) -> np.ndarray:
        return np.array([[0], [0], [self.a_rest], [self.tau1_rest], [self.km_rest]])

    @property
    def name_dof(self) -> list:
        return ["Cn", "F", "A", "Tau1", "Km"]

    @property
    def nb_state(self) -> int:
        return 5

    def serialize(self):
        keys = ("tauc", "a_rest", "tau1_rest", "km_rest", "tau2", "alpha_a", "alpha_tau1", "alpha_km", "tau_fat")
        return type(self), {k: getattr(self, k) for k in keys}

    @property
    def identifiable_parameters(self):
        return super().identifiable_parameters | {"alpha_a": self.alpha_a, "alpha_tau1": self.alpha_tau1,
                                                  "alpha_km": self.alpha_km, "tau_fat": self.tau_fat}

    def set_alpha_a(self, model, alpha_a):
        self.alpha_a = alpha_a

    def set_alpha_km(self, model, alpha_km):
        self.alpha_km = alpha_km

    def set_alpha_tau1(self, model, alpha_tau1):
        self.alpha_tau1 = alpha_tau1

    def set_tau_fat(self, model, tau_fat):
        self.tau_fat = tau_fat


def _set_fatigue_defaults(model):
    # ding2003_with_fatigue.py:50-59 (same literals in ding2007/hmed2018 fatigue variants)
    model.alpha_a = -4.0 * 10e-2
    model.alpha_tau1 = 2.1 * 10e-6
    model.tau_fat = 127
    model.alpha_km = 1.9 * 10e-6


class DingModelPulseWidthFrequency(DingModelFrequency):
    """Ding 2007: pulse width per pulse scales A (cocofest/models/ding2007.py:17-308).

    Control: ``last_pulse_width`` (one per interval, the width of the last pulse at or before the node).
    """

    def __init__(self, model_name: str = "ding_2007", muscle_name: str = None, stim_time: list = None,
                 previous_stim: dict = None, sum_stim_truncation: int = None, **_unused):
        super().__init__(model_name=model_name, muscle_name=muscle_name, stim_time=stim_time,
                         previous_stim=previous_stim, sum_stim_truncation=sum_stim_truncation)
        self._with_fatigue = False
        self.pulse_width = None
        self.previous_stim = previous_stim if previous_stim else {"time": []}
        self.stim_time = stim_time
        # ding2007.py:63-79
        self.a_scale = 4920
        self.pd0 = 0.000131405
        self.pdt = 0.000194138
        self.tau1_rest = 0.060601
        self.tau2 = 0.001
        self.km_rest = 0.137
        self.tauc = 0.011

    @property
    def identifiable_parameters(self):
        return {"a_scale": self.a_scale, "tau1_rest": self.tau1_rest, "km_rest": self.km_rest, "tau2": self.tau2,
                "pd0": self.pd0, "pdt": self.pdt}

    def set_a_scale(self, model, a_scale):
        self.a_scale = a_scale

    def set_pd0(self, model, pd0):
        self.pd0 = pd0

    def set_pdt(self, model, pdt):
        self.pdt = pdt

    def set_impulse_width(self, value):
        self.pulse_width = value

    def serialize(self):
        keys = ("tauc", "a_rest", "tau1_rest", "km_rest", "tau2", "a_scale", "pd0", "pdt", "stim_time", "previous_stim")
        return type(self), {k: getattr(self, k) for k in keys}

    @property
    def cfx_model_id(self) -> int:
        return MODEL_IDS["ding2007_with_fatigue" if self._with_fatigue else "ding2007"]


class DingModelPulseWidthFrequencyWithFatigue(DingModelPulseWidthFrequency):
    """Ding 2007 with fatigue; A relaxes to a_scale (cocofest/models/ding2007_with_fatigue.py:19-328)."""

    def __init__(self, model_name: str = "ding_2007_with_fatigue", muscle_name: str = None, stim_time: list = None,
                 previous_stim: dict = None, sum_stim_truncation: int = 20, **_unused):
        super().__init__(model_name=model_name, muscle_name=muscle_name, stim_time=stim_time,
                         previous_stim=previous_stim, sum_stim_truncation=sum_stim_truncation)
        self._with_fatigue = True
        self.stim_time = stim_time
        _set_fatigue_defaults(self)

    @property
    def name_dof(self) -> list:
        return ["Cn", "F", "A", "Tau1", "Km"]

    @property
    def nb_state(self) -> int:
        return 5

    def standard_rest_values(self) -> np.ndarray:
        return np.array([[0], [0], [self.a_scale], [self.tau1_rest], [self.km_rest]])

    @property
    def identifiable_parameters(self):
        return super().identifiable_parameters | {"alpha_a": self.alpha_a, "alpha_tau1": self.alpha_tau1,
                                                  "alpha_km": self.alpha_km, "tau_fat": self.tau_fat}


class DingModelPulseIntensityFrequency(DingModelFrequency):
    """Hmed 2018: pulse intensity per pulse scales each calcium term by lambda_i
    (cocofest/models/hmed2018.py:17-316).  Control: ``pulse_intensity`` (T per interval, aligned with
    the node's stim row)."""

    def __init__(self, model_name: str = "hmed2018", muscle_name: str = None, stim_time: list = None,
                 previous_stim: dict = None, sum_stim_truncation: int = 20):
        if previous_stim:
            if len(previous_stim["time"]) != len(previous_stim["pulse_intensity"]):
                raise ValueError("The previous_stim time and pulse_intensity must have the same length")
        super().__init__(model_name=model_name, muscle_name=muscle_name, stim_time=stim_time,
                         previous_stim=previous_stim, sum_stim_truncation=sum_stim_truncation)
        self._with_fatigue = False
        self.stim_pulse_intensity_prev = []
        self.previous_stim = previous_stim if previous_stim else {"time": [], "pulse_intensity": []}
        # hmed2018.py:53-63
        self.ar = 0.586
        self.bs = 0.026
        self.Is = 63.1
        self.cr = 0.833
        self.impulse_intensity = None

    @property
    def identifiable_parameters(self):
        return super().identifiable_parameters | {"ar": self.ar, "bs": self.bs, "Is": self.Is, "cr": self.cr}

    @property
    def pulse_intensity_name(self):
        return "pulse_intensity" + ("_" + self.muscle_name if self.muscle_name else "")

    def set_ar(self, model, ar):
        self.ar = ar

    def set_bs(self, model, bs):
        self.bs = bs

    def set_Is(self, model, Is):
        self.Is = Is

    def set_cr(self, model, cr):
        self.cr = cr

    def set_impulse_intensity(self, value):
        self.impulse_intensity = list(value)

    def serialize(self):
        keys = ("tauc", "a_rest", "tau1_rest", "km_rest", "tau2", "ar", "bs", "Is", "cr")
        return type(self), {k: getattr(self, k) for k in keys}

    def min_pulse_intensity(self):
        """Intensity where lambda_i = 0 (hmed2018.py:303-310)."""
        return (np.arctanh(-self.cr) / self.bs) + self.Is

    def _get_additional_previous_stim_time(self):
        while len(self.previous_stim["time"]) < self._sum_stim_truncation:
            self.previous_stim["time"].insert(0, PLACEHOLDER_TIME)
            self.previous_stim["pulse_intensity"].insert(0, PLACEHOLDER_INTENSITY)
        return self.previous_stim

    @property
    def cfx_model_id(self) -> int:
        return MODEL_IDS["hmed2018_with_fatigue" if self._with_fatigue else "hmed2018"]


class DingModelPulseIntensityFrequencyWithFatigue(DingModelPulseIntensityFrequency):
    """Hmed 2018 with fatigue (cocofest/models/hmed2018_with_fatigue.py:20-316)."""

    def __init__(self, model_name: str = "hmed2018_with_fatigue", muscle_name: str = None, stim_time: list = None,
                 previous_stim: dict = None, sum_stim_truncation: int = 20):
        super().__init__(model_name=model_name, muscle_name=muscle_name, stim_time=stim_time,
                         previous_stim=previous_stim, sum_stim_truncation=sum_stim_truncation)
        self._with_fatigue = True
        _set_fatigue_defaults(self)

    @property
    def name_dof(self) -> list:
        return ["Cn", "F", "A", "Tau1", "Km"]

    @property
    def nb_state(self) -> int:
        return 5

    def standard_rest_values(self) -> np.ndarray:
        return np.array([[0], [0], [self.a_rest], [self.tau1_rest], [self.km_rest]])

    @property
    def identifiable_parameters(self):
        return super().identifiable_parameters | {"alpha_a": self.alpha_a, "alpha_tau1": self.alpha_tau1,
                                                  "alpha_km": self.alpha_km, "tau_fat": self.tau_fat}


class ModelMaker:
    """String registry of the six models (cocofest/models/model_maker.py:9-22)."""

    @staticmethod
    def create_model(model_type, **kwargs):
        model_dict = {
            "ding2003": DingModelFrequency,
            "ding2003_with_fatigue": DingModelFrequencyWithFatigue,
            "ding2007": DingModelPulseWidthFrequency,
            "ding2007_with_fatigue": DingModelPulseWidthFrequencyWithFatigue,
            "hmed2018": DingModelPulseIntensityFrequency,
            "hmed2018_with_fatigue": DingModelPulseIntensityFrequencyWithFatigue,
        }
        if model_type not in model_dict:
            raise ValueError(f"Unknown model type: {model_type}")
        return model_dict[model_type](**kwargs)
