"""cocofest_amd — MI355X-native NLP-evaluation engine for cocofest's FES optimal-control problems.

The public names mirror the reference package (Ipuch/cocofest) for the accelerated path: the six FES
models, ``ModelMaker``, ``OcpFes``, ``IvpFes``, ``FourierSeries`` and the bioptim-style ``OdeSolver`` /
``ObjectiveFcn`` / ``ObjectiveList`` / ``Node`` the reference's call sites use, ``FesMskModel`` / ``OcpFesMsk``
(FES muscles driving a bioMod skeleton), ``FesNmpc`` (receding
horizon, every model family) and the batched interior-point driver standing in for Ipopt.  All NLP callbacks and
integrations execute in libcfx (hand-written HIP for gfx950) — there is no CPU evaluation path.
"""

from ._cfx import CfxError, Handle, load_library
from .fes_models import (
    DingModelFrequency,
    DingModelFrequencyWithFatigue,
    DingModelPulseIntensityFrequency,
    DingModelPulseIntensityFrequencyWithFatigue,
    DingModelPulseWidthFrequency,
    DingModelPulseWidthFrequencyWithFatigue,
    FesModel,
    ModelMaker,
)
from .fourier import FourierSeries
from .ivp import IvpFes
from .msk import FesMskModel, FesMskOcp, OcpFesMsk
from .nmpc import FesNmpc, NmpcFesMsk, NmpcResult
from .ocp import Axis, Constraint, ConstraintFcn, ConstraintList, FesOcp, Node, Objective, ObjectiveFcn, ObjectiveList, OcpFes
from .ode_solver import ControlType, OdeSolver
from .solver import BatchedIpm, IpmOptions, IpmResult, Solver

__all__ = [
    "CfxError", "Handle", "load_library", "DingModelFrequency", "DingModelFrequencyWithFatigue",
    "DingModelPulseIntensityFrequency", "DingModelPulseIntensityFrequencyWithFatigue",
    "DingModelPulseWidthFrequency", "DingModelPulseWidthFrequencyWithFatigue", "FesModel", "ModelMaker",
    "FourierSeries", "IvpFes", "FesOcp", "Axis", "Constraint", "ConstraintFcn", "ConstraintList", "Node", "Objective", "ObjectiveFcn", "ObjectiveList", "OcpFes",
    "ControlType", "OdeSolver", "FesMskModel", "FesMskOcp", "OcpFesMsk", "FesNmpc", "NmpcFesMsk", "NmpcResult", "BatchedIpm", "IpmOptions", "IpmResult", "Solver",
]
