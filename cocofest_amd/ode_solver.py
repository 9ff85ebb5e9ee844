"""Transcription choices accepted by OcpFes / IvpFes (the bioptim ``OdeSolver`` / ``ControlType`` names the
reference passes through, cocofest/optimization/fes_ocp.py:120-121, integration/ivp_fes.py:134)."""

from __future__ import annotations

from enum import Enum

from . import _cfx


class _RK:
    scheme = None
    order = None

    def __init__(self, n_integration_steps: int = 5):
        if not isinstance(n_integration_steps, int) or n_integration_steps < 1:
            raise ValueError("n_integration_steps must be a positive int")
        self.n_integration_steps = n_integration_steps

    def __repr__(self):
        return f"{type(self).__name__}(n_integration_steps={self.n_integration_steps})"


class OdeSolver:
    """Explicit Runge-Kutta multiple shooting (RK1 = Euler, RK2 = midpoint, RK4 = classic), m sub-steps per
    shooting interval, piecewise-constant controls (bioptim convention, pinned by the IVP goldens)."""

    class RK1(_RK):
        scheme = _cfx.RK1

    class RK2(_RK):
        scheme = _cfx.RK2

    class RK4(_RK):
        scheme = _cfx.RK4

    class COLLOCATION:
        """Direct collocation (accepted by the reference's sanity check, fes_ocp.py:334-338; bioptim's
        defaults: degree 4, Legendre points): one Lagrange polynomial per shooting interval through the node
        state and ``polynomial_degree`` collocation points (Legendre or Radau IIA), controls held constant."""

        def __init__(self, polynomial_degree: int = 4, method: str = "legendre"):
            if not isinstance(polynomial_degree, int) or not 1 <= polynomial_degree <= 9:
                raise ValueError("polynomial_degree must be an int in [1, 9]")
            if method not in ("legendre", "radau"):
                raise ValueError("method must be 'legendre' or 'radau'")
            self.polynomial_degree = polynomial_degree
            self.method = method
            self.n_integration_steps = polynomial_degree
            self.scheme = _cfx.COLLOCATION_LEGENDRE if method == "legendre" else _cfx.COLLOCATION_RADAU

        def __repr__(self):
            return f"COLLOCATION(polynomial_degree={self.polynomial_degree}, method={self.method!r})"


class ControlType(Enum):
    CONSTANT = 1
