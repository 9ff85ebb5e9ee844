"""Real Fourier series fit used for the force-tracking target (reference: cocofest/fourier_approx.py:8-38).

Host-side data preparation (runs once per problem build), not part of the evaluated hot path.
"""

from __future__ import annotations

import numpy as np
from scipy.integrate import trapezoid


class FourierSeries:
    def __init__(self):
        self.p = 1  # period

    def compute_real_fourier_coeffs(self, x, y, n):
        """(a_i, b_i) for i = 0..n by trapezoidal quadrature over the samples (fourier_approx.py:12-18)."""
        w = 2.0 * np.pi / self.p
        out = np.empty((n + 1, 2))
        for i in range(n + 1):
            out[i, 0] = (2.0 / self.p) * trapezoid(y * np.cos(w * i * x), x)
            out[i, 1] = (2.0 / self.p) * trapezoid(y * np.sin(w * i * x), x)
        return out

    def fit_func_by_fourier_series_with_real_coeffs(self, x, ab, mode="numpy"):
        """a_0/2 + sum_n a_n cos(2 pi n x / p) + b_n sin(2 pi n x / p)  (fourier_approx.py:21-38)."""
        if mode != "numpy":
            raise ValueError("only the numeric evaluation is provided")
        result = 0.0
        for n in range(len(ab)):
            if n == 0:
                result = result + ab[0, 0] / 2.0
            else:
                result = result + ab[n, 0] * np.cos(2.0 * np.pi * n * x / self.p) + ab[n, 1] * np.sin(
                    2.0 * np.pi * n * x / self.p)
        return result
