import json
import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — parity tests through libcfx")


@pytest.fixture(scope="session")
def ivp_goldens():
    return json.loads((GOLDEN / "ivp_goldens.json").read_text())["cases"]


@pytest.fixture(scope="session")
def ref_formulas():
    return json.loads((GOLDEN / "ref_formulas.json").read_text())


def golden_stims(mode, base):
    """Stim list of a test_ivp.py pulse-mode case.  The triplet case runs on the model object the doublet
    case already mutated (ivp_fes.py:240,251), so its base list is the doublet list."""
    s = list(base)
    if mode == "single":
        return s
    s = sorted(s + [round(t + 0.005, 3) for t in s])
    if mode == "doublet":
        return s
    return sorted(s + [round(t + 0.005, 3) for t in s] + [round(t + 0.01, 3) for t in s])


@pytest.fixture(scope="session")
def gpu_available():
    try:
        from cocofest_amd import _cfx

        return _cfx.load_library().cfx_device_count() > 0
    except Exception:
        return False


def rng(seed=0):
    return np.random.default_rng(seed)
