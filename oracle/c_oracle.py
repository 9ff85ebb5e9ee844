"""ctypes wrapper of the plain-C oracle port (oracle/c/fes_oracle.c).

TEST INFRASTRUCTURE ONLY — the CPU baseline leg of bench.py and a cross-check in tests/.
"""

from __future__ import annotations

import ctypes as C
import pathlib
import subprocess

import numpy as np

from . import fes_oracle as O

HERE = pathlib.Path(__file__).parent
LIB = HERE / "c" / "libfes_oracle.so"
CONST_ORDER = ("tauc", "r0_km_relationship", "a_rest", "tau1_rest", "tau2", "km_rest", "a_scale", "pd0", "pdt",
               "ar", "bs", "Is", "cr", "alpha_a", "alpha_tau1", "alpha_km", "tau_fat", "fl", "fv", "fp")
SCHEME = {"RK1": 1, "RK2": 2, "RK4": 4}
_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            subprocess.run(["make", "-C", str(HERE)], check=True, capture_output=True)
        lib = C.CDLL(str(LIB))
        lib.oracle_shooting.restype = C.c_int
        lib.oracle_shooting.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_void_p,
                                        C.c_void_p, C.c_int, C.c_void_p, C.c_double, C.c_int64, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        _lib = lib
    return _lib


def shooting(pb: O.Problem, v, want_g=True, want_jac=True, threads=1):
    """Continuity (+ sliding) residuals and Jacobian values for AoS decision vectors v (B, nv)."""
    lib = load()
    v = np.ascontiguousarray(v, dtype=np.float64)
    B = v.shape[0]
    consts = np.array([pb.c.get(k, 1.0 if k in ("fl", "fv") else 0.0) for k in CONST_ORDER], dtype=np.float64)
    rows = np.ascontiguousarray(pb.rows, dtype=np.float64)
    last = np.ascontiguousarray(pb.last_stim_idx if pb.n_params else [0], dtype=np.int32)
    nnz = O.jac_structure(pb)[0].size
    pattern = O.structural_pattern(pb)
    nz = pb.nx + pb.nu
    jpos = np.full((pb.nx, nz), -1, dtype=np.int32)
    jneg = np.empty(pb.nx, dtype=np.int32)
    off = 0
    for r in range(pb.nx):
        for c in sorted(pattern[r]):
            jpos[r, c] = off
            off += 1
        jneg[r] = off
        off += 1
    g = np.empty((B, pb.ng)) if want_g else None
    jac = np.empty((B, nnz)) if want_jac else None
    model = O.MODEL_NAMES.index(pb.name)
    rc = lib.oracle_shooting(model, SCHEME[pb.scheme], pb.n_steps, pb.n_shooting, pb.truncation, pb.final_time,
                             rows.ctypes.data, consts.ctypes.data, pb.n_params, last.ctypes.data,
                             pb.intensity_floor, B, v.ctypes.data, None if g is None else g.ctypes.data,
                             None if jac is None else jac.ctypes.data, jpos.ctypes.data, jneg.ctypes.data, off,
                             threads)
    if rc != 0:
        raise RuntimeError("oracle_shooting: unsupported size")
    return g, jac
