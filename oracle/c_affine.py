"""ctypes wrapper of oracle/c/fes_affine.c: the CPU baseline in the GPU kernel's own formulation.

TEST INFRASTRUCTURE ONLY — bench.py's same-formulation `cpu_baseline` leg, checked against the oracle in
tests/test_oracle.py.  Two-state Ding families (Ding2003, Ding2007) at RK1 x m, 64-instance tiles.
"""

from __future__ import annotations

import ctypes as C
import pathlib
import subprocess

import numpy as np

from . import fes_oracle as O

HERE = pathlib.Path(__file__).parent
LIB = HERE / "c" / "libfes_affine.so"
_lib = None


class Params(C.Structure):
    _fields_ = [("pw", C.c_int32), ("N", C.c_int32), ("m", C.c_int32), ("nz", C.c_int32), ("km", C.c_double),
                ("tau12", C.c_double), ("tau1km", C.c_double), ("hm", C.c_double), ("hmkm", C.c_double),
                ("hmkmt2", C.c_double), ("a_force", C.c_double), ("pd0", C.c_double), ("pdt", C.c_double)]


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            subprocess.run(["make", "-C", str(HERE)], check=True, capture_output=True)
        lib = C.CDLL(str(LIB))
        lib.affine_shooting.restype = C.c_int
        lib.affine_shooting.argtypes = [C.POINTER(Params), C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int]
        _lib = lib
    return _lib


def tables(pb: O.Problem):
    """cna [m+1] and cnb [N][m+1] of the explicit-Euler calcium recursion cn_{j+1} = cn_j + h (cs(t_j) - cn_j) / tauc,
    run on (slope, offset) pairs from (1, 0); cs from the reference's calcium sum at every sub-step time."""
    if pb.scheme != "RK1" or pb.nx != 2:
        raise ValueError("c_affine: two-state Ding models at RK1 only")
    N, m = pb.n_shooting, pb.n_steps
    dt = pb.final_time / N
    h = dt / m
    al = 1.0 / pb.c["tauc"]
    cna = np.empty(m + 1)
    cnb = np.empty((N, m + 1))
    for k in range(N):
        a, b = 1.0, 0.0
        for j in range(m):
            cna[j], cnb[k, j] = a, b
            cs = float(O.cn_sum(pb.c, k * dt + j * h, np.asarray(pb.rows[k], dtype=np.float64)))
            a, b = a + h * (-al * a), b + h * (al * (cs - b))
        cna[m], cnb[k, m] = a, b
    return cna, cnb


def params(pb: O.Problem) -> Params:
    c = pb.c
    pw = O.control_kind(pb.name) == "pulse_width"
    h = pb.final_time / pb.n_shooting / pb.n_steps
    mult = c.get("fl", 1.0) * c.get("fv", 1.0) + c.get("fp", 0.0)
    P = Params()
    P.pw, P.N, P.m, P.nz = int(pw), pb.n_shooting, pb.n_steps, pb.nx + pb.nu
    P.km, P.tau12, P.tau1km = c["km_rest"], c["tau1_rest"] + c["tau2"], c["tau1_rest"] * c["km_rest"]
    P.hm = h * mult
    P.hmkm = P.hm * c["km_rest"]
    P.hmkmt2 = P.hmkm * c["tau2"]
    P.a_force = c["a_scale"] if pw else c["a_rest"]
    P.pd0, P.pdt = c.get("pd0", 0.0), c.get("pdt", 1.0)
    return P


def structure(pb: O.Problem):
    pattern = O.structural_pattern(pb)
    nz = pb.nx + pb.nu
    jpos = np.full((pb.nx, nz), -1, dtype=np.int32)
    jneg = np.empty(pb.nx, dtype=np.int32)
    off = 0
    for r in range(pb.nx):
        for col in sorted(pattern[r]):
            jpos[r, col] = off
            off += 1
        jneg[r] = off
        off += 1
    return jpos, jneg, off


class Evaluator:
    """Tables and structure built once; __call__ evaluates a tiled batch (B / 64, nv, 64) -> (g, jac) tiles."""

    def __init__(self, pb: O.Problem):
        self.lib = load()
        self.P = params(pb)
        self.cna, self.cnb = tables(pb)
        self.jpos, self.jneg, self.nnzk = structure(pb)
        self.ng, self.nnz = 2 * pb.n_shooting, self.nnzk * pb.n_shooting

    def __call__(self, vt, threads=1, g=None, jac=None):
        vt = np.ascontiguousarray(vt, dtype=np.float64)
        nt = vt.shape[0]
        g = np.empty((nt, self.ng, 64)) if g is None else g
        jac = np.empty((nt, self.nnz, 64)) if jac is None else jac
        rc = self.lib.affine_shooting(C.byref(self.P), self.cna.ctypes.data, self.cnb.ctypes.data, nt * 64,
                                      vt.ctypes.data, g.ctypes.data, jac.ctypes.data, self.jpos.ctypes.data,
                                      self.jneg.ctypes.data, self.nnzk, threads)
        if rc != 0:
            raise RuntimeError("affine_shooting: unsupported problem")
        return g, jac
