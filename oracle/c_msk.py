"""ctypes wrapper of the plain-C port of the musculoskeletal oracle (oracle/c/fes_msk.c).

TEST INFRASTRUCTURE ONLY — the CPU baseline leg of bench.py's musculoskeletal section and a cross-check of
oracle/fes_msk.py in tests/.
"""

from __future__ import annotations

import ctypes as C
import pathlib
import subprocess

import numpy as np

from . import fes_msk as M

HERE = pathlib.Path(__file__).parent
LIB = HERE / "c" / "libfes_msk.so"
SEG, DOF, MUS, PTS = 32, 8, 8, 16
CONST_ORDER = ("tauc", "r0_km_relationship", "a_rest", "tau1_rest", "tau2", "km_rest", "a_scale", "pd0", "pdt",
               "alpha_a", "alpha_tau1", "alpha_km", "tau_fat")
MODEL = {"ding2003": 0, "ding2003_with_fatigue": 1, "ding2007": 2, "ding2007_with_fatigue": 3}
SCHEME = {"RK1": 1, "RK2": 2, "RK4": 4}
_i32, _f64 = C.c_int32, C.c_double


class Desc(C.Structure):
    """Mirror of ms_desc (fes_msk.c)."""

    _fields_ = [("nseg", _i32), ("ndof", _i32), ("parent", _i32 * SEG), ("rt", (_f64 * 16) * SEG),
                ("nrot", _i32 * SEG), ("rot_axis", (_i32 * 3) * SEG), ("mass", _f64 * SEG),
                ("com", (_f64 * 3) * SEG), ("inertia", (_f64 * 9) * SEG), ("grav", _f64 * 3), ("nmus", _i32),
                ("model", _i32 * MUS), ("cst", (_f64 * 13) * MUS), ("npts", _i32 * MUS),
                ("pt_seg", (_i32 * PTS) * MUS), ("pt_pos", ((_f64 * 3) * PTS) * MUS), ("lopt", _f64 * MUS),
                ("slack", _f64 * MUS), ("penn", _f64 * MUS), ("fv_on", _i32), ("fp_on", _i32),
                ("residual", _i32), ("N", _i32), ("m", _i32), ("scheme", _i32), ("T", _i32), ("tf", _f64),
                ("legacy", _i32)]


_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            subprocess.run(["make", "-C", str(HERE)], check=True, capture_output=True)
        lib = C.CDLL(str(LIB))
        lib.ms_shooting.restype = C.c_int
        lib.ms_shooting.argtypes = [C.POINTER(Desc), C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_int]
        _lib = lib
    return _lib


def describe(pb: M.MskProblem) -> Desc:
    """Flatten an oracle MskProblem (full segment tree, muscles by name) into the C descriptor."""
    d = Desc()
    segs = pb.bm["segments"]
    if len(segs) > SEG or pb.nq > DOF or len(pb.muscles) > MUS:
        raise ValueError("problem exceeds the C port's fixed sizes")
    index = {s["name"]: i for i, s in enumerate(segs)}
    d.nseg, d.ndof = len(segs), pb.nq
    for i, s in enumerate(segs):
        d.parent[i] = index[s["parent"]] if s["parent"] else -1
        d.rt[i][:] = list(np.asarray(s["RT"], dtype=float).ravel())
        d.nrot[i] = len(s["rotations"])
        for r, a in enumerate(s["rotations"]):
            d.rot_axis[i][r] = "xyz".index(a)
        d.mass[i] = s["mass"]
        d.com[i][:] = list(map(float, s["com"]))
        d.inertia[i][:] = list(np.asarray(s["inertia"], dtype=float).ravel())
    d.grav[:] = list(map(float, pb.bm["gravity"]))
    d.nmus = len(pb.muscles)
    for j, mus in enumerate(pb.muscles):
        bio = M._bio_muscle(pb, mus.name)
        d.model[j] = MODEL[mus.model]
        d.cst[j][:] = [float(mus.c.get(k, 0.0)) for k in CONST_ORDER]
        path = M.muscle_path(bio)
        if len(path) > PTS:
            raise ValueError("too many path points")
        d.npts[j] = len(path)
        for p, (seg, pos) in enumerate(path):
            d.pt_seg[j][p] = index[seg]
            d.pt_pos[j][p][:] = list(map(float, pos))
        d.lopt[j], d.slack[j], d.penn[j] = bio["optimallength"], bio["tendonslacklength"], bio["pennationangle"]
    d.fv_on, d.fp_on, d.residual = int(pb.fv_on), int(pb.fp_on), int(pb.residual)
    d.N, d.m, d.scheme, d.T = pb.n_shooting, pb.m, SCHEME[pb.scheme], pb.rows.shape[1]
    d.tf = pb.final_time
    d.legacy = int(pb.legacy)
    return d


def shooting(pb: M.MskProblem, v, want_g=True, want_jac=True, threads=1):
    """Continuity rows (B, ng) and dense interval Jacobians (B, N, nx, nz) for decision vectors v (B, nv)."""
    lib = load()
    v = np.ascontiguousarray(v, dtype=np.float64).reshape(-1, pb.nv)
    B = v.shape[0]
    rows = np.ascontiguousarray(pb.rows, dtype=np.float64)
    d = describe(pb)
    g = np.empty((B, pb.ng)) if want_g else None
    jac = np.empty((B, pb.n_shooting, pb.nx, pb.nz)) if want_jac else None
    rc = lib.ms_shooting(C.byref(d), rows.ctypes.data, B, v.ctypes.data, None if g is None else g.ctypes.data,
                         None if jac is None else jac.ctypes.data, threads)
    if rc != 0:
        raise RuntimeError("ms_shooting: unsupported size")
    return g, jac


__all__ = ["describe", "load", "shooting"]
