"""ctypes binding of libcfx (include/cfx.h).

The shared library is built in-tree (``cocofest_amd/libcfx.so``, see ``cocofest_amd/csrc/Makefile``).
There is no CPU fallback: if the library is missing, or no HIP device is visible when a handle is
created, a ``CfxError`` is raised.
"""

from __future__ import annotations

import ctypes as C
import os
import pathlib

import numpy as np

LIB_PATH = pathlib.Path(__file__).with_name("libcfx.so")

ABI_VERSION = 11
OK, EINVAL, EHIP, ENOMEM, EUNSUPPORTED, ENODEV, ECALLBACK = 0, -1, -2, -3, -4, -5, -6
MODEL_IDS = {
    "ding2003": 0,
    "ding2003_with_fatigue": 1,
    "ding2007": 2,
    "ding2007_with_fatigue": 3,
    "hmed2018": 4,
    "hmed2018_with_fatigue": 5,
}
RK1, RK2, RK4 = 1, 2, 4
COLLOCATION_LEGENDRE, COLLOCATION_RADAU = 16, 17
LAYOUT_AOS, LAYOUT_SOA, LAYOUT_TILED64 = 0, 1, 2
DEVICE = 1
KEEP_CONSTANT_JAC = 2
OBJ_LAGRANGE, OBJ_MAYER, OBJ_MAYER_INV = 0, 1, 2
MSK_FORCE_LENGTH, MSK_FORCE_VELOCITY, MSK_PASSIVE_FORCE, MSK_RESIDUAL_TORQUE = 1, 2, 4, 8
MSK_PULSE_WIDTH_PER_PULSE, MSK_LEGACY_CALCIUM = 16, 32
VAR_STATE, VAR_CONTROL = 0, 1


class CfxError(RuntimeError):
    """Error raised by libcfx (carries the integer code)."""

    def __init__(self, code, msg):
        super().__init__(f"libcfx error {code}: {msg}")
        self.code = code


class Constants(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "tauc", "r0_km_relationship", "a_rest", "tau1_rest", "tau2", "km_rest",
        "a_scale", "pd0", "pdt", "ar", "bs", "Is", "cr",
        "alpha_a", "alpha_tau1", "alpha_km", "tau_fat", "fl", "fv", "fp")]


class Objective(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("var_kind", C.c_int32), ("var_index", C.c_int32),
        ("node_first", C.c_int32), ("node_last", C.c_int32),
        ("weight", C.c_double), ("target", C.POINTER(C.c_double)), ("target_value", C.c_double),
    ]


class Problem(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("model", C.c_int32), ("scheme", C.c_int32), ("n_steps", C.c_int32),
        ("n_shooting", C.c_int32), ("truncation", C.c_int32), ("n_params", C.c_int32), ("layout", C.c_int32),
        ("batch", C.c_int64), ("final_time", C.c_double),
        ("stim_rows", C.POINTER(C.c_double)), ("last_stim_idx", C.POINTER(C.c_int32)),
        ("intensity_floor", C.c_double), ("constants", Constants),
        ("n_objectives", C.c_int32), ("objectives", C.POINTER(Objective)), ("device", C.c_int32),
    ]


class MskMuscle(C.Structure):
    _fields_ = [("model", C.c_int32), ("constants", Constants), ("n_points", C.c_int32),
                ("point_frame", C.POINTER(C.c_int32)), ("point_pos", C.POINTER(C.c_double)),
                ("optimal_length", C.c_double), ("tendon_slack_length", C.c_double), ("pennation_angle", C.c_double)]


class MskMarkerPair(C.Structure):
    _fields_ = [("node", C.c_int32), ("axes", C.c_int32), ("frame", C.c_int32 * 2), ("pos", (C.c_double * 3) * 2)]


class MskProblem(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("scheme", C.c_int32), ("n_steps", C.c_int32), ("n_shooting", C.c_int32),
        ("truncation", C.c_int32), ("layout", C.c_int32), ("batch", C.c_int64), ("final_time", C.c_double),
        ("stim_rows", C.POINTER(C.c_double)), ("n_dof", C.c_int32), ("dof_axis", C.POINTER(C.c_int32)),
        ("dof_frame", C.POINTER(C.c_double)), ("gravity", C.c_double * 3), ("body_mass", C.POINTER(C.c_double)),
        ("body_com", C.POINTER(C.c_double)), ("body_inertia", C.POINTER(C.c_double)), ("n_muscles", C.c_int32),
        ("muscles", C.POINTER(MskMuscle)), ("flags", C.c_uint32), ("n_objectives", C.c_int32),
        ("objectives", C.POINTER(Objective)), ("device", C.c_int32), ("n_params", C.c_int32),
        ("last_stim_idx", C.POINTER(C.c_int32)), ("param_offset", C.POINTER(C.c_int32)),
        ("n_marker_pairs", C.c_int32), ("marker_pairs", C.POINTER(MskMarkerPair)),
    ]


class Sizes(C.Structure):
    _fields_ = [("nv", C.c_int64), ("ng", C.c_int64), ("nnz_jac", C.c_int64), ("nnz_hess", C.c_int64),
                ("nx", C.c_int32), ("nu", C.c_int32)]


class LaunchShape(C.Structure):
    _fields_ = [("intervals_per_thread", C.c_int32), ("intervals_fast", C.c_int32), ("instances_per_lane", C.c_int32),
                ("instances_per_lane_g", C.c_int32), ("msk_intervals_per_block", C.c_int32)]


class IpmOptions(C.Structure):
    _fields_ = [("tol", C.c_double), ("max_iter", C.c_int32), ("acceptable_tol", C.c_double),
                ("acceptable_iter", C.c_int32), ("mu_init", C.c_double), ("bound_relax_factor", C.c_double),
                ("bound_push", C.c_double), ("tau_min", C.c_double), ("kappa_eps", C.c_double),
                ("kappa_mu", C.c_double), ("theta_mu", C.c_double), ("s_max", C.c_double), ("armijo", C.c_double),
                ("max_backtrack", C.c_int32), ("delta_c", C.c_double), ("curv_min", C.c_double),
                ("max_soc", C.c_int32), ("kappa_soc", C.c_double), ("watchdog_shortened_iter_trigger", C.c_int32),
                ("watchdog_trial_iter_max", C.c_int32), ("hessian_approximation", C.c_int32),
                ("limited_memory_max_history", C.c_int32), ("restoration", C.c_int32),
                ("max_resto_iter", C.c_int32), ("resto_penalty", C.c_double),
                ("required_infeasibility_reduction", C.c_double), ("filter_reset_trigger", C.c_int32),
                ("max_filter_resets", C.c_int32), ("max_wall_time", C.c_double), ("print_frequency_time", C.c_double),
                ("soft_resto_pderror_reduction_factor", C.c_double), ("max_soft_resto_iters", C.c_int32),
                ("resto_failure_restart", C.c_int32), ("constr_viol_tol", C.c_double),
                ("dual_inf_tol", C.c_double), ("compl_inf_tol", C.c_double),
                ("acceptable_constr_viol_tol", C.c_double), ("acceptable_dual_inf_tol", C.c_double),
                ("acceptable_compl_inf_tol", C.c_double), ("warm_start_bound_push", C.c_double),
                ("warm_start_bound_frac", C.c_double), ("warm_start_mult_bound_push", C.c_double),
                ("warm_start_init_point", C.c_int32), ("honor_original_bounds", C.c_int32),
                ("range_scaling", C.c_int32), ("bound_mult_init_method", C.c_int32),
                ("bound_mult_init_val", C.c_double), ("inertia_test", C.c_int32),
                # ABI 11: Ipopt's barrier-parameter strategies, NLP scaling method, bound_frac
                ("mu_strategy", C.c_int32), ("adaptive_mu_globalization", C.c_int32), ("mu_max_fact", C.c_double),
                ("mu_max", C.c_double), ("mu_min", C.c_double), ("adaptive_mu_monotone_init_factor", C.c_double),
                ("sigma_max", C.c_double), ("sigma_min", C.c_double),
                ("quality_function_section_sigma_tol", C.c_double), ("quality_function_section_qf_tol", C.c_double),
                ("quality_function_max_section_steps", C.c_int32), ("mu_change_resets_filter", C.c_int32),
                ("filter_margin_fact", C.c_double), ("filter_max_margin", C.c_double),
                ("monotone_mu_floor", C.c_int32), ("nlp_scaling_method", C.c_int32),
                ("nlp_scaling_max_gradient", C.c_double), ("nlp_scaling_min_value", C.c_double),
                ("bound_frac", C.c_double)]


# cfx_ipm_get_status values (Ipopt's ApplicationReturnStatus)
IPM_STATUS = {0: "Solve_Succeeded", 1: "Solved_To_Acceptable_Level", 2: "Infeasible_Problem_Detected",
              -1: "Maximum_Iterations_Exceeded", -2: "Restoration_Failed", -5: "Maximum_WallTime_Exceeded"}


class IpmStats(C.Structure):
    _fields_ = [("eval_all", C.c_int64), ("eval_g_f", C.c_int64), ("eval_h", C.c_int64), ("kkt_factor", C.c_int64),
                ("iterations", C.c_int64), ("host_syncs", C.c_int64), ("wall_s", C.c_double),
                ("kkt_n", C.c_int64), ("kkt_kl", C.c_int64), ("kkt_ku", C.c_int64), ("kkt_band_n", C.c_int64),
                ("kkt_border", C.c_int64), ("kkt_blocks", C.c_int64), ("resto_phases", C.c_int64),
                ("resto_iterations", C.c_int64), ("soft_steps", C.c_int64), ("kkt_chain_nodes", C.c_int64),
                ("kkt_chain_sp", C.c_int64), ("mu_mode_switches", C.c_int64)]


# cfx_evaluator / cfx_nlp_desc (cfx_ipm_create_ext): caller-supplied callbacks of an NLP the solver runs on
EVAL_ALL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p)
EVAL_H_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p)


class Evaluator(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("eval_all", EVAL_ALL_FN), ("eval_h", EVAL_H_FN)]


class NlpDesc(C.Structure):
    _fields_ = [("batch", C.c_int64), ("nv", C.c_int64), ("ng", C.c_int64), ("nnz_jac", C.c_int64),
                ("nnz_hess", C.c_int64), ("jac_row", C.POINTER(C.c_int32)), ("jac_col", C.POINTER(C.c_int32)),
                ("hess_row", C.POINTER(C.c_int32)), ("hess_col", C.POINTER(C.c_int32)), ("device", C.c_int32),
                ("hip_stream", C.c_void_p)]


# exported symbols and their signatures (must match include/cfx.h)
_P = C.c_void_p
_D = C.POINTER(C.c_double)
SIGNATURES = {
    "cfx_create": (C.c_int, [C.POINTER(Problem), C.POINTER(_P)]),
    "cfx_destroy": (None, [_P]),
    "cfx_get_sizes": (C.c_int, [_P, C.POINTER(Sizes)]),
    "cfx_get_launch_shape": (C.c_int, [_P, C.POINTER(LaunchShape)]),
    "cfx_set_stream": (C.c_int, [_P, _P]),
    "cfx_synchronize": (C.c_int, [_P]),
    "cfx_last_error": (C.c_char_p, [_P]),
    "cfx_abi_version": (C.c_int, []),
    "cfx_device_count": (C.c_int, []),
    "cfx_jac_structure": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "cfx_jac_constant_mask": (C.c_int, [_P, C.POINTER(C.c_uint8)]),
    "cfx_hess_structure": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "cfx_eval_g": (C.c_int, [_P, _P, _P, C.c_uint32]),
    "cfx_eval_jac_g": (C.c_int, [_P, _P, _P, C.c_uint32]),
    "cfx_eval_f": (C.c_int, [_P, _P, _P, C.c_uint32]),
    "cfx_eval_grad_f": (C.c_int, [_P, _P, _P, C.c_uint32]),
    "cfx_eval_h": (C.c_int, [_P, _P, _P, _P, _P, C.c_uint32]),
    "cfx_eval_all": (C.c_int, [_P, _P, _P, _P, _P, _P, C.c_uint32]),
    "cfx_eval_all_h": (C.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, C.c_uint32]),
    "cfx_integrate": (C.c_int, [_P, _P, _P, _P, C.c_uint32]),
    "cfx_msk_create": (C.c_int, [C.POINTER(MskProblem), C.POINTER(_P)]),
    "cfx_band_lu": (C.c_int, [C.c_int64, C.c_int32, C.c_int32, C.c_int64, _P, _P, _P, C.c_int32, _P, _P]),
    "cfx_band_lu_solve": (C.c_int, [C.c_int64, C.c_int32, C.c_int32, C.c_int64, _P, _P, C.c_int32, _P, _P]),
    "cfx_ipm_default_options": (None, [C.POINTER(IpmOptions)]),
    "cfx_ipm_create": (C.c_int, [_P, _P, _P, C.c_int32, C.POINTER(IpmOptions), C.POINTER(_P)]),
    "cfx_ipm_solve": (C.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, C.c_uint32]),
    "cfx_ipm_get_stats": (C.c_int, [_P, C.POINTER(IpmStats)]),
    "cfx_ipm_get_status": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "cfx_ipm_set_warm_start": (C.c_int, [_P, _P, _P, _P, C.c_uint32]),
    "cfx_ipm_get_bound_multipliers": (C.c_int, [_P, _P, _P, C.c_uint32]),
    "cfx_btri_factor": (C.c_int, [C.c_int64, C.c_int32, C.c_int32, _P, _P, _P, _P, _P, _P]),
    "cfx_btri_solve": (C.c_int, [C.c_int64, C.c_int32, C.c_int32, _P, _P, _P, _P, C.c_int32, _P, _P, _P]),
    "cfx_btri_inertia": (C.c_int, [C.c_int64, C.c_int32, C.c_int32, _P, _P, _P]),
    "cfx_ipm_create_ext": (C.c_int, [C.POINTER(NlpDesc), C.POINTER(Evaluator), _P, _P, C.c_int32,
                                     C.POINTER(IpmOptions), C.POINTER(_P)]),
    "cfx_gather_sum": (C.c_int, [C.c_int64, C.c_int64, _P, _P, _P, C.c_int64, _P, _P]),
    "cfx_ipm_n_fixed": (C.c_int, [_P]),
    "cfx_ipm_last_error": (C.c_char_p, [_P]),
    "cfx_ipm_destroy": (None, [_P]),
}

_lib = None


def load_library(path: str | os.PathLike | None = None):
    """Load libcfx.so (once) and declare every exported signature; raise if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = pathlib.Path(path) if path else pathlib.Path(os.environ.get("CFX_LIB", LIB_PATH))
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's).  Load it
    # first so libcfx binds to the already-loaded runtime instead of pulling in a second one.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not p.exists():
        raise CfxError(ENODEV, f"{p} not found: build it with `make -C cocofest_amd/csrc` (no CPU fallback)")
    lib = C.CDLL(str(p))
    variant = bool(os.environ.get("CFX_LIB")) and not path  # an A/B build may predate later entry points
    for name, (res, args) in SIGNATURES.items():
        if variant and not hasattr(lib, name):
            continue  # calling it raises AttributeError
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.cfx_abi_version() != ABI_VERSION:
        raise CfxError(EINVAL, "libcfx ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def _is_tensor(a):
    """True for a torch.Tensor (torch imported lazily: host-only callers never load it)."""
    if type(a).__module__.split(".")[0] != "torch":
        return False
    import torch

    return isinstance(a, torch.Tensor)


def _ptr(a):
    """Address of a numpy array / torch tensor (None -> NULL)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()


def _band_check(ab, ipiv, rhs, kl, ku):
    import torch

    if not (ab.is_cuda and ab.dtype == torch.float64 and ab.is_contiguous() and ab.dim() == 3):
        raise CfxError(EINVAL, "band: ab must be a contiguous (B, n, 2kl+ku+1) float64 device tensor")
    B, n, ldab = ab.shape
    if ldab != 2 * kl + ku + 1:
        raise CfxError(EINVAL, f"band: ab.shape[2] = {ldab} != 2*kl+ku+1 = {2 * kl + ku + 1}")
    if not (ipiv.is_cuda and ipiv.dtype == torch.int32 and ipiv.is_contiguous() and tuple(ipiv.shape) == (B, n)):
        raise CfxError(EINVAL, "band: ipiv must be a contiguous (B, n) int32 device tensor")
    if rhs is not None and not (rhs.is_cuda and rhs.dtype == torch.float64 and rhs.is_contiguous()
                                and rhs.shape[0] == B and rhs.shape[-1] == n and rhs.dim() in (2, 3)):
        raise CfxError(EINVAL, "band: rhs must be a contiguous (B, n) or (B, nrhs, n) float64 device tensor")
    nrhs = 0 if rhs is None else (1 if rhs.dim() == 2 else rhs.shape[1])
    return B, n, nrhs


def band_lu(ab, ipiv, info, kl: int, ku: int, rhs=None):
    """Factor B banded systems in place (cfx_band_lu) on torch's current stream and, with ``rhs``, solve in
    place.  ab: (B, n, 2kl+ku+1) float64 LAPACK band storage per instance, ipiv: (B, n) int32, info: (B,) int32."""
    import torch

    lib = load_library()
    B, n, nrhs = _band_check(ab, ipiv, rhs, kl, ku)
    if not (info.is_cuda and info.dtype == torch.int32 and info.numel() == B):
        raise CfxError(EINVAL, "band: info must be a (B,) int32 device tensor")
    rc = lib.cfx_band_lu(n, kl, ku, B, _ptr(ab), _ptr(ipiv), _ptr(info), nrhs, _ptr(rhs),
                         torch.cuda.current_stream().cuda_stream)
    if rc != OK:
        raise CfxError(rc, lib.cfx_last_error(None).decode())


def band_lu_solve(ab, ipiv, kl: int, ku: int, rhs):
    """Solve in place with factors from band_lu (cfx_band_lu_solve)."""
    import torch

    lib = load_library()
    B, n, nrhs = _band_check(ab, ipiv, rhs, kl, ku)
    rc = lib.cfx_band_lu_solve(n, kl, ku, B, _ptr(ab), _ptr(ipiv), nrhs, _ptr(rhs),
                               torch.cuda.current_stream().cuda_stream)
    if rc != OK:
        raise CfxError(rc, lib.cfx_last_error(None).decode())


def _objective_array(objectives, keep, n_shooting):
    """ctypes array of objective terms; a term's target array must hold one value per node (n_shooting + 1):
    libcfx reads exactly that many."""
    objs = (Objective * max(1, len(objectives)))()
    for i, o in enumerate(objectives):
        objs[i].kind = o["kind"]
        objs[i].var_kind = o["var_kind"]
        objs[i].var_index = o["var_index"]
        objs[i].node_first = o["node_first"]
        objs[i].node_last = o["node_last"]
        objs[i].weight = o["weight"]
        if o.get("target") is not None:
            t = np.ascontiguousarray(o["target"], dtype=np.float64).reshape(-1)
            if t.size != n_shooting + 1:
                raise CfxError(EINVAL, f"objective term {i}: target has {t.size} values, expected n_shooting + 1 = "
                                       f"{n_shooting + 1}")
            keep.append(t)
            objs[i].target = t.ctypes.data_as(_D)
        objs[i].target_value = float(o.get("target_value", 0.0))
    keep.append(objs)
    return objs


class Handle:
    """One libcfx handle: a batch of B instances of one transcribed FES problem on one GPU.

    Host numpy arrays are copied to the GPU and back synchronously; torch CUDA tensors (float64,
    contiguous) are used in place and the call is enqueued on torch's current stream.
    """

    def __init__(self, *, model_id, constants: dict, scheme, n_steps, n_shooting, truncation, final_time,
                 stim_rows, batch, layout=LAYOUT_SOA, n_params=0, last_stim_idx=None, intensity_floor=0.0,
                 objectives=(), device=0):
        self.lib = load_library()
        self._keep = []
        rows = np.ascontiguousarray(stim_rows, dtype=np.float64).reshape(-1)
        self._keep.append(rows)
        pb = Problem()
        pb.abi_version = ABI_VERSION
        pb.model = model_id
        pb.scheme = scheme
        pb.n_steps = n_steps
        pb.n_shooting = n_shooting
        pb.truncation = truncation
        pb.n_params = n_params
        pb.layout = layout
        pb.batch = batch
        pb.final_time = final_time
        pb.stim_rows = rows.ctypes.data_as(_D)
        if last_stim_idx is not None:
            li = np.ascontiguousarray(last_stim_idx, dtype=np.int32)
            self._keep.append(li)
            pb.last_stim_idx = li.ctypes.data_as(C.POINTER(C.c_int32))
        pb.intensity_floor = intensity_floor
        cst = Constants()
        for name, _ in Constants._fields_:
            setattr(cst, name, float(constants.get(name, 0.0)))
        pb.constants = cst
        objs = _objective_array(objectives, self._keep, n_shooting)
        pb.n_objectives = len(objectives)
        pb.objectives = objs
        pb.device = device
        h = C.c_void_p()
        rc = self.lib.cfx_create(C.byref(pb), C.byref(h))
        self._attach(rc, h, batch, layout, n_shooting, n_steps, device)

    def _attach(self, rc, h, batch, layout, n_shooting, n_steps, device):
        if rc != OK:
            raise CfxError(rc, self.lib.cfx_last_error(None).decode())
        self.h = h
        sz = Sizes()
        self._check(self.lib.cfx_get_sizes(self.h, C.byref(sz)))
        self.nv, self.ng, self.nnz_jac, self.nnz_hess = sz.nv, sz.ng, sz.nnz_jac, sz.nnz_hess
        self.nx, self.nu = sz.nx, sz.nu
        self.batch, self.layout, self.n_shooting, self.n_steps = batch, layout, n_shooting, n_steps
        self.device = device

    def _check(self, rc):
        if rc != OK:
            raise CfxError(rc, self.lib.cfx_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            self.lib.cfx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def launch_shape(self) -> dict:
        """The g + J_g kernels' launch shape fixed at creation (cfx_get_launch_shape)."""
        ls = LaunchShape()
        self._check(self.lib.cfx_get_launch_shape(self.h, C.byref(ls)))
        return {name: int(getattr(ls, name)) for name, _ in LaunchShape._fields_}

    # ---- structure ----
    def jac_structure(self):
        r = np.empty(self.nnz_jac, dtype=np.int32)
        c = np.empty(self.nnz_jac, dtype=np.int32)
        self._check(self.lib.cfx_jac_structure(self.h, r.ctypes.data_as(C.POINTER(C.c_int32)),
                                               c.ctypes.data_as(C.POINTER(C.c_int32))))
        return r, c

    def jac_constant_mask(self):
        """Boolean mask over the J_g values that depend on neither the instance nor the point (cfx_jac_constant_mask):
        the values ``keep_constant_jac=True`` evaluations leave in place."""
        m = np.empty(self.nnz_jac, dtype=np.uint8)
        self._check(self.lib.cfx_jac_constant_mask(self.h, m.ctypes.data_as(C.POINTER(C.c_uint8))))
        return m.astype(bool)

    def hess_structure(self):
        r = np.empty(self.nnz_hess, dtype=np.int32)
        c = np.empty(self.nnz_hess, dtype=np.int32)
        self._check(self.lib.cfx_hess_structure(self.h, r.ctypes.data_as(C.POINTER(C.c_int32)),
                                                c.ctypes.data_as(C.POINTER(C.c_int32))))
        return r, c

    # ---- evaluation ----
    def _buffers(self, *slots):
        """Check every buffer of one call against its slot before libcfx sees it; return (buffers, flags).

        ``slots``: (name, buffer or None, per-instance length, is_output).  libcfx reads / writes exactly
        batch * length doubles per buffer, so a wrong size, dtype or stride would be an out-of-bounds host
        access, and a CPU tensor sent as a device pointer a GPU fault: all of these raise ``CfxError``.
        Host inputs may be any array-like (converted to C-contiguous float64); host outputs must already be
        C-contiguous float64 numpy arrays (results are written in place).  Device buffers must be contiguous
        float64 CUDA tensors on the handle's device."""
        out, kinds = [], []
        for name, a, n, is_out in slots:
            if a is None:
                out.append(None)
                continue
            want = self.batch * n
            if _is_tensor(a):
                if not a.is_cuda:
                    raise CfxError(EINVAL, f"{name}: CPU tensor; pass a numpy array (host) or a CUDA tensor (device)")
                if a.device.index != self.device:
                    raise CfxError(EINVAL, f"{name}: tensor on cuda:{a.device.index}, handle on cuda:{self.device}")
                if str(a.dtype) != "torch.float64" or not a.is_contiguous():
                    raise CfxError(EINVAL, f"{name}: device buffers must be contiguous float64 tensors")
                if a.numel() != want:
                    raise CfxError(EINVAL, f"{name}: {a.numel()} elements, expected batch * {n} = {want}")
                kinds.append(True)
            else:
                if is_out:
                    if not (isinstance(a, np.ndarray) and a.dtype == np.float64 and a.flags.c_contiguous):
                        raise CfxError(EINVAL, f"{name}: host outputs must be C-contiguous float64 numpy arrays")
                else:
                    a = np.ascontiguousarray(a, dtype=np.float64)
                if a.size != want:
                    raise CfxError(EINVAL, f"{name}: {a.size} elements, expected batch * {n} = {want}")
                kinds.append(False)
            out.append(a)
        if kinds and any(kinds) != all(kinds):
            raise CfxError(EINVAL, "mix of host and device buffers in one call")
        return out, (DEVICE if kinds and kinds[0] else 0)

    def set_stream(self, stream_ptr):
        self._check(self.lib.cfx_set_stream(self.h, stream_ptr))

    def _torch_stream(self, flags):
        if flags & DEVICE:
            import torch

            self._check(self.lib.cfx_set_stream(self.h, torch.cuda.current_stream().cuda_stream))

    def _shape(self, n):
        if self.layout == LAYOUT_AOS:
            return (self.batch, n)
        if self.layout == LAYOUT_TILED64:  # (tile, element, instance in tile)
            return (self.batch // 64, n, 64) if n > 1 else (self.batch,)
        return (n, self.batch)

    def eval_all(self, v, g=None, jac=None, f=None, grad=None, keep_constant_jac=False):
        """keep_constant_jac: CFX_KEEP_CONSTANT_JAC — the constant J_g values (jac_constant_mask) are not written;
        ``jac`` (device call) or the handle's staging buffer (host call) must hold them from a full evaluation."""
        (v, g, jac, f, grad), fl = self._buffers(("v", v, self.nv, False), ("g", g, self.ng, True),
                                                  ("jac", jac, self.nnz_jac, True), ("f", f, 1, True),
                                                  ("grad", grad, self.nv, True))
        self._torch_stream(fl)
        fl |= KEEP_CONSTANT_JAC if keep_constant_jac else 0
        self._check(self.lib.cfx_eval_all(self.h, _ptr(v), _ptr(g), _ptr(jac), _ptr(f), _ptr(grad), fl))

    def eval_g(self, v, g=None):
        g = np.empty(self._shape(self.ng)) if g is None else g
        self.eval_all(v, g=g)
        return g

    def eval_jac_g(self, v, jac=None, keep_constant_jac=False):
        jac = np.empty(self._shape(self.nnz_jac)) if jac is None else jac
        self.eval_all(v, jac=jac, keep_constant_jac=keep_constant_jac)
        return jac

    def eval_f(self, v, f=None):
        f = np.empty(self.batch) if f is None else f
        self.eval_all(v, f=f)
        return f

    def eval_grad_f(self, v, grad=None):
        grad = np.empty(self._shape(self.nv)) if grad is None else grad
        self.eval_all(v, grad=grad)
        return grad

    def eval_h(self, v, obj_factor, lam, hess=None):
        hess = np.empty(self._shape(self.nnz_hess)) if hess is None else hess
        (v, obj_factor, lam, hess), fl = self._buffers(("v", v, self.nv, False), ("obj_factor", obj_factor, 1, False),
                                                       ("lam", lam, self.ng, False), ("hess", hess, self.nnz_hess, True))
        self._torch_stream(fl)
        self._check(self.lib.cfx_eval_h(self.h, _ptr(v), _ptr(obj_factor), _ptr(lam), _ptr(hess), fl))
        return hess

    def eval_all_h(self, v, obj_factor, lam, g=None, jac=None, f=None, grad=None, hess=None, keep_constant_jac=False):
        """g, J_g, (f, grad f) and the Lagrangian Hessian at one point (cfx_eval_all_h: one launch on the shooting
        transcriptions).  Returns (g, jac, hess)."""
        if _is_tensor(v):  # device call: the missing outputs on the handle's device
            import torch

            new = lambda n: torch.empty(self._shape(n), dtype=torch.float64, device=v.device)  # noqa: E731
        else:
            new = lambda n: np.empty(self._shape(n))  # noqa: E731
        g = new(self.ng) if g is None else g
        jac = new(self.nnz_jac) if jac is None else jac
        hess = new(self.nnz_hess) if hess is None else hess
        (v, obj_factor, lam, g, jac, f, grad, hess), fl = self._buffers(
            ("v", v, self.nv, False), ("obj_factor", obj_factor, 1, False), ("lam", lam, self.ng, False),
            ("g", g, self.ng, True), ("jac", jac, self.nnz_jac, True), ("f", f, 1, True),
            ("grad", grad, self.nv, True), ("hess", hess, self.nnz_hess, True))
        self._torch_stream(fl)
        fl |= KEEP_CONSTANT_JAC if keep_constant_jac else 0
        self._check(self.lib.cfx_eval_all_h(self.h, _ptr(v), _ptr(obj_factor), _ptr(lam), _ptr(g), _ptr(jac),
                                            _ptr(f), _ptr(grad), _ptr(hess), fl))
        return g, jac, hess

    def integrate(self, x0=None, u=None, traj=None):
        n = (self.n_shooting * self.n_steps + 1) * self.nx
        traj = np.empty(self._shape(n)) if traj is None else traj
        (x0, u, traj), fl = self._buffers(("x0", x0, self.nx, False), ("u", u, self.n_shooting * self.nu, False),
                                          ("traj", traj, n, True))
        self._torch_stream(fl)
        self._check(self.lib.cfx_integrate(self.h, _ptr(x0), _ptr(u), _ptr(traj), fl))
        return traj

    def synchronize(self):
        self._check(self.lib.cfx_synchronize(self.h))


class MskHandle(Handle):
    """A libcfx handle for a musculoskeletal problem (cfx_msk_create): FES muscles driving a serial chain of
    revolute dofs.  Same evaluation interface as :class:`Handle`.

    ``chain``: dict with ``axis`` (nq,), ``frame`` (nq, 12), ``gravity`` (3,), ``mass`` (nq,), ``com`` (nq, 3),
    ``inertia`` (nq, 9); ``muscles``: list of dicts with ``model_id``, ``constants``, ``point_frame``,
    ``point_pos`` (n, 3), ``optimal_length``, ``tendon_slack_length``, ``pennation_angle``; ``marker_pairs``: dicts
    ``node``, ``axes`` (bit mask), ``frame`` (2,), ``pos`` (2, 3) (cfx_msk_marker_pair)."""

    def __init__(self, *, chain, muscles, scheme, n_steps, n_shooting, truncation, final_time, stim_rows, batch,
                 flags=0, layout=LAYOUT_SOA, objectives=(), device=0, n_params=0, last_stim_idx=None,
                 param_offset=None, marker_pairs=()):
        self.lib = load_library()
        self._keep = []

        def arr(a, dt=np.float64):
            a = np.ascontiguousarray(a, dtype=dt).reshape(-1)
            self._keep.append(a)
            return a.ctypes.data_as(C.POINTER(C.c_int32 if dt == np.int32 else C.c_double))

        pb = MskProblem()
        pb.abi_version = ABI_VERSION
        pb.scheme, pb.n_steps, pb.n_shooting, pb.truncation = scheme, n_steps, n_shooting, truncation
        pb.layout, pb.batch, pb.final_time = layout, batch, final_time
        pb.stim_rows = arr(stim_rows)
        pb.n_dof = len(chain["axis"])
        pb.dof_axis = arr(chain["axis"], np.int32)
        pb.dof_frame = arr(chain["frame"])
        for i in range(3):
            pb.gravity[i] = float(chain["gravity"][i])
        pb.body_mass, pb.body_com, pb.body_inertia = arr(chain["mass"]), arr(chain["com"]), arr(chain["inertia"])
        mus = (MskMuscle * len(muscles))()
        for i, m in enumerate(muscles):
            mus[i].model = m["model_id"]
            cst = Constants()
            for name, _ in Constants._fields_:
                setattr(cst, name, float(m["constants"].get(name, 0.0)))
            mus[i].constants = cst
            mus[i].n_points = len(m["point_frame"])
            mus[i].point_frame = arr(m["point_frame"], np.int32)
            mus[i].point_pos = arr(m["point_pos"])
            mus[i].optimal_length = m["optimal_length"]
            mus[i].tendon_slack_length = m["tendon_slack_length"]
            mus[i].pennation_angle = m["pennation_angle"]
        self._keep.append(mus)
        pb.n_muscles = len(muscles)
        pb.muscles = mus
        pb.flags = flags
        pb.objectives = _objective_array(objectives, self._keep, n_shooting)
        pb.n_objectives = len(objectives)
        pb.device = device
        pb.n_params = int(n_params)
        if n_params:
            pb.last_stim_idx = arr(last_stim_idx, np.int32)
            pb.param_offset = arr(param_offset, np.int32)
        if marker_pairs:
            mk = (MskMarkerPair * len(marker_pairs))()
            for i, c in enumerate(marker_pairs):
                mk[i].node, mk[i].axes = int(c["node"]), int(c["axes"])
                for j in range(2):
                    mk[i].frame[j] = int(c["frame"][j])
                    for e in range(3):
                        mk[i].pos[j][e] = float(c["pos"][j][e])
            self._keep.append(mk)
            pb.n_marker_pairs, pb.marker_pairs = len(marker_pairs), mk
        h = C.c_void_p()
        rc = self.lib.cfx_msk_create(C.byref(pb), C.byref(h))
        self._attach(rc, h, batch, layout, n_shooting, n_steps, device)


class Ipm:
    """A libcfx interior-point solver (cfx_ipm_*) bound to a handle (CFX_LAYOUT_AOS, or batch 1): the whole
    iteration runs on the handle's GPU.  ``options``: a dict of cfx_ipm_options fields (libcfx defaults for the
    rest).  Host (numpy) inputs and outputs; the call returns when the solve is done."""

    def __init__(self, handle: Handle, lb, ub, n_params: int = 0, options: dict | None = None):
        self.lib = handle.lib
        self.handle = handle  # keeps the handle alive
        self.batch, self.nv, self.ng = handle.batch, handle.nv, handle.ng
        if handle.batch > 1 and handle.layout != LAYOUT_AOS:
            raise CfxError(EINVAL, "Ipm: the handle must use the AoS layout (or batch 1)")
        lb = np.ascontiguousarray(lb, dtype=np.float64).reshape(-1)
        ub = np.ascontiguousarray(ub, dtype=np.float64).reshape(-1)
        if lb.size != self.nv or ub.size != self.nv:
            raise CfxError(EINVAL, f"Ipm: bounds must hold nv = {self.nv} values")
        opt = IpmOptions()
        self.lib.cfx_ipm_default_options(C.byref(opt))
        for k, v in (options or {}).items():
            if k not in dict(IpmOptions._fields_):
                raise CfxError(EINVAL, f"Ipm: unknown option {k!r}")
            setattr(opt, k, v)
        s = C.c_void_p()
        rc = self.lib.cfx_ipm_create(handle.h, lb.ctypes.data, ub.ctypes.data, int(n_params), C.byref(opt), C.byref(s))
        if rc != OK:
            raise CfxError(rc, self.lib.cfx_last_error(None).decode())
        self.s = s
        self.n_fixed = self.lib.cfx_ipm_n_fixed(self.s)

    @classmethod
    def external(cls, batch, nv, ng, jac_structure, hess_structure, eval_all, eval_h, lb, ub, n_params=0,
                 options=None, device=0, stream=0):
        """The solver over caller-supplied callbacks (cfx_ipm_create_ext): ``eval_all(v, g, jac, f, grad)`` and
        ``eval_h(v, obj_factor, lam, hess)`` receive device pointers (ints; 0 for an output not wanted) of AoS arrays
        on ``stream`` and return 0 on success.  Used by the interval-sharded path (distributed.ShardedNativeIpm)."""
        self = cls.__new__(cls)
        self.lib = load_library()
        self.handle = None
        self.batch, self.nv, self.ng = int(batch), int(nv), int(ng)
        jr, jc = (np.ascontiguousarray(a, dtype=np.int32) for a in jac_structure)
        hr, hc = (np.ascontiguousarray(a, dtype=np.int32) for a in hess_structure)
        i32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
        desc = NlpDesc(self.batch, self.nv, self.ng, len(jr), len(hr), i32(jr), i32(jc), i32(hr), i32(hc), int(device),
                       C.c_void_p(int(stream)))

        def _all(ctx, v, g, jac, f, grad):
            try:
                return int(eval_all(v or 0, g or 0, jac or 0, f or 0, grad or 0))
            except Exception as e:  # noqa: BLE001 — reported through CFX_ECALLBACK, re-raised by solve()
                self._cb_error = e
                return -1

        def _h(ctx, v, of, lam, hess):
            try:
                return int(eval_h(v or 0, of or 0, lam or 0, hess or 0))
            except Exception as e:  # noqa: BLE001
                self._cb_error = e
                return -1

        self._cb = (EVAL_ALL_FN(_all), EVAL_H_FN(_h))  # kept alive with the solver
        self._cb_error = None
        ev = Evaluator(None, self._cb[0], self._cb[1])
        lb = np.ascontiguousarray(lb, dtype=np.float64).reshape(-1)
        ub = np.ascontiguousarray(ub, dtype=np.float64).reshape(-1)
        if lb.size != self.nv or ub.size != self.nv:
            raise CfxError(EINVAL, f"Ipm.external: bounds must hold nv = {self.nv} values")
        opt = IpmOptions()
        self.lib.cfx_ipm_default_options(C.byref(opt))
        for k, v in (options or {}).items():
            if k not in dict(IpmOptions._fields_):
                raise CfxError(EINVAL, f"Ipm: unknown option {k!r}")
            setattr(opt, k, v)
        s = C.c_void_p()
        rc = self.lib.cfx_ipm_create_ext(C.byref(desc), C.byref(ev), lb.ctypes.data, ub.ctypes.data, int(n_params),
                                         C.byref(opt), C.byref(s))
        if rc != OK:
            raise CfxError(rc, self.lib.cfx_last_error(None).decode())
        self.s = s
        self.n_fixed = self.lib.cfx_ipm_n_fixed(self.s)
        return self

    def solve(self, v0, fixed_values=None):
        """Returns (v, y, f, converged, iterations, kkt_error) as numpy arrays."""
        B = self.batch
        v0 = np.ascontiguousarray(v0, dtype=np.float64)
        if v0.size != B * self.nv:
            raise CfxError(EINVAL, f"Ipm.solve: v0 has {v0.size} values, expected batch * nv = {B * self.nv}")
        fv = None
        if fixed_values is not None:
            fv = np.ascontiguousarray(fixed_values, dtype=np.float64)
            if fv.size != B * self.n_fixed:
                raise CfxError(EINVAL, f"Ipm.solve: fixed_values has {fv.size} values, expected batch * n_fixed = "
                                       f"{B * self.n_fixed}")
        v = np.empty((B, self.nv))
        y = np.empty((B, self.ng))
        f = np.empty(B)
        conv = np.empty(B, dtype=np.int32)
        its = np.empty(B, dtype=np.int32)
        kkt = np.empty(B)
        rc = self.lib.cfx_ipm_solve(self.s, v0.ctypes.data, None if fv is None else fv.ctypes.data, v.ctypes.data,
                                    y.ctypes.data, f.ctypes.data, conv.ctypes.data, its.ctypes.data, kkt.ctypes.data, 0)
        if rc != OK:
            err = getattr(self, "_cb_error", None)
            if err is not None:
                self._cb_error = None
                raise CfxError(rc, f"{self.lib.cfx_ipm_last_error(self.s).decode()}: {err!r}") from err
            raise CfxError(rc, self.lib.cfx_ipm_last_error(self.s).decode())
        return v, y, f, conv.astype(bool), its.astype(np.int64), kkt

    def set_warm_start(self, y, z_l, z_u):
        """Ipopt's warm_start_init_point inputs (cfx_ipm_set_warm_start): y (B, ng) constraint multipliers, z_l / z_u
        (B, nv) bound multipliers of the unscaled problem; used by solves with the warm_start_init_point option."""
        B = self.batch
        y = np.ascontiguousarray(y, dtype=np.float64)
        zl = np.ascontiguousarray(z_l, dtype=np.float64)
        zu = np.ascontiguousarray(z_u, dtype=np.float64)
        if y.size != B * self.ng or zl.size != B * self.nv or zu.size != B * self.nv:
            raise CfxError(EINVAL, "Ipm.set_warm_start: y must hold batch * ng values, z_l / z_u batch * nv")
        rc = self.lib.cfx_ipm_set_warm_start(self.s, y.ctypes.data, zl.ctypes.data, zu.ctypes.data, 0)
        if rc != OK:
            raise CfxError(rc, self.lib.cfx_ipm_last_error(self.s).decode())

    def bound_multipliers(self):
        """(z_l, z_u), each (B, nv): the last solve's bound multipliers of the unscaled problem."""
        zl = np.empty((self.batch, self.nv))
        zu = np.empty((self.batch, self.nv))
        rc = self.lib.cfx_ipm_get_bound_multipliers(self.s, zl.ctypes.data, zu.ctypes.data, 0)
        if rc != OK:
            raise CfxError(rc, self.lib.cfx_ipm_last_error(self.s).decode())
        return zl, zu

    def stats(self):
        st = IpmStats()
        rc = self.lib.cfx_ipm_get_stats(self.s, C.byref(st))
        if rc != OK:
            raise CfxError(rc, "cfx_ipm_get_stats")
        return {k: getattr(st, k) for k, _ in IpmStats._fields_}

    def status(self):
        """(B,) int32: the CFX_IPM_* outcome (IPM_STATUS) of every instance of the last solve."""
        out = np.empty(self.batch, dtype=np.int32)
        rc = self.lib.cfx_ipm_get_status(self.s, out.ctypes.data_as(C.POINTER(C.c_int32)))
        if rc != OK:
            raise CfxError(rc, "cfx_ipm_get_status")
        return out

    def close(self):
        if getattr(self, "s", None):
            self.lib.cfx_ipm_destroy(self.s)
            self.s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
