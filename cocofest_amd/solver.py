"""Batched primal-dual interior-point driver over the libcfx callbacks (the Ipopt role of the reference's
`ocp.solve(Solver.IPOPT(...))`, SURVEY.md section 3 stack B).

All B instances of one transcribed problem iterate in lockstep on the GPU: the callbacks (g, J_g, f, grad f,
Lagrangian Hessian) come from libcfx in one launch each for the whole batch, everything else is kept in the
callbacks' sparse (triplet) form, and the Newton/KKT system of every instance is assembled directly in
band storage and factored by libcfx's batched band LU (cfx_band_lu: one wave per instance, band in LDS).
The band comes from ordering the KKT unknowns stage by stage — each constraint row sits between the
variables it couples (x_k, u_k | g_k | x_{k+1}) — which makes the half-bandwidth a few times nx + nu
instead of n.  This plays the part of the sparse LDL^T (MUMPS) Ipopt factors the same matrix with.

Algorithm (Ipopt's, simplified — monotone Fiacco-McCormick barrier, filter line search with one
second-order correction, curvature-based inertia correction, gradient-based problem scaling): minimise
f(v) - mu sum ln(v - lb) - mu sum ln(ub - v) s.t. g(v) = 0; fixed variables (lb == ub, e.g. the initial
state) are removed; default tol 1e-6 on the scaled KKT error as Ipopt's `tol`.
"""

from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np


@dataclass
class IpmOptions:
    tol: float = 1e-6
    max_iter: int = 200
    acceptable_tol: float = 1e-6  # Ipopt "solved to acceptable level": err <= acceptable_tol for
    acceptable_iter: int = 15     # acceptable_iter consecutive iterations
    mu_init: float = 0.1
    # Ipopt's bound relaxation (its default is 1e-8); off by default here: it leaves cfg 5's iteration count within
    # run-to-run noise and moves cfg 3's optimum by 0.02 % through the unscaled pulse-width bound
    bound_relax_factor: float = 0.0
    bound_push: float = 1e-2
    tau_min: float = 0.99
    kappa_eps: float = 10.0
    kappa_mu: float = 0.2
    theta_mu: float = 1.5
    s_max: float = 100.0
    armijo: float = 1e-4
    max_backtrack: int = 30
    delta_c: float = 1e-9
    curv_min: float = 1e-8  # inertia-free test: dx^T (W + Sigma + dw) dx >= curv_min |dx|^2 (scaled space)
    # iterative-refinement steps on each Newton solve (as Ipopt refines its KKT solves); off by default: on cfg 5 /
    # cfg 3 it leaves the iteration counts unchanged and costs a band solve per step (scripts/ipm_refine_probe.py)
    refine: int = 0
    max_soc: int = 4        # second-order corrections per iteration (Ipopt max_soc)
    kappa_soc: float = 0.99  # required infeasibility decrease between corrections (Ipopt kappa_soc)
    # Ipopt's watchdog (on by default there): after this many consecutive shortened line searches the full step is
    # taken for up to watchdog_trial_iter_max iterations, judged against the iterate where the watchdog started;
    # if none is acceptable the solver returns there and backtracks.  0 disables it
    watchdog_shortened_iter_trigger: int = 10
    watchdog_trial_iter_max: int = 3
    # Ipopt's hessian_approximation: "exact" (the callbacks' Lagrangian Hessian) or "limited-memory" (L-BFGS of
    # limited_memory_max_history pairs, Ipopt's defaults)
    hessian_approximation: str = "exact"
    limited_memory_max_history: int = 6
    # what a failed line search starts: "phase" (default; None means it too) — Ipopt's feasibility-restoration phase,
    # an NLP over the constraint violation; "step" — one minimum-norm step on g = 0 then least-squares multipliers
    restoration: str | None = None
    max_resto_iter: int = 200
    resto_penalty: float = 1000.0            # Ipopt resto_penalty_parameter (rho)
    required_infeasibility_reduction: float = 0.9
    # Ipopt's filter reset heuristic: after filter_reset_trigger successive iterations whose line search last rejected a
    # trial point because of the filter, the filter is cleared, at most max_filter_resets times (0: off).  Ipopt's
    # default is 5 resets; off by default here (measured on the fatigue-family RK4 test problem
    # and cfg 5's multistart)
    filter_reset_trigger: int = 5
    max_filter_resets: int = 0
    # Ipopt's soft restoration (IpBacktrackingLineSearch::TrySoftRestoStep): a failed line search first tries the step
    # at the smaller of the primal and dual fractions to the boundary, primal and dual together, accepted when the
    # original filter takes it (at alpha 0: the sufficient-decrease test) or when it cuts the primal-dual system error
    # (mean of |grad L|, |c| and |s z - mu|) by this factor (Ipopt's default 0.9999; 0: off).  An accepted step the
    # filter did not take keeps the instance on such steps — no line search — for up to max_soft_resto_iters
    # iterations, until one satisfies the filter; a rejected one starts the restoration phase.  Phase mode only
    soft_resto_pderror_reduction_factor: float = 0.0
    max_soft_resto_iters: int = 10
    # extension (not Ipopt): a failed restoration phase restarts the main iteration from the phase's last point (zero
    # constraint multipliers, empty filter) instead of stopping the instance with Restoration_Failed; the iteration
    # budget still bounds it.  Off by default (Ipopt's behaviour); DESIGN.md section 5 has the multistart numbers
    resto_failure_restart: bool = False
    # Ipopt's max_wall_time (s): the instances still iterating stop there (status -5); print_frequency_time (s, 0:
    # off): the native solver prints a progress line (iteration, instances iterating, in restoration) this often
    max_wall_time: float = 1e20
    print_frequency_time: float = 0.0
    # Ipopt's termination tests on the unscaled problem (IpOptErrorConv), beside tol on the scaled error: converged
    # needs max|g| <= constr_viol_tol, max|grad L| <= dual_inf_tol and max|s z| <= compl_inf_tol; the acceptable level
    # (acceptable_tol held acceptable_iter iterations, or a restoration phase called at an acceptable point) the
    # acceptable_* ones.  Ipopt's defaults
    constr_viol_tol: float = 1e-4
    dual_inf_tol: float = 1.0
    compl_inf_tol: float = 1e-4
    acceptable_constr_viol_tol: float = 1e-2
    acceptable_dual_inf_tol: float = 1e10
    acceptable_compl_inf_tol: float = 1e-2
    # Ipopt's honor_original_bounds (3.14's default "no"): with bound_relax_factor > 0, True moves the returned point
    # into the original bounds, False returns the iterate as it is (the reference's stored reaching-task widths sit
    # 1e-8 outside their bounds: its Ipopt returned the iterate)
    honor_original_bounds: bool = False
    # variable scaling by the bound range (x = d x~, d = ub - lb when below 1: pulse widths ~1e-4 s become O(1)); an
    # extension — Ipopt scales only f and g (nlp_scaling_method gradient-based), which range_scaling=False reproduces
    range_scaling: bool = True
    # Ipopt's bound_mult_init_method: "mu-based" (z = mu_init / slack; the default here) or "constant" (Ipopt's
    # default: z = bound_mult_init_val)
    bound_mult_init_method: str = "mu-based"
    bound_mult_init_val: float = 1.0
    # inertia correction (NativeIpm, stage-chain layout): False the curvature test above; True Ipopt's test on the KKT
    # matrix's inertia (exactly m negative eigenvalues, else dw grows), counted from the chain's pivot blocks.  Layouts
    # without an inertia count (NativeIpm's band layouts, every BatchedIpm solve) keep the curvature test
    inertia_test: bool = False
    # Ipopt's warm start (NativeIpm: solve(..., warm_start=(y, z_l, z_u))): no least-squares multipliers; x pushed from
    # its bounds by warm_start_bound_push max(1, |bound|) (at most warm_start_bound_frac of the range), bound
    # multipliers raised to warm_start_mult_bound_push; mu starts at mu_init
    warm_start_init_point: bool = False
    warm_start_bound_push: float = 1e-3
    warm_start_bound_frac: float = 1e-3
    warm_start_mult_bound_push: float = 1e-3
    # cold-start push: x_L + min(bound_push max(1, |x_L|), bound_frac (x_U - x_L)) (Ipopt's bound_frac is 0.01; this
    # library's 0.5 pushes narrow-range variables to at most the middle of their range)
    bound_frac: float = 0.5
    # Ipopt's barrier-parameter strategy (IpAdaptiveMuUpdate / IpMonotoneMuUpdate).  "monotone": Fiacco-McCormick, mu
    # decreased while the barrier problem's error is below kappa_eps mu (this library's default); "adaptive" (bioptim's
    # Solver.IPOPT default, recalled — external/bioptim is not in the reference tree): the free-mu mode of Nocedal,
    # Waechter & Waltz (2009) — every iteration mu = sigma * (average complementarity), sigma minimising Ipopt's quality
    # function (mu_oracle "quality-function": the predicted 2-norm-squared dual infeasibility, primal infeasibility and
    # complementarity after a step of mu's direction, golden-section search over log sigma); globalised by
    # adaptive_mu_globalization: "obj-constr-filter" (Ipopt's default: an iterate not acceptable to a filter of the
    # (f, ||c||_1) of the accepted free-mode iterates switches to the monotone mode at mu = adaptive_mu_monotone_init_factor
    # * average complementarity, which returns to the free mode once an iterate is acceptable again) or
    # "never-monotone-mode".  "kkt-error" globalisation and the probing / loqo oracles are not restated
    mu_strategy: str = "monotone"
    mu_oracle: str = "quality-function"
    adaptive_mu_globalization: str = "obj-constr-filter"
    mu_max_fact: float = 1000.0  # mu_max = mu_max_fact * average complementarity at the first iteration (mu_max <= 0)
    mu_max: float = -1.0
    mu_min: float = 1e-11
    adaptive_mu_monotone_init_factor: float = 0.8
    sigma_max: float = 100.0
    sigma_min: float = 1e-6
    quality_function_max_section_steps: int = 8
    quality_function_section_sigma_tol: float = 1e-2
    quality_function_section_qf_tol: float = 0.0
    filter_margin_fact: float = 1e-5
    filter_max_margin: float = 1.0
    # Ipopt resets the line search's filter whenever the barrier parameter changes (linesearch_->Reset() in both mu
    # updates: the filter's phi values belong to the old barrier function).  The adaptive strategy always does; for the
    # monotone strategy this flag (off in this library's profile, which keeps the filter across mu decreases)
    mu_change_resets_filter: bool = False
    # floor of the monotone mu update: "library" tol / 10; "ipopt" min(tol, compl_inf_tol) / (kappa_eps + 1)
    monotone_mu_floor: str = "library"
    # Ipopt's nlp_scaling_method: "gradient-based" (f and each row of g scaled so that their largest gradient entry at
    # the starting point is at most nlp_scaling_max_gradient, factors at least nlp_scaling_min_value) or "none"
    nlp_scaling_method: str = "gradient-based"
    nlp_scaling_max_gradient: float = 100.0
    nlp_scaling_min_value: float = 1e-8
    verbose: bool = False

    # Ipopt 3.14's defaults where bioptim's Solver.IPOPT leaves them, bioptim's values where it sets them (recalled, see
    # DESIGN.md "Solver profiles"): the options Solver.IPOPT() applies by default.  Everything not listed keeps its
    # IpmOptions default, which equals Ipopt's (tol on the unscaled problem, watchdog, second-order corrections, ...)
    IPOPT_PROFILE = dict(
        tol=1e-6, max_iter=1000, acceptable_tol=1e-6, acceptable_iter=15, mu_init=0.1,  # bioptim
        mu_strategy="adaptive",  # bioptim (Ipopt's own default is "monotone")
        limited_memory_max_history=50,  # bioptim (Ipopt: 6)
        bound_relax_factor=1e-8, bound_push=1e-2, bound_frac=1e-2, honor_original_bounds=False,
        range_scaling=False, bound_mult_init_method="constant", bound_mult_init_val=1.0,
        max_resto_iter=3_000_000, max_filter_resets=5, filter_reset_trigger=5,
        soft_resto_pderror_reduction_factor=0.9999, max_soft_resto_iters=10, resto_failure_restart=False,
        mu_change_resets_filter=True, monotone_mu_floor="ipopt", nlp_scaling_method="gradient-based",
        inertia_test=True)

    @classmethod
    def ipopt(cls, **overrides) -> "IpmOptions":
        """The Ipopt / bioptim profile (IPOPT_PROFILE) with ``overrides``."""
        return cls(**{**cls.IPOPT_PROFILE, **overrides})

    def mu_floor(self) -> float:
        """Lower bound of the monotone barrier parameter."""
        if self.monotone_mu_floor == "ipopt":
            return min(self.tol, self.compl_inf_tol) / (self.kappa_eps + 1.0)
        return self.tol / 10

    def __post_init__(self):
        if self.filter_reset_trigger < 1 or self.max_filter_resets < 0:
            raise ValueError("filter_reset_trigger must be >= 1 and max_filter_resets >= 0")
        if not self.max_wall_time > 0 or not self.print_frequency_time >= 0:
            raise ValueError("max_wall_time must be > 0 and print_frequency_time >= 0")
        if not self.soft_resto_pderror_reduction_factor >= 0 or self.max_soft_resto_iters < 0:
            raise ValueError("soft_resto_pderror_reduction_factor must be >= 0 and max_soft_resto_iters >= 0")
        for k in ("constr_viol_tol", "dual_inf_tol", "compl_inf_tol", "acceptable_constr_viol_tol",
                  "acceptable_dual_inf_tol", "acceptable_compl_inf_tol"):
            if not getattr(self, k) > 0:
                raise ValueError(f"{k} must be > 0")
        choices = {"mu_strategy": ("monotone", "adaptive"), "mu_oracle": ("quality-function",),
                   "adaptive_mu_globalization": ("obj-constr-filter", "never-monotone-mode"),
                   "monotone_mu_floor": ("library", "ipopt"), "nlp_scaling_method": ("gradient-based", "none"),
                   "bound_mult_init_method": ("constant", "mu-based"),
                   "hessian_approximation": ("exact", "limited-memory")}
        for k, allowed in choices.items():
            if getattr(self, k) not in allowed:
                raise ValueError(f"{k} must be one of {allowed} (got {getattr(self, k)!r}; Ipopt's other choices are not "
                                 "restated here)")
        if not (self.mu_min > 0 and self.mu_max_fact > 0 and 0 < self.sigma_min <= 1 <= self.sigma_max and
                0 < self.adaptive_mu_monotone_init_factor and self.quality_function_max_section_steps >= 0 and
                0 < self.quality_function_section_sigma_tol < 1 and self.quality_function_section_qf_tol >= 0 and
                self.filter_margin_fact > 0 and self.filter_max_margin > 0):
            raise ValueError("invalid adaptive barrier-parameter options")
        if not (self.nlp_scaling_max_gradient > 0 and self.nlp_scaling_min_value > 0):
            raise ValueError("nlp_scaling_max_gradient and nlp_scaling_min_value must be > 0")
        if not (0 < self.bound_frac <= 0.5 and self.bound_push > 0):
            raise ValueError("bound_push must be > 0 and 0 < bound_frac <= 0.5")


class Solver:
    """bioptim's solver namespace as cocofest uses it: ``ocp.solve(Solver.IPOPT(_max_iter=..., _tol=...,
    _hessian_approximation="limited-memory"))`` (examples/getting_started/frequency_optimization.py:22,
    pulse_duration_optimization.py:41).  The options map onto the native interior point's (IpmOptions); the
    ones that only steer Ipopt's own output or its external linear solver are accepted and ignored.

    ``profile`` names the option set the explicit options start from: "ipopt" (the default — IpmOptions.IPOPT_PROFILE,
    Ipopt 3.14's defaults with bioptim's Solver.IPOPT values where bioptim sets them, so a cocofest script is solved
    with the reference's solver settings) or "cfx" (this library's tuned set, the IpmOptions defaults)."""

    class IPOPT:
        _PROFILES = ("ipopt", "cfx")
        _OPTIONS = {"_tol": "tol", "_max_iter": "max_iter", "_acceptable_tol": "acceptable_tol",
                    "_acceptable_iter": "acceptable_iter", "_mu_init": "mu_init",
                    "_bound_relax_factor": "bound_relax_factor", "_bound_push": "bound_push",
                    "_hessian_approximation": "hessian_approximation",
                    "_limited_memory_max_history": "limited_memory_max_history", "_max_soc": "max_soc",
                    "_watchdog_shortened_iter_trigger": "watchdog_shortened_iter_trigger",
                    "_watchdog_trial_iter_max": "watchdog_trial_iter_max", "_max_resto_iter": "max_resto_iter",
                    "_resto_penalty_parameter": "resto_penalty",
                    "_required_infeasibility_reduction": "required_infeasibility_reduction",
                    "_filter_reset_trigger": "filter_reset_trigger", "_max_filter_resets": "max_filter_resets",
                    "_max_wall_time": "max_wall_time", "_print_frequency_time": "print_frequency_time",
                    "_soft_resto_pderror_reduction_factor": "soft_resto_pderror_reduction_factor",
                    "_max_soft_resto_iters": "max_soft_resto_iters", "_constr_viol_tol": "constr_viol_tol",
                    "_dual_inf_tol": "dual_inf_tol", "_compl_inf_tol": "compl_inf_tol",
                    "_acceptable_constr_viol_tol": "acceptable_constr_viol_tol",
                    "_acceptable_dual_inf_tol": "acceptable_dual_inf_tol",
                    "_acceptable_compl_inf_tol": "acceptable_compl_inf_tol",
                    "_mu_strategy": "mu_strategy", "_mu_oracle": "mu_oracle",
                    "_adaptive_mu_globalization": "adaptive_mu_globalization", "_mu_max_fact": "mu_max_fact",
                    "_mu_max": "mu_max", "_mu_min": "mu_min", "_nlp_scaling_method": "nlp_scaling_method",
                    "_nlp_scaling_max_gradient": "nlp_scaling_max_gradient", "_bound_frac": "bound_frac",
                    "_bound_mult_init_method": "bound_mult_init_method", "_bound_mult_init_val": "bound_mult_init_val",
                    "_honor_original_bounds": "honor_original_bounds",
                    "_warm_start_init_point": "warm_start_init_point", "_warm_start_bound_push": "warm_start_bound_push",
                    "_warm_start_bound_frac": "warm_start_bound_frac",
                    "_warm_start_mult_bound_push": "warm_start_mult_bound_push"}
        _IGNORED = {"show_online_optim", "show_options", "_print_level", "_linear_solver",
                    "_check_derivatives_for_naninf", "_c_compile", "_print_timing_statistics", "_output_file",
                    "_warm_start_slack_bound_push", "_warm_start_slack_bound_frac"}
        # Ipopt's yes / no options
        _YESNO = {"_honor_original_bounds", "_warm_start_init_point"}

        def __init__(self, show_online_optim: bool = False, show_options: dict | None = None, profile: str = "ipopt",
                     **kwargs):
            if profile not in self._PROFILES:
                raise ValueError(f"Solver.IPOPT: profile must be one of {self._PROFILES}")
            self.profile = profile
            base = IpmOptions.ipopt() if profile == "ipopt" else IpmOptions()
            self._tol = base.tol
            self._max_iter = 1000  # bioptim's _max_iter, in either profile
            self._hessian_approximation = "exact"
            self._limited_memory_max_history = base.limited_memory_max_history
            self._print_level = 5
            self._linear_solver = "mumps"
            for k, v in kwargs.items():
                if k not in self._OPTIONS and k not in self._IGNORED:
                    raise TypeError(f"Solver.IPOPT: unknown option {k!r}")
                if k in self._YESNO and isinstance(v, str):
                    if v not in ("yes", "no"):
                        raise ValueError(f"Solver.IPOPT: {k} must be 'yes' or 'no'")
                    v = v == "yes"
                setattr(self, k, v)
            if self._hessian_approximation not in ("exact", "limited-memory"):
                raise ValueError("hessian_approximation must be 'exact' or 'limited-memory'")
            self.options()  # validates every option now (unknown choices raise ValueError)

        # bioptim's setters
        def set_maximum_iterations(self, n: int):
            self._max_iter = int(n)

        def set_tol(self, tol: float):
            self._tol = float(tol)

        def set_hessian_approximation(self, value: str):
            if value not in ("exact", "limited-memory"):
                raise ValueError("hessian_approximation must be 'exact' or 'limited-memory'")
            self._hessian_approximation = value

        def set_limited_memory_max_history(self, n: int):
            self._limited_memory_max_history = int(n)

        def set_print_level(self, n: int):
            self._print_level = int(n)

        def set_linear_solver(self, name: str):
            self._linear_solver = name

        # the plain names the round-1 facade read
        @property
        def tol(self):
            return self._tol

        @property
        def max_iter(self):
            return self._max_iter

        def set_mu_strategy(self, value: str):
            self._mu_strategy = value
            self.options()

        def set_nlp_scaling_method(self, value: str):
            self._nlp_scaling_method = value
            self.options()

        def apply(self, opts: "IpmOptions") -> "IpmOptions":
            """The profile's options, then the explicit ones, onto ``opts`` (fields neither sets keep their value)."""
            if self.profile == "ipopt":
                for name, v in IpmOptions.IPOPT_PROFILE.items():
                    setattr(opts, name, v)
            for k, name in self._OPTIONS.items():
                if hasattr(self, k):
                    setattr(opts, name, getattr(self, k))
            opts.__post_init__()
            return opts

        def options(self) -> "IpmOptions":
            """The IpmOptions this solver object stands for."""
            return self.apply(IpmOptions())


def apply_solver(opts: "IpmOptions", solver) -> "IpmOptions":
    """Options of a Solver.IPOPT (or any object with tol / max_iter attributes) onto IpmOptions."""
    if solver is None:
        return opts
    if isinstance(solver, Solver.IPOPT):
        return solver.apply(opts)
    for k in ("tol", "max_iter"):
        if hasattr(solver, k):
            setattr(opts, k, getattr(solver, k))
    return opts


@dataclass
class IpmResult:
    v: np.ndarray
    y: np.ndarray
    f: np.ndarray
    converged: np.ndarray
    iterations: np.ndarray
    kkt_error: np.ndarray
    wall_time: float
    n_callbacks: dict = field(default_factory=dict)
    # per instance, Ipopt's ApplicationReturnStatus (cocofest_amd._cfx.IPM_STATUS): 0 solved, 1 solved to acceptable
    # level, 2 local infeasibility, -1 maximum iterations, -2 restoration failed, -5 maximum wall time
    status: np.ndarray | None = None


class _SegmentSum:
    """Deterministic `out.index_add_(1, idx, src)` for a fixed index: the sources of each output position are
    gathered in a fixed order from a padded (n_out_used, k_max) table and summed, so the KKT assembly (and with it
    the iteration path) is the same on every run, which GPU atomics do not guarantee."""

    def __init__(self, torch, idx, device):
        idx = np.asarray(idx, dtype=np.int64)
        order = np.argsort(idx, kind="stable")
        uniq, counts = np.unique(idx, return_counts=True)
        kmax = int(counts.max()) if counts.size else 1
        table = np.full((uniq.size, kmax), idx.size, dtype=np.int64)  # padding points at a zero column
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
        for k in range(kmax):
            has = counts > k
            table[has, k] = order[starts[has] + k]
        self.torch = torch
        self.uniq = torch.as_tensor(uniq, device=device)
        self.table = torch.as_tensor(table, device=device)

    def add_(self, out, src):
        srcp = self.torch.cat([src, src.new_zeros((src.shape[0], 1))], dim=1)
        out[:, self.uniq] += srcp[:, self.table].sum(-1)
        return out


class BatchedIpm:
    """Interior-point solver for B instances of one FesOcp on one GPU."""

    def __init__(self, ocp, batch: int = 1, device: int = 0, options: IpmOptions | None = None, handle=None,
                 torch_device=None, band=None):
        """``handle`` / ``torch_device`` / ``band`` let tests drive the same algorithm with another evaluator and
        linear solver on the CPU; the product path always opens a libcfx handle and uses libcfx's band LU on
        GPU ``device``."""
        import torch

        self.torch = torch
        self.ocp = ocp
        self.B = batch
        self.opt = options or IpmOptions()
        self.opt.__post_init__()  # options set after construction (Solver.IPOPT.apply) are checked too
        if self.opt.restoration not in (None, "step", "phase"):
            raise ValueError("restoration must be 'phase' or 'step'")
        self._phase = self.opt.restoration in (None, "phase")  # the native solver's default too
        # what only the native interior point implements is refused here rather than silently ignored
        if self.opt.hessian_approximation != "exact":
            raise ValueError("BatchedIpm: hessian_approximation='limited-memory' is implemented by the native interior "
                             "point (NativeIpm / cfx_ipm) only")
        if self.opt.warm_start_init_point:
            raise ValueError("BatchedIpm: warm_start_init_point is implemented by NativeIpm only")
        # (inertia_test: the band factorisation here has no inertia count, so the curvature test stands in for it, as
        # on NativeIpm's band layouts)
        self.dev = torch.device(torch_device) if torch_device is not None else torch.device("cuda", device)
        self.h = handle if handle is not None else ocp.nlp(batch=batch, layout="aos", device=device)
        h = self.h
        self.n, self.m = h.nv, h.ng
        lb, ub = ocp.bounds_vector()
        self.fixed = np.where(lb == ub)[0]
        self.free = np.where(lb != ub)[0]
        t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=self.dev)  # noqa: E731
        self.lb_full, self.ub_full = t(lb), t(ub)
        self.lbF, self.ubF = self.lb_full[self.free], self.ub_full[self.free]
        self.hasL = torch.isfinite(self.lbF)
        self.hasU = torch.isfinite(self.ubF)
        self.freeT = torch.as_tensor(self.free, device=self.dev)
        # Variable scaling (x = d * x~): variables whose bound range is below 1 (pulse widths ~1e-4 s, fatigue
        # time constants) are mapped to O(1); the iteration works in x~, bounds and derivatives follow.
        width = self.ubF - self.lbF
        self.d = torch.where(torch.isfinite(width) & (width < 1.0) & bool(self.opt.range_scaling), width,
                             torch.ones_like(width))
        self.lbF, self.ubF = self.lbF / self.d, self.ubF / self.d
        # Ipopt's bound_relax_factor: the iteration sees the bounds relaxed by eps * max(1, |bound|) (in the user's
        # units, as Ipopt), meant for bounds the solution touches only asymptotically (a fatigue state a hair above
        # its rest value); the result is projected back onto the original bounds (Ipopt's honor_original_bounds)
        rel = self.opt.bound_relax_factor
        self.lbF0, self.ubF0 = self.lbF, self.ubF
        self.lbF = self.lbF - rel * torch.clamp((self.lbF * self.d).abs(), min=1.0) / self.d
        self.ubF = self.ubF + rel * torch.clamp((self.ubF * self.d).abs(), min=1.0) / self.d
        # gradient-based function scaling (Ipopt nlp_scaling_method): set at the starting point
        self.sf = torch.ones((batch,), dtype=torch.float64, device=self.dev)
        self.sg = torch.ones((batch, h.ng), dtype=torch.float64, device=self.dev)
        self._build_kkt_maps(*h.jac_structure(), *h.hess_structure())
        self.band = band if band is not None else GpuBandSolver()
        self.calls = {"eval_all": 0, "eval_h": 0, "eval_g_f": 0, "kkt_factor": 0}

    def _build_kkt_maps(self, jr, jc, hr, hc):
        """Triplet maps of J_g and the Hessian restricted to the free variables, the stage-wise ordering of the
        KKT unknowns (free variables, then the multipliers of g) and the band-storage position of every
        KKT entry."""
        torch = self.torch
        nf, m = len(self.free), self.m
        posF = np.full(self.n, -1, dtype=np.int64)
        posF[self.free] = np.arange(nf)
        jr, jc, hr, hc = (np.asarray(a, dtype=np.int64) for a in (jr, jc, hr, hc))
        jsel = np.where(posF[jc] >= 0)[0]
        hsel = np.where((posF[hr] >= 0) & (posF[hc] >= 0))[0]
        jrF, jcF = jr[jsel], posF[jc[jsel]]
        hrF, hcF = posF[hr[hsel]], posF[hc[hsel]]
        # unknown u: variable j -> key j; constraint row i -> midpoint of the keys of the free columns it couples.
        # Parameters sit at the end of the decision vector but each is used by a few neighbouring rows only
        # (the Hmed sliding windows): they take the mean key of the rows that use them.
        vkey = np.arange(nf, dtype=np.float64)
        n_par = int(getattr(self.ocp, "n_params", 0) or 0)
        par = np.zeros(nf, dtype=bool)
        if n_par:
            par = self.free >= self.n - n_par

        def row_keys(vk, skip):
            sel = ~skip[jcF]
            cmin = np.full(m, np.inf)
            cmax = np.full(m, -np.inf)
            np.minimum.at(cmin, jrF[sel], vk[jcF[sel]])
            np.maximum.at(cmax, jrF[sel], vk[jcF[sel]])
            return np.where(np.isfinite(cmin), 0.5 * (cmin + cmax) + 0.25, nf)

        ckey = row_keys(vkey, par)
        if par.any():
            ssum = np.zeros(nf)
            cnt = np.zeros(nf)
            np.add.at(ssum, jcF, ckey[jrF])
            np.add.at(cnt, jcF, 1.0)
            vkey = np.where(par & (cnt > 0), ssum / np.maximum(cnt, 1.0) + 0.1, vkey)
            ckey = row_keys(vkey, np.zeros(nf, dtype=bool))
        key = np.concatenate([vkey, ckey])
        order = np.argsort(key, kind="stable")
        pos = np.empty(nf + m, dtype=np.int64)
        pos[order] = np.arange(nf + m)
        # KKT entries (row, col) in band order: H (both triangles), J, J^T, the two diagonals
        off = hrF != hcF
        rows = np.concatenate([pos[hrF], pos[hcF[off]], pos[nf + jrF], pos[jcF], pos[:nf], pos[nf:]])
        cols = np.concatenate([pos[hcF], pos[hrF[off]], pos[jcF], pos[nf + jrF], pos[:nf], pos[nf:]])
        kl = int(max(0, (rows - cols).max()))
        ku = int(max(0, (cols - rows).max()))
        ldab = 2 * kl + ku + 1
        flat = cols * ldab + kl + ku + rows - cols
        nh, nho, nj = len(hsel), int(off.sum()), len(jsel)
        sl = np.cumsum([0, nh, nho, nj, nj, nf, m])
        L = lambda a: torch.as_tensor(a, device=self.dev, dtype=torch.long)  # noqa: E731
        self.nK, self.kl, self.ku, self.ldab = nf + m, kl, ku, ldab
        self.jselT, self.jrF, self.jcF = L(jsel), L(jrF), L(jcF)
        self.hselT, self.hrF, self.hcF, self.hoff = L(hsel), L(hrF), L(hcF), torch.as_tensor(off, device=self.dev)
        self.posT = L(pos)
        self.idx_h, self.idx_ht = L(flat[sl[0]:sl[1]]), L(flat[sl[1]:sl[2]])
        self.idx_j, self.idx_jt = L(flat[sl[2]:sl[3]]), L(flat[sl[3]:sl[4]])
        self.idx_dx, self.idx_dy = L(flat[sl[4]:sl[5]]), L(flat[sl[5]:sl[6]])
        self.seg_kkt = _SegmentSum(torch, flat[sl[0]:sl[5]], self.dev)  # H, H^T, J, J^T, diag_x entries
        self.seg_jt = _SegmentSum(torch, jcF, self.dev)  # J^T y
        self.seg_j = _SegmentSum(torch, jrF, self.dev)  # J dx
        self.seg_h = _SegmentSum(torch, np.concatenate([hrF, hcF[off]]), self.dev)  # W dx

    # ---- callbacks (device, AoS); _scaled_* return the scaled problem in x~ ---------------------------------
    def _scaled_all(self, v):
        """g, J_g values over the free columns (triplets jrF, jcF), f, grad f of the scaled problem."""
        g, jac, f, grad = self._eval_all(v)
        gF = grad[:, self.freeT] * self.d * self.sf[:, None]
        jv = jac[:, self.jselT] * self.d[self.jcF] * self.sg[:, self.jrF]
        return g * self.sg, jv, f * self.sf, gF

    def _scaled_gf(self, v):
        g, f = self._eval_gf(v)
        return g * self.sg, f * self.sf

    def _scaled_hess(self, v, y, of=None):
        """Lagrangian Hessian values over the free variables (triplets hrF >= hcF) of the scaled problem (objective
        factor ``of``, default the objective scaling)."""
        hv = self._eval_h(v, y * self.sg, self.sf if of is None else of)
        return hv[:, self.hselT] * self.d[self.hrF] * self.d[self.hcF]

    def _jt_mul(self, jv, y):
        """J^T y over the free variables."""
        out = self.torch.zeros((self.B, len(self.free)), dtype=self.torch.float64, device=self.dev)
        return self.seg_jt.add_(out, jv * y[:, self.jrF])

    def _quad_w(self, hv, dx):
        """dx^T W dx from the lower-triangle triplets."""
        t = hv * dx[:, self.hrF] * dx[:, self.hcF]
        return (t * (1.0 + self.hoff.to(t.dtype))).sum(1)

    def _set_function_scaling(self, v):
        """Ipopt's gradient-based NLP scaling at the starting point: s = min(1, max_gradient / max |grad|), at least
        nlp_scaling_min_value; nlp_scaling_method "none": s = 1."""
        torch = self.torch
        g, jac, f, grad = self._eval_all(v)
        opt = self.opt
        if opt.nlp_scaling_method == "none":
            self.sf = torch.ones((self.B,), dtype=torch.float64, device=self.dev)
            self.sg = torch.ones((self.B, self.m), dtype=torch.float64, device=self.dev)
            return
        gF = grad[:, self.freeT] * self.d
        ja = (jac[:, self.jselT] * self.d[self.jcF]).abs()
        rmax = torch.zeros((self.B, self.m), dtype=torch.float64, device=self.dev)
        rmax.scatter_reduce_(1, self.jrF.expand(self.B, -1), ja, reduce="amax")
        gm, lo = opt.nlp_scaling_max_gradient, opt.nlp_scaling_min_value
        self.sf = torch.clamp(torch.clamp(gm / torch.clamp(gF.abs().amax(1), min=1e-300), max=1.0), min=lo)
        self.sg = torch.clamp(torch.clamp(gm / torch.clamp(rmax, min=1e-300), max=1.0), min=lo)

    def _kkt_matvec(self, hv, diag_x, jv, dx, dy):
        """[[W + diag_x, J^T], [J, -delta_c I]] [dx; dy] from the triplets (the residual of iterative refinement)."""
        torch = self.torch
        wx = self.seg_h.add_(diag_x * dx, torch.cat([hv * dx[:, self.hcF], (hv * dx[:, self.hrF])[:, self.hoff]], 1))
        top = wx + self._jt_mul(jv, dy)
        jd = self.seg_j.add_(torch.zeros((self.B, self.m), dtype=torch.float64, device=self.dev),
                             jv * dx[:, self.jcF])
        return torch.cat([top, jd - self.opt.delta_c * dy], dim=1)

    def _kkt_band(self, hv, diag_x, jv, diag_y=None):
        """Band storage (B, nK, ldab) of [[W + diag_x, J^T], [J, -delta_c I + diag_y]] in the stage-wise order."""
        torch = self.torch
        ab = torch.zeros((self.B, self.nK * self.ldab), dtype=torch.float64, device=self.dev)
        self.seg_kkt.add_(ab, torch.cat([hv, hv[:, self.hoff], jv, jv, diag_x], dim=1))
        ab[:, self.idx_dy] -= self.opt.delta_c
        if diag_y is not None:
            ab[:, self.idx_dy] += diag_y
        self.calls["kkt_factor"] += 1
        return ab.view(self.B, self.nK, self.ldab)

    def _eval_all(self, v):
        torch = self.torch
        B = self.B
        g = torch.empty((B, self.m), dtype=torch.float64, device=self.dev)
        jac = torch.empty((B, self.h.nnz_jac), dtype=torch.float64, device=self.dev)
        f = torch.empty((B,), dtype=torch.float64, device=self.dev)
        grad = torch.empty((B, self.n), dtype=torch.float64, device=self.dev)
        self.h.eval_all(v, g=g, jac=jac, f=f, grad=grad)
        self.calls["eval_all"] += 1
        return g, jac, f, grad

    def _eval_gf(self, v):
        torch = self.torch
        g = torch.empty((self.B, self.m), dtype=torch.float64, device=self.dev)
        f = torch.empty((self.B,), dtype=torch.float64, device=self.dev)
        self.h.eval_all(v, g=g, f=f)
        self.calls["eval_g_f"] += 1
        return g, f

    def _eval_h(self, v, y, of):
        torch = self.torch
        hv = torch.empty((self.B, self.h.nnz_hess), dtype=torch.float64, device=self.dev)
        self.h.eval_h(v, of.contiguous(), y.contiguous(), hv)
        self.calls["eval_h"] += 1
        return hv

    # ---- main loop --------------------------------------------------------------------------------------
    def solve(self, v0=None, fixed_values=None):
        """Solve from ``v0`` (B, nv) (default: the problem's initial guess).  ``fixed_values`` (B, n_fixed)
        overrides, per instance, the variables whose bounds coincide (e.g. each NMPC scenario's own initial
        state); by default they take their bound."""
        torch = self.torch
        opt = self.opt
        B, nf, m = self.B, len(self.free), self.m
        t0 = time.perf_counter()
        if v0 is None:
            v0 = np.tile(self.ocp.initial_guess_vector(), (B, 1))
        v = torch.as_tensor(np.asarray(v0, dtype=np.float64), device=self.dev).clone()
        if fixed_values is None:
            v[:, self.fixed] = self.lb_full[self.fixed]
        else:
            v[:, self.fixed] = torch.as_tensor(np.asarray(fixed_values, dtype=np.float64), device=self.dev)
        self._set_function_scaling(v)
        x = v[:, self.freeT] / self.d
        # push the start strictly inside the bounds (Ipopt bound_push / bound_frac)
        # per-instance bounds: Ipopt moves a bound by slack_move when a slack falls below machine precision
        lbF, ubF, hasL, hasU = self.lbF.expand(B, -1).clone(), self.ubF.expand(B, -1).clone(), self.hasL, self.hasU
        self._lbI, self._ubI = lbF, ubF
        pl = opt.bound_push * torch.clamp(torch.where(hasL, lbF.abs(), torch.ones_like(lbF)), min=1.0)
        pu = opt.bound_push * torch.clamp(torch.where(hasU, ubF.abs(), torch.ones_like(ubF)), min=1.0)
        both = hasL & hasU
        width = torch.where(both, ubF - lbF, torch.full_like(lbF, np.inf))
        pl = torch.minimum(pl, opt.bound_frac * width)
        pu = torch.minimum(pu, opt.bound_frac * width)
        x = torch.where(hasL, torch.maximum(x, lbF + pl), x)
        x = torch.where(hasU, torch.minimum(x, ubF - pu), x)
        mu = torch.full((B,), opt.mu_init, dtype=torch.float64, device=self.dev)
        sl = torch.where(hasL, x - lbF, torch.ones_like(x))
        su = torch.where(hasU, ubF - x, torch.ones_like(x))
        if opt.bound_mult_init_method == "constant":  # Ipopt's default
            zl = torch.where(hasL, torch.full_like(x, opt.bound_mult_init_val), torch.zeros_like(x))
            zu = torch.where(hasU, torch.full_like(x, opt.bound_mult_init_val), torch.zeros_like(x))
        else:
            zl = torch.where(hasL, mu[:, None] / sl, torch.zeros_like(x))
            zu = torch.where(hasU, mu[:, None] / su, torch.zeros_like(x))
        y = torch.zeros((B, m), dtype=torch.float64, device=self.dev)
        reinit_y = torch.ones((B,), dtype=torch.bool, device=self.dev) if m else torch.zeros((B,), dtype=torch.bool,
                                                                                          device=self.dev)
        delta_w_last = torch.zeros((B,), dtype=torch.float64, device=self.dev)
        done = torch.zeros((B,), dtype=torch.bool, device=self.dev)
        stopped = torch.zeros((B,), dtype=torch.bool, device=self.dev)
        status = torch.full((B,), -1, dtype=torch.int32, device=self.dev)  # Ipopt ApplicationReturnStatus
        iters = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        acc_count = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        err0 = torch.full((B,), np.inf, dtype=torch.float64, device=self.dev)
        filt = torch.full((B, 64, 2), np.inf, dtype=torch.float64, device=self.dev)  # (theta, phi) pairs
        filt[:, :, 1] = -np.inf
        fpos = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        # watchdog state (Ipopt IpBacktrackingLineSearch: StartWatchDog / StopWatchDog)
        wd_short = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        wd_on = torch.zeros((B,), dtype=torch.bool, device=self.dev)
        wd_trial = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        skip_first = torch.zeros((B,), dtype=torch.bool, device=self.dev)
        wd = None
        # Ipopt's filter reset heuristic: successive iterations whose last rejection was the filter's, resets done
        f_succ = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        f_resets = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        # soft restoration: instances taking soft steps, and how many they have taken
        soft_on = torch.zeros((B,), dtype=torch.bool, device=self.dev)
        soft_cnt = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        soft_fac = opt.soft_resto_pderror_reduction_factor if (m and self._phase) else 0.0
        self.soft_steps = 0  # soft-restoration steps taken (all instances)
        # adaptive barrier update: free-mu mode per instance, the (f, theta) filter of its globalisation, mu_max
        adaptive = opt.mu_strategy == "adaptive"
        mfree = torch.full((B,), adaptive, dtype=torch.bool, device=self.dev)
        mfilt = torch.full((B, 64, 2), np.inf, dtype=torch.float64, device=self.dev)
        mfpos = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        mu_max = torch.full((B,), -1.0, dtype=torch.float64, device=self.dev)
        self.mode_switches = torch.zeros((B,), dtype=torch.int64, device=self.dev)  # free -> monotone switches
        mufl = opt.mu_floor()

        self._v_template = v

        def full(xf):  # scaled free variables -> full decision vector
            return self._full(xf)

        it = -1
        while it + 1 < opt.max_iter:
            it += 1
            if time.perf_counter() - t0 > opt.max_wall_time:  # Ipopt max_wall_time
                status = torch.where(done, status, torch.full_like(status, -5))
                break
            vfull = full(x)
            g, jv, f, gF = self._scaled_all(vfull)
            sl = torch.where(hasL, x - lbF, torch.ones_like(x))
            su = torch.where(hasU, ubF - x, torch.ones_like(x))
            if bool(reinit_y.any()):  # least-squares multipliers (Ipopt's constr_mult_init), start and restoration
                y = torch.where(reinit_y[:, None], self._ls_multipliers(jv, gF - zl + zu), y)
                reinit_y = torch.zeros_like(reinit_y)
            # KKT error (Ipopt scaling s_d, s_c)
            jty = self._jt_mul(jv, y)
            rd = gF + jty - zl + zu
            zsum = zl.abs().sum(1) + zu.abs().sum(1) + y.abs().sum(1)
            sd = torch.clamp(zsum / (2 * nf + m), min=opt.s_max) / opt.s_max
            sc = torch.clamp((zl.abs().sum(1) + zu.abs().sum(1)) / (2 * nf), min=opt.s_max) / opt.s_max
            compl_l = torch.where(hasL, sl * zl, torch.zeros_like(x))
            compl_u = torch.where(hasU, su * zu, torch.zeros_like(x))
            e_d = rd.abs().amax(1) / sd
            e_p = g.abs().amax(1) if m else torch.zeros_like(mu)
            e_c0 = torch.maximum(compl_l.abs().amax(1), compl_u.abs().amax(1)) / sc
            err0 = torch.maximum(torch.maximum(e_d, e_p), e_c0)
            # Ipopt's unscaled tests: x = d x_s, g = g_s / sg, the multipliers of the scaled problem over sf
            e_pu = (g / self.sg).abs().amax(1) if m else torch.zeros_like(mu)
            e_du = (rd / self.d).abs().amax(1) / self.sf
            e_cu = torch.maximum(compl_l.abs().amax(1), compl_u.abs().amax(1)) / self.sf
            conv = (err0 <= opt.tol) & (e_pu <= opt.constr_viol_tol) & (e_du <= opt.dual_inf_tol) & \
                (e_cu <= opt.compl_inf_tol)
            acc_ok = (err0 <= opt.acceptable_tol) & (e_pu <= opt.acceptable_constr_viol_tol) & \
                (e_du <= opt.acceptable_dual_inf_tol) & (e_cu <= opt.acceptable_compl_inf_tol)
            acc_count = torch.where(acc_ok, acc_count + 1, torch.zeros_like(acc_count))
            newly = (~done) & (conv | (acc_count >= opt.acceptable_iter))
            status = torch.where(newly, torch.where(conv, 0, 1).to(status.dtype), status)
            done = done | newly
            # an instance whose iterations (restoration-phase ones included) reach max_iter stops, unconverged
            out_of_iters = (~done) & (iters >= opt.max_iter)
            status = torch.where(out_of_iters, torch.full_like(status, -1), status)
            stopped = stopped | out_of_iters
            done = done | out_of_iters
            if bool(done.all()):
                break
            # barrier update.  Adaptive strategy (IpAdaptiveMuUpdate): the globalisation decides the mode first — a
            # free-mode iterate not acceptable to the (f, theta) filter switches to the monotone mode, a monotone-mode
            # iterate acceptable to it returns to the free mode; acceptable iterates enter the filter.  The free mode's
            # mu comes from the quality-function oracle once the KKT matrix is factored (below)
            mu_prev = mu
            mono = ~done
            max_passes = 5  # the monotone strategy's fast decrease (mu_allow_fast_monotone_decrease)
            if adaptive:
                zB = torch.zeros_like(mu)
                theta_c = g.abs().sum(1) if m else zB
                ncomp = int(hasL.sum()) + int(hasU.sum())
                avg = (compl_l.sum(1) + compl_u.sum(1)) / max(ncomp, 1)
                mu_max = torch.where(mu_max < 0, torch.full_like(mu_max, opt.mu_max) if opt.mu_max > 0 else
                                     opt.mu_max_fact * avg, mu_max)
                act = ~done
                ok = (torch.ones_like(done) if opt.adaptive_mu_globalization == "never-monotone-mode"
                      else self._mfilter_ok(mfilt, f, theta_c))
                to_mono = act & mfree & ~ok
                back = act & ~mfree & ok
                mfilt, mfpos = self._mfilter_add(mfilt, mfpos, act & ok, f, theta_c)
                mfree = (mfree | back) & ~to_mono
                mu = torch.where(to_mono, torch.minimum(torch.clamp(opt.adaptive_mu_monotone_init_factor * avg,
                                                                    min=opt.mu_min), mu_max), mu)
                self.mode_switches = self.mode_switches + to_mono.long()
                mono = act & ~mfree & ~to_mono
                max_passes = 1
            # monotone update: while the barrier sub-problem is solved, decrease mu
            for _ in range(max_passes):
                e_cmu = torch.maximum((compl_l - torch.where(hasL, mu[:, None], 0 * mu[:, None])).abs().amax(1),
                                      (compl_u - torch.where(hasU, mu[:, None], 0 * mu[:, None])).abs().amax(1)) / sc
                e_mu = torch.maximum(torch.maximum(e_d, e_p), e_cmu)
                dec = mono & (e_mu <= opt.kappa_eps * mu) & (mu > mufl)
                if not bool(dec.any()):
                    break
                mu = torch.where(dec, torch.clamp(torch.minimum(opt.kappa_mu * mu, mu ** opt.theta_mu), min=mufl), mu)
            # Ipopt restarts the line search's filter whenever mu changes (and so in every free-mode iteration)
            reset_ls = (~done) & (mu != mu_prev) & bool(adaptive or opt.mu_change_resets_filter)
            if adaptive:
                reset_ls = reset_ls | (mfree & ~done)
            if bool(reset_ls.any()):
                filt = torch.where(reset_ls[:, None, None], torch.tensor([np.inf, -np.inf], dtype=torch.float64,
                                                                         device=self.dev), filt)

            W = self._scaled_hess(vfull, y)
            sig = torch.where(hasL, zl / sl, torch.zeros_like(x)) + torch.where(hasU, zu / su, torch.zeros_like(x))
            if adaptive:
                # the Newton step is affine in mu: rhs = [-(grad f + J^T y) + mu cen; -c], cen = 1 / s_L - 1 / s_U.  The
                # free-mode instances solve mu = 0 and cen alone, the oracle picks mu, the step is their combination
                cen_x = torch.where(hasL, 1.0 / sl, torch.zeros_like(x)) - torch.where(hasU, 1.0 / su, torch.zeros_like(x))
                rhs_ax = -(gF + jty)
                osel = mfree & ~done
                murhs = torch.where(osel, torch.zeros_like(mu), mu)
                rhs = torch.cat([rhs_ax + murhs[:, None] * cen_x, -g], dim=1)
                rhs_c = torch.cat([cen_x, torch.zeros_like(g)], dim=1)
                rd2 = (rd * rd).sum(1)
                c2 = (g * g).sum(1) if m else zB
            else:
                bar = torch.where(hasL, mu[:, None] / sl, torch.zeros_like(x)) - torch.where(hasU, mu[:, None] / su,
                                                                                             torch.zeros_like(x))
                rhs_x = -(gF + jty - bar)
                rhs = torch.cat([rhs_x, -g], dim=1)
            # inertia correction by curvature test: increase delta_w until dx^T (W + Sigma + dw) dx > 0
            dw = torch.zeros((B,), dtype=torch.float64, device=self.dev)
            for attempt in range(12):
                dxx = sig + dw[:, None]
                K = self.band.factor(self._kkt_band(W, dxx, jv), self.kl, self.ku)
                sol = self._kkt_solve(K, rhs)
                for _ in range(opt.refine):
                    sol = sol + self._kkt_solve(K, rhs - self._kkt_matvec(W, dxx, jv, sol[:, :nf], sol[:, nf:]))
                if adaptive and bool(osel.any()):
                    solc = self._kkt_solve(K, rhs_c)
                    for _ in range(opt.refine):
                        solc = solc + self._kkt_solve(K, rhs_c - self._kkt_matvec(W, dxx, jv, solc[:, :nf],
                                                                                  solc[:, nf:]))
                    mu_o = self._mu_oracle(osel, sl, su, zl, zu, sol[:, :nf], solc[:, :nf], rd2, c2, avg, mu_max)
                    mu = torch.where(osel, mu_o, mu)
                    sol = torch.where(osel[:, None], sol + mu[:, None] * solc, sol)
                dx, dy = sol[:, :nf], sol[:, nf:]
                curv = self._quad_w(W, dx) + (dxx * dx * dx).sum(1)
                # a zero pivot (LAPACK info != 0) or a non-finite solution counts as wrong inertia: more delta_w
                bad = (~done) & ((curv <= opt.curv_min * (dx * dx).sum(1)) | ~torch.isfinite(curv) |
                                 self.band.singular(K) | ~torch.isfinite(sol).all(1))
                if not bool(bad.any()):
                    break
                first = dw == 0
                dw = torch.where(bad, torch.where(first, torch.where(delta_w_last > 0,
                                                                     torch.clamp(delta_w_last / 3, min=1e-20),
                                                                     torch.full_like(dw, 1e-4)), dw * 8), dw)
            delta_w_last = dw
            tau = torch.clamp(1.0 - mu, min=opt.tau_min)
            if adaptive:  # the final mu's barrier gradient and Newton right-hand side (line search, corrections)
                bar = torch.where(hasL, mu[:, None] / sl, torch.zeros_like(x)) - torch.where(hasU, mu[:, None] / su,
                                                                                             torch.zeros_like(x))
                rhs_x = rhs_ax + mu[:, None] * cen_x
            dzl = torch.where(hasL, mu[:, None] / sl - zl - zl / sl * dx, torch.zeros_like(x))
            dzu = torch.where(hasU, mu[:, None] / su - zu + zu / su * dx, torch.zeros_like(x))
            # fraction to the boundary
            a_p = torch.minimum(self._max_step(sl, dx, hasL, tau), self._max_step(su, -dx, hasU, tau))
            a_z = torch.minimum(self._max_step(zl, dzl, hasL, tau), self._max_step(zu, dzu, hasU, tau))
            # filter line search with one second-order correction (Waechter & Biegler 2006, Ipopt's defaults)
            theta = g.abs().sum(1)
            phi = self._barrier_obj(f, x, mu)
            dphi = (gF - bar).mul(dx).sum(1)
            if it == 0:
                theta_max = 1e4 * torch.clamp(theta, min=1.0)
                theta_min = 1e-4 * torch.clamp(theta, min=1.0)
            # watchdog start: remember this iterate, its direction and its line-search reference values
            wd_start = (~done) & (~wd_on) & (wd_short >= opt.watchdog_shortened_iter_trigger) & \
                (opt.watchdog_shortened_iter_trigger > 0)
            if bool(wd_start.any()):
                cur = dict(x=x, y=y, zl=zl, zu=zu, mu=mu, theta=theta, phi=phi, dphi=dphi, a_p=a_p)
                if wd is None:
                    wd = {k: t.clone() for k, t in cur.items()}
                for k, t in cur.items():
                    c = wd_start.view(-1, *([1] * (t.dim() - 1)))
                    wd[k] = torch.where(c, t, wd[k])
                wd_on = wd_on | wd_start
                wd_trial = torch.where(wd_start, torch.zeros_like(wd_trial), wd_trial)
            if wd is not None:  # in the watchdog, trial points are judged against the watchdog iterate
                r_theta = torch.where(wd_on, wd["theta"], theta)
                r_phi = torch.where(wd_on, wd["phi"], phi)
                r_dphi = torch.where(wd_on, wd["dphi"], dphi)
            else:
                r_theta, r_phi, r_dphi = theta, phi, dphi
            alpha = torch.where(skip_first, 0.5 * a_p, a_p)
            accepted = done | soft_on  # instances taking soft steps skip the line search (TrySoftRestoStep below)
            forced = torch.zeros_like(done)
            armijo_step = torch.zeros_like(done)
            rej_f = torch.zeros_like(done)  # Ipopt's InitThisLineSearch
            x_acc = x.clone()
            dx_acc = dx.clone()
            for ls in range(opt.max_backtrack):
                xt = x + alpha[:, None] * dx
                gt, ft = self._scaled_gf(full(xt))
                a_test = torch.where(wd_on, wd["a_p"], alpha) if wd is not None else alpha
                ok, arm = self._filter_accept(gt, ft, xt, r_theta, r_phi, r_dphi, a_test, mu, theta_max, theta_min,
                                              filt)
                rej_f = rej_f | (self._rejf & ~accepted)
                ok = ok & ~accepted
                if ls == 0:
                    # watchdog iterations take the full step whether or not it is acceptable (no corrections)
                    forced = wd_on & ~ok & ~accepted
                    x_acc = torch.where(forced[:, None], xt, x_acc)
                    accepted = accepted | forced
                    # second-order corrections for rejected full steps that increased the infeasibility: up to
                    # max_soc of them while each cuts the infeasibility by kappa_soc (Ipopt's defaults 4 / 0.99)
                    soc_try = (~accepted) & (~ok) & (gt.abs().sum(1) >= theta) & ~skip_first
                    c_soc = alpha[:, None] * g + gt
                    theta_soc = gt.abs().sum(1)
                    for _ in range(opt.max_soc):
                        if not bool(soc_try.any()):
                            break
                        sol_c = self._kkt_solve(K, torch.cat([rhs_x * alpha[:, None], -c_soc], dim=1))
                        dxc = sol_c[:, :nf]
                        a_c = torch.minimum(self._max_step(sl, dxc, hasL, tau), self._max_step(su, -dxc, hasU, tau))
                        xc = x + a_c[:, None] * dxc
                        gc, fc = self._scaled_gf(full(xc))
                        okc, armc = self._filter_accept(gc, fc, xc, theta, phi, dphi, alpha, mu, theta_max,
                                                        theta_min, filt)
                        rej_f = rej_f | (self._rejf & soc_try & ~accepted)
                        okc = okc & soc_try & (a_c >= 0.99)
                        x_acc = torch.where(okc[:, None], xc, x_acc)
                        dx_acc = torch.where(okc[:, None], (xc - x) / alpha.clamp(min=1e-300)[:, None], dx_acc)
                        armijo_step = torch.where(okc, armc, armijo_step)
                        accepted = accepted | okc
                        theta_c = gc.abs().sum(1)
                        soc_try = soc_try & ~okc & (a_c >= 0.99) & (theta_c <= opt.kappa_soc * theta_soc)
                        theta_soc = theta_c
                        c_soc = a_c[:, None] * c_soc + gc
                x_acc = torch.where(ok[:, None], xt, x_acc)
                armijo_step = torch.where(ok, arm, armijo_step)
                accepted = accepted | ok
                if bool(accepted.all()):
                    break
                alpha = torch.where(accepted, alpha, alpha * 0.5)
            failed = ~accepted
            # watchdog bookkeeping: an acceptable point ends it; after watchdog_trial_iter_max unacceptable full
            # steps the solver returns to the watchdog iterate, and the next line search starts at half its step
            wd_ok = wd_on & accepted & ~forced
            wd_trial = torch.where(forced, wd_trial + 1, wd_trial)
            wd_back = forced & (wd_trial > opt.watchdog_trial_iter_max)
            wd_on = wd_on & ~wd_ok & ~wd_back
            shortened = accepted & ~forced & (alpha < a_p)
            wd_short = torch.where(wd_ok | wd_back | failed | ~shortened, torch.zeros_like(wd_short), wd_short + 1)
            skip_first = wd_back.clone()
            # Ipopt's filter reset heuristic (FilterLSAcceptor::UpdateForNextIteration), before the augmentation
            upd = (~done) & accepted & ~forced & ~soft_on & (f_resets < opt.max_filter_resets)
            f_succ = torch.where(upd, torch.where(rej_f, f_succ + 1, torch.zeros_like(f_succ)), f_succ)
            f_reset = upd & rej_f & (f_succ >= opt.filter_reset_trigger)
            f_succ = torch.where(f_reset, torch.zeros_like(f_succ), f_succ)
            f_resets = f_resets + f_reset.long()
            self.filter_resets = f_resets.cpu().numpy()
            filt = torch.where(f_reset[:, None, None], torch.tensor([np.inf, -np.inf], dtype=torch.float64,
                                                                    device=self.dev), filt)
            # filter augmentation for h-type (non-Armijo) steps
            grow = (~done) & accepted & ~armijo_step & ~forced & ~soft_on
            filt, fpos = self._augment_filter(filt, fpos, grow, theta, phi)
            # a failed search: a feasibility-restoration step (minimum-norm Newton step on g = 0 in the metric
            # Sigma + I, backtracking on ||g||_1 only), then a fresh filter and least-squares multipliers
            x_new = x_acc
            failed = failed & ~done
            soft_acc = torch.zeros_like(done)
            if soft_fac > 0:
                # Ipopt's soft restoration, for the failed searches and the instances already taking soft steps
                was_soft = soft_on & ~done
                soft_cnt = torch.where(was_soft, soft_cnt + 1, soft_cnt)
                over = was_soft & (soft_cnt > opt.max_soft_resto_iters)
                cand = (failed & ~wd_on) | (was_soft & ~over)
                failed = failed | over
                if bool(cand.any()):
                    a_s = torch.minimum(a_p, a_z)
                    xs = x + a_s[:, None] * dx
                    ys, zls, zus = y + a_s[:, None] * dy, zl + a_s[:, None] * dzl, zu + a_s[:, None] * dzu
                    gs, jvs, fs, gFs = self._scaled_all(full(xs))
                    ok_orig, _ = self._filter_accept(gs, fs, xs, theta, phi, dphi, torch.zeros_like(alpha), mu,
                                                     theta_max, theta_min, filt)
                    pd_c = self._pd_error(gF, jv, y, zl, zu, g, x, mu)
                    pd_t = self._pd_error(gFs, jvs, ys, zls, zus, gs, xs, mu)
                    soft_acc = cand & torch.isfinite(pd_t) & (ok_orig | (pd_t <= soft_fac * pd_c))
                    self.soft_steps += int(soft_acc.sum())
                    failed = (failed | cand) & ~soft_acc
                    x_new = torch.where(soft_acc[:, None], xs, x_new)
                    # a step the filter takes ends the soft steps (and augments it, as an h-type step would)
                    filt, fpos = self._augment_filter(filt, fpos, soft_acc & ok_orig, theta, phi)
                    soft_on = torch.where(cand, soft_acc & ~ok_orig, soft_on)
                    wd_short = torch.where(cand, torch.zeros_like(wd_short), wd_short)
                soft_on = soft_on & ~over
                soft_cnt = torch.where(soft_on, soft_cnt, torch.zeros_like(soft_cnt))
            if self._phase:
                # Ipopt: "Restoration phase called at acceptable point" ends the solve, solved to the acceptable level
                at_acc = failed & acc_ok
                status = torch.where(at_acc, torch.ones_like(status), status)
                done = done | at_acc
                failed = failed & ~at_acc
            if bool(failed.any()) and m and self._phase:
                # Ipopt's restoration phase; its iterations count among the solve's.  An instance whose budget is
                # spent does not enter it (and does not move); a phase that fails (its line search, max_resto_iter)
                # or finds a point of local infeasibility stops the instance where it is, as Ipopt's solve stops
                entered = failed & (iters < opt.max_iter)
                xr, zl, zu, filt, fpos, its_r, rexit = self._restoration_phase(failed, x, zl, zu, g, theta, phi, mu,
                                                                                tau, filt, fpos, iters)
                back = entered & ((rexit == self.RS_OK) | (rexit == self.RS_BUDGET) |
                                  ((rexit == self.RS_FAILED) & bool(opt.resto_failure_restart)))
                rstop = entered & ~back
                x_new = torch.where(back[:, None], xr, x_acc)
                iters = iters + its_r + rstop.long()  # a stopped instance takes no step below: count its iteration
                status = torch.where(rstop, torch.where(rexit == self.RS_INFEASIBLE, torch.full_like(status, 2),
                                                        torch.full_like(status, -2)), status)
                done = done | rstop
                stopped = stopped | rstop
                # after the phase: zero constraint multipliers (Ipopt's constr_mult_reset_threshold = 0 ignores the
                # least-squares estimate) and a fresh filter (measured: cfg 5 from 16 perturbed starts converges
                # 13 / 16 with it against 9 / 16 keeping the augmented filter; round-3 probe, in git history at 4131d45)
                y = torch.where(back[:, None], torch.zeros_like(y), y)
                filt = torch.where(back[:, None, None], torch.tensor([np.inf, -np.inf], dtype=torch.float64,
                                                                     device=self.dev), filt)
                alpha = torch.where(failed, torch.zeros_like(alpha), alpha)
            elif bool(failed.any()) and m:
                xr = self._restoration_step(x, g, jv, sig, tau)
                x_new = torch.where(failed[:, None], xr, x_acc)
                filt = torch.where(failed[:, None, None], torch.tensor([np.inf, -np.inf], dtype=torch.float64,
                                                                       device=self.dev), filt)
                reinit_y = reinit_y | failed
                alpha = torch.where(failed, torch.zeros_like(alpha), alpha)  # y and z stay put this iteration
            if soft_fac > 0 and bool(soft_acc.any()):
                alpha = torch.where(soft_acc, a_s, alpha)  # the soft step moves y (and z, below) by the same step
            step = (~done)
            alpha = torch.where(step, alpha, torch.zeros_like(alpha))
            if opt.verbose:  # (and the variable whose bound cuts the primal step most: fraction to the boundary)
                rl = torch.where(hasL & (dx < 0), -tau[:, None] * sl / dx, torch.full_like(dx, np.inf))
                ru = torch.where(hasU & (dx > 0), tau[:, None] * su / dx, torch.full_like(dx, np.inf))
                rr = torch.minimum(rl, ru)[0]
                jb = int(rr.argmin())
                print(f"    blocking v[{int(self.free[jb])}] ({'lower' if bool(rl[0, jb] <= ru[0, jb]) else 'upper'}) "
                      f"ratio {float(rr[jb]):.2e} x {float(x[0, jb] * self.d[jb]):.4e} dx {float(dx[0, jb] * self.d[jb]):.3e}; "
                      f"ratios < 1e-2: {int((rr < 1e-2).sum())}")
                print(f"it {it:3d} f {float(f[0]):.6e} err {float(err0[0]):.3e} e_d {float(e_d[0]):.2e} "
                      f"e_p {float(e_p[0]):.2e} mu {float(mu[0]):.1e} alpha {float(alpha[0]):.2e} "
                      f"a_p {float(a_p[0]):.2e} dw {float(dw[0]):.1e} "
                      f"argmax|rd| v[{int(self.free[int(rd[0].abs().argmax())])}]")
            x = torch.where(step[:, None], x_new, x)
            # updates only where a step is taken and finite (0 * NaN would poison a finished instance for good)
            mv = (alpha > 0) & torch.isfinite(dy).all(1)
            y = torch.where(mv[:, None], y + alpha[:, None] * dy, y)
            az = torch.where(step & ~failed, torch.where(soft_acc, alpha, a_z), torch.zeros_like(a_z))
            mz = (az > 0) & torch.isfinite(dzl).all(1) & torch.isfinite(dzu).all(1)
            zl = torch.where(mz[:, None], zl + az[:, None] * dzl, zl)
            zu = torch.where(mz[:, None], zu + az[:, None] * dzu, zu)
            self._adjust_bounds(x, mu)
            # keep z within [mu / (kappa s), kappa mu / s] (Ipopt kappa_Sigma = 1e10)
            sl = torch.where(hasL, x - lbF, torch.ones_like(x))
            su = torch.where(hasU, ubF - x, torch.ones_like(x))
            zl = torch.where(hasL, torch.clamp(zl, min=mu[:, None] / (1e10 * sl), max=1e10 * mu[:, None] / sl), zl)
            zu = torch.where(hasU, torch.clamp(zu, min=mu[:, None] / (1e10 * su), max=1e10 * mu[:, None] / su), zu)
            if wd is not None and bool(wd_back.any()):  # back to the watchdog iterate
                c = wd_back[:, None]
                x, y = torch.where(c, wd["x"], x), torch.where(c, wd["y"], y)
                zl, zu = torch.where(c, wd["zl"], zl), torch.where(c, wd["zu"], zu)
                mu = torch.where(wd_back, wd["mu"], mu)
            iters = iters + step.long()
        if opt.honor_original_bounds:
            x = torch.minimum(torch.maximum(x, self.lbF0), self.ubF0)  # inf bounds leave x as is
        vfinal = full(x)
        g, f = self._eval_gf(vfinal)
        y = y * self.sg / self.sf[:, None]  # multipliers of the unscaled problem
        if self.dev.type == "cuda":
            torch.cuda.synchronize()
        return IpmResult(v=vfinal.cpu().numpy(), y=y.cpu().numpy(), f=f.cpu().numpy(),
                         converged=(done & ~stopped).cpu().numpy(),
                         iterations=iters.cpu().numpy(), kkt_error=err0.cpu().numpy(),
                         wall_time=time.perf_counter() - t0, n_callbacks=dict(self.calls),
                         status=status.cpu().numpy())

    def _augment_filter(self, filt, fpos, grow, theta, phi):
        """Add (theta, phi) of the instances ``grow`` to their filter (a ring of filt.shape[1] pairs)."""
        torch = self.torch
        slot = torch.arange(filt.shape[1], device=self.dev) == (fpos % filt.shape[1])[:, None]
        filt = torch.where(grow[:, None, None] & slot[:, :, None],
                           torch.stack([(1 - 1e-5) * theta, phi - 1e-5 * theta], dim=1)[:, None, :], filt)
        return filt, fpos + grow.long()

    # ---- adaptive barrier parameter (Ipopt's IpAdaptiveMuUpdate, IpQualityFunctionMuOracle; recalled) -------------
    @staticmethod
    def _mfilter_ok(mfilt, f, theta):
        """Acceptable to the mu globalisation's filter (IpFilter::Acceptable): against every entry (f_i, theta_i),
        f <= f_i or theta < theta_i (empty entries are +inf)."""
        return ((f[:, None] <= mfilt[:, :, 0]) | (theta[:, None] < mfilt[:, :, 1])).all(1)

    def _mfilter_add(self, mfilt, mfpos, on, f, theta):
        """RememberCurrentPointAsAccepted: (f - margin, theta - margin), margin = filter_margin_fact
        min(filter_max_margin, theta), enters the filter of the instances ``on``; entries it dominates leave it.  A ring
        of mfilt.shape[1] slots: the first free slot, else slot mfpos."""
        torch = self.torch
        opt = self.opt
        margin = opt.filter_margin_fact * torch.clamp(theta, max=opt.filter_max_margin)
        fe, te = f - margin, theta - margin
        dom = on[:, None] & (fe[:, None] <= mfilt[:, :, 0]) & (te[:, None] <= mfilt[:, :, 1])
        mfilt = torch.where(dom[:, :, None], torch.full_like(mfilt, np.inf), mfilt)
        free_slot = torch.isinf(mfilt[:, :, 0]) & torch.isinf(mfilt[:, :, 1])
        nslot = mfilt.shape[1]
        first = torch.where(free_slot.any(1), free_slot.long().argmax(1), mfpos % nslot)
        slot = torch.arange(nslot, device=self.dev)[None, :] == first[:, None]
        mfilt = torch.where((on[:, None] & slot)[:, :, None], torch.stack([fe, te], 1)[:, None, :], mfilt)
        return mfilt, mfpos + on.long()

    def _mu_oracle(self, sel, sl, su, zl, zu, dxa, dxc, rd2, c2, avg, mu_max):
        """Ipopt's quality-function mu oracle (QualityFunctionMuOracle::CalculateMu, 2-norm-squared, no centrality or
        balancing term) for the instances ``sel``.  The step for mu = sigma avg (avg: the average complementarity) is
        dx = dxa + mu dxc (affine and unit-centering solutions of the factored KKT system), dz as in the iteration; the
        quality of sigma is the predicted (1 - a_d)^2 |grad L|^2 / n_x + (1 - a_p)^2 |c|^2 / m + |(s + a_p ds)(z + a_d
        dz)|^2 / n_bounds, a_p / a_d the fractions to the boundary (tau = max(tau_min, 1 - mu)).  sigma: if q(1 - 1e-2)
        > q(1) a golden-section search over log sigma in [1, min(sigma_max, mu_max / avg)], else over
        [max(sigma_min, mu_min / avg), 1 - 1e-2] (quality_function_max_section_steps sections, stopping once the
        bracket is within quality_function_section_sigma_tol of its upper end); the best of the two inner points, or
        of an end point never moved.  Returns mu per instance (the others: anything)."""
        torch = self.torch
        opt = self.opt
        hasL, hasU = self.hasL, self.hasU
        nd = max(int(sl.shape[1]), 1)
        nc = int(hasL.sum()) + int(hasU.sum())
        z = torch.zeros_like(sl)

        def q(sig):
            mu = (sig * avg)[:, None]
            dx = dxa + mu * dxc
            dzl = torch.where(hasL, mu / sl - zl - zl / sl * dx, z)
            dzu = torch.where(hasU, mu / su - zu + zu / su * dx, z)
            tau = torch.clamp(1.0 - mu[:, 0], min=opt.tau_min)
            ap = torch.minimum(self._max_step(sl, dx, hasL, tau), self._max_step(su, -dx, hasU, tau))
            ad = torch.minimum(self._max_step(zl, dzl, hasL, tau), self._max_step(zu, dzu, hasU, tau))
            a, d = ap[:, None], ad[:, None]
            cl = torch.where(hasL, (sl + a * dx) * (zl + d * dzl), z)
            cu = torch.where(hasU, (su - a * dx) * (zu + d * dzu), z)
            val = (1.0 - ad) ** 2 * rd2 / nd
            if self.m:
                val = val + (1.0 - ap) ** 2 * c2 / self.m
            if nc:
                val = val + ((cl * cl).sum(1) + (cu * cu).sum(1)) / nc
            return val

        ones = torch.ones_like(avg)
        s1m = 1.0 - max(1e-4, opt.quality_function_section_sigma_tol)
        safe = avg > 0
        avgs = torch.where(safe, avg, ones)
        q1m, q1 = q(s1m * ones), q(ones)
        up = q1m > q1  # the quality decreases beyond sigma = 1
        s_hi = torch.where(up, torch.clamp(mu_max / avgs, max=opt.sigma_max), torch.clamp(opt.mu_min / avgs,
                                                                                           min=opt.sigma_min))
        # bracket [lo, hi] in sigma, with the known end values (-1: unknown)
        lo = torch.where(up, ones, s_hi)
        hi = torch.where(up, s_hi, torch.maximum(s_hi, s1m * ones))
        q_lo = torch.where(up, q1, -ones)
        q_hi = torch.where(up, -ones, q1m)
        trivial = lo >= hi
        sig_triv = torch.where(up, hi, lo)
        a, b = torch.log(lo), torch.log(torch.maximum(hi, lo))
        a0, b0 = a.clone(), b.clone()
        gfac = (3.0 - np.sqrt(5.0)) / 2.0
        m1, m2 = a + gfac * (b - a), a + (1.0 - gfac) * (b - a)
        qm1, qm2 = q(torch.exp(m1)), q(torch.exp(m2))
        live = sel & ~trivial
        for _ in range(opt.quality_function_max_section_steps):
            qs = torch.stack([q_lo, q_hi, qm1, qm2], 1)
            known = qs >= 0
            qmin = torch.where(known, qs, torch.full_like(qs, np.inf)).amin(1)
            qmax = torch.where(known, qs, torch.full_like(qs, -np.inf)).amax(1)
            live = live & (torch.exp(b) - torch.exp(a) >= opt.quality_function_section_sigma_tol * torch.exp(b)) & \
                (1.0 - qmin / qmax >= opt.quality_function_section_qf_tol)
            if not bool(live.any()):
                break
            right = qm1 > qm2  # the minimum is in [m1, b]
            na = torch.where(right, m1, a)
            nq_lo = torch.where(right, qm1, q_lo)
            nb = torch.where(right, b, m2)
            nq_hi = torch.where(right, q_hi, qm2)
            nm1 = torch.where(right, m2, na + gfac * (nb - na))
            nm2 = torch.where(right, na + (1.0 - gfac) * (nb - na), m1)
            qn = q(torch.exp(torch.where(right, nm2, nm1)))
            nqm1 = torch.where(right, qm2, qn)
            nqm2 = torch.where(right, qn, qm1)
            c = live
            a, b, q_lo, q_hi = (torch.where(c, new, old) for new, old in ((na, a), (nb, b), (nq_lo, q_lo), (nq_hi, q_hi)))
            m1, m2, qm1, qm2 = (torch.where(c, new, old) for new, old in ((nm1, m1), (nm2, m2), (nqm1, qm1), (nqm2, qm2)))
        best = torch.where(qm1 < qm2, m1, m2)
        qbest = torch.where(qm1 < qm2, qm1, qm2)
        # an end point never moved competes with the inner points (its value computed if unknown)
        hi_end = b == b0
        lo_end = (a == a0) & ~hi_end
        q_end = torch.where(hi_end, q_hi, q_lo)
        need = (hi_end | lo_end) & (q_end < 0)
        if bool((need & sel & ~trivial).any()):
            q_end = torch.where(need, q(torch.exp(torch.where(hi_end, b, a))), q_end)
        take = (hi_end | lo_end) & (q_end < qbest)
        best = torch.where(take, torch.where(hi_end, b, a), best)
        sig = torch.where(trivial, sig_triv, torch.exp(best))
        mu = torch.clamp(torch.minimum(sig * avg, mu_max), min=opt.mu_min)
        return torch.where(safe, mu, torch.full_like(mu, opt.mu_min))

    def _pd_error(self, gF, jv, y, zl, zu, g, x, mu):
        """Ipopt's primal-dual system error (IpoptCalculatedQuantities::curr_primal_dual_system_error) of the scaled
        problem: (||grad L||_1 + ||c||_1 + sum |s z - mu|) over the number of those terms."""
        torch = self.torch
        hasL, hasU = self.hasL, self.hasU
        sl = torch.where(hasL, x - self._lbI, torch.ones_like(x))
        su = torch.where(hasU, self._ubI - x, torch.ones_like(x))
        rd = gF + self._jt_mul(jv, y) - zl + zu
        cl = torch.where(hasL, (sl * zl - mu[:, None]).abs(), torch.zeros_like(x))
        cu = torch.where(hasU, (su * zu - mu[:, None]).abs(), torch.zeros_like(x))
        n = x.shape[1] + self.m + int(hasL.sum()) + int(hasU.sum())
        return (rd.abs().sum(1) + g.abs().sum(1) + cl.sum(1) + cu.sum(1)) / n

    def _full(self, xf):
        vv = self._v_template.clone()
        vv[:, self.freeT] = xf * self.d
        return vv

    def _ls_multipliers(self, jv, r):
        """y minimising ||r + J^T y||: [[I, J^T], [J, 0]] [w; y] = [-r; 0]; dropped when |y| > 1e3 (Ipopt)."""
        torch = self.torch
        B, nf = self.B, len(self.free)
        K = self.band.factor(self._kkt_band(torch.zeros((B, self.hrF.numel()), dtype=torch.float64, device=self.dev),
                                            torch.ones((B, nf), dtype=torch.float64, device=self.dev), jv),
                             self.kl, self.ku)
        sol = self._kkt_solve(K, torch.cat([-r, torch.zeros((B, self.m), dtype=torch.float64, device=self.dev)], 1))
        y = sol[:, nf:]
        ok = torch.isfinite(y).all(1) & (y.abs().amax(1) <= 1e3)
        return torch.where(ok[:, None], y, torch.zeros_like(y))

    def _restoration_step(self, x, g, jv, sig, tau):
        """Minimum-norm step towards g = 0 ([[Sigma + I, J^T], [J, 0]]), kept inside the bounds by the fraction
        to the boundary and halved until ||g||_1 decreases."""
        torch = self.torch
        B, nf = self.B, len(self.free)
        K = self.band.factor(self._kkt_band(torch.zeros((B, self.hrF.numel()), dtype=torch.float64, device=self.dev),
                                            sig + 1.0, jv), self.kl, self.ku)
        dx = self._kkt_solve(K, torch.cat([torch.zeros((B, nf), dtype=torch.float64, device=self.dev), -g], 1))[:, :nf]
        sl = torch.where(self.hasL, x - self._lbI, torch.ones_like(x))
        su = torch.where(self.hasU, self._ubI - x, torch.ones_like(x))
        a = torch.minimum(self._max_step(sl, dx, self.hasL, tau), self._max_step(su, -dx, self.hasU, tau))
        theta = g.abs().sum(1)
        out = x.clone()
        todo = torch.ones((B,), dtype=torch.bool, device=self.dev)
        for _ in range(20):
            xt = x + a[:, None] * dx
            gt, _ = self._scaled_gf(self._full(xt))
            ok = todo & torch.isfinite(gt).all(1) & (gt.abs().sum(1) < theta)
            out = torch.where(ok[:, None], xt, out)
            todo = todo & ~ok
            if not bool(todo.any()):
                break
            a = a * 0.5
        return out

    RS_OK, RS_FAILED, RS_INFEASIBLE, RS_BUDGET = 1, 2, 3, 4  # how a restoration phase ended (cfx_ipm.hip rs_exit)

    def _restoration_phase(self, on, x, zl, zu, g, theta, phi, mu, tau, filt, fpos, iters):
        """Ipopt's feasibility-restoration phase for the instances ``on`` (their line search failed):
        min rho sum(p + n) + 1/2 sum_i zeta D_i^2 (x_i - x_r,i)^2 s.t. c(x) - p + n = 0, p, n >= 0 and the bounds
        (c the scaled constraints, x_r = x, zeta = sqrt(mu_R), D_i = min(1, 1 / |x_r,i|)), by this interior point
        with its own barrier mu_R, filter and line search; p, n and the bound multipliers' steps are eliminated, so
        the Newton system is the original band KKT with W = Hessian of y^T c + zeta D^2 and the (2,2) block
        -(p / zp + n / zn).  It ends when a point is acceptable to the original filter (augmented with x) with
        ||c||_1 <= required_infeasibility_reduction * theta, when its own sub-problem has converged (a local
        minimiser of the infeasibility), after a failed line search of its own, after max_resto_iter iterations, or
        when the instance's iterations (``iters`` + the phase's) reach max_iter — the budget is per instance: one
        instance's phase does not use up the batch's main iterations.  The exit code (RS_*) says which: the caller
        stops the instances whose phase failed (RS_FAILED: its line search or max_resto_iter) or found local
        infeasibility (RS_INFEASIBLE), as Ipopt does.  On success the original bound multipliers take a Newton step for complementarity over the
        phase's dx (fraction to the boundary; reset to 1 above 1e3); the caller then restarts the constraint
        multipliers from zero and the filter from empty.  The executable specification of
        csrc/cfx_ipm.hip's k_rs_* kernels (which run each instance's phase iterations inside the host's main
        iterations instead of a nested loop: the same per-instance arithmetic).  Returns (x_r, zl, zu, filt, fpos,
        iterations per instance, exit code per instance)."""
        torch = self.torch
        opt = self.opt
        B, nf, m = self.B, len(self.free), self.m
        hasL, hasU = self.hasL, self.hasU
        lbI, ubI = self._lbI, self._ubI
        rho = opt.resto_penalty
        zeros_x = torch.zeros_like(x)
        on = on & (iters < opt.max_iter)
        # the original filter takes the point where the phase starts
        slot = (torch.arange(filt.shape[1], device=self.dev) == (fpos % filt.shape[1])[:, None])[:, :, None]
        filt = torch.where(on[:, None, None] & slot,
                           torch.stack([(1 - 1e-5) * theta, phi - 1e-5 * theta], dim=1)[:, None, :], filt)
        fpos = fpos + on.long()
        th0 = theta
        c = g
        muR = torch.maximum(mu, c.abs().amax(1))
        mR = muR[:, None]
        sR = torch.hypot(mR, rho * c)
        n = torch.where(c > 0, (mR + mR * mR / (sR + rho * c)) / (2 * rho), (mR - rho * c + sR) / (2 * rho))
        p = torch.where(c < 0, (mR + mR * mR / (sR - rho * c)) / (2 * rho), (mR + rho * c + sR) / (2 * rho))
        zp, zn = mR / p, mR / n
        yR = torch.zeros_like(c)
        xR = x.clone()
        xref = x
        rzl = torch.where(hasL, torch.clamp(zl, max=rho), zeros_x)
        rzu = torch.where(hasU, torch.clamp(zu, max=rho), zeros_x)
        rfilt = torch.full((B, filt.shape[1], 2), np.inf, dtype=torch.float64, device=self.dev)
        rfilt[:, :, 1] = -np.inf
        its = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        dwl = torch.zeros((B,), dtype=torch.float64, device=self.dev)
        tmax = tmin = None
        dref = torch.clamp(xref.abs(), min=1.0) ** 2
        of0 = torch.zeros((B,), dtype=torch.float64, device=self.dev)
        rexit = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        rr_last = torch.zeros_like(on)  # the last phase iteration reset p, n (Ipopt's RestoRestorationPhase)

        def pn_closed_form(cc, muR_):
            mR_ = muR_[:, None]
            s_ = torch.hypot(mR_, rho * cc)
            nn_ = torch.where(cc > 0, (mR_ + mR_ * mR_ / (s_ + rho * cc)) / (2 * rho), (mR_ - rho * cc + s_) / (2 * rho))
            pp_ = torch.where(cc < 0, (mR_ + mR_ * mR_ / (s_ - rho * cc)) / (2 * rho), (mR_ + rho * cc + s_) / (2 * rho))
            return pp_, nn_

        def merit(xx, pp, nn, mu_):
            w = mu_.sqrt()[:, None] / dref
            prox = (w * (xx - xref) ** 2).sum(1)
            bad = ((pp <= 0) | (nn <= 0)).any(1)
            lg = (torch.log(torch.clamp(pp, min=1e-300)) + torch.log(torch.clamp(nn, min=1e-300))).sum(1)
            fx = self._barrier_obj(rho * (pp + nn).sum(1) + 0.5 * prox, xx, mu_)
            return torch.where(bad, torch.full_like(fx, np.inf), fx - mu_ * lg)

        for r in range(opt.max_resto_iter):
            if not bool(on.any()):
                break
            vfull = self._full(xR)
            gS, jv, _, _ = self._scaled_all(vfull)
            sl = torch.where(hasL, xR - lbI, torch.ones_like(xR))
            su = torch.where(hasU, ubI - xR, torch.ones_like(xR))
            jty = self._jt_mul(jv, yR)
            w = muR.sqrt()[:, None] / dref
            ed = torch.maximum((w * (xR - xref) + jty - rzl + rzu).abs().amax(1),
                               torch.maximum((rho - yR - zp).abs().amax(1), (rho + yR - zn).abs().amax(1)))
            ep = (gS - p + n).abs().amax(1)
            # the phase's monotone barrier update
            looping = on.clone()
            e_last = torch.full_like(muR, np.inf)
            for _ in range(5):
                mR = muR[:, None]
                ecm = torch.maximum(
                    torch.maximum(torch.where(hasL, (sl * rzl - mR).abs(), zeros_x).amax(1),
                                  torch.where(hasU, (su * rzu - mR).abs(), zeros_x).amax(1)),
                    torch.maximum((p * zp - mR).abs().amax(1), (n * zn - mR).abs().amax(1)))
                e_mu = torch.maximum(torch.maximum(ed, ep), ecm)
                e_last = torch.where(looping, e_mu, e_last)
                dec = looping & (e_mu <= opt.kappa_eps * muR) & (muR > opt.tol / 10)
                looping = dec
                if not bool(dec.any()):
                    break
                muR = torch.where(dec, torch.clamp(torch.minimum(opt.kappa_mu * muR, muR ** opt.theta_mu),
                                                   min=opt.tol / 10), muR)
            # its sub-problem solved without a point the original problem accepts: local infeasibility
            infeas = on & (muR <= opt.tol / 10) & (e_last <= opt.kappa_eps * muR)
            rexit = torch.where(infeas, torch.full_like(rexit, self.RS_INFEASIBLE), rexit)
            on = on & ~infeas
            if not bool(on.any()):
                break
            mR = muR[:, None]
            tauR = torch.clamp(1.0 - muR, min=opt.tau_min)
            w = muR.sqrt()[:, None] / dref
            sig = torch.where(hasL, rzl / sl, zeros_x) + torch.where(hasU, rzu / su, zeros_x)
            bar = torch.where(hasL, mR / sl, zeros_x) - torch.where(hasU, mR / su, zeros_x)
            Sp, Sn = zp / p, zn / n
            ap, an = mR / p - rho + yR, mR / n - rho - yR
            rhs = torch.cat([-(w * (xR - xref) + jty - bar), -(gS - p + n) + ap / Sp - an / Sn], dim=1)
            dc = -(1.0 / Sp + 1.0 / Sn)
            W = self._scaled_hess(vfull, yR, of0)
            dw = torch.zeros((B,), dtype=torch.float64, device=self.dev)
            for _ in range(12):
                dxx = sig + dw[:, None] + w
                K = self.band.factor(self._kkt_band(W, dxx, jv, dc), self.kl, self.ku)
                sol = self._kkt_solve(K, rhs)
                dx, dy = sol[:, :nf], sol[:, nf:]
                curv = self._quad_w(W, dx) + (dxx * dx * dx).sum(1)
                bad = on & ((curv <= opt.curv_min * (dx * dx).sum(1)) | ~torch.isfinite(curv) |
                            self.band.singular(K) | ~torch.isfinite(sol).all(1))
                if not bool(bad.any()):
                    break
                first = dw == 0
                dw = torch.where(bad, torch.where(first, torch.where(dwl > 0, torch.clamp(dwl / 3, min=1e-20),
                                                                     torch.full_like(dw, 1e-4)), dw * 8), dw)
            dwl = dw
            dp, dn = (dy + ap) / Sp, (-dy + an) / Sn
            dzp, dzn = mR / p - zp - Sp * dp, mR / n - zn - Sn * dn
            dzl = torch.where(hasL, mR / sl - rzl - rzl / sl * dx, zeros_x)
            dzu = torch.where(hasU, mR / su - rzu + rzu / su * dx, zeros_x)
            all_m = torch.ones_like(p, dtype=torch.bool)
            a_p = torch.minimum(torch.minimum(self._max_step(sl, dx, hasL, tauR), self._max_step(su, -dx, hasU, tauR)),
                                torch.minimum(self._max_step(p, dp, all_m, tauR), self._max_step(n, dn, all_m, tauR)))
            a_z = torch.minimum(torch.minimum(self._max_step(rzl, dzl, hasL, tauR), self._max_step(rzu, dzu, hasU, tauR)),
                                torch.minimum(self._max_step(zp, dzp, all_m, tauR), self._max_step(zn, dzn, all_m, tauR)))
            thR = (gS - p + n).abs().sum(1)
            phR = merit(xR, p, n, muR)
            dphR = ((w * (xR - xref) - bar) * dx).sum(1) + ((rho - mR / p) * dp + (rho - mR / n) * dn).sum(1)
            if tmax is None:
                tmax, tmin = 1e4 * torch.clamp(thR, min=1.0), 1e-4 * torch.clamp(thR, min=1.0)
            alpha = a_p.clone()
            acc = torch.zeros_like(on)
            arm_acc = torch.zeros_like(on)
            x_a, p_a, n_a = xR.clone(), p.clone(), n.clone()
            g_a = torch.zeros_like(gS)
            f_a = torch.zeros_like(muR)
            for _ in range(opt.max_backtrack):
                xt = xR + alpha[:, None] * dx
                pt, nt = p + alpha[:, None] * dp, n + alpha[:, None] * dn
                gt, ft = self._scaled_gf(self._full(xt))
                ok, arm = self._filter_core((gt - pt + nt).abs().sum(1), merit(xt, pt, nt, muR), thR, phR, dphR, alpha,
                                            tmax, tmin, rfilt)
                ok = ok & on & ~acc
                c1 = ok[:, None]
                x_a, p_a, n_a = torch.where(c1, xt, x_a), torch.where(c1, pt, p_a), torch.where(c1, nt, n_a)
                g_a, f_a = torch.where(c1, gt, g_a), torch.where(ok, ft, f_a)
                arm_acc = torch.where(ok, arm, arm_acc)
                acc = acc | ok
                if not bool((on & ~acc).any()):
                    break
                alpha = torch.where(acc, alpha, alpha * 0.5)
            its = its + on.long()
            # a failed line search of the phase: Ipopt's RestoRestorationPhase — x stays, p and n take their closed
            # form at x (the phase's constraints then hold) and the phase's filter takes the point (below); a second
            # failed search in a row fails the phase
            lsfail = on & ~acc
            rexit = torch.where(lsfail & rr_last, torch.full_like(rexit, self.RS_FAILED), rexit)
            on = on & ~(lsfail & rr_last)
            rr = lsfail & ~rr_last
            if bool(rr.any()):
                pN, nN = pn_closed_form(gS, muR)
                c2 = rr[:, None]
                p, n = torch.where(c2, pN, p), torch.where(c2, nN, n)
                zp, zn = torch.where(c2, mR / p, zp), torch.where(c2, mR / n, zn)
            rr_last = rr
            grow = on & ~arm_acc  # h-type steps, and the points the reset starts from
            rslot = (torch.arange(rfilt.shape[1], device=self.dev) == (r % rfilt.shape[1]))[None, :, None]
            rfilt = torch.where(grow[:, None, None] & rslot,
                                torch.stack([(1 - 1e-5) * thR, phR - 1e-5 * thR], dim=1)[:, None, :], rfilt)
            stepped = on & acc
            c1 = stepped[:, None]
            xR = torch.where(c1, x_a, xR)
            slN = torch.where(hasL, xR - lbI, torch.ones_like(xR))
            suN = torch.where(hasU, ubI - xR, torch.ones_like(xR))
            azc = a_z[:, None]
            rzl = torch.where(c1 & hasL, torch.clamp(rzl + azc * dzl, min=mR / (1e10 * slN), max=1e10 * mR / slN), rzl)
            rzu = torch.where(c1 & hasU, torch.clamp(rzu + azc * dzu, min=mR / (1e10 * suN), max=1e10 * mR / suN), rzu)
            p, n = torch.where(c1, p_a, p), torch.where(c1, n_a, n)
            yR = torch.where(c1, yR + alpha[:, None] * dy, yR)
            zp = torch.where(c1, torch.clamp(zp + azc * dzp, min=mR / (1e10 * p), max=1e10 * mR / p), zp)
            zn = torch.where(c1, torch.clamp(zn + azc * dzn, min=mR / (1e10 * n), max=1e10 * mR / n), zn)
            # exit test on the original problem at the accepted point
            th = g_a.abs().sum(1)
            ph = self._barrier_obj(f_a, xR, mu)
            dominated = ((th[:, None] >= filt[:, :, 0]) & (ph[:, None] >= filt[:, :, 1])).any(1)
            done_r = stepped & torch.isfinite(th) & torch.isfinite(ph) & \
                (th <= opt.required_infeasibility_reduction * th0) & ~dominated
            if bool(done_r.any()):  # the original bound multipliers: Newton step over the phase's whole dx
                sl0 = torch.where(hasL, x - lbI, torch.ones_like(x))
                su0 = torch.where(hasU, ubI - x, torch.ones_like(x))
                d = xR - x
                m0 = mu[:, None]
                dzl0 = torch.where(hasL, m0 / sl0 - zl - zl / sl0 * d, zeros_x)
                dzu0 = torch.where(hasU, m0 / su0 - zu + zu / su0 * d, zeros_x)
                ad = torch.minimum(self._max_step(zl, dzl0, hasL, tau), self._max_step(zu, dzu0, hasU, tau))[:, None]
                zl1 = torch.where(hasL, zl + ad * dzl0, zl)
                zu1 = torch.where(hasU, zu + ad * dzu0, zu)
                big = torch.maximum(zl1.amax(1), zu1.amax(1)) > 1e3
                zl1 = torch.where(big[:, None], hasL.to(zl.dtype).expand_as(zl), zl1)
                zu1 = torch.where(big[:, None], hasU.to(zu.dtype).expand_as(zu), zu1)
                zl = torch.where(done_r[:, None], zl1, zl)
                zu = torch.where(done_r[:, None], zu1, zu)
            if opt.verbose:
                print(f"  resto {r:3d} on {int(on[0])} acc {int(acc[0])} muR {float(muR[0]):.2e} thR {float(thR[0]):.3e} "
                      f"th {float(th[0]):.3e} th0 {float(th0[0]):.3e} dom {int(dominated[0])} a {float(alpha[0]):.2e} "
                      f"ap {float(a_p[0]):.2e} az {float(a_z[0]):.2e} dw {float(dw[0]):.1e} done {int(done_r[0])} ed {float(ed[0]):.2e} "
                      f"ep {float(ep[0]):.2e} emu {float(e_last[0]):.2e}")
            rexit = torch.where(done_r, torch.full_like(rexit, self.RS_OK), rexit)
            budget = on & ~done_r & (iters + its >= opt.max_iter)
            rexit = torch.where(budget, torch.full_like(rexit, self.RS_BUDGET), rexit)
            on = on & ~done_r & ~budget
        # max_resto_iter iterations of the phase: Ipopt's Restoration_Failed
        rexit = torch.where(on, torch.full_like(rexit, self.RS_FAILED), rexit)
        return xR, zl, zu, filt, fpos, its, rexit

    def _kkt_solve(self, K, rhs):
        """Solve with factored KKT K for a natural-order right-hand side (free variables, then g rows)."""
        rb = self.torch.empty_like(rhs)
        rb[:, self.posT] = rhs
        xb = self.band.solve(K, rb)
        return xb[:, self.posT]

    def _max_step(self, s, ds, has, tau):
        torch = self.torch
        ratio = torch.where(has & (ds < 0), -tau[:, None] * s / ds, torch.full_like(s, np.inf))
        return torch.clamp(ratio.amin(1), max=1.0)

    SLACK_MOVE = np.finfo(np.float64).eps ** 0.75  # Ipopt slack_move

    def _safe_slacks(self, x, mu):
        """Slacks to the current bounds, and for those below eps min(1, mu) (a trial point that lands on a bound
        in floating point) the bound moved outwards by slack_move max(1, |bound|) (Ipopt's CalculateSafeSlack /
        AdjustVariableBounds).  Returns (sl, su, lb, ub) with the moved bounds."""
        torch = self.torch
        s_min = np.finfo(np.float64).eps * torch.clamp(mu, max=1.0)[:, None]
        lb, ub = self._lbI, self._ubI
        sl = torch.where(self.hasL, x - lb, torch.ones_like(x))
        su = torch.where(self.hasU, ub - x, torch.ones_like(x))
        ml = self.hasL & (sl < s_min) & (sl >= 0)
        mu_ = self.hasU & (su < s_min) & (su >= 0)
        if bool(ml.any()) or bool(mu_.any()):
            lb = torch.where(ml, lb - self.SLACK_MOVE * torch.clamp(lb.abs(), min=1.0), lb)
            ub = torch.where(mu_, ub + self.SLACK_MOVE * torch.clamp(ub.abs(), min=1.0), ub)
            sl = torch.where(self.hasL, x - lb, sl)
            su = torch.where(self.hasU, ub - x, su)
        return sl, su, lb, ub

    def _adjust_bounds(self, x, mu):
        """Make the bound moves of an accepted point permanent (per instance)."""
        _, _, lb, ub = self._safe_slacks(x, mu)
        self._lbI.copy_(lb)
        self._ubI.copy_(ub)

    def _barrier_obj(self, f, x, mu):
        torch = self.torch
        sl, su, _, _ = self._safe_slacks(x, mu)
        bad = ((sl <= 0) & self.hasL).any(1) | ((su <= 0) & self.hasU).any(1)
        barrier = torch.where(self.hasL, torch.log(torch.clamp(sl, min=1e-300)), torch.zeros_like(x)).sum(1) + \
            torch.where(self.hasU, torch.log(torch.clamp(su, min=1e-300)), torch.zeros_like(x)).sum(1)
        return torch.where(bad, torch.full_like(f, np.inf), f - mu * barrier)

    def _filter_accept(self, gt, ft, xt, theta, phi, dphi, alpha, mu, theta_max, theta_min, filt):
        """Ipopt acceptance test of a trial point: (accepted, by the Armijo/f-type rule)."""
        return self._filter_core(gt.abs().sum(1), self._barrier_obj(ft, xt, mu), theta, phi, dphi, alpha, theta_max,
                                 theta_min, filt)

    def _filter_core(self, tt, pt, theta, phi, dphi, alpha, theta_max, theta_min, filt):
        """The filter test of a trial (tt = ||c||_1, pt = barrier objective) against the current point."""
        torch = self.torch
        opt = self.opt
        finite = torch.isfinite(pt) & torch.isfinite(tt)
        s_phi, s_theta, delta = 2.3, 1.1, 1.0
        switching = (dphi < 0) & (alpha * (-dphi).clamp(min=0) ** s_phi > delta * theta ** s_theta) & (theta <= theta_min)
        # Ipopt's Compare_le(lhs, rhs, base): lhs - rhs <= 10 eps |base|, so that round-off in phi near an optimum
        # does not reject a step
        tol_phi = 10 * np.finfo(np.float64).eps * phi.abs()
        armijo_ok = (pt - phi) - opt.armijo * alpha * dphi <= tol_phi
        suff = (tt - (1 - 1e-5) * theta <= 10 * np.finfo(np.float64).eps * theta) | \
            ((pt - phi) + 1e-5 * theta <= tol_phi)
        in_filter = ((tt[:, None] >= filt[:, :, 0]) & (pt[:, None] >= filt[:, :, 1])).any(1)
        ok = finite & (tt <= theta_max) & ~in_filter & torch.where(switching, armijo_ok, suff)
        # rejected by the filter alone (Ipopt's last_rejection_due_to_filter: the other tests passed)
        self._rejf = finite & (tt <= theta_max) & in_filter & torch.where(switching, armijo_ok, suff)
        return ok, switching & armijo_ok

    def close(self):
        self.h.close()


class GpuBandSolver:
    """Batched band LU of libcfx (cfx_band_lu / cfx_band_lu_solve) on torch's current stream."""

    def factor(self, ab, kl, ku):
        import torch

        from . import _cfx

        ab = ab.contiguous()
        B, n, _ = ab.shape
        ipiv = torch.empty((B, n), dtype=torch.int32, device=ab.device)
        info = torch.empty((B,), dtype=torch.int32, device=ab.device)
        _cfx.band_lu(ab, ipiv, info, kl, ku)
        return (ab, ipiv, info, kl, ku)

    @staticmethod
    def singular(fac):
        """(B,) bool: instances whose factorisation hit an exactly zero pivot (LAPACK info != 0)."""
        return fac[2] != 0

    def solve(self, fac, rhs):
        from . import _cfx

        ab, ipiv, _info, kl, ku = fac
        x = rhs.contiguous().clone()
        _cfx.band_lu_solve(ab, ipiv, kl, ku, x)
        return x


_NATIVE_OPTIONS = ("tol", "max_iter", "acceptable_tol", "acceptable_iter", "mu_init", "bound_relax_factor",
                   "bound_push", "tau_min", "kappa_eps", "kappa_mu", "theta_mu", "s_max", "armijo", "max_backtrack",
                   "delta_c", "curv_min", "max_soc", "kappa_soc", "watchdog_shortened_iter_trigger",
                   "watchdog_trial_iter_max", "limited_memory_max_history", "max_resto_iter", "resto_penalty",
                   "required_infeasibility_reduction", "filter_reset_trigger", "max_filter_resets", "max_wall_time",
                   "print_frequency_time", "soft_resto_pderror_reduction_factor", "max_soft_resto_iters",
                   "resto_failure_restart", "constr_viol_tol", "dual_inf_tol", "compl_inf_tol",
                   "acceptable_constr_viol_tol", "acceptable_dual_inf_tol", "acceptable_compl_inf_tol",
                   "warm_start_bound_push", "warm_start_bound_frac", "warm_start_mult_bound_push", "inertia_test",
                   "mu_max_fact", "mu_max", "mu_min", "adaptive_mu_monotone_init_factor", "sigma_max", "sigma_min",
                   "quality_function_section_sigma_tol", "quality_function_section_qf_tol",
                   "quality_function_max_section_steps", "mu_change_resets_filter", "filter_margin_fact",
                   "filter_max_margin", "nlp_scaling_max_gradient", "nlp_scaling_min_value", "bound_frac",
                   "warm_start_init_point", "honor_original_bounds", "range_scaling", "bound_mult_init_val")
_HESSIAN_APPROXIMATION = {"exact": 0, "limited-memory": 1}
_RESTORATION = {"step": 0, "phase": 1, None: 1}
_ENUMS = {"hessian_approximation": _HESSIAN_APPROXIMATION, "restoration": _RESTORATION,
          "bound_mult_init_method": {"constant": 0, "mu-based": 1}, "mu_strategy": {"monotone": 0, "adaptive": 1},
          "adaptive_mu_globalization": {"obj-constr-filter": 0, "never-monotone-mode": 1},
          "monotone_mu_floor": {"library": 0, "ipopt": 1}, "nlp_scaling_method": {"none": 0, "gradient-based": 1}}


def native_options(opt: IpmOptions) -> dict:
    """cfx_ipm_options fields of ``opt`` (NativeIpm and distributed.ShardedNativeIpm: one mapping, so that the same
    IpmOptions give the same algorithm in both).  BatchedIpm-only options (refine) are refused."""
    opt.__post_init__()
    if opt.refine:
        raise ValueError("the native interior point has no iterative refinement (refine > 0): BatchedIpm only")
    out = {}
    for k in _NATIVE_OPTIONS:
        v = getattr(opt, k)
        out[k] = int(v) if isinstance(v, bool) else v
    for k, table in _ENUMS.items():
        out[k] = table[getattr(opt, k)]
    return out


class NativeIpm:
    """The interior point of :class:`BatchedIpm`, run by libcfx itself (``cfx_ipm_*``, csrc/cfx_ipm.hip): the whole
    iteration stays on the GPU — callbacks, fused barrier-algebra kernels, band assembly, band LU — and the host
    reads a 16-byte counter twice per iteration instead of issuing ~1,500 tensor operations.  Same constructor,
    ``solve`` and result as :class:`BatchedIpm`, which remains the algorithm's executable specification (CPU-testable
    with the oracle, cross-checked against scipy).  Iterative refinement (``refine``) is BatchedIpm-only."""

    def __init__(self, ocp, batch: int = 1, device: int = 0, options: IpmOptions | None = None):
        from . import _cfx

        self.ocp = ocp
        self.B = batch
        self.opt = options or IpmOptions()
        nopt = native_options(self.opt)
        self.h = ocp.nlp(batch=batch, layout="aos", device=device)
        self.n, self.m = self.h.nv, self.h.ng
        lb, ub = ocp.bounds_vector()
        self.fixed = np.where(lb == ub)[0]
        self.free = np.where(lb != ub)[0]
        self.ipm = _cfx.Ipm(self.h, lb, ub, int(getattr(ocp, "n_params", 0) or 0), nopt)
        self.calls = {"eval_all": 0, "eval_h": 0, "eval_g_f": 0, "kkt_factor": 0}

    def solve(self, v0=None, fixed_values=None, warm_start=None):
        """``warm_start``: (y, z_l, z_u) multipliers of the unscaled problem ((B, ng), (B, nv), (B, nv)) for a solve
        with ``warm_start_init_point``; ``last_bound_multipliers`` holds the solve's (z_l, z_u) afterwards."""
        t0 = time.perf_counter()
        if v0 is None:
            v0 = np.tile(self.ocp.initial_guess_vector(), (self.B, 1))
        if warm_start is not None:
            self.ipm.set_warm_start(*warm_start)
        elif self.opt.warm_start_init_point:
            raise ValueError("NativeIpm.solve: warm_start_init_point needs warm_start=(y, z_l, z_u)")
        v, y, f, conv, its, kkt = self.ipm.solve(v0, fixed_values)
        self.last_bound_multipliers = self.ipm.bound_multipliers()
        wall = time.perf_counter() - t0
        st = self.ipm.stats()
        self.calls = {k: int(st[k]) for k in ("eval_all", "eval_h", "eval_g_f", "kkt_factor")}
        self.last_stats = st
        return IpmResult(v=v, y=y, f=f, converged=conv, iterations=its, kkt_error=kkt, wall_time=wall,
                         n_callbacks=dict(self.calls), status=self.ipm.status())

    def close(self):
        self.ipm.close()
        self.h.close()


def solve_ocp(ocp, solver=None, batch: int = 1, device: int = 0, v0=None, **kwargs):
    """`FesOcp.solve`: interior-point solve of `batch` instances (multi-start when v0 differs per row)."""
    opts = apply_solver(IpmOptions(**{k: v for k, v in kwargs.items() if hasattr(IpmOptions, k)}), solver)
    # the product path is libcfx's own solver; BatchedIpm only for what it alone offers (iterative refinement)
    ipm = (BatchedIpm if opts.refine else NativeIpm)(ocp, batch=batch, device=device, options=opts)
    try:
        return ipm.solve(v0)
    finally:
        ipm.close()
