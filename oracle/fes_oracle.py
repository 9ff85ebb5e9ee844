"""CPU oracle for the cocofest FES NLP-evaluation hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``cocofest_amd``) imports,
links or executes this module; only ``tests/``, ``__graft_entry__.smoke()`` and
the ``cpu_baseline`` leg of ``bench.py`` may use it, and only as the checker.

It is a plain numpy restatement of the reference algorithm (Ipuch/cocofest
@ 2025-02-24), written from the reference's formulas, with every function
citing the reference file:line it follows.  The reference delegates
transcription to bioptim and evaluation to CasADi (neither vendored nor
installed); the parts that live there are restated from the conventions the
reference's own IVP golden vectors pin down ("validated
semantics"), and are marked "bioptim convention" below.

Parity pinning: the IVP trajectories are checked against the 9 golden vectors
of ``tests/shard1/test_ivp.py`` (copied as data into ``tests/golden/``) and the
formula-level functions against fixtures generated from the reference's own
formula code (``tests/golden/make_golden.py``).  The transcription layout
(decision-vector ordering, continuity sign, Lagrange weighting) is the build's
documented choice; OCP optima are "parity unpinned" by the reference's tests
except config 2 (0 DOF: optimum == forward integration).

Derivatives are computed by the complex-step method (analytic functions
only: exp, tanh, rational), which is independent of the forward-mode dual
numbers used by the HIP kernels; second derivatives are central differences
of complex-step gradients.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from fractions import Fraction
from math import gcd

import numpy as np

# cocofest/models/ding2003.py:394-397 (time placeholder that left-pads the history)
PLACEHOLDER_TIME = -10000000.0
# cocofest/models/hmed2018.py:312-316 (intensity placeholder for padded history)
PLACEHOLDER_INTENSITY = 50.0

MODEL_NAMES = (
    "ding2003",
    "ding2003_with_fatigue",
    "ding2007",
    "ding2007_with_fatigue",
    "hmed2018",
    "hmed2018_with_fatigue",
)


def model_constants(name: str) -> dict:
    """Default constants of each model.

    ding2003.py:51-66, ding2003_with_fatigue.py:50-59, ding2007.py:63-79,
    ding2007_with_fatigue.py:60-69, hmed2018.py:53-63, hmed2018_with_fatigue.py:50-59.
    """
    if name not in MODEL_NAMES:
        raise ValueError(f"Unknown model type: {name}")
    c = dict(tauc=0.020, r0_km_relationship=1.04, a_rest=3009.0, tau1_rest=0.050957, tau2=0.060, km_rest=0.103)
    if name.startswith("ding2007"):
        c.update(a_scale=4920.0, pd0=0.000131405, pdt=0.000194138, tau1_rest=0.060601, tau2=0.001, km_rest=0.137,
                 tauc=0.011)
    if name.startswith("hmed2018"):
        c.update(ar=0.586, bs=0.026, Is=63.1, cr=0.833)
    if name.endswith("with_fatigue"):
        c.update(alpha_a=-4.0 * 10e-2, tau_fat=127.0, alpha_tau1=2.1 * 10e-6, alpha_km=1.9 * 10e-6)
    return c


def n_states(name: str) -> int:
    return 5 if name.endswith("with_fatigue") else 2


def control_kind(name: str) -> str:
    if name.startswith("ding2007"):
        return "pulse_width"  # state_configure.py:256-273, one control per interval
    if name.startswith("hmed2018"):
        return "pulse_intensity"  # state_configure.py:275-292, T controls per interval
    return "none"


def min_pulse_intensity(c: dict) -> float:
    """hmed2018.py:303-310."""
    return np.arctanh(-c["cr"]) / c["bs"] + c["Is"]


def rest_values(name: str, c: dict) -> np.ndarray:
    """standard_rest_values: ding2003.py:81-87, ding2003_with_fatigue.py:73-79,
    ding2007_with_fatigue.py:102-108 (A rests at a_scale), hmed2018_with_fatigue.py:94-100."""
    if not name.endswith("with_fatigue"):
        return np.zeros(2)
    a0 = c["a_scale"] if name.startswith("ding2007") else c["a_rest"]
    return np.array([0.0, 0.0, a0, c["tau1_rest"], c["km_rest"]])


# --------------------------------------------------------------------------------------
# a1 / a2: shooting count and stimulation table
# --------------------------------------------------------------------------------------


def prepare_n_shooting(stim_time, final_time) -> int:
    """cocofest/optimization/fes_ocp.py:192-222 (LCM of the reduced denominators of t_i / T)."""
    tf = Fraction(final_time).limit_denominator()
    n = 1
    for t in stim_time:
        d = (Fraction(t).limit_denominator() / tf).denominator
        n = n * d // gcd(n, d)
    return n


@dataclass
class StimTable:
    rows: np.ndarray  # (N+1, T) stim times per node (numerical_data_timeseries transposed)
    src: np.ndarray  # (N+1, T) index into all_stim of every row entry
    all_stim: list  # history placeholders + previous stims + stims
    stim_idx_at_node: list  # reference's stim_idx_at_node_list
    n_prefix: int  # len(previous_stim after padding)


def stim_table(stim_time, n_shooting, final_time, truncation, previous_stim=None, lookup="exact") -> StimTable:
    """cocofest/models/ding2003.py:394-429.

    For node k (time k*T/N) keep the last ``truncation`` entries of
    [placeholders, previous stims, stims] whose time is <= the node time.
    ``lookup="exact"`` compares in exact rational arithmetic (this matches the
    reference's golden vectors); ``lookup="float"`` is
    the literal float ``<=`` of ding2003.py:411.
    """
    prev = list(previous_stim or [])
    while len(prev) < truncation:
        prev.insert(0, PLACEHOLDER_TIME)
    all_stim = prev + list(stim_time)
    arr = np.array(all_stim, dtype=np.float64)
    n = n_shooting
    node_idx = []
    if lookup == "exact":
        fs = [Fraction(s).limit_denominator() for s in all_stim]
        tf = Fraction(final_time).limit_denominator()
        for k in range(n + 1):
            tk = tf * k / n
            node_idx.append(max(i for i, s in enumerate(fs) if s <= tk))
    else:
        dt = final_time / n
        for k in range(n + 1):
            node_idx.append(int(np.where(arr <= k * dt)[0][-1]))
    rows = np.empty((n + 1, truncation))
    src = np.empty((n + 1, truncation), dtype=np.int64)
    for k, idx in enumerate(node_idx):
        lo = idx + 1 - truncation
        src[k] = np.arange(lo, idx + 1)
        rows[k] = arr[lo: idx + 1]
    node_list = list(range(n + 1))
    stim_idx = [node_list[: idx - truncation + 1][-truncation:] for idx in node_idx]
    return StimTable(rows=rows, src=src, all_stim=all_stim, stim_idx_at_node=stim_idx, n_prefix=len(prev))


# --------------------------------------------------------------------------------------
# a3-a9: right-hand sides
# --------------------------------------------------------------------------------------


def cn_sum(c, t, row, lam=None, legacy_skip_first=False):
    """ding2003.py:200-252 (ri_fun, exp_time_fun, cn_sum_fun); r0 = km_rest + 1.04 (268-272).

    ``row`` has shape (T, ...) broadcastable against ``t``; ``lam`` likewise or None (lambda_i = 1,
    ding2003.py:148-150).  ``legacy_skip_first``: the convention of the revision that wrote the reference's stored
    reaching-task solutions (examples/dynamics/reaching_task/result_file/*.pkl), measured from their calcium
    trajectories (tests/test_reference_solution.py): once a window holds more than one real pulse its first term is
    left out of the sum (the later terms keep their r_i).  Test infrastructure only; the product follows the current
    cn_sum_fun.
    """
    r0 = c["km_rest"] + c["r0_km_relationship"]
    total = 0
    n_real = np.sum(np.asarray(row) > -1e6, axis=0) if legacy_skip_first else None
    for i in range(row.shape[0]):
        if legacy_skip_first and i == row.shape[0] - n_real and n_real > 1:
            continue
        ri = 1 if i == 0 else 1 + (r0 - 1) * np.exp(-(row[i] - row[i - 1]) / c["tauc"])
        term = ri * np.exp(-(t - row[i]) / c["tauc"])
        total = total + (term if lam is None else term * lam[i])
    return total


def lambda_i(c, intensity):
    """hmed2018.py:169-180."""
    return c["ar"] * (np.tanh(c["bs"] * (intensity - c["Is"])) + c["cr"])


def a_calculation(c, a_scale, pulse_width):
    """ding2007.py:172-188."""
    return a_scale * (1 - np.exp(-(pulse_width - c["pd0"]) / c["pdt"]))


def rhs(name, c, t, x, u, row, fl=1.0, fv=1.0, fp=0.0, legacy=False):
    """system_dynamics of the six models.

    ding2003.py:153-198, ding2003_with_fatigue.py:138-240, ding2007.py:121-170,
    ding2007_with_fatigue.py:133-241, hmed2018.py:119-167, hmed2018_with_fatigue.py:124-229.
    x: (nx, ...); u: (nu, ...) or None; row: (T, ...).
    ``legacy``: the conventions of the revision that wrote the reference's stored reaching-task solutions (measured
    from their trajectories, tests/test_reference_solution.py): the calcium sum skips a window's first pulse once it
    holds several (cn_sum), and the fatigue models take r0 from the Km state instead of km_rest.  Test infrastructure
    only; the product follows the current reference.
    """
    fatigue = name.endswith("with_fatigue")
    cn, f = x[0], x[1]
    lam = None
    if name.startswith("hmed2018"):
        lam = [lambda_i(c, u[i]) for i in range(row.shape[0])]
    cs = cn_sum(dict(c, km_rest=x[4]) if (legacy and fatigue) else c, t, row, lam, legacy)
    cn_dot = (1 / c["tauc"]) * cs - (cn / c["tauc"])  # ding2003.py:254-266
    if fatigue:
        a, tau1, km = x[2], x[3], x[4]
    else:
        a = c["a_scale"] if name.startswith("ding2007") else c["a_rest"]
        tau1, km = c["tau1_rest"], c["km_rest"]
    if name.startswith("ding2007"):
        a = a_calculation(c, a, u[0])
    s = cn / (km + cn)
    f_dot = (a * s - (f / (tau1 + c["tau2"] * s))) * (fl * fv + fp)  # ding2003.py:274-311
    parts = [cn_dot, f_dot]
    if fatigue:
        a_rest = c["a_scale"] if name.startswith("ding2007") else c["a_rest"]
        parts.append(-(x[2] - a_rest) / c["tau_fat"] + c["alpha_a"] * f)
        parts.append(-(tau1 - c["tau1_rest"]) / c["tau_fat"] + c["alpha_tau1"] * f)
        parts.append(-(km - c["km_rest"]) / c["tau_fat"] + c["alpha_km"] * f)
    shape = np.broadcast(*parts).shape
    return np.stack([np.broadcast_to(p, shape) for p in parts])


# --------------------------------------------------------------------------------------
# a15 / a16: explicit Runge-Kutta sub-stepping (bioptim convention)
# --------------------------------------------------------------------------------------


def _step(scheme, f, t, h, x):
    """One sub-step.  bioptim convention (validated by the IVP goldens): RK1 = explicit Euler,
    RK2 = explicit midpoint, RK4 = classic with stage times (t, t+h/2, t+h/2, t+h); the control is
    held constant over the interval."""
    if scheme == "RK1":
        return x + h * f(t, x)
    if scheme == "RK2":
        k1 = f(t, x)
        return x + h * f(t + h / 2, x + h / 2 * k1)
    if scheme == "RK4":
        k1 = f(t, x)
        k2 = f(t + h / 2, x + h / 2 * k1)
        k3 = f(t + h / 2, x + h / 2 * k2)
        k4 = f(t + h, x + h * k3)
        return x + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
    raise ValueError(f"unknown scheme {scheme}")


def integrate_interval(name, c, scheme, m, t0, dt, x, u, row, keep_substeps=False):
    """Phi_m(x_k, u_k): m sub-steps of RK-s over [t0, t0 + dt] (bioptim RK integrator)."""
    h = dt / m
    f = lambda t, xx: rhs(name, c, t, xx, u, row)  # noqa: E731
    out = [x] if keep_substeps else None
    for j in range(m):
        x = _step(scheme, f, t0 + j * h, h, x)
        if keep_substeps:
            out.append(x)
    return out if keep_substeps else x


# --------------------------------------------------------------------------------------
# Problem description + NLP callbacks (bioptim multiple shooting, build's layout)
# --------------------------------------------------------------------------------------


@dataclass
class Objective:
    """One quadratic tracking term  weight * c_k * (z_k - target_k)^2  summed over ``nodes``.

    kind "lagrange": c_k = dt (rectangle-left quadrature, bioptim convention, unverified);
    kind "mayer": c_k = 1.  ``var`` = ("x", state index) or ("u", control index).
    fes_ocp.py:531-569 (force tracking: Lagrange TRACK_STATE F, weight 100, Node.ALL;
    end force: Mayer MINIMIZE_STATE F at Node.END, weight 1).
    """

    kind: str
    var: tuple
    weight: float
    target: np.ndarray  # (N+1,) or (N,) per node target
    nodes: list


@dataclass
class Problem:
    name: str
    c: dict
    n_shooting: int
    final_time: float
    truncation: int
    rows: np.ndarray  # (N+1, T)
    scheme: str = "RK1"
    n_steps: int = 10
    n_params: int = 0
    last_stim_idx: list = field(default_factory=list)
    intensity_floor: float = 0.0
    objectives: list = field(default_factory=list)

    @property
    def nx(self):
        return n_states(self.name)

    @property
    def nu(self):
        k = control_kind(self.name)
        return 0 if k == "none" else (1 if k == "pulse_width" else self.truncation)

    @property
    def n_slide(self):
        return self.nu if (self.n_params > 0 and control_kind(self.name) == "pulse_intensity") else 0

    @property
    def nv(self):
        return self.n_shooting * (self.nx + self.nu) + self.nx + self.n_params

    @property
    def ng(self):
        return self.n_shooting * (self.nx + self.n_slide)

    @property
    def dt(self):
        return self.final_time / self.n_shooting

    def x_off(self, k):
        return k * (self.nx + self.nu)

    def u_off(self, k):
        return k * (self.nx + self.nu) + self.nx

    @property
    def p_off(self):
        return self.n_shooting * (self.nx + self.nu) + self.nx

    def unpack(self, v):
        """v: (B, nv) -> X (B, N+1, nx), U (B, N, nu), P (B, n_params)."""
        B = v.shape[0]
        N, nx, nu = self.n_shooting, self.nx, self.nu
        body = v[:, : N * (nx + nu)].reshape(B, N, nx + nu)
        X = np.concatenate([body[:, :, :nx], v[:, None, N * (nx + nu): N * (nx + nu) + nx]], axis=1)
        U = body[:, :, nx:]
        P = v[:, self.p_off:]
        return X, U, P


def _phi_all(pb: Problem, X, U):
    """Phi for every (instance, interval); returns (B, N, nx)."""
    B, N = X.shape[0], pb.n_shooting
    L = B * N
    x = X[:, :N, :].reshape(L, pb.nx).T
    u = U.reshape(L, pb.nu).T if pb.nu else None
    t0 = np.tile(np.arange(N) * pb.dt, B)
    rows = np.tile(pb.rows[:N].T, (1, B))  # (T, L) interval k uses the node-k row
    xe = integrate_interval(pb.name, pb.c, pb.scheme, pb.n_steps, t0, pb.dt, x, u, rows)
    return xe.T.reshape(B, N, pb.nx)


def sliding_window(pb: Problem, P, k):
    """custom_constraints.py:102-119: the last-T intensity parameters up to the last stim at node k,
    left-padded with the minimal intensity; returns (B, T)."""
    idx = pb.last_stim_idx[k]
    cols = [P[:, i] for i in range(idx + 1)]
    while len(cols) < pb.nu:
        cols.insert(0, np.full(P.shape[0], pb.intensity_floor, dtype=P.dtype))
    cols = cols[len(cols) - pb.nu:]
    return np.stack(cols, axis=1)


def eval_g(pb: Problem, v):
    """Constraint vector.  Per interval k: continuity Phi(x_k, u_k) - x_{k+1} (nx rows), then (Hmed with
    intensity parameters) the sliding-window rows u_k - window_k (fes_ocp.py:413-438)."""
    X, U, P = pb.unpack(v)
    cont = _phi_all(pb, X, U) - X[:, 1:, :]
    if not pb.n_slide:
        return cont.reshape(v.shape[0], -1)
    parts = []
    for k in range(pb.n_shooting):
        parts.append(cont[:, k, :])
        parts.append(U[:, k, :] - sliding_window(pb, P, k))
    return np.concatenate(parts, axis=1)


def continuity_blocks(pb: Problem, v, h=1e-30):
    """Dense per-interval Jacobian blocks dPhi_k/d(x_k, u_k): (B, N, nx, nx+nu), by complex step."""
    X, U, _ = pb.unpack(v)
    nz = pb.nx + pb.nu
    out = np.empty((v.shape[0], pb.n_shooting, pb.nx, nz))
    for j in range(nz):
        Xc = X.astype(np.complex128)
        Uc = U.astype(np.complex128)
        if j < pb.nx:
            Xc[:, :-1, j] += 1j * h
        else:
            Uc[:, :, j - pb.nx] += 1j * h
        out[:, :, :, j] = _phi_all(pb, Xc, Uc).imag / h
    return out


def structural_pattern(pb: Problem):
    """Symbolic (CasADi-style) sparsity of dPhi/d(x_k, u_k): the set of z-indices each state of the interval
    end depends on, propagated through the RHS dependencies of a3-a9 and the RK stages.  Returns a list of
    sets, one per state.  Placeholder history terms keep their (numerically zero) structural entries, as a
    symbolic evaluation of cn_sum_fun with the stim times as inputs would."""
    nx, nu = pb.nx, pb.nu
    kind = control_kind(pb.name)
    fatigue = pb.name.endswith("with_fatigue")

    def f(x):
        out = [x[0] | (set(range(nx, nx + nu)) if kind == "pulse_intensity" else set())]
        fdep = x[0] | x[1]
        if fatigue:
            fdep = fdep | x[2] | x[3] | x[4]
        if kind == "pulse_width":
            fdep = fdep | {nx}
        out.append(fdep)
        if fatigue:
            out += [x[2] | x[1], x[3] | x[1], x[4] | x[1]]
        return out

    x = [{r} for r in range(nx)]
    n_stage = {"RK1": 1, "RK2": 2, "RK4": 4}[pb.scheme]
    for _ in range(pb.n_steps):
        k = f(x)
        acc = [set(a) for a in k]
        for _ in range(n_stage - 1):
            k = f([x[r] | k[r] for r in range(nx)])
            acc = [acc[r] | k[r] for r in range(nx)]
        x = [x[r] | acc[r] for r in range(nx)]
    return x


def jac_structure(pb: Problem):
    """Triplet structure (row, col) of J_g, in the build's value order: per interval k, for every
    continuity row r its structurally non-zero (x_k, u_k) entries (ascending) then the -1 on x_{k+1}[r];
    then, after all intervals, the sliding-window entries (+1 on u_k[j], -1 on the parameter it equals)."""
    rows, cols = [], []
    nx, nu, ns = pb.nx, pb.nu, pb.n_slide
    pattern = structural_pattern(pb)
    for k in range(pb.n_shooting):
        g0 = k * (nx + ns)
        for r in range(nx):
            for c in sorted(pattern[r]):
                rows.append(g0 + r)
                cols.append(pb.x_off(k) + c)
            rows.append(g0 + r)
            cols.append(pb.x_off(k + 1) + r)
    if ns:
        for k in range(pb.n_shooting):
            g0 = k * (nx + ns) + nx
            idx = pb.last_stim_idx[k]
            first_param = idx + 1 - nu  # parameter index at window slot 0 (may be < 0: padding)
            for j in range(nu):
                rows.append(g0 + j)
                cols.append(pb.u_off(k) + j)
                pi = first_param + j
                if 0 <= pi <= idx:
                    rows.append(g0 + j)
                    cols.append(pb.p_off + pi)
    return np.array(rows, dtype=np.int64), np.array(cols, dtype=np.int64)


def eval_jac_g(pb: Problem, v):
    """J_g values in ``jac_structure`` order, shape (B, nnz)."""
    blocks = continuity_blocks(pb, v)
    B = v.shape[0]
    pattern = structural_pattern(pb)
    cols = []
    for k in range(pb.n_shooting):
        for r in range(pb.nx):
            cols += [blocks[:, k, r, c] for c in sorted(pattern[r])]
            cols.append(-np.ones(B))
    vals = [np.stack(cols, axis=1)]
    if pb.n_slide:
        sl = []
        for k in range(pb.n_shooting):
            idx = pb.last_stim_idx[k]
            first_param = idx + 1 - pb.nu
            for j in range(pb.nu):
                sl.append(1.0)
                if 0 <= first_param + j <= idx:
                    sl.append(-1.0)
        vals.append(np.tile(np.array(sl), (B, 1)))
    return np.concatenate(vals, axis=1)


def _obj_terms(pb: Problem, v):
    X, U, _ = pb.unpack(v)
    for ob in pb.objectives:
        scale = pb.dt if ob.kind == "lagrange" else 1.0
        kind, idx = ob.var
        for k in ob.nodes:
            z = X[:, k, idx] if kind == "x" else U[:, k, idx]
            off = (pb.x_off(k) if kind == "x" else pb.u_off(k)) + idx
            yield ob.weight * scale, z, ob.target[k], off


def eval_f(pb: Problem, v):
    f = np.zeros(v.shape[0])
    for w, z, tgt, _ in _obj_terms(pb, v):
        f = f + w * (z - tgt) ** 2
    return f


def eval_grad_f(pb: Problem, v):
    g = np.zeros_like(v)
    for w, z, tgt, off in _obj_terms(pb, v):
        g[:, off] += 2 * w * (z - tgt)
    return g


def lagrangian_hessian_blocks(pb: Problem, v, obj_factor, lam, delta=1e-3):
    """Hessian of obj_factor*f + lam^T g restricted to the build's structure:
    per interval k the dense (x_k,u_k) block (B, N, nz, nz) and the x_N diagonal (B, nx).
    The continuity part is a central difference of complex-step gradients of lam_k^T Phi_k (the gradients
    are exact to rounding), Richardson-extrapolated over steps delta and delta/2: O(delta^4) truncation."""
    H1, HN = _lagrangian_hessian_fd(pb, v, obj_factor, lam, delta)
    H2, _ = _lagrangian_hessian_fd(pb, v, obj_factor, lam, delta / 2)
    return (4 * H2 - H1) / 3, HN


def hess_structure(pb: Problem):
    """(row, col) of the Hessian values in the build's packed order (row >= col)."""
    nz = pb.nx + pb.nu
    rows, cols = [], []
    for k in range(pb.n_shooting):
        for i in range(nz):
            for j in range(i + 1):
                rows.append(pb.x_off(k) + i)
                cols.append(pb.x_off(k) + j)
    for r in range(pb.nx):
        rows.append(pb.x_off(pb.n_shooting) + r)
        cols.append(pb.x_off(pb.n_shooting) + r)
    return np.array(rows), np.array(cols)


def hessian_values(pb: Problem, v, obj_factor, lam):
    """Lagrangian Hessian in the build's packed order: per interval the lower triangle (i, j <= i) of the
    (x_k, u_k) block row-major, then the x_N diagonal; shape (B, N*nz(nz+1)/2 + nx)."""
    H, HN = lagrangian_hessian_blocks(pb, v, obj_factor, lam)
    nz = pb.nx + pb.nu
    il, jl = np.tril_indices(nz)
    order = np.argsort(il * (il + 1) // 2 + jl)
    blocks = H[:, :, il[order], jl[order]].reshape(v.shape[0], -1)
    return np.concatenate([blocks, HN], axis=1)


def _lagrangian_hessian_fd(pb: Problem, v, obj_factor, lam, delta):
    B = v.shape[0]
    nx, nu, nz, N = pb.nx, pb.nu, pb.nx + pb.nu, pb.n_shooting
    ng_k = nx + pb.n_slide
    L = lam.reshape(B, N, ng_k)[:, :, :nx]

    def grad_lphi(vv):
        blocks = continuity_blocks(pb, vv)  # (B,N,nx,nz)
        return np.einsum("bkr,bkrc->bkc", L, blocks)

    H = np.zeros((B, N, nz, nz))
    X, U, _ = pb.unpack(v)
    for j in range(nz):
        vp, vm = v.copy(), v.copy()
        offs = [(pb.x_off(k) + j) if j < nx else (pb.u_off(k) + j - nx) for k in range(N)]
        scale = np.maximum(1e-4, np.abs(v[:, offs]))  # relative steps (pulse widths are ~1e-4 s)
        step = delta * scale  # (B, N)
        for kk, off in enumerate(offs):
            vp[:, off] += step[:, kk]
            vm[:, off] -= step[:, kk]
        H[:, :, :, j] = (grad_lphi(vp) - grad_lphi(vm)) / (2 * step[:, :, None])
    H = 0.5 * (H + H.transpose(0, 1, 3, 2))
    obj_factor = np.broadcast_to(np.asarray(obj_factor, dtype=float), (B,))
    HN = np.zeros((B, nx))
    for w, _, _, off in _obj_terms(pb, v):
        k, r = divmod(off, nx + nu)
        if off >= pb.p_off:
            continue
        if k == N:
            HN[:, r] += obj_factor * 2 * w
        else:
            H[:, k, r, r] += obj_factor * 2 * w
    return H, HN


# --------------------------------------------------------------------------------------
# IVP (a16): single shooting, every sub-step returned
# --------------------------------------------------------------------------------------


def ivp_controls(name, table: StimTable, n_shooting, truncation, pulse_width=None, pulse_intensity=None):
    """Per-interval controls of an IvpFes run, (N, nu).

    Ding2007: width of the last pulse at or before the node (ivp_fes.py:344-351).
    Hmed2018: the T intensities aligned with the node's stim row, history placeholders at 50 mA
    (hmed2018.py:312-316; equals ivp_fes.py:324-342 whenever N == n_stim, the golden-vector case).
    """
    kind = control_kind(name)
    if kind == "none":
        return np.zeros((n_shooting, 0))
    n_prefix = table.n_prefix
    if kind == "pulse_width":
        pw = pulse_width if isinstance(pulse_width, (list, tuple, np.ndarray)) else None
        out = np.empty((n_shooting, 1))
        for k in range(n_shooting):
            if pw is not None and len(pw) != 1:
                out[k, 0] = pw[table.stim_idx_at_node[k][-1]]
            else:
                out[k, 0] = pw[0] if pw is not None else pulse_width
        return out
    pi = pulse_intensity
    out = np.empty((n_shooting, truncation))
    for k in range(n_shooting):
        for j in range(truncation):
            s = table.src[k, j] - n_prefix
            if s < 0:
                out[k, j] = PLACEHOLDER_INTENSITY
            elif isinstance(pi, (list, tuple, np.ndarray)):
                out[k, j] = pi[s] if len(pi) != 1 else pi[0]
            else:
                out[k, j] = pi
    return out


def ivp_integrate(name, c, rows, controls, final_time, scheme="RK4", m=10, x0=None):
    """IvpFes.integrate (ivp_fes.py:282-297): sequential propagation from the rest state over the N
    intervals, returning all N*m+1 sub-step samples as (nx, N*m+1)."""
    N = controls.shape[0]
    dt = final_time / N
    x = (rest_values(name, c) if x0 is None else np.asarray(x0, dtype=np.float64)).copy()
    samples = [x]
    for k in range(N):
        u = controls[k] if controls.shape[1] else None
        sub = integrate_interval(name, c, scheme, m, k * dt, dt, x, u, rows[k], keep_substeps=True)
        samples.extend(sub[1:])
        x = sub[-1]
    return np.stack(samples, axis=1)


# --------------------------------------------------------------------------------------
# Bounds (a12) and Fourier target (a13)
# --------------------------------------------------------------------------------------


def state_bounds(name, c):
    """fes_ocp.py:452-499 -> (lb, ub) each (nx, 3) for columns (first node, middle, last)."""
    rest = rest_values(name, c)
    dofs = ["Cn", "F", "A", "Tau1", "Km"][: n_states(name)]
    lo, hi = rest.copy(), rest.copy()
    for i, d in enumerate(dofs):
        if d == "Cn":
            hi[i] = 2
        if d == "F":
            hi[i] = 1000
        elif d in ("Tau1", "Km"):
            hi[i] = 1
        elif d == "A":
            lo[i] = 0
    return np.stack([rest, lo, lo], axis=1), np.stack([rest, hi, hi], axis=1)


def fourier_target(time, force, n_shooting, n_harmonics=50):
    """fourier_approx.py:12-38 evaluated at linspace(0, 1, N+1) as in fes_ocp.py:539-548."""
    from scipy.integrate import trapezoid

    coeffs = []
    for i in range(n_harmonics + 1):
        an = 2.0 * trapezoid(force * np.cos(2 * np.pi * i * time), time)
        bn = 2.0 * trapezoid(force * np.sin(2 * np.pi * i * time), time)
        coeffs.append((an, bn))
    ab = np.array(coeffs)
    x = np.linspace(0, 1, n_shooting + 1)
    out = 0.0
    for n in range(len(ab)):
        out = out + (ab[n, 0] / 2.0 if n == 0 else ab[n, 0] * np.cos(2 * np.pi * n * x) + ab[n, 1] * np.sin(
            2 * np.pi * n * x))
    return out
