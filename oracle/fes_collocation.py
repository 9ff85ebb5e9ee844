"""Direct-collocation transcription of the FES OCPs, restated on the CPU (numpy) — TEST INFRASTRUCTURE ONLY
(the product never imports this module; tests/ and the smoke check use it as the checker).

The reference accepts ``OdeSolver.COLLOCATION`` for OcpFes / IvpFes (cocofest/optimization/fes_ocp.py:334-338,
cocofest/integration/ivp_fes.py:223-227) and hands it to bioptim, which is absent here (SURVEY.md section
8(c)).  This module restates the published Lagrange-basis scheme bioptim implements (one interpolating
polynomial of degree d per shooting interval through the node state and d collocation points, Legendre
(Gauss) or Radau IIA points, controls held constant over the interval):

    tau_0 = 0, tau_1..tau_d = the collocation points on (0, 1]
    l_i(tau) = prod_{r != i} (tau - tau_r) / (tau_i - tau_r)       (Lagrange basis)
    C[i][j] = l_i'(tau_j),  D[i] = l_i(1)
    defect (k, j), j = 1..d:   sum_i C[i][j] x_k^i - dt f(t_k + tau_j dt, x_k^j, u_k) = 0
    continuity k:              sum_i D[i] x_k^i - x_{k+1}^0 = 0

with f the model right-hand side of fes_oracle.rhs (the reference's system_dynamics, a3-a9).  Parity with
bioptim's own collocation is UNPINNED (no bioptim, no reference fixture for it); the build's kernels are
checked against this restatement.

Layout (the build's choice): per interval k, z_k = [x_k^0, x_k^1, ..., x_k^d, u_k] (nx each, then nu), then
x_N, then the Hmed intensity parameters.  Rows per interval: the d defect blocks (nx each), the
continuity block (nx), then (Hmed with parameters) the sliding-window rows.  Interior points share the
node bounds of the intermediate nodes.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import fes_oracle as O


def collocation_points(d: int, method: str = "legendre") -> np.ndarray:
    """The d collocation points on (0, 1]: Gauss-Legendre, or Radau IIA (right end point included)."""
    if d < 1:
        raise ValueError("polynomial degree must be >= 1")
    if method == "legendre":
        x = np.polynomial.legendre.leggauss(d)[0]
    elif method == "radau":
        # right Radau points: roots of P_d(x) - P_{d-1}(x) on [-1, 1]
        c = np.zeros(d + 1)
        c[d] = 1.0
        c[d - 1] = -1.0
        x = np.sort(np.real(np.polynomial.legendre.legroots(c)))
        dc = np.polynomial.legendre.legder(c)
        for _ in range(4):  # Newton polish: companion-matrix roots are only good to ~1e-14
            x[:-1] -= np.polynomial.legendre.legval(x[:-1], c) / np.polynomial.legendre.legval(x[:-1], dc)
        x[-1] = 1.0
    else:
        raise ValueError(f"unknown collocation method {method}")
    return (np.asarray(x) + 1.0) / 2.0


def coefficients(d: int, method: str = "legendre"):
    """(tau (d+1,), C (d+1, d+1) with C[i][j] = l_i'(tau_j), D (d+1,) with D[i] = l_i(1))."""
    tau = np.concatenate([[0.0], collocation_points(d, method)])
    C = np.zeros((d + 1, d + 1))
    D = np.zeros(d + 1)
    idx = range(d + 1)
    for i in idx:
        D[i] = np.prod([(1.0 - tau[r]) / (tau[i] - tau[r]) for r in idx if r != i])
        for j in idx:
            if j == i:  # l_i'(tau_i) = sum_{r != i} 1 / (tau_i - tau_r)
                C[i, j] = sum(1.0 / (tau[i] - tau[r]) for r in idx if r != i)
            else:  # l_i'(tau_j) = prod_{r != i, j} (tau_j - tau_r) / (tau_i - tau_r) / (tau_i - tau_j)
                C[i, j] = np.prod([(tau[j] - tau[r]) / (tau[i] - tau[r]) for r in idx if r not in (i, j)]) / (
                    tau[i] - tau[j])
    return tau, C, D


@dataclass
class ColProblem(O.Problem):
    degree: int = 4
    method: str = "legendre"

    @property
    def nzc(self):
        return (self.degree + 1) * self.nx + self.nu

    @property
    def nv(self):
        return self.n_shooting * self.nzc + self.nx + self.n_params

    @property
    def ngk(self):
        return (self.degree + 1) * self.nx + self.n_slide

    @property
    def ng(self):
        return self.n_shooting * self.ngk

    def x_off(self, k):
        return k * self.nzc

    def xc_off(self, k, j):
        return k * self.nzc + j * self.nx

    def u_off(self, k):
        return k * self.nzc + (self.degree + 1) * self.nx

    @property
    def p_off(self):
        return self.n_shooting * self.nzc + self.nx

    def unpack(self, v):
        """v (B, nv) -> node states X (B, N+1, nx), U (B, N, nu), P (B, n_params)."""
        B, N, nx, nu, d = v.shape[0], self.n_shooting, self.nx, self.nu, self.degree
        body = v[:, : N * self.nzc].reshape(B, N, self.nzc)
        X = np.concatenate([body[:, :, :nx], v[:, None, N * self.nzc: N * self.nzc + nx]], axis=1)
        U = body[:, :, (d + 1) * nx:]
        return X, U, v[:, self.p_off:]

    def unpack_points(self, v):
        """(B, N, d+1, nx): node state and collocation states of every interval."""
        B, N, nx, d = v.shape[0], self.n_shooting, self.nx, self.degree
        return v[:, : N * self.nzc].reshape(B, N, self.nzc)[:, :, : (d + 1) * nx].reshape(B, N, d + 1, nx)

    def pack(self, XC, X_end, U=None, P=None):
        B, N = XC.shape[0], self.n_shooting
        v = np.zeros((B, self.nv), dtype=XC.dtype)
        body = v[:, : N * self.nzc].reshape(B, N, self.nzc)
        body[:, :, : (self.degree + 1) * self.nx] = XC.reshape(B, N, -1)
        if self.nu:
            body[:, :, (self.degree + 1) * self.nx:] = U
        v[:, N * self.nzc: N * self.nzc + self.nx] = X_end
        if self.n_params:
            v[:, self.p_off:] = P
        return v


def _point_rhs(pb: ColProblem, XC, U, j):
    """f at collocation point j (1..d) of every (instance, interval): (B, N, nx)."""
    tau, _, _ = coefficients(pb.degree, pb.method)
    B, N = XC.shape[0], pb.n_shooting
    L = B * N
    x = XC[:, :, j, :].reshape(L, pb.nx).T
    u = U.reshape(L, pb.nu).T if pb.nu else None
    t = np.tile(np.arange(N) * pb.dt + tau[j] * pb.dt, B)
    rows = np.tile(pb.rows[:N].T, (1, B))
    return O.rhs(pb.name, pb.c, t, x, u, rows).T.reshape(B, N, pb.nx)


def eval_g(pb: ColProblem, v):
    _, C, D = coefficients(pb.degree, pb.method)
    XC = pb.unpack_points(v)
    X, U, P = pb.unpack(v)
    d = pb.degree
    blocks = []
    for j in range(1, d + 1):
        poly = np.einsum("i,bkir->bkr", C[:, j], XC)
        blocks.append(poly - pb.dt * _point_rhs(pb, XC, U, j))
    blocks.append(np.einsum("i,bkir->bkr", D, XC) - X[:, 1:, :])
    if pb.n_slide:
        blocks.append(np.stack([U[:, k, :] - O.sliding_window(pb, P, k) for k in range(pb.n_shooting)], axis=1))
    return np.concatenate(blocks, axis=2).reshape(v.shape[0], -1)


def rhs_deps(pb: ColProblem):
    """Structural dependencies of each RHS row on (x (nx), u (nu)) at one point: list of (x set, u set)."""
    nx, nu = pb.nx, pb.nu
    kind = O.control_kind(pb.name)
    fat = pb.name.endswith("with_fatigue")
    deps = [({0}, set(range(nu)) if kind == "pulse_intensity" else set())]
    deps.append(({0, 1} | ({2, 3, 4} if fat else set()), {0} if kind == "pulse_width" else set()))
    if fat:
        deps += [({r, 1}, set()) for r in (2, 3, 4)]
    return deps


def jac_structure(pb: ColProblem):
    """Per interval: defect row (j, r): x_k^0..x_k^d of state r, then the other states of point j it depends
    on (ascending), then its controls (ascending); continuity row r: x_k^0..x_k^d of r, then x_{k+1}^0[r].
    The sliding-window entries follow all intervals (as in the shooting transcription)."""
    rows, cols = [], []
    nx, d = pb.nx, pb.degree
    deps = rhs_deps(pb)
    for k in range(pb.n_shooting):
        g0 = k * pb.ngk
        for j in range(1, d + 1):
            for r in range(nx):
                row = g0 + (j - 1) * nx + r
                for i in range(d + 1):
                    rows.append(row)
                    cols.append(pb.xc_off(k, i) + r)
                for c in sorted(deps[r][0] - {r}):
                    rows.append(row)
                    cols.append(pb.xc_off(k, j) + c)
                for c in sorted(deps[r][1]):
                    rows.append(row)
                    cols.append(pb.u_off(k) + c)
        for r in range(nx):
            row = g0 + d * nx + r
            for i in range(d + 1):
                rows.append(row)
                cols.append(pb.xc_off(k, i) + r)
            rows.append(row)
            cols.append(pb.x_off(k + 1) + r)
    if pb.n_slide:
        nu = pb.nu
        for k in range(pb.n_shooting):
            g0 = k * pb.ngk + (d + 1) * nx
            idx = pb.last_stim_idx[k]
            first = idx + 1 - nu
            for j in range(nu):
                rows.append(g0 + j)
                cols.append(pb.u_off(k) + j)
                if 0 <= first + j <= idx:
                    rows.append(g0 + j)
                    cols.append(pb.p_off + first + j)
    return np.array(rows, dtype=np.int64), np.array(cols, dtype=np.int64)


def _rhs_jacobians(pb: ColProblem, XC, U, j, h=1e-30):
    """Complex-step df/dx (B, N, nx, nx) and df/du (B, N, nx, nu) at point j."""
    B, N, nx, nu = XC.shape[0], pb.n_shooting, pb.nx, pb.nu
    fx = np.empty((B, N, nx, nx))
    fu = np.empty((B, N, nx, nu))
    for c in range(nx):
        Xc = XC.astype(np.complex128)
        Xc[:, :, j, c] += 1j * h
        fx[:, :, :, c] = _point_rhs(pb, Xc, U.astype(np.complex128), j).imag / h
    for c in range(nu):
        Uc = U.astype(np.complex128)
        Uc[:, :, c] += 1j * h
        fu[:, :, :, c] = _point_rhs(pb, XC.astype(np.complex128), Uc, j).imag / h
    return fx, fu


def eval_jac_g(pb: ColProblem, v):
    _, C, D = coefficients(pb.degree, pb.method)
    XC = pb.unpack_points(v)
    _, U, _ = pb.unpack(v)
    B, nx, d = v.shape[0], pb.nx, pb.degree
    deps = rhs_deps(pb)
    jac = [_rhs_jacobians(pb, XC, U, j) for j in range(1, d + 1)]
    vals = []
    for k in range(pb.n_shooting):
        for j in range(1, d + 1):
            fx, fu = jac[j - 1]
            for r in range(nx):
                for i in range(d + 1):
                    val = np.full(B, C[i, j])
                    if i == j:
                        val = val - pb.dt * fx[:, k, r, r]
                    vals.append(val)
                for c in sorted(deps[r][0] - {r}):
                    vals.append(-pb.dt * fx[:, k, r, c])
                for c in sorted(deps[r][1]):
                    vals.append(-pb.dt * fu[:, k, r, c])
        for r in range(nx):
            for i in range(d + 1):
                vals.append(np.full(B, D[i]))
            vals.append(-np.ones(B))
    if pb.n_slide:
        for k in range(pb.n_shooting):
            idx = pb.last_stim_idx[k]
            first = idx + 1 - pb.nu
            for j in range(pb.nu):
                vals.append(np.ones(B))
                if 0 <= first + j <= idx:
                    vals.append(-np.ones(B))
    return np.stack(vals, axis=1)


def eval_f(pb: ColProblem, v):
    return O.eval_f(pb, v)


def eval_grad_f(pb: ColProblem, v):
    return O.eval_grad_f(pb, v)


def hess_structure(pb: ColProblem):
    """Per interval k: the x_k^0 diagonal (objective terms only); for each point j = 1..d the lower triangle
    over x_k^j then the (u_k, x_k^j) block (row u, column x); then the lower triangle over u_k.  Finally the
    x_N diagonal."""
    rows, cols = [], []
    nx, nu, d = pb.nx, pb.nu, pb.degree
    for k in range(pb.n_shooting):
        for r in range(nx):
            rows.append(pb.x_off(k) + r)
            cols.append(pb.x_off(k) + r)
        for j in range(1, d + 1):
            for a in range(nx):
                for b in range(a + 1):
                    rows.append(pb.xc_off(k, j) + a)
                    cols.append(pb.xc_off(k, j) + b)
            for a in range(nu):
                for b in range(nx):
                    rows.append(pb.u_off(k) + a)
                    cols.append(pb.xc_off(k, j) + b)
        for a in range(nu):
            for b in range(a + 1):
                rows.append(pb.u_off(k) + a)
                cols.append(pb.u_off(k) + b)
    for r in range(nx):
        rows.append(pb.x_off(pb.n_shooting) + r)
        cols.append(pb.x_off(pb.n_shooting) + r)
    return np.array(rows, dtype=np.int64), np.array(cols, dtype=np.int64)


def _weighted_point_gradient(pb, XC, U, j, w, h=1e-30):
    """Complex-step gradient over (x^j, u) of phi = sum_r w[b, k, r] f_r(x^j, u): (B, N, nx + nu)."""
    nx, nu = pb.nx, pb.nu
    out = np.empty(XC.shape[:2] + (nx + nu,))
    for c in range(nx + nu):
        Xc = XC.astype(np.complex128)
        Uc = U.astype(np.complex128)
        if c < nx:
            Xc[:, :, j, c] += 1j * h
        else:
            Uc[:, :, c - nx] += 1j * h
        out[:, :, c] = (w * _point_rhs(pb, Xc, Uc, j)).sum(-1).imag / h
    return out


def _point_hessians(pb, XC, U, j, w):
    """Hessian over (x^j, u) of sum_r w_r f_r at point j: central differences of the complex-step gradient with
    relative steps, Richardson-extrapolated (O(delta^4)); (B, N, nz, nz) symmetric."""
    nx, nu = pb.nx, pb.nu
    nz = nx + nu
    H = np.empty(XC.shape[:2] + (nz, nz))
    for c in range(nz):
        base = XC[:, :, j, c] if c < nx else U[:, :, c - nx]
        step = 1e-3 * np.maximum(1e-4, np.abs(base))

        def grad_at(s):
            Xc, Uc = XC.copy(), U.copy()
            if c < nx:
                Xc[:, :, j, c] = Xc[:, :, j, c] + s
            else:
                Uc[:, :, c - nx] = Uc[:, :, c - nx] + s
            return _weighted_point_gradient(pb, Xc, Uc, j, w)

        d1 = (grad_at(step) - grad_at(-step)) / (2 * step)[..., None]
        d2 = (grad_at(step / 2) - grad_at(-step / 2)) / step[..., None]
        H[:, :, :, c] = (4 * d2 - d1) / 3
    return 0.5 * (H + np.swapaxes(H, -1, -2))


def hessian_values(pb: ColProblem, v, obj_factor, lam):
    """Values of obj_factor * Hess(f) + sum lam * Hess(g) in ``hess_structure`` order, (B, nnz)."""
    XC = pb.unpack_points(v)
    _, U, _ = pb.unpack(v)
    B, N, nx, nu, d = v.shape[0], pb.n_shooting, pb.nx, pb.nu, pb.degree
    L = lam.reshape(B, N, pb.ngk)
    pts = [_point_hessians(pb, XC, U, j, -pb.dt * L[:, :, (j - 1) * nx: j * nx]) for j in range(1, d + 1)]
    # objective diagonal (quadratic tracking terms)
    diag = np.zeros((B, pb.nv))
    for w, _, _, off in O._obj_terms(pb, v):
        diag[:, off] += 2 * w * obj_factor
    vals = []
    for k in range(N):
        for r in range(nx):
            vals.append(diag[:, pb.x_off(k) + r])
        for j in range(1, d + 1):
            Hj = pts[j - 1][:, k]
            for a in range(nx):
                for b in range(a + 1):
                    vals.append(Hj[:, a, b])
            for a in range(nu):
                for b in range(nx):
                    vals.append(Hj[:, nx + a, b])
        Huu = sum(pts[j - 1][:, k, nx:, nx:] for j in range(1, d + 1)) if nu else None
        for a in range(nu):
            for b in range(a + 1):
                extra = diag[:, pb.u_off(k) + a] if a == b else 0.0
                vals.append(Huu[:, a, b] + extra)
    for r in range(nx):
        vals.append(diag[:, pb.x_off(N) + r])
    return np.stack(vals, axis=1)
