"""Batched primal-dual interior-point driver over the libcfx callbacks (the Ipopt role of the reference's
`ocp.solve(Solver.IPOPT(...))`, SURVEY.md section 3 stack B).

All B instances of one transcribed problem iterate in lockstep on the GPU: the callbacks (g, J_g, f, grad f,
Lagrangian Hessian) come from libcfx in one launch each for the whole batch, the Newton/KKT systems are
assembled densely per instance and solved with batched FP64 LU (torch.linalg on ROCm), and every scalar
decision (step length, barrier update, convergence) is taken per instance with masks.  Dense KKT is the
right shape here: the transcribed FES problems have 40-600 free variables per instance.

Algorithm (Ipopt's, simplified — monotone Fiacco-McCormick barrier, l1-merit backtracking instead of the
filter, curvature-based inertia correction): minimise f(v) - mu sum ln(v - lb) - mu sum ln(ub - v) s.t.
g(v) = 0; fixed variables (lb == ub, e.g. the initial state) are removed; default tol 1e-6 on the scaled
KKT error as Ipopt's `tol`.
"""

from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np


@dataclass
class IpmOptions:
    tol: float = 1e-6
    max_iter: int = 200
    mu_init: float = 0.1
    bound_push: float = 1e-2
    tau_min: float = 0.99
    kappa_eps: float = 10.0
    kappa_mu: float = 0.2
    theta_mu: float = 1.5
    s_max: float = 100.0
    armijo: float = 1e-4
    max_backtrack: int = 30
    delta_c: float = 1e-9
    verbose: bool = False


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


class BatchedIpm:
    """Interior-point solver for B instances of one FesOcp on one GPU."""

    def __init__(self, ocp, batch: int = 1, device: int = 0, options: IpmOptions | None = None, handle=None,
                 torch_device=None):
        """``handle`` / ``torch_device`` let tests drive the same algorithm with another evaluator on the CPU;
        the product path always opens a libcfx handle on GPU ``device``."""
        import torch

        self.torch = torch
        self.ocp = ocp
        self.B = batch
        self.opt = options or IpmOptions()
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
        self.d = torch.where(torch.isfinite(width) & (width < 1.0), width, torch.ones_like(width))
        self.lbF, self.ubF = self.lbF / self.d, self.ubF / self.d
        # gradient-based function scaling (Ipopt nlp_scaling_method): set at the starting point
        self.sf = torch.ones((batch,), dtype=torch.float64, device=self.dev)
        self.sg = torch.ones((batch, h.ng), dtype=torch.float64, device=self.dev)
        jr, jc = h.jac_structure()
        hr, hc = h.hess_structure()
        self.jr, self.jc = torch.as_tensor(jr, device=self.dev).long(), torch.as_tensor(jc, device=self.dev).long()
        self.hr, self.hc = torch.as_tensor(hr, device=self.dev).long(), torch.as_tensor(hc, device=self.dev).long()
        self.calls = {"eval_all": 0, "eval_h": 0, "eval_g_f": 0}

    # ---- callbacks (device, AoS); _scaled_* return the scaled problem in x~ ---------------------------------
    def _scaled_all(self, v):
        g, jac, f, grad = self._eval_all(v)
        gF = grad[:, self.freeT] * self.d * self.sf[:, None]
        JF = self._dense_jac(jac) * self.d[None, None, :] * self.sg[:, :, None]
        return g * self.sg, JF, f * self.sf, gF

    def _scaled_gf(self, v):
        g, f = self._eval_gf(v)
        return g * self.sg, f * self.sf

    def _scaled_hess(self, v, y):
        hv = self._eval_h(v, y * self.sg, self.sf)
        return self._dense_hess(hv) * self.d[None, :, None] * self.d[None, None, :]

    def _set_function_scaling(self, v):
        g, jac, f, grad = self._eval_all(v)
        gF = grad[:, self.freeT] * self.d
        JF = self._dense_jac(jac) * self.d[None, None, :]
        torch = self.torch
        self.sf = torch.clamp(100.0 / torch.clamp(gF.abs().amax(1), min=1e-300), max=1.0)
        self.sg = torch.clamp(100.0 / torch.clamp(JF.abs().amax(2), min=1e-300), max=1.0)

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

    # ---- dense assembly ---------------------------------------------------------------------------------
    def _dense_jac(self, jac):
        J = self.torch.zeros((self.B, self.m, self.n), dtype=self.torch.float64, device=self.dev)
        J[:, self.jr, self.jc] = jac
        return J[:, :, self.freeT]

    def _dense_hess(self, hv):
        torch = self.torch
        H = torch.zeros((self.B, self.n, self.n), dtype=torch.float64, device=self.dev)
        H.index_put_((torch.arange(self.B, device=self.dev)[:, None], self.hr[None, :], self.hc[None, :]), hv,
                     accumulate=True)
        off = self.hr != self.hc
        H.index_put_((torch.arange(self.B, device=self.dev)[:, None], self.hc[off][None, :], self.hr[off][None, :]),
                     hv[:, off], accumulate=True)
        return H[:, self.freeT][:, :, self.freeT]

    # ---- main loop --------------------------------------------------------------------------------------
    def solve(self, v0=None):
        torch = self.torch
        opt = self.opt
        B, nf, m = self.B, len(self.free), self.m
        t0 = time.perf_counter()
        if v0 is None:
            v0 = np.tile(self.ocp.initial_guess_vector(), (B, 1))
        v = torch.as_tensor(np.asarray(v0, dtype=np.float64), device=self.dev).clone()
        v[:, self.fixed] = self.lb_full[self.fixed]
        self._set_function_scaling(v)
        x = v[:, self.freeT] / self.d
        # push the start strictly inside the bounds (Ipopt bound_push / bound_frac)
        lbF, ubF, hasL, hasU = self.lbF, self.ubF, self.hasL, self.hasU
        pl = opt.bound_push * torch.clamp(torch.where(hasL, lbF.abs(), torch.ones_like(lbF)), min=1.0)
        pu = opt.bound_push * torch.clamp(torch.where(hasU, ubF.abs(), torch.ones_like(ubF)), min=1.0)
        both = hasL & hasU
        width = torch.where(both, ubF - lbF, torch.full_like(lbF, np.inf))
        pl = torch.minimum(pl, 0.5 * width)
        pu = torch.minimum(pu, 0.5 * width)
        x = torch.where(hasL, torch.maximum(x, lbF + pl), x)
        x = torch.where(hasU, torch.minimum(x, ubF - pu), x)
        mu = torch.full((B,), opt.mu_init, dtype=torch.float64, device=self.dev)
        sl = torch.where(hasL, x - lbF, torch.ones_like(x))
        su = torch.where(hasU, ubF - x, torch.ones_like(x))
        zl = torch.where(hasL, mu[:, None] / sl, torch.zeros_like(x))
        zu = torch.where(hasU, mu[:, None] / su, torch.zeros_like(x))
        y = torch.zeros((B, m), dtype=torch.float64, device=self.dev)
        delta_w_last = torch.zeros((B,), dtype=torch.float64, device=self.dev)
        done = torch.zeros((B,), dtype=torch.bool, device=self.dev)
        iters = torch.zeros((B,), dtype=torch.int64, device=self.dev)
        err0 = torch.full((B,), np.inf, dtype=torch.float64, device=self.dev)
        I_n = torch.eye(nf, dtype=torch.float64, device=self.dev)
        filt = torch.full((B, 64, 2), np.inf, dtype=torch.float64, device=self.dev)  # (theta, phi) pairs
        filt[:, :, 1] = -np.inf
        fpos = torch.zeros((B,), dtype=torch.int64, device=self.dev)

        def full(xf):  # scaled free variables -> full decision vector
            vv = v.clone()
            vv[:, self.freeT] = xf * self.d
            return vv

        for it in range(opt.max_iter):
            vfull = full(x)
            g, JF, f, gF = self._scaled_all(vfull)
            sl = torch.where(hasL, x - lbF, torch.ones_like(x))
            su = torch.where(hasU, ubF - x, torch.ones_like(x))
            # KKT error (Ipopt scaling s_d, s_c)
            rd = gF + torch.einsum("bmn,bm->bn", JF, y) - zl + zu
            zsum = zl.abs().sum(1) + zu.abs().sum(1) + y.abs().sum(1)
            sd = torch.clamp(zsum / (2 * nf + m), min=opt.s_max) / opt.s_max
            sc = torch.clamp((zl.abs().sum(1) + zu.abs().sum(1)) / (2 * nf), min=opt.s_max) / opt.s_max
            compl_l = torch.where(hasL, sl * zl, torch.zeros_like(x))
            compl_u = torch.where(hasU, su * zu, torch.zeros_like(x))
            e_d = rd.abs().amax(1) / sd
            e_p = g.abs().amax(1) if m else torch.zeros_like(mu)
            e_c0 = torch.maximum(compl_l.abs().amax(1), compl_u.abs().amax(1)) / sc
            err0 = torch.maximum(torch.maximum(e_d, e_p), e_c0)
            newly = (~done) & (err0 <= opt.tol)
            done = done | newly
            if bool(done.all()):
                break
            # barrier update (monotone): while the barrier sub-problem is solved, decrease mu
            for _ in range(5):
                e_cmu = torch.maximum((compl_l - torch.where(hasL, mu[:, None], 0 * mu[:, None])).abs().amax(1),
                                      (compl_u - torch.where(hasU, mu[:, None], 0 * mu[:, None])).abs().amax(1)) / sc
                e_mu = torch.maximum(torch.maximum(e_d, e_p), e_cmu)
                dec = (~done) & (e_mu <= opt.kappa_eps * mu) & (mu > opt.tol / 10)
                if not bool(dec.any()):
                    break
                mu = torch.where(dec, torch.clamp(torch.minimum(opt.kappa_mu * mu, mu ** opt.theta_mu), min=opt.tol / 10),
                                 mu)
            tau = torch.clamp(1.0 - mu, min=opt.tau_min)

            W = self._scaled_hess(vfull, y)
            sig = torch.where(hasL, zl / sl, torch.zeros_like(x)) + torch.where(hasU, zu / su, torch.zeros_like(x))
            bar = torch.where(hasL, mu[:, None] / sl, torch.zeros_like(x)) - torch.where(hasU, mu[:, None] / su,
                                                                                         torch.zeros_like(x))
            rhs_x = -(gF + torch.einsum("bmn,bm->bn", JF, y) - bar)
            rhs = torch.cat([rhs_x, -g], dim=1)
            # inertia correction by curvature test: increase delta_w until dx^T (W + Sigma + dw) dx > 0
            dw = torch.zeros((B,), dtype=torch.float64, device=self.dev)
            for attempt in range(12):
                Kxx = W + torch.diag_embed(sig) + dw[:, None, None] * I_n
                top = torch.cat([Kxx, JF.transpose(1, 2)], dim=2)
                bot = torch.cat([JF, -opt.delta_c * torch.eye(m, dtype=torch.float64, device=self.dev).expand(B, m, m)],
                                dim=2)
                K = torch.cat([top, bot], dim=1)
                sol = torch.linalg.solve(K, rhs)
                dx, dy = sol[:, :nf], sol[:, nf:]
                curv = torch.einsum("bi,bij,bj->b", dx, Kxx, dx)
                bad = (~done) & ((curv <= 1e-12 * (dx * dx).sum(1)) | ~torch.isfinite(curv))
                if not bool(bad.any()):
                    break
                first = dw == 0
                dw = torch.where(bad, torch.where(first, torch.where(delta_w_last > 0,
                                                                     torch.clamp(delta_w_last / 3, min=1e-20),
                                                                     torch.full_like(dw, 1e-4)), dw * 8), dw)
            delta_w_last = dw
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
            alpha = a_p.clone()
            accepted = done.clone()
            armijo_step = torch.zeros_like(done)
            x_acc = x.clone()
            dx_acc = dx.clone()
            for ls in range(opt.max_backtrack):
                xt = x + alpha[:, None] * dx
                gt, ft = self._scaled_gf(full(xt))
                ok, arm = self._filter_accept(gt, ft, xt, theta, phi, dphi, alpha, mu, theta_max, theta_min, filt)
                ok = ok & ~accepted
                if ls == 0:
                    # second-order correction for rejected full steps that increased the infeasibility
                    soc_try = (~accepted) & (~ok) & (gt.abs().sum(1) >= theta)
                    if bool(soc_try.any()):
                        c_soc = alpha[:, None] * g + gt
                        sol_c = torch.linalg.solve(K, torch.cat([rhs_x * alpha[:, None], -c_soc], dim=1))
                        dxc = sol_c[:, :nf]
                        a_c = torch.minimum(self._max_step(sl, dxc, hasL, tau), self._max_step(su, -dxc, hasU, tau))
                        xc = x + a_c[:, None] * dxc
                        gc, fc = self._scaled_gf(full(xc))
                        okc, armc = self._filter_accept(gc, fc, xc, theta, phi, dphi, alpha, mu, theta_max,
                                                        theta_min, filt)
                        okc = okc & soc_try & (a_c >= 0.99)
                        x_acc = torch.where(okc[:, None], xc, x_acc)
                        dx_acc = torch.where(okc[:, None], (xc - x) / alpha.clamp(min=1e-300)[:, None], dx_acc)
                        armijo_step = torch.where(okc, armc, armijo_step)
                        accepted = accepted | okc
                x_acc = torch.where(ok[:, None], xt, x_acc)
                armijo_step = torch.where(ok, arm, armijo_step)
                accepted = accepted | ok
                if bool(accepted.all()):
                    break
                alpha = torch.where(accepted, alpha, alpha * 0.5)
            failed = ~accepted
            # filter augmentation for h-type (non-Armijo) steps
            grow = (~done) & accepted & ~armijo_step
            filt = torch.where(grow[:, None, None] & (torch.arange(filt.shape[1], device=self.dev) ==
                                                      (fpos % filt.shape[1])[:, None])[:, :, None],
                               torch.stack([(1 - 1e-5) * theta, phi - 1e-5 * theta], dim=1)[:, None, :], filt)
            fpos = fpos + grow.long()
            # a failed search takes the shortest step anyway (restoration-free fallback)
            x_new = torch.where(failed[:, None], x + alpha[:, None] * dx, x_acc)
            alpha_eff = torch.where(failed, alpha, torch.where(accepted, alpha, alpha))
            step = (~done)
            alpha = torch.where(step, alpha_eff, torch.zeros_like(alpha_eff))
            if opt.verbose:
                print(f"it {it:3d} f {float(f[0]):.6e} err {float(err0[0]):.3e} e_d {float(e_d[0]):.2e} "
                      f"e_p {float(e_p[0]):.2e} mu {float(mu[0]):.1e} alpha {float(alpha[0]):.2e} "
                      f"a_p {float(a_p[0]):.2e} dw {float(dw[0]):.1e}")
            x = torch.where(step[:, None], x_new, x)
            y = y + alpha[:, None] * dy
            az = torch.where(step, a_z, torch.zeros_like(a_z))
            zl = zl + az[:, None] * dzl
            zu = zu + az[:, None] * dzu
            # keep z within [mu / (kappa s), kappa mu / s] (Ipopt kappa_Sigma = 1e10)
            sl = torch.where(hasL, x - lbF, torch.ones_like(x))
            su = torch.where(hasU, ubF - x, torch.ones_like(x))
            zl = torch.where(hasL, torch.clamp(zl, min=mu[:, None] / (1e10 * sl), max=1e10 * mu[:, None] / sl), zl)
            zu = torch.where(hasU, torch.clamp(zu, min=mu[:, None] / (1e10 * su), max=1e10 * mu[:, None] / su), zu)
            iters = iters + step.long()
        vfinal = full(x)
        g, f = self._eval_gf(vfinal)
        y = y * self.sg / self.sf[:, None]  # multipliers of the unscaled problem
        if self.dev.type == "cuda":
            torch.cuda.synchronize()
        return IpmResult(v=vfinal.cpu().numpy(), y=y.cpu().numpy(), f=f.cpu().numpy(), converged=done.cpu().numpy(),
                         iterations=iters.cpu().numpy(), kkt_error=err0.cpu().numpy(),
                         wall_time=time.perf_counter() - t0, n_callbacks=dict(self.calls))

    def _max_step(self, s, ds, has, tau):
        torch = self.torch
        ratio = torch.where(has & (ds < 0), -tau[:, None] * s / ds, torch.full_like(s, np.inf))
        return torch.clamp(ratio.amin(1), max=1.0)

    def _barrier_obj(self, f, x, mu):
        torch = self.torch
        sl = torch.where(self.hasL, x - self.lbF, torch.ones_like(x))
        su = torch.where(self.hasU, self.ubF - x, torch.ones_like(x))
        bad = ((sl <= 0) & self.hasL).any(1) | ((su <= 0) & self.hasU).any(1)
        barrier = torch.where(self.hasL, torch.log(torch.clamp(sl, min=1e-300)), torch.zeros_like(x)).sum(1) + \
            torch.where(self.hasU, torch.log(torch.clamp(su, min=1e-300)), torch.zeros_like(x)).sum(1)
        return torch.where(bad, torch.full_like(f, np.inf), f - mu * barrier)

    def _filter_accept(self, gt, ft, xt, theta, phi, dphi, alpha, mu, theta_max, theta_min, filt):
        """Ipopt acceptance test of a trial point: (accepted, by the Armijo/f-type rule)."""
        torch = self.torch
        opt = self.opt
        tt = gt.abs().sum(1)
        pt = self._barrier_obj(ft, xt, mu)
        finite = torch.isfinite(pt) & torch.isfinite(tt)
        s_phi, s_theta, delta = 2.3, 1.1, 1.0
        switching = (dphi < 0) & (alpha * (-dphi).clamp(min=0) ** s_phi > delta * theta ** s_theta) & (theta <= theta_min)
        armijo_ok = pt <= phi + opt.armijo * alpha * dphi
        suff = (tt <= (1 - 1e-5) * theta) | (pt <= phi - 1e-5 * theta)
        in_filter = ((tt[:, None] >= filt[:, :, 0]) & (pt[:, None] >= filt[:, :, 1])).any(1)
        ok = finite & (tt <= theta_max) & ~in_filter & torch.where(switching, armijo_ok, suff)
        return ok, switching & armijo_ok

    def _merit(self, f, g, x, mu, nu):
        torch = self.torch
        sl = torch.where(self.hasL, x - self.lbF, torch.ones_like(x))
        su = torch.where(self.hasU, self.ubF - x, torch.ones_like(x))
        bad = ((sl <= 0) & self.hasL).any(1) | ((su <= 0) & self.hasU).any(1)
        barrier = torch.where(self.hasL, torch.log(torch.clamp(sl, min=1e-300)), torch.zeros_like(x)).sum(1) + \
            torch.where(self.hasU, torch.log(torch.clamp(su, min=1e-300)), torch.zeros_like(x)).sum(1)
        phi = f - mu * barrier + nu * g.abs().sum(1)
        return torch.where(bad, torch.full_like(phi, np.inf), phi)

    def close(self):
        self.h.close()


def solve_ocp(ocp, solver=None, batch: int = 1, device: int = 0, v0=None, **kwargs):
    """`FesOcp.solve`: interior-point solve of `batch` instances (multi-start when v0 differs per row)."""
    opts = IpmOptions(**{k: v for k, v in kwargs.items() if hasattr(IpmOptions, k)})
    if solver is not None:
        for k in ("tol", "max_iter"):
            if hasattr(solver, k):
                setattr(opts, k, getattr(solver, k))
    ipm = BatchedIpm(ocp, batch=batch, device=device, options=opts)
    try:
        return ipm.solve(v0)
    finally:
        ipm.close()
