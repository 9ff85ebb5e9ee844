// cfx_hessian.h — Lagrangian Hessian blocks of the multiple-shooting constraints on gfx950.
//
// For interval k, H_k = sum_r lambda_{k,r} d^2 Phi_r / dz^2 over z = (x_k, u_k) (lower triangle, packed
// row-major: entry (i, j), j <= i, at k*nhk + i(i+1)/2 + j).  Second-order forward mode: the RK recursion
// runs on Jet<DJ> numbers (value, DJ first-order and DJ(DJ+1)/2 second-order terms) over a SUBSET of the
// nz directions.  The nz directions are cut into blocks of BS; a task (I, J), I <= J, carries blocks I and
// J (DJ = 2 BS slots) and writes the within-block entries when I == J, the cross entries when I < J, so
// every entry is written exactly once while the per-lane register footprint stays bounded (Hmed has up to
// 5 + 32 directions).  Thread = (instance, interval, task).  Objective terms are added afterwards by
// k_objective_hess.
#pragma once

#include "cfx_kernels.h"

namespace cfx {

// direction slot s of task (I, J) -> global direction, or -1
struct HTask {
    int16_t I, J;
};

// Force / fatigue right-hand side in generic arithmetic (S = double or Jet<D>); same formulas as rhs_force.
template <int MODEL, class S>
CFX_HD void rhs_force_gen(const KParams& P, const S& cn, const S* x, const S& afac, S* f) {
    constexpr bool FAT = is_fatigue(MODEL), PW = is_pw(MODEL);
    const S& F = x[1];
    if constexpr (FAT) {
        const S& A = x[2];
        const S& tau1 = x[3];
        const S& km = x[4];
        const S s = cn / (km + cn);
        const S Aeff = PW ? A * afac : A;
        f[1] = (Aeff * s - F / (tau1 + P.tau2 * s)) * P.mult;
        f[2] = P.alpha_a * F - (A - P.a_fat_rest) * P.inv_tau_fat;
        f[3] = P.alpha_tau1 * F - (tau1 - P.tau1_rest) * P.inv_tau_fat;
        f[4] = P.alpha_km * F - (km - P.km_rest) * P.inv_tau_fat;
    } else {
        const S s = cn / (P.km_rest + cn);
        if constexpr (PW) {
            f[1] = ((P.a_scale * afac) * s - F / (P.tau1_rest + P.tau2 * s)) * P.mult;
        } else {
            f[1] = (P.a_rest * s - F / (P.tau1_rest + P.tau2 * s)) * P.mult;
        }
    }
}

template <int DJ, int TMAX>
struct CsHmedJet {
    const double* coef;
    double lamv[TMAX];
    double l1[DJ], l2[DJ];  // lambda' and lambda'' of the intensity carried by slot s
    int uidx[DJ];
    CFX_HD Jet<DJ> eval(int q) const {
        const double* c = coef + (int64_t)q * TMAX;
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < TMAX; ++i) s += c[i] * lamv[i];
        Jet<DJ> r = jconst<DJ>(s);
#pragma unroll
        for (int d = 0; d < DJ; ++d)
            if (uidx[d] >= 0) {
                const double ci = c[uidx[d]];
                r.g[d] = ci * l1[d];
                r.h[d * (d + 1) / 2 + d] = ci * l2[d];  // intensities act separately: no cross terms
            }
        return r;
    }
};

// GJ: the same launch also writes the continuity rows g and every J_g value of the interval (cfx_eval_all_h, the
// north star's residuals + Jacobian + Hessian in one launch): the jets' first-order parts are the Jacobian columns of
// the task's own block (diagonal tasks, each block's columns written by exactly one thread), task (0, 0) writes the
// g rows and the -1 on x_{k+1}; the calcium row of the Ding families is the affine recursion (cfx_kernels.h).
template <int MODEL, int SCHEME, int DJ, int TMAX, bool GJ>
__global__ void __launch_bounds__(256) k_hessian(const KParams P, const HTask* __restrict__ tasks, int bs,
                                                 const double* __restrict__ V, const double* __restrict__ LAM,
                                                 double* __restrict__ H, double* __restrict__ G,
                                                 double* __restrict__ J) {
    constexpr int NX = nx_of(MODEL);
    constexpr bool LIN = !is_int(MODEL);
    constexpr int S = stages_of(SCHEME);
    using J_t = Jet<DJ>;
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int k = blockIdx.y;
    const HTask task = tasks[blockIdx.z];
    // layout (SoA or 64-instance tiles): element stride ES, per-buffer instance bases
    const int64_t ES = lay_stride(P), vb = lay_base(P, P.nv_tot, b), lb = lay_base(P, P.ng_tot, b),
                  hb = lay_base(P, P.nh_tot, b), jb = lay_base(P, P.nnz_tot, b);
    auto Vat = [&](int64_t e) { return V[vb + e * ES]; };
    const int xo = k * P.nz;

    int gd[DJ];
#pragma unroll
    for (int s = 0; s < DJ; ++s) {
        const int blk = s < bs ? task.I : task.J;
        const int g = blk * bs + (s < bs ? s : s - bs);
        gd[s] = (task.I == task.J && s >= bs) ? -1 : (g < P.nz ? g : -1);
    }
    auto seed = [&](double v, int dir) {
        J_t r = jconst<DJ>(v);
#pragma unroll
        for (int s = 0; s < DJ; ++s)
            if (gd[s] == dir) r.g[s] = 1.0;
        return r;
    };

    J_t x[NX];
#pragma unroll
    for (int r = 0; r < NX; ++r) x[r] = seed(Vat(xo + r), r);
    const J_t cn0 = x[0];

    J_t afac = jconst<DJ>(1.0);
    if constexpr (is_pw(MODEL)) {
        const double pw = Vat(xo + NX);
        const double ex = exp(-(pw - P.pd0) / P.pdt);
        // E = 1 - exp(-(pw - pd0)/pdt): E' = ex/pdt, E'' = -ex/pdt^2
        afac = jchain(seed(pw, NX), 1.0 - ex, ex / P.pdt, -ex / (P.pdt * P.pdt));
    }
    CsHmedJet<DJ, TMAX> csh;
    if constexpr (!LIN) {
        csh.coef = P.tab;
#pragma unroll
        for (int i = 0; i < TMAX; ++i) {
            const double ui = i < P.T ? Vat(xo + NX + i) : P.Is;
            csh.lamv[i] = i < P.T ? P.ar * (tanh(P.bs * (ui - P.Is)) + P.cr) : 0.0;
        }
#pragma unroll
        for (int s = 0; s < DJ; ++s) {
            csh.uidx[s] = -1;
            csh.l1[s] = csh.l2[s] = 0.0;
            if (gd[s] >= NX) {
                const double th = tanh(P.bs * (Vat(xo + gd[s]) - P.Is));
                const double d1 = P.bs * (1.0 - th * th);
                csh.l1[s] = P.ar * d1;
                csh.l2[s] = -2.0 * P.ar * P.bs * th * d1;
                csh.uidx[s] = gd[s] - NX;
            }
        }
    }
    const double* cnb = P.tab + (int64_t)k * P.tstride;
    auto stage = [&](const J_t* xs, int slot, J_t* kk) {
        J_t cn;
        if constexpr (LIN) {
            cn = P.cna[slot] * cn0 + cnb[slot];
        } else {
            cn = xs[0];
            kk[0] = P.inv_tauc * (csh.eval(k * P.Q + slot) - cn);
        }
        rhs_force_gen<MODEL>(P, cn, xs, afac, kk);
    };
    constexpr int R0 = LIN ? 1 : 0;
    const double h = P.h, h2 = 0.5 * P.h, h6 = P.h / 6.0;
    for (int j = 0; j < P.m; ++j) {
        const int slot = j * S;
        J_t k1[NX];
        stage(x, slot, k1);
        if constexpr (SCHEME == 1) {
#pragma unroll
            for (int r = R0; r < NX; ++r) x[r] = x[r] + h * k1[r];
        } else if constexpr (SCHEME == 2) {
            J_t xs[NX], k2[NX];
#pragma unroll
            for (int r = R0; r < NX; ++r) xs[r] = x[r] + h2 * k1[r];
            stage(xs, slot + 1, k2);
#pragma unroll
            for (int r = R0; r < NX; ++r) x[r] = x[r] + h * k2[r];
        } else {
            J_t xs[NX], acc[NX], kk[NX];
#pragma unroll
            for (int r = R0; r < NX; ++r) {
                acc[r] = k1[r];
                xs[r] = x[r] + h2 * k1[r];
            }
#pragma unroll
            for (int sg = 1; sg < 4; ++sg) {
                stage(xs, slot + sg, kk);
                if (sg < 3) {
                    const double c = sg == 1 ? h2 : h;
#pragma unroll
                    for (int r = R0; r < NX; ++r) {
                        acc[r] = acc[r] + 2.0 * kk[r];
                        xs[r] = x[r] + c * kk[r];
                    }
                }
            }
#pragma unroll
            for (int r = R0; r < NX; ++r) x[r] = x[r] + h6 * (acc[r] + kk[r]);
        }
    }
    // the calcium row of the Ding families is affine in cn0: no second-order term

    if constexpr (GJ) {
        const int end = P.m * S;  // the interval end's calcium slot (LIN)
        const int64_t jo = (int64_t)k * P.nnzk;
        if (task.I == task.J) {  // this block's Jacobian columns
#pragma unroll
            for (int sl = 0; sl < DJ; ++sl) {
                const int g = sl < bs ? gd[sl] : -1;
                if (g < 0) continue;
                if constexpr (LIN) {
                    if (g == 0 && P.jpos[0][0] >= 0 && !P.keepc) J[jb + (jo + P.jpos[0][0]) * ES] = P.cna[end];
                }
#pragma unroll
                for (int r = R0; r < NX; ++r) {
                    const int pos = P.jpos[r][g];
                    if (pos >= 0) J[jb + (jo + pos) * ES] = x[r].g[sl];
                }
            }
        }
        if (blockIdx.z == 0) {  // g rows and the -1 on x_{k+1}
            const int xn = (k + 1) * P.nz;
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                const double phi = (LIN && r == 0) ? fma(P.cna[end], cn0.v, cnb[end]) : x[r].v;
                G[lb + (int64_t)(k * P.ngk + r) * ES] = phi - Vat(xn + r);
                if (!P.keepc) J[jb + (jo + P.jneg[r]) * ES] = -1.0;
            }
        }
    }

    double lam[NX];
#pragma unroll
    for (int r = 0; r < NX; ++r) lam[r] = LAM[lb + (int64_t)(k * P.ngk + r) * ES];
    const int64_t ho = (int64_t)k * P.nhk;
#pragma unroll
    for (int s1 = 0; s1 < DJ; ++s1) {
#pragma unroll
        for (int s2 = 0; s2 <= s1; ++s2) {
            const int g1 = gd[s1], g2 = gd[s2];
            if (g1 < 0 || g2 < 0) continue;
            const bool cross = task.I != task.J;
            if (cross && !((s1 >= bs) && (s2 < bs))) continue;  // only (block J, block I) pairs
            double acc = 0.0;
#pragma unroll
            for (int r = R0; r < NX; ++r) acc += lam[r] * x[r].h[s1 * (s1 + 1) / 2 + s2];
            const int i = g1 > g2 ? g1 : g2, jj = g1 > g2 ? g2 : g1;
            H[hb + (ho + i * (i + 1) / 2 + jj) * ES] = acc;
        }
    }
    // x_N has no interval block: its (objective-only) diagonal starts from zero
    if (k == P.N - 1 && blockIdx.z == 0) {
#pragma unroll
        for (int r = 0; r < NX; ++r) H[hb + ((int64_t)P.N * P.nhk + r) * ES] = 0.0;
    }
}

}  // namespace cfx
