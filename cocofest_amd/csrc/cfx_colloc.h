// cfx_colloc.h — direct-collocation transcription of the FES OCPs on gfx950 (bioptim OdeSolver.COLLOCATION,
// the option the reference accepts at cocofest/optimization/fes_ocp.py:334-338).
//
// Per interval k the decision block is z_k = [x_k^0, x_k^1, ..., x_k^d, u_k]; with tau_0 = 0 and the d
// Legendre / Radau points tau_j, C[i][j] = l_i'(tau_j) and D[i] = l_i(1) of the Lagrange basis:
//   defect (k, j), j = 1..d :  sum_i C[i][j] x_k^i - dt f(t_k + tau_j dt, x_k^j, u_k)
//   continuity k            :  sum_i D[i] x_k^i - x_{k+1}^0
// Unlike multiple shooting there is no recursion: each point costs ONE right-hand side and its partials, and
// most Jacobian entries are the constants C and D.  Thread = (instance, interval); the collocation states
// are read straight from HBM (L1/L2 serve the d re-reads of the polynomial sums).  The calcium sum at every
// point is precomputed on the host like the RK stage sums (tab[k*d + j-1]: the value for Ding, the Hmed
// coefficient row otherwise).
//
// J_g value order per interval (mirrored by the host structure): for j = 1..d, r = 0..nx-1 the defect row
// [x^0_r .. x^d_r, the other states of point j it depends on (ascending), its controls (ascending)]; then
// the continuity rows [x^0_r .. x^d_r, the -1 on x_{k+1}^0_r].
// Hessian value order per interval: the x_k^0 diagonal (objective terms only), for each point the lower
// triangle over x_k^j and the (u_k, x_k^j) block, then the lower triangle over u_k.
#pragma once

#include "cfx_hessian.h"
#include "cfx_kernels.h"

namespace cfx {

// states each RHS row depends on at one point (bit c = state c): cn <- cn; F <- cn, F (+ A, Tau1, Km);
// A / Tau1 / Km <- itself, F
constexpr uint32_t col_xdeps(int model, int r) {
    return r == 0 ? 1u : (r == 1 ? (is_fatigue(model) ? 0x1Fu : 0x3u) : ((1u << r) | 2u));
}
// controls each RHS row depends on: the calcium row on every Hmed intensity, the force row on the pulse width
constexpr int col_udeps(int model, int r, int nu) {
    return r == 0 ? (is_int(model) ? nu : 0) : ((r == 1 && is_pw(model)) ? 1 : 0);
}
constexpr int col_rowlen(int model, int r, int deg, int nu) {
    return deg + 1 + __builtin_popcount(col_xdeps(model, r) & ~(1u << r)) + col_udeps(model, r, nu);
}

// DEG > 0: the degree is a compile-time constant and every input of the interval (x^0..x^d, x_{k+1}, the
// controls) is loaded into registers before the first store — on CDNA vmcnt counts stores too, so a load
// issued after stores waits for them; DEG == 0: any degree, states re-read from memory per point.
template <int MODEL, int TMAX, int DEG>
__global__ void __launch_bounds__(256) k_colloc(const KParams P, const double* __restrict__ V, double* __restrict__ G,
                                                double* __restrict__ J) {
    constexpr int NX = nx_of(MODEL);
    constexpr bool PW = is_pw(MODEL), HM = is_int(MODEL);
    constexpr int DD = NX + (PW ? 1 : 0);  // directions of the RHS partials: the point's states (+ pulse width)
    constexpr int XS = DEG > 0 ? DEG + 1 : 1;
    constexpr int UN = DEG > 0 ? DEG + 1 : 1;  // unroll factor of the point / basis loops
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int k = blockIdx.y;
    const int d = DEG > 0 ? DEG : P.deg;
    const double* Vb = V + b;
    const int64_t xo = (int64_t)k * P.nz;
    auto ld = [&](int64_t e) { return Vb[(xo + e) * B]; };

    double xs[XS][NX], xn[NX];
    if constexpr (DEG > 0) {
#pragma unroll
        for (int i = 0; i <= DEG; ++i)
#pragma unroll
            for (int r = 0; r < NX; ++r) xs[i][r] = ld(i * NX + r);
    }
#pragma unroll
    for (int r = 0; r < NX; ++r) xn[r] = Vb[((int64_t)(k + 1) * P.nz + r) * B];
    auto X = [&](int i, int r) { return DEG > 0 ? xs[i][r] : ld(i * NX + r); };

    Amp amp{1.0, 0.0, -1};
    double lam[TMAX], lamd[TMAX];
    if constexpr (PW) {
        const double ex = exp(-(ld(P.uoff) - P.pd0) / P.pdt);
        amp.E = 1.0 - ex;
        amp.dE = ex / P.pdt;
        amp.pwdir = NX;
    }
    if constexpr (HM) {
#pragma unroll
        for (int i = 0; i < TMAX; ++i) {
            const double th = i < P.T ? tanh(P.bs * (ld(P.uoff + i) - P.Is)) : 0.0;
            lam[i] = i < P.T ? P.ar * (th + P.cr) : 0.0;
            lamd[i] = i < P.T ? P.ar * P.bs * (1.0 - th * th) : 0.0;
        }
    }
    int sumrow = 0;
#pragma unroll
    for (int r = 0; r < NX; ++r) sumrow += col_rowlen(MODEL, r, d, P.nu);
    const int64_t jo = (int64_t)k * P.nnzk;
    const int64_t go = (int64_t)k * P.ngk;

#pragma unroll UN
    for (int j = 1; j <= d; ++j) {
        double x[NX];
#pragma unroll
        for (int r = 0; r < NX; ++r) x[r] = X(j, r);
        const int q = k * d + j - 1;
        double cs;
        const double* coef = P.tab + (int64_t)q * (HM ? TMAX : 1);
        if constexpr (HM) {
            cs = 0.0;
#pragma unroll
            for (int i = 0; i < TMAX; ++i) cs += coef[i] * lam[i];
        } else {
            cs = coef[0];
        }
        double xd[NX][DD], cnd[DD], f[NX], fd[NX][DD];
#pragma unroll
        for (int r = 0; r < NX; ++r)
#pragma unroll
            for (int c = 0; c < DD; ++c) xd[r][c] = r == c ? 1.0 : 0.0;
#pragma unroll
        for (int c = 0; c < DD; ++c) cnd[c] = c == 0 ? 1.0 : 0.0;
        rhs_force<MODEL, DD, true>(P, x[0], cnd, x, xd, amp, f, fd);
        f[0] = P.inv_tauc * (cs - x[0]);
        if (G) {
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                double poly = 0.0;
#pragma unroll UN
                for (int i = 0; i <= d; ++i) poly = fma(P.colC[i][j], X(i, r), poly);
                st_nt(G + (go + (j - 1) * NX + r) * B + b, fma(-P.dt, f[r], poly));
            }
        }
        if (J) {
            int64_t o = jo + (int64_t)(j - 1) * sumrow;
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                const double diag = r == 0 ? -P.inv_tauc : fd[r][r];
#pragma unroll UN
                for (int i = 0; i <= d; ++i)
                    st_nt(J + (o + i) * B + b, i == j ? fma(-P.dt, diag, P.colC[i][j]) : P.colC[i][j]);
                o += d + 1;
#pragma unroll
                for (int c = 0; c < NX; ++c)
                    if (c != r && (col_xdeps(MODEL, r) >> c & 1u)) st_nt(J + (o++) * B + b, -P.dt * fd[r][c]);
                if constexpr (HM) {
                    if (r == 0) {
#pragma unroll
                        for (int i = 0; i < TMAX; ++i)  // register-resident lamd: no dynamic indexing
                            if (i < P.T) st_nt(J + (o + i) * B + b, -P.dt * P.inv_tauc * coef[i] * lamd[i]);
                        o += P.T;
                    }
                }
                if constexpr (PW) {
                    if (r == 1) st_nt(J + (o++) * B + b, -P.dt * fd[1][NX]);
                }
            }
        }
    }
    // continuity
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        if (G) {
            double e = 0.0;
#pragma unroll UN
            for (int i = 0; i <= d; ++i) e = fma(P.colD[i], X(i, r), e);
            st_nt(G + (go + d * NX + r) * B + b, e - xn[r]);
        }
        if (J) {
            const int64_t o = jo + (int64_t)d * sumrow + (int64_t)r * (d + 2);
#pragma unroll UN
            for (int i = 0; i <= d; ++i) st_nt(J + (o + i) * B + b, P.colD[i]);
            st_nt(J + (o + d + 1) * B + b, -1.0);
        }
    }
}

// Lagrangian Hessian of the collocation defects: sum_{j,r} lambda_{k,j,r} (-dt) d^2 f_r(x_k^j, u_k).  Local
// directions of a point: its nx states then the nu controls; a task (I, J) carries direction blocks I and J
// (as k_hessian).  States of different points never meet, so point j's (x, x) and (u, x) entries are written
// per point; the (u, u) entries are summed over the points in registers and written once.
template <int MODEL, int DJ, int TMAX>
__global__ void __launch_bounds__(256) k_colloc_hess(const KParams P, const HTask* __restrict__ tasks, int bs,
                                                     const double* __restrict__ V, const double* __restrict__ LAM,
                                                     double* __restrict__ H) {
    constexpr int NX = nx_of(MODEL);
    constexpr bool HM = is_int(MODEL);
    using J_t = Jet<DJ>;
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int k = blockIdx.y;
    const HTask task = tasks[blockIdx.z];
    const int d = P.deg, nu = P.nu, nzl = NX + P.nu;
    const double* Vb = V + b;
    const int64_t xo = (int64_t)k * P.nz;

    int gd[DJ];
#pragma unroll
    for (int s = 0; s < DJ; ++s) {
        const int blk = s < bs ? task.I : task.J;
        const int g = blk * bs + (s < bs ? s : s - bs);
        gd[s] = (task.I == task.J && s >= bs) ? -1 : (g < nzl ? g : -1);
    }
    auto seed = [&](double v, int dir) {
        J_t r = jconst<DJ>(v);
#pragma unroll
        for (int s = 0; s < DJ; ++s)
            if (gd[s] == dir) r.g[s] = 1.0;
        return r;
    };
    J_t afac = jconst<DJ>(1.0);
    if constexpr (is_pw(MODEL)) {
        const double pw = Vb[(xo + P.uoff) * B];
        const double ex = exp(-(pw - P.pd0) / P.pdt);
        afac = jchain(seed(pw, NX), 1.0 - ex, ex / P.pdt, -ex / (P.pdt * P.pdt));
    }
    CsHmedJet<DJ, TMAX> csh;
    if constexpr (HM) {
        csh.coef = P.tab;
#pragma unroll
        for (int i = 0; i < TMAX; ++i) {
            const double ui = i < P.T ? Vb[(xo + P.uoff + i) * B] : P.Is;
            csh.lamv[i] = i < P.T ? P.ar * (tanh(P.bs * (ui - P.Is)) + P.cr) : 0.0;
        }
#pragma unroll
        for (int s = 0; s < DJ; ++s) {
            csh.uidx[s] = -1;
            csh.l1[s] = csh.l2[s] = 0.0;
            if (gd[s] >= NX) {
                const double th = tanh(P.bs * (Vb[(xo + P.uoff + gd[s] - NX) * B] - P.Is));
                const double d1 = P.bs * (1.0 - th * th);
                csh.l1[s] = P.ar * d1;
                csh.l2[s] = -2.0 * P.ar * P.bs * th * d1;
                csh.uidx[s] = gd[s] - NX;
            }
        }
    }
    const bool cross = task.I != task.J;
    auto wanted = [&](int s1, int s2) { return gd[s1] >= 0 && gd[s2] >= 0 && (!cross || (s1 >= bs && s2 < bs)); };
    const int64_t hk = (int64_t)k * P.nhk;
    const int per_point = NX * (NX + 1) / 2 + nu * NX;
    const int64_t uu0 = hk + NX + (int64_t)d * per_point;
    double uu[DJ * (DJ + 1) / 2];
#pragma unroll
    for (int t = 0; t < DJ * (DJ + 1) / 2; ++t) uu[t] = 0.0;

    for (int j = 1; j <= d; ++j) {
        J_t x[NX];
#pragma unroll
        for (int r = 0; r < NX; ++r) x[r] = seed(Vb[(xo + j * NX + r) * B], r);
        J_t f[NX];
        const int q = k * d + j - 1;
        const J_t cs = HM ? csh.eval(q) : jconst<DJ>(P.tab[q]);
        f[0] = P.inv_tauc * (cs - x[0]);
        rhs_force_gen<MODEL>(P, x[0], x, afac, f);
        double w[NX];
#pragma unroll
        for (int r = 0; r < NX; ++r) w[r] = -P.dt * LAM[(int64_t)(k * P.ngk + (j - 1) * NX + r) * B + b];
        const int64_t pj = hk + NX + (int64_t)(j - 1) * per_point;
#pragma unroll
        for (int s1 = 0; s1 < DJ; ++s1) {
#pragma unroll
            for (int s2 = 0; s2 <= s1; ++s2) {
                if (!wanted(s1, s2)) continue;
                double acc = 0.0;
#pragma unroll
                for (int r = 0; r < NX; ++r) acc += w[r] * f[r].h[s1 * (s1 + 1) / 2 + s2];
                const int g1 = gd[s1] > gd[s2] ? gd[s1] : gd[s2], g2 = gd[s1] > gd[s2] ? gd[s2] : gd[s1];
                if (g1 < NX) {
                    H[(pj + g1 * (g1 + 1) / 2 + g2) * B + b] = acc;
                } else if (g2 < NX) {
                    H[(pj + NX * (NX + 1) / 2 + (int64_t)(g1 - NX) * NX + g2) * B + b] = acc;
                } else {
                    uu[s1 * (s1 + 1) / 2 + s2] += acc;
                }
            }
        }
    }
#pragma unroll
    for (int s1 = 0; s1 < DJ; ++s1) {
#pragma unroll
        for (int s2 = 0; s2 <= s1; ++s2) {
            if (!wanted(s1, s2)) continue;
            const int g1 = gd[s1] > gd[s2] ? gd[s1] : gd[s2], g2 = gd[s1] > gd[s2] ? gd[s2] : gd[s1];
            if (g2 >= NX) {
                const int a = g1 - NX, c = g2 - NX;
                H[(uu0 + a * (a + 1) / 2 + c) * B + b] = uu[s1 * (s1 + 1) / 2 + s2];
            }
        }
    }
    // the node-state diagonal of interval k (and x_N) carries objective terms only: start from zero
    if (blockIdx.z == 0) {
#pragma unroll
        for (int r = 0; r < NX; ++r) H[(hk + r) * B + b] = 0.0;
        if (k == P.N - 1) {
#pragma unroll
            for (int r = 0; r < NX; ++r) H[((int64_t)P.N * P.nhk + r) * B + b] = 0.0;
        }
    }
}

}  // namespace cfx
