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

// One interval of g (defects + continuity) and J_g for NI adjacent instances per lane (16-byte accesses when NI = 2).
// DEG > 0: the degree is a compile-time constant and every input of the interval (x^1..x^d, x_{k+1}, the controls)
// is loaded into registers before the first store — on CDNA vmcnt counts stores too, so a load issued after stores
// waits for them; x^0 is the previous interval's x_{k+1} (xc, carried by the caller's interval loop).  DEG == 0: any
// degree, NI = 1, states re-read from memory per point.  ES / vb / gb / jb: element stride and the instances' bases
// of V, G, J (SoA or 64-instance tiles, lay_stride / lay_base).  Shared by k_colloc and the fused g + J_g + Hessian
// launch (k_colloc_hess<GJ>), so the two write the same bits.
template <int MODEL, int TMAX, int DEG, int NI, bool PLAIN = false>
__device__ __forceinline__ void colloc_interval(const KParams& P, const double* __restrict__ V, double* __restrict__ G,
                                                double* __restrict__ J, int k, int64_t ES, int64_t vb, int64_t gb,
                                                int64_t jb, double (&xc)[nx_of(MODEL)][NI]) {
    constexpr int NX = nx_of(MODEL);
    constexpr bool PW = is_pw(MODEL), HM = is_int(MODEL);
    constexpr int DD = NX + (PW ? 1 : 0);  // directions of the RHS partials: the point's states (+ pulse width)
    constexpr int XS = DEG > 0 ? DEG + 1 : 1;
    constexpr int UN = DEG > 0 ? DEG + 1 : 1;  // unroll factor of the point / basis loops
    static_assert(DEG > 0 || NI == 1, "the generic-degree body runs one instance per lane");
    const int d = DEG > 0 ? DEG : P.deg;
    const int64_t xo = (int64_t)k * P.nz;
    auto ld = [&](int64_t e, double(&o)[NI]) { ld_lane<NI>(V + vb + (xo + e) * ES, o); };

    double xs[XS][NX][NI], xn[NX][NI];
    if constexpr (DEG > 0) {
#pragma unroll
        for (int r = 0; r < NX; ++r)
#pragma unroll
            for (int n = 0; n < NI; ++n) xs[0][r][n] = xc[r][n];
#pragma unroll
        for (int i = 1; i <= DEG; ++i)
#pragma unroll
            for (int r = 0; r < NX; ++r) ld(i * NX + r, xs[i][r]);
    }
#pragma unroll
    for (int r = 0; r < NX; ++r) ld_lane<NI>(V + vb + ((int64_t)(k + 1) * P.nz + r) * ES, xn[r]);
    auto X = [&](int i, int r, int n) { return DEG > 0 ? xs[i][r][n] : V[vb + (xo + i * NX + r) * ES]; };

    Amp amp[NI];
    double lam[NI][TMAX], lamd[NI][TMAX];
#pragma unroll
    for (int n = 0; n < NI; ++n) amp[n] = Amp{1.0, 0.0, -1};
    if constexpr (PW) {
        double pw[NI];
        ld(P.uoff, pw);
#pragma unroll
        for (int n = 0; n < NI; ++n) {
            const double ex = exp(-(pw[n] - P.pd0) / P.pdt);
            amp[n].E = 1.0 - ex;
            amp[n].dE = ex / P.pdt;
            amp[n].pwdir = NX;
        }
    }
    if constexpr (HM) {
#pragma unroll
        for (int i = 0; i < TMAX; ++i) {
            double u[NI];
#pragma unroll
            for (int n = 0; n < NI; ++n) u[n] = P.Is;
            if (i < P.T) ld(P.uoff + i, u);
#pragma unroll
            for (int n = 0; n < NI; ++n) {
                const double th = i < P.T ? tanh(P.bs * (u[n] - P.Is)) : 0.0;
                lam[n][i] = i < P.T ? P.ar * (th + P.cr) : 0.0;
                lamd[n][i] = i < P.T ? P.ar * P.bs * (1.0 - th * th) : 0.0;
            }
        }
    }
    int sumrow = 0;
#pragma unroll
    for (int r = 0; r < NX; ++r) sumrow += col_rowlen(MODEL, r, d, P.nu);
    const int64_t jo = (int64_t)k * P.nnzk;
    const int64_t go = (int64_t)k * P.ngk;

#pragma unroll UN
    for (int j = 1; j <= d; ++j) {
        const int q = k * d + j - 1;
        const double* coef = P.tab + (int64_t)q * (HM ? TMAX : 1);
        double f[NI][NX], fd[NI][NX][DD];
#pragma unroll
        for (int n = 0; n < NI; ++n) {
            double x[NX];
#pragma unroll
            for (int r = 0; r < NX; ++r) x[r] = X(j, r, n);
            double cs;
            if constexpr (HM) {
                cs = 0.0;
#pragma unroll
                for (int i = 0; i < TMAX; ++i) cs += coef[i] * lam[n][i];
            } else {
                cs = coef[0];
            }
            double xd[NX][DD], cnd[DD];
#pragma unroll
            for (int r = 0; r < NX; ++r)
#pragma unroll
                for (int c = 0; c < DD; ++c) xd[r][c] = r == c ? 1.0 : 0.0;
#pragma unroll
            for (int c = 0; c < DD; ++c) cnd[c] = c == 0 ? 1.0 : 0.0;
            rhs_force<MODEL, DD, true>(P, x[0], cnd, x, xd, amp[n], f[n], fd[n]);
            f[n][0] = P.inv_tauc * (cs - x[0]);
        }
        if (G) {
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                double t[NI];
#pragma unroll
                for (int n = 0; n < NI; ++n) {
                    double poly = 0.0;
#pragma unroll UN
                    for (int i = 0; i <= d; ++i) poly = fma(P.colC[i][j], X(i, r, n), poly);
                    t[n] = fma(-P.dt, f[n][r], poly);
                }
                st_lane_p<NI, PLAIN>(G + gb + (go + (j - 1) * NX + r) * ES, t);
            }
        }
        if (J) {
            int64_t o = jo + (int64_t)(j - 1) * sumrow;
#pragma unroll
            for (int r = 0; r < NX; ++r) {
#pragma unroll UN
                for (int i = 0; i <= d; ++i) {
                    // CFX_KEEP_CONSTANT_JAC: only the point's own non-calcium states vary (cfx_jac_constant_mask)
                    if (P.keepc && (r == 0 || i != j)) continue;
                    double t[NI];
#pragma unroll
                    for (int n = 0; n < NI; ++n) {
                        const double diag = r == 0 ? -P.inv_tauc : fd[n][r][r];
                        t[n] = i == j ? fma(-P.dt, diag, P.colC[i][j]) : P.colC[i][j];
                    }
                    st_lane_p<NI, PLAIN>(J + jb + (o + i) * ES, t);
                }
                o += d + 1;
#pragma unroll
                for (int c = 0; c < NX; ++c)
                    if (c != r && (col_xdeps(MODEL, r) >> c & 1u)) {
                        double t[NI];
#pragma unroll
                        for (int n = 0; n < NI; ++n) t[n] = -P.dt * fd[n][r][c];
                        st_lane_p<NI, PLAIN>(J + jb + (o++) * ES, t);
                    }
                if constexpr (HM) {
                    if (r == 0) {
#pragma unroll
                        for (int i = 0; i < TMAX; ++i)  // register-resident lamd: no dynamic indexing
                            if (i < P.T) {
                                double t[NI];
#pragma unroll
                                for (int n = 0; n < NI; ++n) t[n] = -P.dt * P.inv_tauc * coef[i] * lamd[n][i];
                                st_lane_p<NI, PLAIN>(J + jb + (o + i) * ES, t);
                            }
                        o += P.T;
                    }
                }
                if constexpr (PW) {
                    if (r == 1) {
                        double t[NI];
#pragma unroll
                        for (int n = 0; n < NI; ++n) t[n] = -P.dt * fd[n][1][NX];
                        st_lane_p<NI, PLAIN>(J + jb + (o++) * ES, t);
                    }
                }
            }
        }
    }
    // continuity
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        if (G) {
            double t[NI];
#pragma unroll
            for (int n = 0; n < NI; ++n) {
                double e = 0.0;
#pragma unroll UN
                for (int i = 0; i <= d; ++i) e = fma(P.colD[i], X(i, r, n), e);
                t[n] = e - xn[r][n];
            }
            st_lane_p<NI, PLAIN>(G + gb + (go + d * NX + r) * ES, t);
        }
        if (J && !P.keepc) {
            const int64_t o = jo + (int64_t)d * sumrow + (int64_t)r * (d + 2);
#pragma unroll UN
            for (int i = 0; i <= d; ++i) {
                double t[NI];
#pragma unroll
                for (int n = 0; n < NI; ++n) t[n] = P.colD[i];
                st_lane_p<NI, PLAIN>(J + jb + (o + i) * ES, t);
            }
            double m1[NI];
#pragma unroll
            for (int n = 0; n < NI; ++n) m1[n] = -1.0;
            st_lane_p<NI, PLAIN>(J + jb + (o + d + 1) * ES, m1);
        }
    }
#pragma unroll
    for (int r = 0; r < NX; ++r)
#pragma unroll
        for (int n = 0; n < NI; ++n) xc[r][n] = xn[r][n];
}

// g + J_g of the collocation transcription.  Thread = (NI adjacent instances, intervals [k0, k0 + kpt)); grid as the
// shooting launch (interval chunks on grid.x when P.ifast, instance blocks on grid.y).  Each interval reads its own
// block (x^0 carried from the previous interval's x_{k+1}) and x_{k+1}^0; no recursion, so the intervals per thread
// only shape the launch (fewer, longer waves; the carried x^0 is read once).
template <int MODEL, int TMAX, int DEG, int NI, bool PLAIN>
__device__ __forceinline__ void colloc_thread(const KParams& P, const double* __restrict__ V, double* __restrict__ G,
                                              double* __restrict__ J) {
    constexpr int NX = nx_of(MODEL);
    const unsigned bi = P.ifast ? blockIdx.y : blockIdx.x, bk = P.ifast ? blockIdx.x : blockIdx.y;
    const int64_t b0 = ((int64_t)bi * blockDim.x + threadIdx.x) * NI;
    if (b0 >= P.B) return;
    const int k0 = bk * P.kpt;
    const int k1 = min(P.N, k0 + P.kpt);
    const int64_t ES = lay_stride(P);
    const int64_t vb = lay_base(P, P.nv_tot, b0), gb = lay_base(P, P.ng_tot, b0), jb = lay_base(P, P.nnz_tot, b0);
    double xc[NX][NI];
    if constexpr (DEG > 0) {
#pragma unroll
        for (int r = 0; r < NX; ++r) ld_lane<NI>(V + vb + ((int64_t)k0 * P.nz + r) * ES, xc[r]);
    }
    for (int k = k0; k < k1; ++k) colloc_interval<MODEL, TMAX, DEG, NI, PLAIN>(P, V, G, J, k, ES, vb, gb, jb, xc);
}
template <int MODEL, int TMAX, int DEG, int NI, bool PLAIN = false>
__global__ void __launch_bounds__(256) k_colloc(const KParams P, const double* __restrict__ V, double* __restrict__ G,
                                                double* __restrict__ J) {
    colloc_thread<MODEL, TMAX, DEG, NI, PLAIN>(P, V, G, J);
}
// The bench's launch shapes under names of their own (one kernel name mixed the SoA, tiled and
// keep-constant launches in the traces, so no roofline fraction could be recomputed per launch): the same body.
#define CFX_COLLOC_NAMED(NAME)                                                                                        \
    template <int MODEL, int TMAX, int DEG, int NI>                                                                 \
    __global__ void __launch_bounds__(256) NAME(const KParams P, const double* __restrict__ V,                       \
                                                double* __restrict__ G, double* __restrict__ J) {                   \
        colloc_thread<MODEL, TMAX, DEG, NI, false>(P, V, G, J);                                                     \
    }
CFX_COLLOC_NAMED(k_colloc_soa)
CFX_COLLOC_NAMED(k_colloc_tiles)
CFX_COLLOC_NAMED(k_colloc_soa_keepj)
CFX_COLLOC_NAMED(k_colloc_tiles_keepj)
#undef CFX_COLLOC_NAMED
// occupancy probe (CFX_COLLOC_STORE=w4 / w4plain): the same thread body held to 128 VGPRs (4 waves per SIMD; the
// default instantiation of the bench's shape takes 198 VGPRs, 2 waves)
template <int MODEL, int TMAX, int DEG, int NI, bool PLAIN>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_colloc_w4(
    const KParams P, const double* __restrict__ V, double* __restrict__ G, double* __restrict__ J) {
    colloc_thread<MODEL, TMAX, DEG, NI, PLAIN>(P, V, G, J);
}

// Lagrangian Hessian of the collocation defects: sum_{j,r} lambda_{k,j,r} (-dt) d^2 f_r(x_k^j, u_k).  Local
// directions of a point: its nx states then the nu controls; a task (I, J) carries direction blocks I and J
// (as k_hessian).  States of different points never meet, so point j's (x, x) and (u, x) entries are written
// per point; the (u, u) entries are summed over the points in registers and written once.
// GJ: the same launch also writes g and J_g (cfx_eval_all_h: defects, continuity, Jacobian and Hessian of every
// interval from one launch, the north star's contract): task 0 of each interval runs the k_colloc body
// (colloc_interval, generic degree), so its values are k_colloc's bits.
template <int MODEL, int DJ, int TMAX, bool GJ>
__global__ void __launch_bounds__(256) k_colloc_hess(const KParams P, const HTask* __restrict__ tasks, int bs,
                                                     const double* __restrict__ V, const double* __restrict__ LAM,
                                                     double* __restrict__ H, double* __restrict__ G,
                                                     double* __restrict__ J) {
    constexpr int NX = nx_of(MODEL);
    constexpr bool HM = is_int(MODEL);
    using J_t = Jet<DJ>;
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int k = blockIdx.y;
    const HTask task = tasks[blockIdx.z];
    const int d = P.deg, nu = P.nu, nzl = NX + P.nu;
    // layout (SoA or 64-instance tiles): element stride ES, per-buffer instance bases
    const int64_t ES = lay_stride(P), vb = lay_base(P, P.nv_tot, b), lb = lay_base(P, P.ng_tot, b),
                  hb = lay_base(P, P.nh_tot, b);
    auto Vat = [&](int64_t e) { return V[vb + e * ES]; };
    const int64_t xo = (int64_t)k * P.nz;
    if constexpr (GJ) {
        if (blockIdx.z == 0) {
            double xc[NX][1];
            colloc_interval<MODEL, TMAX, 0, 1>(P, V, G, J, k, ES, vb, lb, lay_base(P, P.nnz_tot, b), xc);
        }
    }

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
        const double pw = Vat(xo + P.uoff);
        const double ex = exp(-(pw - P.pd0) / P.pdt);
        afac = jchain(seed(pw, NX), 1.0 - ex, ex / P.pdt, -ex / (P.pdt * P.pdt));
    }
    CsHmedJet<DJ, TMAX> csh;
    if constexpr (HM) {
        csh.coef = P.tab;
#pragma unroll
        for (int i = 0; i < TMAX; ++i) {
            const double ui = i < P.T ? Vat(xo + P.uoff + i) : P.Is;
            csh.lamv[i] = i < P.T ? P.ar * (tanh(P.bs * (ui - P.Is)) + P.cr) : 0.0;
        }
#pragma unroll
        for (int s = 0; s < DJ; ++s) {
            csh.uidx[s] = -1;
            csh.l1[s] = csh.l2[s] = 0.0;
            if (gd[s] >= NX) {
                const double th = tanh(P.bs * (Vat(xo + P.uoff + gd[s] - NX) - P.Is));
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
        for (int r = 0; r < NX; ++r) x[r] = seed(Vat(xo + j * NX + r), r);
        J_t f[NX];
        const int q = k * d + j - 1;
        const J_t cs = HM ? csh.eval(q) : jconst<DJ>(P.tab[q]);
        f[0] = P.inv_tauc * (cs - x[0]);
        rhs_force_gen<MODEL>(P, x[0], x, afac, f);
        double w[NX];
#pragma unroll
        for (int r = 0; r < NX; ++r) w[r] = -P.dt * LAM[lb + (int64_t)(k * P.ngk + (j - 1) * NX + r) * ES];
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
                    H[hb + (pj + g1 * (g1 + 1) / 2 + g2) * ES] = acc;
                } else if (g2 < NX) {
                    H[hb + (pj + NX * (NX + 1) / 2 + (int64_t)(g1 - NX) * NX + g2) * ES] = acc;
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
                H[hb + (uu0 + a * (a + 1) / 2 + c) * ES] = uu[s1 * (s1 + 1) / 2 + s2];
            }
        }
    }
    // the node-state diagonal of interval k (and x_N) carries objective terms only: start from zero
    if (blockIdx.z == 0) {
#pragma unroll
        for (int r = 0; r < NX; ++r) H[hb + (hk + r) * ES] = 0.0;
        if (k == P.N - 1) {
#pragma unroll
            for (int r = 0; r < NX; ++r) H[hb + ((int64_t)P.N * P.nhk + r) * ES] = 0.0;
        }
    }
}

}  // namespace cfx
