// cfx_kernels.h — gfx950 kernels of the FES multiple-shooting NLP callbacks.
//
// Data layout in HBM (SoA, "element-major, instance-minor"): element e of instance b lives at
// buf[e * B + b], so the 64 lanes of a wave (64 consecutive instances) read/write 512 contiguous bytes
// per access.  One thread owns one instance, a run of KPT consecutive shooting intervals (the end state
// of interval k is the loaded start state of interval k+1, so x is read once) and one chunk of
// Jacobian directions.  Interval index and chunk are wave-uniform, so every read of the per-interval
// stimulation coefficient table is a scalar (SMEM) load shared by the whole wave.
//
// The stimulation sum of the reference (cn_sum_fun, cocofest/models/ding2003.py:230-252) depends only
// on time and on the stim table row, never on a decision variable (Ding2003/Ding2007), or linearly on
// lambda_i(u) (Hmed2018, hmed2018.py:97-98,169-180).  It is therefore evaluated once per problem on the
// host, at every RK stage time of every interval, with the reference's own operation order
// (r_i * exp(-(t - t_i)/tauc), summed over i).  What remains per RHS on the GPU: two reciprocals and
// ~15 FP64 ops, plus a handful of FMAs per Jacobian direction with hand-derived partial derivatives.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cfx_dual.h"

namespace cfx {

enum { M_D03 = 0, M_D03F = 1, M_D07 = 2, M_D07F = 3, M_H18 = 4, M_H18F = 5 };

constexpr int nx_of(int m) { return (m & 1) ? 5 : 2; }
constexpr bool is_fatigue(int m) { return (m & 1) != 0; }
constexpr bool is_pw(int m) { return m == M_D07 || m == M_D07F; }
constexpr bool is_int(int m) { return m == M_H18 || m == M_H18F; }
constexpr int stages_of(int scheme) { return scheme == 4 ? 4 : (scheme == 2 ? 2 : 1); }


constexpr int kMaxNz = 5 + 32;  // nx + truncation
constexpr int kMaxDeg = 9;      // collocation polynomial degree
constexpr int kMaxGridY = 65535;  // launch grid y / z limit

// Everything a kernel needs, passed by value (kernel argument segment).
struct KParams {
    int64_t B;       // batch = SoA leading dimension
    int32_t nx;      // states
    int32_t N;       // shooting intervals
    int32_t m;       // RK sub-steps per interval
    int32_t nu;      // controls per interval
    int32_t nz;      // nx + nu
    int32_t T;       // truncation
    int32_t Q;       // RHS slots per interval (m * stages)
    int32_t ngk;     // constraint rows per interval (nx + n_slide)
    int32_t nnzk;    // J_g entries per interval (structural pattern + the -I)
    int32_t nhk;     // Hessian entries per interval (nz (nz+1) / 2)
    int32_t n_slide; // sliding-window rows per interval
    int32_t n_params;
    int32_t kpt;     // shooting intervals per thread
    int32_t ifast;   // shooting launch: interval chunks on grid.x (fast), instance blocks on grid.y
    int32_t keepc;   // CFX_KEEP_CONSTANT_JAC: the instance- and point-invariant J_g values (the -1 on x_{k+1}, the
                     // Ding calcium row's cna) are not stored; the output already holds them (cfx_jac_constant_mask)
    double dt, h;
    // model constants (reciprocals precomputed on the host)
    double inv_tauc, tau2, km_rest, tau1_rest, a_rest, a_scale, pd0, pdt;
    double ar, bs, Is, cr;
    double alpha_a, alpha_tau1, alpha_km, inv_tau_fat, a_fat_rest, mult;
    double neg_mult, mult_km;  // -mult, mult * km_rest
    // fused Euler step of the two-state Ding families (euler_force): tau1 + tau2, tau1 km, h mult, h mult km,
    // h mult km tau2 (rest values)
    double tau12, tau1km, hm, hmkm, hmkmt2;
    const double* tab;  // Ding: cnb[N*(Q+1)] affine calcium offsets; Hmed: coef[N*Q*TMAX] (zero padded past T)
    const double* cna;  // Ding: affine calcium slopes per slot [Q+1] (identical for every interval)
    int32_t tstride;    // per-interval stride of tab (Ding: Q+1)
    const double* rest; // rest state [nx] (IVP default x0)
    // J_g value offset, inside an interval block, of dPhi_r/dz_c (-1: structural zero) and of the -1 on x_{k+1}[r]
    int16_t jpos[5][kMaxNz];
    int16_t jneg[5];
    // offset of u_k inside an interval's decision block (nx for shooting, (deg+1) nx for collocation)
    int32_t uoff;
    // direct collocation (cfx_colloc.h): polynomial degree, C[i][j] = l_i'(tau_j), D[i] = l_i(1)
    int32_t deg;
    double colC[kMaxDeg + 1][kMaxDeg + 1];
    double colD[kMaxDeg + 1];
    // Hessian value index of the diagonal entry of (node k, element e), e < nx + nu, k <= N (objective terms)
    const int32_t* hdiag;
    // CFX_LAYOUT_TILED64: element e of instance b at ((b / 64) * len + e) * 64 + b % 64 (len = nv, ng or
    // nnz_jac per instance); otherwise SoA e * B + b
    int32_t tiled;
    int64_t nv_tot, ng_tot, nnz_tot, nh_tot;  // per-instance lengths of v, g, J_g and Hessian buffers (layout bases)
};

// Element stride and the offset of instance b's element 0 in a buffer of `len` doubles per instance.
CFX_HD int64_t lay_stride(const KParams& P) { return P.tiled ? 64 : P.B; }
CFX_HD int64_t lay_base(const KParams& P, int64_t len, int64_t b) {
    return P.tiled ? ((b >> 6) * len) * 64 + (b & 63) : b;
}

// 1/x from v_rcp_f64 (relative error <= 4.6e-8 measured on MI355X) and one cubic correction
// y (1 + e + e^2), e = 1 - x y: residual O(e^3) ~ 1e-22, i.e. the FP64 rounding of the last FMAs.
// Inputs here are positive and well scaled (no special-value handling).
CFX_HD double frcp(double x) {
    const double y = __builtin_amdgcn_rcp(x);
    const double e = fma(-x, y, 1.0);
    return fma(y, fma(e, e, e), y);
}

// Pulse-width amplitude factor of Ding2007 (ding2007.py:172-188) for one interval:
// E = 1 - exp(-(pw - pd0)/pdt) and dE/dpw; pwdir = lane direction carrying d/dpw (-1: none).
struct Amp {
    double E, dE;
    int pwdir;
};

// ---------------------------------------------------------------------------------------------------
// Force (and fatigue) right-hand side with its directional derivatives, for a given calcium value cn and
// its tangent cnd (the calcium row itself is handled by the integrator).
//   F_dot  = (A s - F / (tau1 + tau2 s)) (fl fv + fp),  s = cn / (Km + cn)     (ding2003.py:274-311)
//   A_dot  = alpha_A F - (A - A_rest) / tau_fat, same for Tau1, Km          (ding2003_with_fatigue.py:197-240)
// Ding2007 scales A by E(pw) (ding2007.py:172-188).  With d1 = Km + cn and d2 = tau1 d1 + tau2 cn:
// s = cn / d1 and 1 / (tau1 + tau2 s) = d1 / d2, so a single reciprocal R = 1 / (d1 d2) serves both
// quotients (1/d1 = d2 R, 1/d2 = d1 R); the partial derivatives below are exact rearrangements:
//   dF/dcn = Km W, dF/dKm = -cn W with W = fl fv (A / d1^2 + F tau2 / d2^2);  dF/dF = -d1/d2;
//   dF/dTau1 = F (d1/d2)^2;  dF/dA = s (E);  dF/dpw = s A dE/dpw.
// xd[r][j] = d x_r / d z along lane direction j; fd likewise for the output (rows 1..nx-1 written).
// ---------------------------------------------------------------------------------------------------
template <int MODEL, int D, bool CN_SPARSE>
CFX_HD void rhs_force(const KParams& P, double cn, const double* cnd, const double* x,
                      const double (*xd)[D > 0 ? D : 1], const Amp& amp, double* f, double (*fd)[D > 0 ? D : 1]) {
    // CN_SPARSE: the calcium tangent is cnd[0] along lane direction 0 and exactly zero elsewhere
    constexpr bool FAT = is_fatigue(MODEL), PW = is_pw(MODEL);
    const double F = x[1];
    const double km = FAT ? x[4] : P.km_rest;
    const double tau1 = FAT ? x[3] : P.tau1_rest;
    const double A = FAT ? x[2] : (PW ? P.a_scale : P.a_rest);
    const double Aeff = PW ? A * amp.E : A;
    const double d1 = km + cn;
    const double d2 = fma(tau1, d1, P.tau2 * cn);
    const double R = frcp(d1 * d2);
    const double q1 = d2 * R;  // 1 / d1
    const double q2 = d1 * R;  // 1 / d2
    const double t1 = cn * q1; // s
    const double t2 = d1 * q2; // 1 / (tau1 + tau2 s)
    f[1] = P.mult * (Aeff * t1 - F * t2);
    if (FAT) {
        f[2] = P.alpha_a * F - (A - P.a_fat_rest) * P.inv_tau_fat;
        f[3] = P.alpha_tau1 * F - (tau1 - P.tau1_rest) * P.inv_tau_fat;
        f[4] = P.alpha_km * F - (km - P.km_rest) * P.inv_tau_fat;
    }
    if constexpr (D > 0) {
        const double W0 = fma(Aeff, q1 * q1, (F * P.tau2) * (q2 * q2));
        const double g_cn = (FAT ? P.mult * km : P.mult_km) * W0;
        const double g_F = P.neg_mult * t2;
        const double g_A = P.mult * t1 * (PW ? amp.E : 1.0);
        const double g_tau = P.mult * F * (t2 * t2);
        const double g_km = -cn * P.mult * W0;
        const double g_pw = PW ? P.mult * t1 * A * amp.dE : 0.0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            double t = g_F * xd[1][j];
            if (!CN_SPARSE || j == 0) t = fma(g_cn, cnd[j], t);
            if (FAT) t += g_A * xd[2][j] + g_tau * xd[3][j] + g_km * xd[4][j];
            if (PW && j == amp.pwdir) t += g_pw;
            fd[1][j] = t;
            if (FAT) {
                fd[2][j] = P.alpha_a * xd[1][j] - P.inv_tau_fat * xd[2][j];
                fd[3][j] = P.alpha_tau1 * xd[1][j] - P.inv_tau_fat * xd[3][j];
                fd[4][j] = P.alpha_km * xd[1][j] - P.inv_tau_fat * xd[4][j];
            }
        }
    }
}

// Hmed2018 stimulation sum: cs = sum_i coef[q][i] * lambda_i(u_i) with lambda_i held in registers
// (cn_sum_fun with lambda_i, ding2003.py:230-252 / hmed2018.py:97-98); its derivative exists only along
// this lane's u-directions (uidx >= 0): d cs / d u_i = coef[q][i] * lambda_i'(u_i).
// Lane direction j carries intensity ubase + j (ubase = chunk * D - nx, wave-uniform, so the coefficient
// c[ubase + j] is a scalar load); lamd[j] = 0 for directions that are not intensities.
template <int DMAX, int TMAX>
struct CsHmed {
    const double* coef;
    double lamv[TMAX];
    double lamd[DMAX > 0 ? DMAX : 1];
    int ubase;
    template <int D>
    CFX_HD double eval(int q, double* csd) const {
        const double* c = coef + (int64_t)q * TMAX;
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < TMAX; ++i) s += c[i] * lamv[i];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const int ui = ubase + j;
            csd[j] = (ui >= 0 && ui < TMAX) ? c[ui] * lamd[j] : 0.0;
        }
        return s;
    }
};

// Per-instance integration state carried by a thread: states, tangents, calcium start value, Ding2007
// amplitude factor.  A thread integrates NI independent instances side by side (ILP for the long FP64
// dependency chains; the per-slot coefficient loads are shared).
template <int NX, int D>
struct IState {
    double x[NX];
    double xd[NX][D > 0 ? D : 1];
    double cn0;
    Amp amp;
};

// ---------------------------------------------------------------------------------------------------
// One explicit Euler sub-step of the force row of Ding2003 / Ding2007 without fatigue (the default RK1 of
// OcpFes), fused with its tangents: the same right-hand side as rhs_force with h, mult, km and tau1 folded
// into host constants and the force row written in its linear-in-F form
//   F+ = F (1 - u) + h mult A s,  u = h mult d1 / d2,  s = cn / d1,  d2 = (tau1 + tau2) cn + tau1 km,
//   dF+/dz = (1 - u) dF/dz + h mult km (A / d1^2 + F tau2 / d2^2) dcn/dz  (+ h mult s A dE/dpw along pw),
// 23 FP64 operations per instance and sub-step instead of 27 (the reassociation moves results by a few ulp).
// The calcium row is affine in cn0 (see integrate): cn = a cn0 + b, dcn/dcn0 = a on lane direction 0.
// ---------------------------------------------------------------------------------------------------
template <int MODEL, int D>
CFX_HD void euler_force(const KParams& P, double a, double b, bool dir0, IState<2, D>& st) {
    constexpr bool PW = is_pw(MODEL);
    const double A = PW ? P.a_scale * st.amp.E : P.a_rest;  // loop-invariant over the sub-steps
    const double cn = fma(a, st.cn0, b);
    const double d1 = cn + P.km_rest;
    const double d2 = fma(P.tau12, cn, P.tau1km);
    const double R = frcp(d1 * d2);
    const double q1 = d2 * R;  // 1 / d1
    const double q2 = d1 * R;  // 1 / d2
    const double u = (P.hm * d1) * q2;
    const double s = cn * q1;
    const double F = st.x[1];
    st.x[1] = fma(P.hm * A, s, fma(-u, F, F));
    if constexpr (D > 0) {
        const double w = fma(P.hmkm * A, q1 * q1, (F * P.hmkmt2) * (q2 * q2));
#pragma unroll
        for (int j = 0; j < D; ++j) {
            double t = fma(-u, st.xd[1][j], st.xd[1][j]);
            if (j == 0 && dir0) t = fma(w, a, t);
            if (PW && j == st.amp.pwdir) t = fma(P.hm * P.a_scale * st.amp.dE, s, t);
            st.xd[1][j] = t;
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// Sub-steps [j0, j0 + msteps) of RK-s over interval k (bioptim RK1 = Euler, RK2 = midpoint, RK4 = classic;
// stage times t, t+h/2, t+h/2, t+h; control held constant), carrying D tangent directions, for NI
// instances at once.
//
// Ding2003 / Ding2007 (with or without fatigue): the calcium ODE cn_dot = (cs(t) - cn) / tauc is linear
// with a decision-independent forcing, so under any explicit RK scheme every stage value is affine in the
// interval's start value: cn = cna[slot] * cn0 + cnb[k][slot], precomputed on the host (slot = j*S + stage;
// slot j*S is the start of sub-step j, slot m*S the interval end).  Its tangent is cna along the cn0
// direction and zero elsewhere.  Hmed2018 (cs depends on the intensities) integrates cn like the others.
// ---------------------------------------------------------------------------------------------------
template <int MODEL, int SCHEME, int D, int TMAX, int NI>
CFX_HD void integrate(const KParams& P, int k, int j0, int msteps, int chunk, IState<nx_of(MODEL), D> (&st)[NI],
                      CsHmed<D, TMAX> (&csh)[NI]) {
    constexpr int NX = nx_of(MODEL);
    constexpr int DD = D > 0 ? D : 1;
    constexpr bool LIN = !is_int(MODEL);
    constexpr int S = stages_of(SCHEME);
    constexpr int R0 = LIN ? 1 : 0;  // first integrated state row
    const double h = P.h, h2 = 0.5 * P.h, h6 = P.h / 6.0;
    const double* cnb = P.tab + (int64_t)k * P.tstride;
    const bool dir0 = chunk == 0;  // lane direction 0 is d/dcn0 only in chunk 0

    // one RHS evaluation of instance i at stage slot `slot` with stage-input state (xs, xsd)
    auto stage = [&](int i, const double* xs, const double (*xsd)[DD], int slot, double* kk, double (*kkd)[DD]) {
        double cn, cnd[DD];
        if constexpr (LIN) {
            const double a = P.cna[slot];
            cn = fma(a, st[i].cn0, cnb[slot]);
#pragma unroll
            for (int d = 0; d < D; ++d) cnd[d] = (dir0 && d == 0) ? a : 0.0;
        } else {
            double csd[DD];
            const double cs = csh[i].template eval<D>(k * P.Q + slot, csd);
            cn = xs[0];
            kk[0] = P.inv_tauc * (cs - cn);
#pragma unroll
            for (int d = 0; d < D; ++d) {
                cnd[d] = xsd[0][d];
                kkd[0][d] = P.inv_tauc * (csd[d] - cnd[d]);
            }
        }
        rhs_force<MODEL, D, LIN>(P, cn, cnd, xs, xsd, st[i].amp, kk, kkd);
    };

    for (int j = j0; j < j0 + msteps; ++j) {
        const int slot = j * S;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            double* x = st[i].x;
            double(*xd)[DD] = st[i].xd;
            if constexpr (SCHEME == 1 && LIN && !is_fatigue(MODEL)) {
                euler_force<MODEL, D>(P, P.cna[slot], cnb[slot], dir0, st[i]);
                continue;
            }
            double k1[NX], k1d[NX][DD];
            stage(i, x, xd, slot, k1, k1d);
            if constexpr (SCHEME == 1) {
#pragma unroll
                for (int r = R0; r < NX; ++r) {
                    x[r] = x[r] + h * k1[r];
#pragma unroll
                    for (int d = 0; d < D; ++d) xd[r][d] = xd[r][d] + h * k1d[r][d];
                }
            } else if constexpr (SCHEME == 2) {
                double xs[NX], xsd[NX][DD], k2[NX], k2d[NX][DD];
#pragma unroll
                for (int r = R0; r < NX; ++r) {
                    xs[r] = x[r] + h2 * k1[r];
#pragma unroll
                    for (int d = 0; d < D; ++d) xsd[r][d] = xd[r][d] + h2 * k1d[r][d];
                }
                stage(i, xs, xsd, slot + 1, k2, k2d);
#pragma unroll
                for (int r = R0; r < NX; ++r) {
                    x[r] = x[r] + h * k2[r];
#pragma unroll
                    for (int d = 0; d < D; ++d) xd[r][d] = xd[r][d] + h * k2d[r][d];
                }
            } else {
                double xs[NX], xsd[NX][DD], acc[NX], accd[NX][DD], kk[NX], kkd[NX][DD];
#pragma unroll
                for (int r = R0; r < NX; ++r) {
                    acc[r] = k1[r];
                    xs[r] = x[r] + h2 * k1[r];
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        accd[r][d] = k1d[r][d];
                        xsd[r][d] = xd[r][d] + h2 * k1d[r][d];
                    }
                }
#pragma unroll
                for (int sg = 1; sg < 4; ++sg) {
                    stage(i, xs, xsd, slot + sg, kk, kkd);
                    if (sg < 3) {
                        const double c = sg == 1 ? h2 : h;
#pragma unroll
                        for (int r = R0; r < NX; ++r) {
                            acc[r] = acc[r] + 2.0 * kk[r];
                            xs[r] = x[r] + c * kk[r];
#pragma unroll
                            for (int d = 0; d < D; ++d) {
                                accd[r][d] = accd[r][d] + 2.0 * kkd[r][d];
                                xsd[r][d] = xd[r][d] + c * kkd[r][d];
                            }
                        }
                    }
                }
#pragma unroll
                for (int r = R0; r < NX; ++r) {
                    x[r] = x[r] + h6 * (acc[r] + kk[r]);
#pragma unroll
                    for (int d = 0; d < D; ++d) xd[r][d] = xd[r][d] + h6 * (accd[r][d] + kkd[r][d]);
                }
            }
        }
    }
    if constexpr (LIN) {
        const int se = (j0 + msteps) * S;
        const double a = P.cna[se];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            st[i].x[0] = fma(a, st[i].cn0, cnb[se]);
#pragma unroll
            for (int d = 0; d < D; ++d) st[i].xd[0][d] = (dir0 && d == 0) ? a : 0.0;
        }
    }
}

// Per-interval control set-up: Ding2007 amplitude factor, Hmed lambdas.  Lane direction j carries global
// direction chunk * D + j; u directions start at NX.  Controls of the interval are read at
// Vb[(xo + NX + i) * B].
template <int MODEL, int D, int TMAX>
CFX_HD void load_controls(const KParams& P, const double* Vb, int64_t B, int xo, int chunk, Amp& amp,
                          CsHmed<D, TMAX>& csh) {
    constexpr int NX = nx_of(MODEL);
    amp.E = 1.0;
    amp.dE = 0.0;
    amp.pwdir = -1;
    if constexpr (is_pw(MODEL)) {
        const double pw = Vb[(int64_t)(xo + NX) * B];
        const double ex = exp(-(pw - P.pd0) / P.pdt);
        amp.E = 1.0 - ex;
        amp.dE = ex / P.pdt;
        const int j = NX - chunk * D;
        amp.pwdir = (j >= 0 && j < D) ? j : -1;
    }
    if constexpr (is_int(MODEL)) {
        csh.coef = P.tab;
#pragma unroll
        for (int i = 0; i < TMAX; ++i) {
            const double ui = i < P.T ? Vb[(int64_t)(xo + NX + i) * B] : P.Is;
            csh.lamv[i] = i < P.T ? P.ar * (tanh(P.bs * (ui - P.Is)) + P.cr) : 0.0;
        }
        csh.ubase = chunk * D - NX;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const int gd = chunk * D + j;
            csh.lamd[j] = 0.0;
            if (gd >= NX && gd < P.nz) {
                const double th = tanh(P.bs * (Vb[(int64_t)(xo + gd) * B] - P.Is));
                csh.lamd[j] = P.ar * P.bs * (1.0 - th * th);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// Kernel 1: continuity residuals g_k = Phi(x_k, u_k) - x_{k+1} and the structurally non-zero entries of
// dPhi/d(x_k, u_k) (+ the -1 on x_{k+1}).  Thread = (instance b, intervals [k0, k0+kpt), direction chunk);
// D directions per lane (D = 0: g only).
// ---------------------------------------------------------------------------------------------------
// NI adjacent instances per lane: element e of instances b0 .. b0+NI-1 is NI contiguous doubles, moved as
// NI/2 16-byte accesses per lane (1 KiB per wave instruction).  Requires B % NI == 0 and 16-byte aligned
// buffers for NI > 1 (checked on the host).
template <int NI>
CFX_HD void ld_lane(const double* p, double (&o)[NI]) {
    if constexpr (NI == 1) {
        o[0] = p[0];
    } else {
#pragma unroll
        for (int i = 0; i < NI; i += 2) {
            const double2 t = *reinterpret_cast<const double2*>(p + i);
            o[i] = t.x;
            o[i + 1] = t.y;
        }
    }
}
// Output stores are non-temporal (`global_store … nt`): the callback outputs are a write stream far larger than the
// 256 MiB Infinity Cache.  cfg 2, B = 2^20: 0.315 -> 0.287 ms together with the shorter interval chunks of
// cfx_create (scripts/store_probe.py, profiles/round2/store_probe.jsonl).  The lines stay in the XCD's L2 (a
// consumer launched next still hits there).
CFX_HD void st_nt(double* p, double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
template <int NI>
CFX_HD void st_lane(double* p, const double (&v)[NI]) {
    if constexpr (NI == 1) {
        st_nt(p, v[0]);
    } else {
#if defined(__HIP_DEVICE_COMPILE__)
        typedef double nt2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int i = 0; i < NI; i += 2) __builtin_nontemporal_store(nt2{v[i], v[i + 1]}, reinterpret_cast<nt2*>(p + i));
#else
#pragma unroll
        for (int i = 0; i < NI; i += 2) *reinterpret_cast<double2*>(p + i) = make_double2(v[i], v[i + 1]);
#endif
    }
}
// st_lane with a store policy: PLAIN = ordinary (write-back) 16-byte stores, for the collocation store-policy probe
template <int NI, bool PLAIN>
CFX_HD void st_lane_p(double* p, const double (&v)[NI]) {
    if constexpr (PLAIN) {
        if constexpr (NI == 1) {
            *p = v[0];
        } else {
#pragma unroll
            for (int i = 0; i < NI; i += 2) *reinterpret_cast<double2*>(p + i) = make_double2(v[i], v[i + 1]);
        }
    } else {
        st_lane<NI>(p, v);
    }
}
template <int NI>
CFX_HD void st_lane_const(double* p, double c) {
    double v[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) v[i] = c;
    st_lane<NI>(p, v);
}

// The interval loop of one thread.  WG: g is written (G != nullptr, direction chunk 0); J != nullptr whenever
// D > 0 (the launcher picks D = 0 for g-only calls).  WG is a template parameter so that each loop body is
// branch-free around its loads: on CDNA vmcnt counts stores as well as loads, and with a runtime "is G present"
// branch the compiler had to place the wait for x_{k+1} at the merge point after the interval's stores, where it
// waited for all of them to complete before the next interval could start.  With WG the g rows consume x_{k+1}
// before any store of the interval is issued.
template <int MODEL, int SCHEME, int D, int TMAX, int NI, bool WG>
__device__ __forceinline__ void shoot_run(const KParams& P, const double* __restrict__ V, double* __restrict__ G,
                                          double* __restrict__ J, int k0, int k1, int chunk, int64_t ES, int64_t vb,
                                          int64_t gb, int64_t jb) {
    constexpr int NX = nx_of(MODEL);
    IState<NX, D> st[NI];
    CsHmed<D, TMAX> csh[NI];
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        double t[NI];
        ld_lane<NI>(V + vb + (int64_t)(k0 * P.nz + r) * ES, t);
#pragma unroll
        for (int i = 0; i < NI; ++i) st[i].x[r] = t[i];
    }
    // Consume the start state here, before the loop: the wait the compiler places for these loads would otherwise
    // sit at the loop header (its pending state merges the preheader's loads with the back edge) and run every
    // interval, where vmcnt then also waits for the previous interval's stores.  Not volatile and no memory
    // clobber: the table reads stay scalar loads.
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int r = 0; r < NX; ++r) asm("" : "+v"(st[i].x[r]));

    for (int k = k0; k < k1; ++k) {
        const int xo = k * P.nz;
        const int xn = (k + 1) * P.nz;
        double xnext[NX][NI];  // issued before the integration so its latency hides under it
#pragma unroll
        for (int r = 0; r < NX; ++r) ld_lane<NI>(V + vb + (int64_t)(xn + r) * ES, xnext[r]);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
#pragma unroll
            for (int r = 0; r < NX; ++r)
#pragma unroll
                for (int j = 0; j < D; ++j) st[i].xd[r][j] = (chunk * D + j == r) ? 1.0 : 0.0;
            st[i].cn0 = st[i].x[0];
            load_controls<MODEL, D, TMAX>(P, V + vb + i, ES, xo, chunk, st[i].amp, csh[i]);
        }
        integrate<MODEL, SCHEME, D, TMAX, NI>(P, k, 0, P.m, chunk, st, csh);
        if constexpr (WG) {
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                double t[NI];
#pragma unroll
                for (int i = 0; i < NI; ++i) t[i] = st[i].x[r] - xnext[r][i];
                st_lane<NI>(G + gb + (int64_t)(k * P.ngk + r) * ES, t);
            }
        } else {
            // no g rows: consume x_{k+1} explicitly before the stores (see above)
#pragma unroll
            for (int r = 0; r < NX; ++r)
#pragma unroll
                for (int i = 0; i < NI; ++i) asm("" : "+v"(xnext[r][i]));
        }
        if constexpr (D > 0) {
            const int64_t jo = (int64_t)k * P.nnzk;
#pragma unroll
            for (int r = 0; r < NX; ++r) {
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const int gd = chunk * D + j;
                    if (gd < P.nz) {
                        const int pos = P.jpos[r][gd];
                        // the Ding calcium row's only entry, dCn+/dCn0 = cna[m S], is constant (integrate)
                        const bool cst = !is_int(MODEL) && r == 0 && gd == 0 && P.keepc;
                        if (pos >= 0 && !cst) {
                            double t[NI];
#pragma unroll
                            for (int i = 0; i < NI; ++i) t[i] = st[i].xd[r][j];
                            st_lane<NI>(J + jb + (jo + pos) * ES, t);
                        }
                    }
                }
                if (chunk == 0 && !P.keepc) st_lane_const<NI>(J + jb + (jo + P.jneg[r]) * ES, -1.0);
            }
        }
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < NX; ++r) st[i].x[r] = xnext[r][i];
    }
}

// CFX_SHOOT_WPE: occupancy hint for the shooting kernel (waves per SIMD the register allocation must allow; A/B builds).
// Measured with 8 (63 instead of 78 VGPRs, 6 -> 8 waves per SIMD, no spills): cfg 2 0.274 -> 0.277 ms, cfg 3 0.451 ->
// 0.516 ms (profiles/round3/occupancy/wpe8_ab.jsonl); the default allocation is kept.
#ifdef CFX_SHOOT_WPE
#define CFX_SHOOT_ATTR __attribute__((amdgpu_waves_per_eu(CFX_SHOOT_WPE, CFX_SHOOT_WPE)))
#else
#define CFX_SHOOT_ATTR
#endif
template <int MODEL, int SCHEME, int D, int TMAX, int NI>
__global__ void __launch_bounds__(256) CFX_SHOOT_ATTR k_shooting(const KParams P, const double* __restrict__ V,
                                                  double* __restrict__ G, double* __restrict__ J) {
    const int64_t B = P.B;
    const unsigned bi = P.ifast ? blockIdx.y : blockIdx.x, bk = P.ifast ? blockIdx.x : blockIdx.y;
    const int64_t b0 = ((int64_t)bi * blockDim.x + threadIdx.x) * NI;
    if (b0 >= B) return;
    const int k0 = bk * P.kpt;
    const int k1 = min(P.N, k0 + P.kpt);
    const int chunk = is_int(MODEL) ? (int)blockIdx.z : 0;  // the other models carry every direction in one lane

    // layout: element stride ES, per-buffer instance offsets (SoA: b0; 64-instance tiles: see KParams).  The
    // accesses stay expressed on the __restrict__ arguments (a derived `G ? G + off : nullptr` pointer loses
    // the no-alias fact, and the table reads then turn into vector loads behind every store).
    const int64_t ES = lay_stride(P);
    const int64_t vb = lay_base(P, P.nv_tot, b0), gb = lay_base(P, P.ng_tot, b0), jb = lay_base(P, P.nnz_tot, b0);
    if constexpr (D == 0) {
        shoot_run<MODEL, SCHEME, 0, TMAX, NI, true>(P, V, G, J, k0, k1, chunk, ES, vb, gb, jb);
    } else {
        if (G != nullptr && chunk == 0)
            shoot_run<MODEL, SCHEME, D, TMAX, NI, true>(P, V, G, J, k0, k1, chunk, ES, vb, gb, jb);
        else
            shoot_run<MODEL, SCHEME, D, TMAX, NI, false>(P, V, G, J, k0, k1, chunk, ES, vb, gb, jb);
    }
}

// ---------------------------------------------------------------------------------------------------
// Kernel 2: single-shooting trajectory (IvpFes.integrate).  One thread per instance, sequential over
// intervals, every sub-step written: traj[(s * nx + r) * B + b], s = 0 .. N*m.
// ---------------------------------------------------------------------------------------------------
template <int MODEL, int SCHEME, int TMAX>
__global__ void __launch_bounds__(256) k_ivp(const KParams P, const double* __restrict__ X0,
                                             const double* __restrict__ U, double* __restrict__ TR) {
    constexpr int NX = nx_of(MODEL);
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    IState<NX, 0> st[1];
    CsHmed<0, TMAX> csh[1];
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        st[0].x[r] = X0 ? X0[(int64_t)r * B + b] : P.rest[r];
        TR[(int64_t)r * B + b] = st[0].x[r];
    }
    int64_t s = 1;
    const double* Ub = U ? U + b : nullptr;
    for (int k = 0; k < P.N; ++k) {
        // controls of interval k live at U[(k*nu + i)*B + b]; load_controls reads Vb[(xo + NX + i)*B]
        load_controls<MODEL, 0, TMAX>(P, Ub, B, k * P.nu - NX, 0, st[0].amp, csh[0]);
        st[0].cn0 = st[0].x[0];
        for (int j = 0; j < P.m; ++j) {
            integrate<MODEL, SCHEME, 0, TMAX, 1>(P, k, j, 1, 0, st, csh);
#pragma unroll
            for (int r = 0; r < NX; ++r) TR[(s * NX + r) * B + b] = st[0].x[r];
            ++s;
        }
    }
}

}  // namespace cfx
