// cfx_kernels.h — gfx950 kernels of the FES multiple-shooting NLP callbacks.
//
// Data layout in HBM (SoA, "element-major, instance-minor"): element e of instance b lives at
// buf[e * B + b], so the 64 lanes of a wave (64 consecutive instances) read/write 512 contiguous bytes
// per access.  One thread owns one (instance, shooting interval, direction chunk); the interval index
// and the chunk are blockIdx.y / blockIdx.z, hence wave-uniform, so every read of the per-interval
// stimulation coefficient table is a scalar (SMEM) load shared by the whole wave.
//
// The stimulation sum of the reference (cn_sum_fun, cocofest/models/ding2003.py:230-252) depends only
// on time and on the stim table row, never on a decision variable (Ding2003/Ding2007), or linearly on
// lambda_i(u) (Hmed2018, hmed2018.py:97-98,169-180).  It is therefore evaluated once per problem on the
// host, at every RK stage time of every interval, with the reference's own operation order
// (r_i * exp(-(t - t_i)/tauc), summed over i), leaving 2 divisions and ~20 flops per RHS on the GPU.
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
    int32_t nnzk;    // J_g entries per interval (nx * (nz + 1))
    int32_t nhk;     // Hessian entries per interval (nz (nz+1) / 2)
    int32_t n_slide; // sliding-window rows per interval
    int32_t n_params;
    double dt, h;
    // model constants (reciprocals precomputed on the host)
    double inv_tauc, tau2, km_rest, tau1_rest, a_rest, a_scale, pd0, pdt;
    double ar, bs, Is, cr;
    double alpha_a, alpha_tau1, alpha_km, inv_tau_fat, a_fat_rest, mult;
    const double* tab;  // Ding: cs[N*Q]; Hmed: coef[N*Q*TMAX] (zero padded past T)
    const double* rest; // rest state [nx] (IVP default x0)
};

// ---------------------------------------------------------------------------------------------------
// Right-hand side, written once for double / Dual / Jet.
//   cn_dot = (cs - cn) / tauc                                  (ding2003.py:254-266)
//   F_dot  = (A * s - F / (tau1 + tau2 * s)) * (fl*fv + fp),  s = cn / (Km + cn)   (ding2003.py:274-311)
//   A_dot  = -(A - A_rest)/tau_fat + alpha_A F, same for Tau1, Km  (ding2003_with_fatigue.py:197-240)
// Ding2007: A is scaled by afac = 1 - exp(-(pw - pd0)/pdt)  (ding2007.py:172-188); for the model
// without fatigue afac already contains a_scale.
// ---------------------------------------------------------------------------------------------------
template <int MODEL, class S, class CS>
CFX_HD void rhs(const KParams& P, const S* x, const CS& cs, const S& afac, S* dx) {
    const S& cn = x[0];
    const S& F = x[1];
    dx[0] = P.inv_tauc * (cs - cn);
    if constexpr (is_fatigue(MODEL)) {
        const S& A = x[2];
        const S& tau1 = x[3];
        const S& km = x[4];
        const S s = cn / (km + cn);
        if constexpr (is_pw(MODEL)) {
            dx[1] = ((A * afac) * s - F / (tau1 + P.tau2 * s)) * P.mult;
        } else {
            dx[1] = (A * s - F / (tau1 + P.tau2 * s)) * P.mult;
        }
        dx[2] = P.alpha_a * F - (A - P.a_fat_rest) * P.inv_tau_fat;
        dx[3] = P.alpha_tau1 * F - (tau1 - P.tau1_rest) * P.inv_tau_fat;
        dx[4] = P.alpha_km * F - (km - P.km_rest) * P.inv_tau_fat;
    } else {
        const S s = cn / (P.km_rest + cn);
        if constexpr (is_pw(MODEL)) {
            dx[1] = (afac * s - F / (P.tau1_rest + P.tau2 * s)) * P.mult;
        } else {
            dx[1] = (P.a_rest * s - F / (P.tau1_rest + P.tau2 * s)) * P.mult;
        }
    }
}

// Stimulation-sum providers: slot q (= ((k*m + j) * stages + stage)) -> cs value (+ derivatives).
struct CsTable {
    const double* tab;
    CFX_HD double operator()(int q) const { return tab[q]; }
};

// Hmed2018: cs = sum_i coef[q][i] * lambda_i(u_i); lambda values held in registers, the derivative
// enters only along this lane's u-directions (uidx >= 0).
template <int D, int TMAX>
struct CsHmed {
    const double* coef;
    double lamv[TMAX];
    double lamd[D > 0 ? D : 1];
    int uidx[D > 0 ? D : 1];
    CFX_HD Dual<D> operator()(int q) const {
        const double* c = coef + (int64_t)q * TMAX;
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < TMAX; ++i) s += c[i] * lamv[i];
        Dual<D> r;
        r.v = s;
#pragma unroll
        for (int j = 0; j < D; ++j) r.d[j] = uidx[j] >= 0 ? c[uidx[j]] * lamd[j] : 0.0;
        return r;
    }
};

// value-only Hmed provider (g, IVP)
template <int TMAX>
struct CsHmedV {
    const double* coef;
    double lamv[TMAX];
    CFX_HD double operator()(int q) const {
        const double* c = coef + (int64_t)q * TMAX;
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < TMAX; ++i) s += c[i] * lamv[i];
        return s;
    }
};

// m sub-steps of RK-s over one interval (bioptim RK1 = Euler, RK2 = midpoint, RK4 = classic;
// stage times t, t+h/2, t+h/2, t+h; control held constant).  q0 = first RHS slot of the interval.
template <int MODEL, int SCHEME, class S, class CSP>
CFX_HD void integrate_interval(const KParams& P, int q0, S* x, const S& afac, const CSP& csp) {
    constexpr int NX = nx_of(MODEL);
    const double h = P.h;
    const double h2 = 0.5 * P.h;
    const double h6 = P.h / 6.0;
    int q = q0;
    for (int j = 0; j < P.m; ++j) {
        S k1[NX];
        rhs<MODEL>(P, x, csp(q), afac, k1);
        if constexpr (SCHEME == 1) {
#pragma unroll
            for (int r = 0; r < NX; ++r) x[r] = x[r] + h * k1[r];
            q += 1;
        } else if constexpr (SCHEME == 2) {
            S xs[NX], k2[NX];
#pragma unroll
            for (int r = 0; r < NX; ++r) xs[r] = x[r] + h2 * k1[r];
            rhs<MODEL>(P, xs, csp(q + 1), afac, k2);
#pragma unroll
            for (int r = 0; r < NX; ++r) x[r] = x[r] + h * k2[r];
            q += 2;
        } else {
            S xs[NX], acc[NX], kk[NX];
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                acc[r] = k1[r];
                xs[r] = x[r] + h2 * k1[r];
            }
            rhs<MODEL>(P, xs, csp(q + 1), afac, kk);
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                acc[r] = acc[r] + 2.0 * kk[r];
                xs[r] = x[r] + h2 * kk[r];
            }
            rhs<MODEL>(P, xs, csp(q + 2), afac, kk);
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                acc[r] = acc[r] + 2.0 * kk[r];
                xs[r] = x[r] + h * kk[r];
            }
            rhs<MODEL>(P, xs, csp(q + 3), afac, kk);
#pragma unroll
            for (int r = 0; r < NX; ++r) x[r] = x[r] + h6 * (acc[r] + kk[r]);
            q += 4;
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// Kernel 1: continuity residuals g_k = Phi(x_k, u_k) - x_{k+1} and the dense Jacobian block
// dPhi/d(x_k, u_k) (+ the -I on x_{k+1}).  Thread = (instance b, interval k = blockIdx.y,
// direction chunk = blockIdx.z); D directions per lane (D = 0: g only).
// ---------------------------------------------------------------------------------------------------
template <int MODEL, int SCHEME, int D, int TMAX>
__global__ void __launch_bounds__(256) k_shooting(const KParams P, const double* __restrict__ V,
                                                  double* __restrict__ G, double* __restrict__ J) {
    constexpr int NX = nx_of(MODEL);
    using S = Dual<D>;
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int k = blockIdx.y;
    const int chunk = blockIdx.z;
    const int xo = k * P.nz;
    const double* Vb = V + b;

    S x[NX];
#pragma unroll
    for (int r = 0; r < NX; ++r) x[r] = dconst<D>(Vb[(int64_t)(xo + r) * B]);
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const int gd = chunk * D + j;
        if (gd < NX) {
#pragma unroll
            for (int r = 0; r < NX; ++r)
                if (r == gd) x[r].d[j] = 1.0;
        }
    }

    S afac = dconst<D>(0.0);
    if constexpr (is_pw(MODEL)) {
        S pw = dconst<D>(Vb[(int64_t)(xo + NX) * B]);
#pragma unroll
        for (int j = 0; j < D; ++j)
            if (chunk * D + j == NX) pw.d[j] = 1.0;
        const S e = 1.0 - sexp((-1.0) * (pw - P.pd0) / P.pdt);
        afac = is_fatigue(MODEL) ? e : P.a_scale * e;
    }

    if constexpr (is_int(MODEL)) {
        CsHmed<D, TMAX> csp;
        csp.coef = P.tab;
#pragma unroll
        for (int i = 0; i < TMAX; ++i) {
            const double ui = i < P.T ? Vb[(int64_t)(xo + NX + i) * B] : P.Is;
            csp.lamv[i] = i < P.T ? P.ar * (tanh(P.bs * (ui - P.Is)) + P.cr) : 0.0;
        }
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const int gd = chunk * D + j;
            if (gd >= NX && gd < P.nz) {
                const double ui = Vb[(int64_t)(xo + gd) * B];
                const double th = tanh(P.bs * (ui - P.Is));
                csp.lamd[j] = P.ar * P.bs * (1.0 - th * th);
                csp.uidx[j] = gd - NX;
            } else {
                csp.lamd[j] = 0.0;
                csp.uidx[j] = -1;
            }
        }
        integrate_interval<MODEL, SCHEME>(P, k * P.Q, x, afac, csp);
    } else {
        integrate_interval<MODEL, SCHEME>(P, k * P.Q, x, afac, CsTable{P.tab});
    }

    if (G != nullptr && chunk == 0) {
        const int xn = (k + 1) * P.nz;
#pragma unroll
        for (int r = 0; r < NX; ++r)
            G[(int64_t)(k * P.ngk + r) * B + b] = value(x[r]) - Vb[(int64_t)(xn + r) * B];
    }
    if constexpr (D > 0) {
        if (J != nullptr) {
            const int64_t jo = (int64_t)k * P.nnzk;
#pragma unroll
            for (int r = 0; r < NX; ++r) {
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const int gd = chunk * D + j;
                    if (gd < P.nz) J[(jo + r * (P.nz + 1) + gd) * B + b] = x[r].d[j];
                }
                if (chunk == 0) J[(jo + r * (P.nz + 1) + P.nz) * B + b] = -1.0;
            }
        }
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
    double x[NX];
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        x[r] = X0 ? X0[(int64_t)r * B + b] : P.rest[r];
        TR[(int64_t)r * B + b] = x[r];
    }
    int64_t s = 1;
    for (int k = 0; k < P.N; ++k) {
        double afac = 0.0;
        if constexpr (is_pw(MODEL)) {
            const double pw = U[(int64_t)(k * P.nu) * B + b];
            const double e = 1.0 - exp(-(pw - P.pd0) / P.pdt);
            afac = is_fatigue(MODEL) ? e : P.a_scale * e;
        }
        // integrate sub-step by sub-step so every sample is stored
        KParams Pk = P;
        Pk.m = 1;
        CsHmedV<TMAX> csh;
        if constexpr (is_int(MODEL)) {
            csh.coef = P.tab;
#pragma unroll
            for (int i = 0; i < TMAX; ++i) {
                const double ui = i < P.T ? U[(int64_t)(k * P.nu + i) * B + b] : P.Is;
                csh.lamv[i] = i < P.T ? P.ar * (tanh(P.bs * (ui - P.Is)) + P.cr) : 0.0;
            }
        }
        for (int j = 0; j < P.m; ++j) {
            const int q0 = (k * P.m + j) * stages_of(SCHEME);
            if constexpr (is_int(MODEL)) {
                integrate_interval<MODEL, SCHEME>(Pk, q0, x, afac, csh);
            } else {
                integrate_interval<MODEL, SCHEME>(Pk, q0, x, afac, CsTable{P.tab});
            }
#pragma unroll
            for (int r = 0; r < NX; ++r) TR[(s * NX + r) * B + b] = x[r];
            ++s;
        }
    }
}

}  // namespace cfx
