// cfx_msk.h — gfx950 kernels of the musculoskeletal FES path (FesMskModel, cocofest/models/dynamical_model.py).
//
// One right-hand side couples NM FES muscles (the Ding calcium/force[/fatigue] ODEs) to a serial chain of NQ
// revolute dofs (biorbd model reduced on the host, see cfx_api.hip:msk_reduce):
//   frames    R_j = R_{j-1} A_j Rot_axis(q_j), o_j = o_{j-1} + R_{j-1} t_j            (constant [A_j | t_j])
//   muscles   points fixed in a frame; muscle-tendon length L = sum |P_{i+1} - P_i|, length Jacobian
//             J_L[k] = sum u_i . (z_k x (P_{i+1} - o_k) - z_k x (P_i - o_k)) over the dofs above each point;
//             fibre length (L - slack) / cos(pennation); velocity J_L qdot; De Groote FL / FV / FP
//             (cocofest/models/hill_coefficients.py:11-126) scale dF/dt (ding2003.py:274-311)
//   torque    tau = -J_L^T F (+ residual torque)                         (dynamical_model.py:206-334)
//   dynamics  qddot = M(q)^-1 (tau - h(q, qdot)); M from body Jacobians, h by recursive Newton-Euler with
//             qddot = 0 (gravity as a base acceleration), one composite rigid body per dof frame.
// Everything is written once over a generic scalar S: double (values), Dual<D> (Jacobian directions), Jet<D>
// (Lagrangian Hessian blocks) and Dep (structural dependency bitmasks, run on the host to get CasADi-style
// sparsity).  Constants come from an MskGeom block in device memory; every index into it is wave-uniform, so
// the reads are scalar loads.  No MFMA: a 2-dof arm has no dense contraction worth a matrix core.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include <type_traits>

#include "cfx_dual.h"

namespace cfx {

#define MSK_HD __host__ __device__ __forceinline__

constexpr int kMskMaxQ = 4;      // dofs of the serial chain
constexpr int kMskMaxMus = 8;    // muscles
constexpr int kMskMaxPts = 16;   // path points per muscle (origin, via points, insertion)
constexpr int kMskMaxX = kMskMaxMus * 5 + 2 * kMskMaxQ;
constexpr int kMskMaxZ = 64;  // decision variables of one interval (the dependency masks are 64-bit)

// ---- structural dependency bitmask (host sparsity pass) ------------------------------------------------------
struct Dep {
    uint64_t m;
};
MSK_HD Dep operator+(Dep a, Dep b) { return Dep{a.m | b.m}; }
MSK_HD Dep operator-(Dep a, Dep b) { return Dep{a.m | b.m}; }
MSK_HD Dep operator*(Dep a, Dep b) { return Dep{a.m | b.m}; }
MSK_HD Dep operator/(Dep a, Dep b) { return Dep{a.m | b.m}; }
MSK_HD Dep operator+(Dep a, double) { return a; }
MSK_HD Dep operator+(double, Dep a) { return a; }
MSK_HD Dep operator-(Dep a, double) { return a; }
MSK_HD Dep operator-(double, Dep a) { return a; }
MSK_HD Dep operator*(Dep a, double) { return a; }
MSK_HD Dep operator*(double, Dep a) { return a; }
MSK_HD Dep operator/(Dep a, double) { return a; }
MSK_HD Dep operator/(double, Dep a) { return a; }
MSK_HD Dep operator-(Dep a) { return a; }
MSK_HD double value(Dep) { return 1.0; }

template <int D>
CFX_HD Dual<D> operator-(const Dual<D>& a) {
    return 0.0 - a;
}
template <int D>
CFX_HD Jet<D> operator-(const Jet<D>& a) {
    return 0.0 - a;
}

// constants of each scalar type
template <class S>
struct Num;
template <>
struct Num<double> {
    static MSK_HD double c(double v) { return v; }
};
template <>
struct Num<Dep> {
    static MSK_HD Dep c(double) { return Dep{0}; }
};
template <int D>
struct Num<Dual<D>> {
    static CFX_HD Dual<D> c(double v) { return dconst<D>(v); }
};
template <int D>
struct Num<Jet<D>> {
    static CFX_HD Jet<D> c(double v) { return jconst<D>(v); }
};

// ---- elementary functions (value, first and second derivative through the generic chain rule) -----------
MSK_HD double mexp(double x) { return exp(x); }
MSK_HD double mlog(double x) { return log(x); }
MSK_HD double msqrt(double x) { return sqrt(x); }
MSK_HD double msin(double x) { return sin(x); }
MSK_HD double mcos(double x) { return cos(x); }
MSK_HD Dep mexp(Dep a) { return a; }
MSK_HD Dep mlog(Dep a) { return a; }
MSK_HD Dep msqrt(Dep a) { return a; }
MSK_HD Dep msin(Dep a) { return a; }
MSK_HD Dep mcos(Dep a) { return a; }
// sin and cos of one angle from one argument reduction (two separate calls reduce twice)
MSK_HD void msincos(double x, double* s, double* c) {
#if defined(__HIP_DEVICE_COMPILE__)
    sincos(x, s, c);
#else
    *s = std::sin(x);
    *c = std::cos(x);
#endif
}
MSK_HD void msincos(Dep a, Dep* s, Dep* c) { *s = *c = a; }

template <int D>
CFX_HD Dual<D> dchain(const Dual<D>& a, double f0, double f1) {
    Dual<D> r;
    r.v = f0;
#pragma unroll
    for (int i = 0; i < D; ++i) r.d[i] = f1 * a.d[i];
    return r;
}
template <int D>
CFX_HD Dual<D> mexp(const Dual<D>& a) {
    const double e = exp(a.v);
    return dchain(a, e, e);
}
template <int D>
CFX_HD Dual<D> mlog(const Dual<D>& a) {
    return dchain(a, log(a.v), drcp(a.v));
}
template <int D>
CFX_HD Dual<D> msqrt(const Dual<D>& a) {
    const double s = sqrt(a.v);
    return dchain(a, s, 0.5 * drcp(s));
}
template <int D>
CFX_HD Dual<D> msin(const Dual<D>& a) {
    return dchain(a, sin(a.v), cos(a.v));
}
template <int D>
CFX_HD Dual<D> mcos(const Dual<D>& a) {
    return dchain(a, cos(a.v), -sin(a.v));
}
template <int D>
CFX_HD void msincos(const Dual<D>& a, Dual<D>* s, Dual<D>* c) {
    double sv, cv;
    msincos(a.v, &sv, &cv);
    *s = dchain(a, sv, cv);
    *c = dchain(a, cv, -sv);
}
template <int D>
CFX_HD Jet<D> mexp(const Jet<D>& a) {
    const double e = exp(a.v);
    return jchain(a, e, e, e);
}
template <int D>
CFX_HD Jet<D> mlog(const Jet<D>& a) {
    const double i = 1.0 / a.v;
    return jchain(a, log(a.v), i, -i * i);
}
template <int D>
CFX_HD Jet<D> msqrt(const Jet<D>& a) {
    const double s = sqrt(a.v);
    return jchain(a, s, 0.5 / s, -0.25 / (s * a.v));
}
template <int D>
CFX_HD Jet<D> msin(const Jet<D>& a) {
    const double s = sin(a.v), c = cos(a.v);
    return jchain(a, s, c, -s);
}
template <int D>
CFX_HD Jet<D> mcos(const Jet<D>& a) {
    const double s = sin(a.v), c = cos(a.v);
    return jchain(a, c, -s, -c);
}
template <int D>
CFX_HD void msincos(const Jet<D>& a, Jet<D>* s, Jet<D>* c) {
    double sv, cv;
    msincos(a.v, &sv, &cv);
    *s = jchain(a, sv, cv, -sv);
    *c = jchain(a, cv, -sv, -cv);
}

// ---- problem constants ----------------------------------------------------------------------------------------
struct MskMuscleConst {
    double inv_tauc, tau2, km_rest, tau1_rest, a_force;  // a_force: A_rest (Ding2003) or a_scale (Ding2007)
    double pd0, inv_pdt;
    double alpha_a, alpha_tau1, alpha_km, inv_tau_fat, a_fat_rest;
    double inv_lopt, slack, inv_cos_penn;
    double ar, bs, Is, cr;  // Hmed2018 recruitment curve lambda(I) (hmed2018.py:169-180)
};

struct MskGeom {
    int32_t axis[kMskMaxQ];        // always 2: cfx_msk_create turns every joint into a rotation about its frame's z
    double A[kMskMaxQ][9];         // constant rotation from frame j-1 (ground for j = 0) to dof j's joint frame
    double t[kMskMaxQ][3];         // its translation, in frame j-1
    double grav[3];
    double mass[kMskMaxQ];         // composite body moving with frame j (mass, com and inertia about the com, in frame j)
    double com[kMskMaxQ][3];
    double inertia[kMskMaxQ][9];
    // muscle paths: only the segments whose ends move with different frames (-1: ground) vary with q; the
    // segments inside one rigid frame contribute a constant length and nothing to the length Jacobian
    int32_t nseg[kMskMaxMus];
    int32_t seg_frame[kMskMaxMus][kMskMaxPts][2];
    double seg_pos[kMskMaxMus][kMskMaxPts][2][3];
    double const_len[kMskMaxMus];
    MskMuscleConst mc[kMskMaxMus];
    int32_t fl_on, fv_on, fp_on;
    int16_t jpos[kMskMaxX * kMskMaxZ];  // J_g value offset of dPhi_r/dz_c inside an interval block (-1: zero)
    int16_t jneg[kMskMaxX];            // offset of the -1 on x_{k+1}[r]
};

struct MskParams {
    int64_t B;
    int32_t N, m, nx, nu, nz, Q, nnzk, nhk, residual, npw;
    int32_t T, ngk;      // truncation; rows per interval (nx continuity rows, then the Hmed sliding-window rows)
    int32_t kpb;         // k_msk_tangents_lds: consecutive intervals per block (fixed by cfx_msk_create)
    int32_t keepc;       // CFX_KEEP_CONSTANT_JAC: the -1 on x_{k+1} is not stored (the output holds it already)
    int32_t hgrp[3];     // k_msk_hpair's task groups (cfx_msk_create orders the tasks so): pairs without q, with one
                         // q (listed first), with two
    double dt, h;
    // calcium sums [N][Q][NM] at every RK stage time (host, reference operation order); Hmed2018: the per-pulse
    // coefficients r_i exp(-(t - t_i) / tau_c) [N][Q][NM][TMAX] of cs = sum_i coef_i lambda(I_i)
    const double* cs;
    // CFX_MSK_LEGACY_CALCIUM (fatigue families): d cs / d Km [N][Q][NM] — the stored revision's r0 = Km + r0_km
    // makes cs affine in the Km state, cs = table + (Km - km_rest) cs1; nullptr: today's r0 = km_rest + r0_km
    const double* cs1;
    const double* rest;  // rest state [nx] (IVP default x0)
    double* scratch;     // k_msk_stagecoef_par -> k_msk_tangents: per-stage Jacobian coefficients [N][Q][NC][B]
};

template <int FAM>
constexpr int msk_nxm() {
    return (FAM & 1) ? 5 : 2;
}
template <int FAM>
constexpr bool msk_pw() {
    return FAM == 2 || FAM == 3;
}
// Hmed2018 families: 4 / 5 (T <= 10), 6 / 7 (T <= 20); bit 0 is fatigue as for the Ding families
template <int FAM>
constexpr bool msk_hmed() {
    return FAM >= 4;
}
template <int FAM>
constexpr int msk_tmax() {
    return FAM < 4 ? 0 : (FAM < 6 ? 10 : 20);
}
// Controls in the kernels' canonical slots: [pulse widths (Ding2007) | TMAX intensities per muscle (Hmed2018) |
// residual torques]; msk_udec maps a slot to its control index in the decision vector (-1: a padding intensity
// past the truncation, or a residual torque the problem does not have).
template <int NM, int FAM>
constexpr int msk_nui() {
    return (msk_pw<FAM>() ? NM : 0) + NM * msk_tmax<FAM>();
}
template <int NQ, int NM, int FAM>
constexpr int msk_numax() {
    return msk_nui<NM, FAM>() + NQ;
}
template <int NM, int FAM>
MSK_HD int msk_udec(int c, int T, int nu) {
    if constexpr (msk_hmed<FAM>()) {
        constexpr int TM = msk_tmax<FAM>();
        if (c < NM * TM) {
            const int m = c / TM, j = c - m * TM;
            return j < T ? m * T + j : -1;
        }
        const int d = NM * T + (c - NM * TM);
        return d < nu ? d : -1;
    } else {
        return c < nu ? c : -1;
    }
}
// stride of the stage table P.cs per (interval, stage)
template <int NM, int FAM>
constexpr int msk_cs_stride() {
    return msk_hmed<FAM>() ? NM * msk_tmax<FAM>() : NM;
}
// Hmed2018 recruitment lambda(I) = ar (tanh(bs (I - Is)) + cr) and its first two derivatives (hmed2018.py:169-180)
MSK_HD void msk_lambda(const MskMuscleConst& L, double I, double& l0, double& l1, double& l2) {
    const double t = tanh(L.bs * (I - L.Is)), s = 1.0 - t * t;
    l0 = L.ar * (t + L.cr);
    l1 = L.ar * L.bs * s;
    l2 = -2.0 * L.ar * L.bs * L.bs * t * s;
}
// the lambdas of one interval's intensities (canonical slots u[mu TMAX + i])
template <int NM, int FAM, class SU>
MSK_HD void msk_interval_lam(const MskGeom& G, const SU* u, double* lam) {
    if constexpr (msk_hmed<FAM>()) {
        constexpr int TM = msk_tmax<FAM>();
#pragma unroll
        for (int mu = 0; mu < NM; ++mu)
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                double l1, l2;
                msk_lambda(G.mc[mu], value(u[mu * TM + i]), lam[mu * TM + i], l1, l2);
            }
    }
}
// the NM calcium sums of stage kq: the table (Ding) or sum_i coef_i lambda_i (Hmed; lam: the NM * TMAX lambdas of
// the interval's intensities, nullptr on the host dependency pass, where only the structure matters)
template <int NM, int FAM>
MSK_HD void msk_stage_cs(const double* __restrict__ tab, int64_t kq, const double* lam, double* cs) {
    if constexpr (msk_hmed<FAM>()) {
        constexpr int TM = msk_tmax<FAM>();
        const double* c = tab + kq * NM * TM;
#pragma unroll
        for (int mu = 0; mu < NM; ++mu) {
            double sum = 0.0;
            if (lam) {
#pragma unroll
                for (int i = 0; i < TM; ++i) sum = sum + c[mu * TM + i] * lam[mu * TM + i];
            }
            cs[mu] = sum;
        }
    } else {
#pragma unroll
        for (int mu = 0; mu < NM; ++mu) cs[mu] = tab[kq * NM + mu];
    }
}

// legacy calcium: the stage's d cs / d Km per muscle (nullptr when off)
template <int NM>
MSK_HD const double* msk_cs1(const MskParams& P, int64_t kq) {
    return P.cs1 ? P.cs1 + kq * NM : nullptr;
}

// ---- small vector helpers ---------------------------------------------------------------------------------------
// c ? a : b field by field: a conditional on whole dual numbers is lowered to a copy from a selected address, which
// keeps the operands in scratch memory
MSK_HD double msel(bool c, double a, double b) { return c ? a : b; }
MSK_HD Dep msel(bool c, Dep a, Dep b) { return c ? a : b; }
template <int D>
CFX_HD Dual<D> msel(bool c, const Dual<D>& a, const Dual<D>& b) {
    Dual<D> r;
    r.v = c ? a.v : b.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.d[i] = c ? a.d[i] : b.d[i];
    return r;
}
template <int D>
CFX_HD Jet<D> msel(bool c, const Jet<D>& a, const Jet<D>& b) {
    Jet<D> r;
    r.v = c ? a.v : b.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.g[i] = c ? a.g[i] : b.g[i];
#pragma unroll
    for (int i = 0; i < Jet<D>::H; ++i) r.h[i] = c ? a.h[i] : b.h[i];
    return r;
}
template <class S>
MSK_HD void cross3(const S* a, const S* b, S* r) {
    r[0] = a[1] * b[2] - a[2] * b[1];
    r[1] = a[2] * b[0] - a[0] * b[2];
    r[2] = a[0] * b[1] - a[1] * b[0];
}
template <class S>
MSK_HD S dot3(const S* a, const S* b) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

// Frames of the chain: R[j] (row-major 3x3), o[j], joint axis z[j] (world).
template <int NQ, class S>
MSK_HD void msk_frames(const MskGeom& G, const S* q, S (*R)[9], S (*o)[3], S (*z)[3]) {
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
        S Rb[9];
        if (j == 0) {
#pragma unroll
            for (int e = 0; e < 9; ++e) Rb[e] = Num<S>::c(G.A[0][e]);
#pragma unroll
            for (int e = 0; e < 3; ++e) o[0][e] = Num<S>::c(G.t[0][e]);
        } else {
#pragma unroll
            for (int r = 0; r < 3; ++r) {
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    Rb[r * 3 + c] = R[j - 1][r * 3] * G.A[j][c] + R[j - 1][r * 3 + 1] * G.A[j][3 + c] +
                                    R[j - 1][r * 3 + 2] * G.A[j][6 + c];
                o[j][r] = o[j - 1][r] + R[j - 1][r * 3] * G.t[j][0] + R[j - 1][r * 3 + 1] * G.t[j][1] +
                          R[j - 1][r * 3 + 2] * G.t[j][2];
            }
        }
        S s, c;
        msincos(q[j], &s, &c);
        // R_j = Rb Rot_z(q): columns 0 and 1 mix, the axis column 2 is kept (cfx_msk_create expresses every joint
        // as a rotation about its frame's z axis, G.axis[j] == 2)
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const S ca = Rb[r * 3 + 0], cb = Rb[r * 3 + 1], cz = Rb[r * 3 + 2];
            R[j][r * 3 + 0] = ca * c + cb * s;
            R[j][r * 3 + 1] = cb * c - ca * s;
            R[j][r * 3 + 2] = cz;
            z[j][r] = cz;
        }
    }
}

// World position of a point fixed in frame f (-1: ground) and its Jacobian columns z_k x (P - o_k), k <= f.
template <int NQ, class S>
MSK_HD void msk_point(const S (*R)[9], const S (*o)[3], const S (*z)[3], int f, const double* p, S* P, S (*dP)[3]) {
#pragma unroll
    for (int e = 0; e < 3; ++e) P[e] = Num<S>::c(p[e]);
#pragma unroll
    for (int k = 0; k < NQ; ++k)
#pragma unroll
        for (int e = 0; e < 3; ++e) dP[k][e] = Num<S>::c(0.0);
    if constexpr (std::is_same<S, double>::value) {
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
            if (f == j) {
#pragma unroll
                for (int e = 0; e < 3; ++e)
                    P[e] = o[j][e] + R[j][e * 3] * p[0] + R[j][e * 3 + 1] * p[1] + R[j][e * 3 + 2] * p[2];
#pragma unroll
                for (int k = 0; k <= j; ++k) {
                    S r[3] = {P[0] - o[k][0], P[1] - o[k][1], P[2] - o[k][2]};
                    cross3(z[k], r, dP[k]);
                }
            }
        }
        return;
    }
    // dual numbers: the point's own frame only, one branch per frame (f is wave-uniform).  Each branch ends in an
    // inline-asm marker of its own: without it the compiler merged the branches' identical tails into copies from
    // R[f] / o[f] with f a run-time index, which kept the frames in scratch memory
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
        if (f == j) {
#pragma unroll
            for (int e = 0; e < 3; ++e)
                P[e] = o[j][e] + R[j][e * 3] * p[0] + R[j][e * 3 + 1] * p[1] + R[j][e * 3 + 2] * p[2];
#pragma unroll
            for (int k = 0; k <= j; ++k) {
                const S r[3] = {P[0] - o[k][0], P[1] - o[k][1], P[2] - o[k][2]};
                cross3(z[k], r, dP[k]);
            }
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("; msk_point frame %0" ::"n"(j));
#endif
        }
    }
}

// De Groote force-length (hill_coefficients.py:11-63), force-velocity (66-96), passive force (99-126).
template <class S>
MSK_HD S hill_fl(const S& nl) {
    const double b1[3] = {0.815, 0.433, 0.100}, b2[3] = {1.055, 0.717, 1.000}, b3[3] = {0.162, -0.030, 0.354},
                 b4[3] = {0.063, 0.200, 0.0};
    S r = Num<S>::c(0.0);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const S d = nl - b2[i];
        const S w = b3[i] + b4[i] * nl;
        r = r + b1[i] * mexp((-0.5 * (d * d)) / (w * w));
    }
    return r;
}
template <class S>
MSK_HD S hill_fv(const S& vel) {
    const S w = (-8.149 * (vel / 10.0)) + (-0.374);
    return -0.318 * mlog(w + msqrt(w * w + 1.0)) + 0.886;
}
template <class S>
MSK_HD S hill_fp(const S& nl) {
    const S fp = (mexp(4.0 * (nl - 1.0) / 0.6) - 1.0) / (exp(4.0) - 1.0);
    return msel(value(fp) > 0.0, fp, Num<S>::c(0.0));
}

// Promotion of a q-only quantity (SQ) to the (q, qdot) scalar (SV): identity when both are the same type, else
// Dual<nq> -> Dual<2 nq> with zero qdot directions.
template <class T>
struct DualN;
template <int D>
struct DualN<Dual<D>> {
    static constexpr int n = D;
};
template <int B, int A>
CFX_HD Dual<B> dual_up(const Dual<A>& a) {
    Dual<B> r = dconst<B>(a.v);
#pragma unroll
    for (int i = 0; i < A; ++i) r.d[i] = a.d[i];
    return r;
}
template <class T>
struct IsJet : std::false_type {};
template <int D>
struct IsJet<Jet<D>> : std::true_type {};
template <class SV, class SQ>
MSK_HD SV up(const SQ& a) {
    if constexpr (std::is_same<SV, SQ>::value) {
        return a;
    } else if constexpr (std::is_same<SQ, double>::value) {
        return Num<SV>::c(a);
    } else if constexpr (IsJet<SV>::value) {  // Dual<1> in the pair's first direction, no second derivatives
        SV r = Num<SV>::c(a.v);
        r.g[0] = a.d[0];
        return r;
    } else {
        return dual_up<DualN<SV>::n>(a);
    }
}
template <class SV, class SQ>
MSK_HD void up3(const SQ* a, SV* r) {
#pragma unroll
    for (int e = 0; e < 3; ++e) r[e] = up<SV>(a[e]);
}

// The skeleton of FesMskModel.muscle_dynamic (dynamical_model.py:133-334) for given muscle forces F: frames,
// every muscle's length / length Jacobian / velocity and its Hill multiplier mult = FL FV (+ FP), the joint
// torques -J_L^T F (+ residual taur, nullable) and the forward dynamics qdd.  Mv / JLv (nullable) receive the
// values of M and J_L.  Quantities that depend on q only (frames, muscle geometry, the body Jacobians, M) are
// computed in SQ, those that also depend on qdot (velocities, Hill FV, Newton-Euler, qdd) in SV: with
// SQ = Dual<nq>, SV = Dual<2 nq> the q-only half of the work carries half the derivative directions.
template <int NQ, int NM, class SV, class SQ>
MSK_HD void msk_skeleton(const MskGeom& G, const SQ* q, const SV* qd, const SV* F, const SV* taur, SV* mult, SV* qdd,
                         double (*Mv)[NQ], double (*JLv)[NQ]) {
    SQ R[NQ][9], o[NQ][3], z[NQ][3];
    msk_frames<NQ>(G, q, R, o, z);
    SV tau[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) tau[k] = taur ? taur[k] : Num<SV>::c(0.0);
#pragma unroll
    for (int mu = 0; mu < NM; ++mu) {
        const MskMuscleConst& C = G.mc[mu];
        // ---- geometry: muscle-tendon length and its Jacobian over the frame-crossing segments
        SQ L = Num<SQ>::c(G.const_len[mu]), JL[NQ];
#pragma unroll
        for (int k = 0; k < NQ; ++k) JL[k] = Num<SQ>::c(0.0);
        const int ns = G.nseg[mu];
        for (int i = 0; i < ns; ++i) {
            SQ P0[3], dP0[NQ][3], P1[3], dP1[NQ][3];
            msk_point<NQ>(R, o, z, G.seg_frame[mu][i][0], G.seg_pos[mu][i][0], P0, dP0);
            msk_point<NQ>(R, o, z, G.seg_frame[mu][i][1], G.seg_pos[mu][i][1], P1, dP1);
            const SQ d[3] = {P1[0] - P0[0], P1[1] - P0[1], P1[2] - P0[2]};
            const SQ n = msqrt(dot3(d, d));
            const SQ inv = 1.0 / n;
            L = L + n;
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                const SQ dd[3] = {dP1[k][0] - dP0[k][0], dP1[k][1] - dP0[k][1], dP1[k][2] - dP0[k][2]};
                JL[k] = JL[k] + dot3(d, dd) * inv;
            }
        }
        // ---- Hill coefficients
        const SQ nl = ((L - C.slack) * C.inv_cos_penn) * C.inv_lopt;
        SV JLu[NQ];
        SV vel = Num<SV>::c(0.0);
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            JLu[k] = up<SV>(JL[k]);
            vel = vel + JLu[k] * qd[k];
        }
        const SV fl = msel(G.fl_on, up<SV>(hill_fl(nl)), Num<SV>::c(1.0));
        const SV fv = msel(G.fv_on, hill_fv(vel), Num<SV>::c(1.0));
        mult[mu] = G.fp_on ? fl * fv + up<SV>(hill_fp(nl)) : fl * fv;
        // ---- joint torque -J_L^T F (dynamical_model.py:331-332)
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            tau[k] = tau[k] - JLu[k] * F[mu];
            if (JLv) JLv[mu][k] = value(JL[k]);
        }
    }
    // ---- rigid-body dynamics: h by Newton-Euler (qddot = 0), M from the body Jacobians
    SV w[3] = {Num<SV>::c(0.0), Num<SV>::c(0.0), Num<SV>::c(0.0)};
    SV al[3] = {Num<SV>::c(0.0), Num<SV>::c(0.0), Num<SV>::c(0.0)};
    SV acc[3] = {Num<SV>::c(-G.grav[0]), Num<SV>::c(-G.grav[1]), Num<SV>::c(-G.grav[2])};
    SV h[NQ];
    SQ M[NQ][NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        h[i] = Num<SV>::c(0.0);
#pragma unroll
        for (int k = 0; k < NQ; ++k) M[i][k] = Num<SQ>::c(0.0);
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
        SV zj[3];
        up3(z[j], zj);
        if (j > 0) {
            const SQ rq[3] = {o[j][0] - o[j - 1][0], o[j][1] - o[j - 1][1], o[j][2] - o[j - 1][2]};
            SV r[3], t1[3], t2[3], t3[3];
            up3(rq, r);
            cross3(al, r, t1);
            cross3(w, r, t2);
            cross3(w, t2, t3);
#pragma unroll
            for (int e = 0; e < 3; ++e) acc[e] = acc[e] + t1[e] + t3[e];
            const SV zq[3] = {zj[0] * qd[j], zj[1] * qd[j], zj[2] * qd[j]};
            SV t4[3];
            cross3(w, zq, t4);
#pragma unroll
            for (int e = 0; e < 3; ++e) {
                al[e] = al[e] + t4[e];
                w[e] = w[e] + zq[e];
            }
        } else {
#pragma unroll
            for (int e = 0; e < 3; ++e) w[e] = zj[e] * qd[0];
        }
        if (G.mass[j] == 0.0) continue;
        // composite body of frame j
        SQ rc[3], c[3];
#pragma unroll
        for (int e = 0; e < 3; ++e) {
            rc[e] = R[j][e * 3] * G.com[j][0] + R[j][e * 3 + 1] * G.com[j][1] + R[j][e * 3 + 2] * G.com[j][2];
            c[e] = o[j][e] + rc[e];
        }
        SQ RI[9], Iw[9];  // Iw = R I R^T
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int cc = 0; cc < 3; ++cc)
                RI[r * 3 + cc] = R[j][r * 3] * G.inertia[j][cc] + R[j][r * 3 + 1] * G.inertia[j][3 + cc] +
                                 R[j][r * 3 + 2] * G.inertia[j][6 + cc];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int cc = 0; cc < 3; ++cc)
                Iw[r * 3 + cc] = RI[r * 3] * R[j][cc * 3] + RI[r * 3 + 1] * R[j][cc * 3 + 1] + RI[r * 3 + 2] * R[j][cc * 3 + 2];
        SV rcu[3], t1[3], t2[3], t3[3], Fb[3], Iwu[9];
        up3(rc, rcu);
#pragma unroll
        for (int e = 0; e < 9; ++e) Iwu[e] = up<SV>(Iw[e]);
        cross3(al, rcu, t1);
        cross3(w, rcu, t2);
        cross3(w, t2, t3);
        const double mj = G.mass[j];
#pragma unroll
        for (int e = 0; e < 3; ++e) Fb[e] = mj * (acc[e] + t1[e] + t3[e]);
        SV Iwa[3], Iww[3], t5[3], Nb[3];
#pragma unroll
        for (int e = 0; e < 3; ++e) {
            Iwa[e] = Iwu[e * 3] * al[0] + Iwu[e * 3 + 1] * al[1] + Iwu[e * 3 + 2] * al[2];
            Iww[e] = Iwu[e * 3] * w[0] + Iwu[e * 3 + 1] * w[1] + Iwu[e * 3 + 2] * w[2];
        }
        cross3(w, Iww, t5);
#pragma unroll
        for (int e = 0; e < 3; ++e) Nb[e] = Iwa[e] + t5[e];
        SQ Jv[NQ][3], IJ[NQ][3];
#pragma unroll
        for (int i = 0; i <= j; ++i) {
            const SQ rq[3] = {c[0] - o[i][0], c[1] - o[i][1], c[2] - o[i][2]};
            SV r[3], zi[3], m1[3];
            up3(rq, r);
            up3(z[i], zi);
            cross3(r, Fb, m1);
            const SV mm[3] = {m1[0] + Nb[0], m1[1] + Nb[1], m1[2] + Nb[2]};
            h[i] = h[i] + dot3(zi, mm);
            cross3(z[i], rq, Jv[i]);
#pragma unroll
            for (int e = 0; e < 3; ++e) IJ[i][e] = Iw[e * 3] * z[i][0] + Iw[e * 3 + 1] * z[i][1] + Iw[e * 3 + 2] * z[i][2];
        }
#pragma unroll
        for (int i = 0; i <= j; ++i)
#pragma unroll
            for (int k = 0; k <= i; ++k) M[i][k] = M[i][k] + mj * dot3(Jv[i], Jv[k]) + dot3(z[i], IJ[k]);
    }
    if (Mv) {
#pragma unroll
        for (int i = 0; i < NQ; ++i)
#pragma unroll
            for (int k = 0; k <= i; ++k) Mv[i][k] = Mv[k][i] = value(M[i][k]);
    }
    // ---- solve M qddot = tau - h (symmetric positive definite, unrolled Cholesky)
    SV rhs[NQ], Mu[NQ][NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        rhs[i] = tau[i] - h[i];
#pragma unroll
        for (int k = 0; k <= i; ++k) Mu[i][k] = up<SV>(M[i][k]);
    }
    if constexpr (NQ == 1) {
        qdd[0] = rhs[0] / Mu[0][0];
    } else if constexpr (NQ == 2) {
        const SV det = Mu[0][0] * Mu[1][1] - Mu[1][0] * Mu[1][0];
        qdd[0] = (Mu[1][1] * rhs[0] - Mu[1][0] * rhs[1]) / det;
        qdd[1] = (Mu[0][0] * rhs[1] - Mu[1][0] * rhs[0]) / det;
    } else {
        SV Lc[NQ][NQ];
#pragma unroll
        for (int i = 0; i < NQ; ++i)
#pragma unroll
            for (int k = 0; k <= i; ++k) {
                SV sum = Mu[i][k];
#pragma unroll
                for (int p = 0; p < k; ++p) sum = sum - Lc[i][p] * Lc[k][p];
                Lc[i][k] = i == k ? msqrt(sum) : sum / Lc[k][k];
            }
        SV y[NQ];
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
            SV sum = rhs[i];
#pragma unroll
            for (int p = 0; p < i; ++p) sum = sum - Lc[i][p] * y[p];
            y[i] = sum / Lc[i][i];
        }
#pragma unroll
        for (int i = NQ - 1; i >= 0; --i) {
            SV sum = y[i];
#pragma unroll
            for (int p = i + 1; p < NQ; ++p) sum = sum - Lc[p][i] * qdd[p];
            qdd[i] = sum / Lc[i][i];
        }
    }
}

// FesMskModel.muscle_dynamic for one state: f = dx/dt.  cs[m]: calcium sum of muscle m at this stage time.
// q (SQ) may carry fewer derivative directions than the rest of the state (k_msk_hpair: the frames of a pair that does
// not involve q are plain values)
template <int NQ, int NM, int FAM, class S, class SQ>
MSK_HD void msk_rhs_q(const MskGeom& G, int residual, const double* cs, const double* cs1, const S* x, const SQ* q,
                      const S* u, S* f) {
    constexpr int NXM = msk_nxm<FAM>();
    constexpr bool FAT = (FAM & 1) != 0, PW = msk_pw<FAM>();
    constexpr int XQ = NM * NXM, XQD = XQ + NQ;
    constexpr int NUI = msk_nui<NM, FAM>();
    S F[NM], mult[NM], qdd[NQ], taur[NQ];
#pragma unroll
    for (int mu = 0; mu < NM; ++mu) F[mu] = x[mu * NXM + 1];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
        if (residual) taur[k] = u[NUI + k];
        else taur[k] = Num<S>::c(0.0);
    }
    msk_skeleton<NQ, NM>(G, q, x + XQD, F, taur, mult, qdd, nullptr, nullptr);
#pragma unroll
    for (int mu = 0; mu < NM; ++mu) {
        const MskMuscleConst& C = G.mc[mu];
        // FES muscle ODE (ding2003.py:254-311, ding2003_with_fatigue.py:197-240, ding2007.py:172-188)
        const S& cn = x[mu * NXM];
        f[mu * NXM] = (cs[mu] - cn) * C.inv_tauc;
        if constexpr (msk_hmed<FAM>() && std::is_same<S, Dep>::value) {
            // structure pass: cn_dot reads the muscle's intensities through cs (hmed2018.py:97-98)
#pragma unroll
            for (int i = 0; i < msk_tmax<FAM>(); ++i) f[mu * NXM] = f[mu * NXM] + u[mu * msk_tmax<FAM>() + i];
        }
        S km = Num<S>::c(C.km_rest), tau1 = Num<S>::c(C.tau1_rest), A = Num<S>::c(C.a_force);
        if constexpr (FAT) {
            A = x[mu * NXM + 2];
            tau1 = x[mu * NXM + 3];
            km = x[mu * NXM + 4];
            if (cs1) f[mu * NXM] = f[mu * NXM] + (km - C.km_rest) * (cs1[mu] * C.inv_tauc);  // legacy r0 = Km + r0_km
        }
        S Aeff = A;
        if constexpr (PW) Aeff = A * (1.0 - mexp(-(u[mu] - C.pd0) * C.inv_pdt));
        const S s = cn / (km + cn);
        f[mu * NXM + 1] = (Aeff * s - F[mu] / (tau1 + C.tau2 * s)) * mult[mu];
        if constexpr (FAT) {
            f[mu * NXM + 2] = C.alpha_a * F[mu] - (A - C.a_fat_rest) * C.inv_tau_fat;
            f[mu * NXM + 3] = C.alpha_tau1 * F[mu] - (tau1 - C.tau1_rest) * C.inv_tau_fat;
            f[mu * NXM + 4] = C.alpha_km * F[mu] - (km - C.km_rest) * C.inv_tau_fat;
        }
    }
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
        f[XQ + k] = x[XQD + k];
        f[XQD + k] = qdd[k];
    }
}

template <int NQ, int NM, int FAM, class S>
MSK_HD void msk_rhs(const MskGeom& G, int residual, const double* cs, const double* cs1, const S* x, const S* u,
                    S* f) {
    msk_rhs_q<NQ, NM, FAM>(G, residual, cs, cs1, x, x + NM * msk_nxm<FAM>(), u, f);
}

// Phi_m(x, u) over interval k: m RK sub-steps (bioptim convention: constant control, RK4 stage times
// t, t + h/2, t + h/2, t + h).  x is overwritten with the end state.  LEG: legacy calcium (P.cs1 set) — a compile-time
// choice, because a pointer chosen at run time between the local stage array and null kept the array in scratch memory.
template <int NQ, int NM, int FAM, int SCHEME, bool LEG, class S>
MSK_HD void msk_interval_t(const MskParams& P, const MskGeom& G, int k, S* x, const S* u, const double* lam) {
    constexpr int NX = NM * msk_nxm<FAM>() + 2 * NQ;
    constexpr int ST = SCHEME == 4 ? 4 : (SCHEME == 2 ? 2 : 1);
    constexpr int NMC = NM;
    const double h = P.h;
    for (int j = 0; j < P.m; ++j) {
        double csv[ST * NMC], csv1[LEG ? ST * NMC : 1];  // the stage sums of this sub-step (and their d / d Km)
#pragma unroll
        for (int st = 0; st < ST; ++st) {
            msk_stage_cs<NM, FAM>(P.cs, (int64_t)k * P.Q + j * ST + st, lam, csv + st * NMC);
            if constexpr (LEG)
#pragma unroll
                for (int mu = 0; mu < NM; ++mu) csv1[st * NMC + mu] = P.cs1[((int64_t)k * P.Q + j * ST + st) * NM + mu];
        }
        const double* cs = csv;
        auto c1s = [&](int st) -> const double* {
            if constexpr (LEG) return csv1 + st * NMC;
            return nullptr;
        };
        if constexpr (SCHEME == 1) {
            S f[NX];
            msk_rhs<NQ, NM, FAM>(G, P.residual, cs, c1s(0), x, u, f);
#pragma unroll
            for (int r = 0; r < NX; ++r) x[r] = x[r] + h * f[r];
        } else if constexpr (SCHEME == 2) {
            S f[NX], xs[NX];
            msk_rhs<NQ, NM, FAM>(G, P.residual, cs, c1s(0), x, u, f);
#pragma unroll
            for (int r = 0; r < NX; ++r) xs[r] = x[r] + (0.5 * h) * f[r];
            msk_rhs<NQ, NM, FAM>(G, P.residual, cs + NMC, c1s(1), xs, u, f);
#pragma unroll
            for (int r = 0; r < NX; ++r) x[r] = x[r] + h * f[r];
        } else {
            S acc[NX], xs[NX], f[NX];
            msk_rhs<NQ, NM, FAM>(G, P.residual, cs, c1s(0), x, u, f);
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                acc[r] = f[r];
                xs[r] = x[r] + (0.5 * h) * f[r];
            }
            msk_rhs<NQ, NM, FAM>(G, P.residual, cs + NMC, c1s(1), xs, u, f);
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                acc[r] = acc[r] + 2.0 * f[r];
                xs[r] = x[r] + (0.5 * h) * f[r];
            }
            msk_rhs<NQ, NM, FAM>(G, P.residual, cs + 2 * NMC, c1s(2), xs, u, f);
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                acc[r] = acc[r] + 2.0 * f[r];
                xs[r] = x[r] + h * f[r];
            }
            msk_rhs<NQ, NM, FAM>(G, P.residual, cs + 3 * NMC, c1s(3), xs, u, f);
#pragma unroll
            for (int r = 0; r < NX; ++r) x[r] = x[r] + (h / 6.0) * (acc[r] + f[r]);
        }
    }
}

template <int NQ, int NM, int FAM, int SCHEME, class S>
MSK_HD void msk_interval(const MskParams& P, const MskGeom& G, int k, S* x, const S* u, const double* lam) {
    if (P.cs1) msk_interval_t<NQ, NM, FAM, SCHEME, true>(P, G, k, x, u, lam);
    else msk_interval_t<NQ, NM, FAM, SCHEME, false>(P, G, k, x, u, lam);
}

// ---- g + J_g: thread = (instance, interval, chunk of D Jacobian directions) ---------------------------------
template <int NQ, int NM, int FAM, int SCHEME, int D>
__global__ void __launch_bounds__(256) k_msk_shooting(const MskParams P, const MskGeom* __restrict__ GG,
                                                      const double* __restrict__ V, double* __restrict__ Gout,
                                                      double* __restrict__ J) {
    constexpr int NX = NM * msk_nxm<FAM>() + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int k = blockIdx.y;
    const int c0 = blockIdx.z * D;
    const MskGeom& G = *GG;
    const int nz = P.nz, nu = P.nu;
    const int64_t zb = (int64_t)k * nz;
    using S = Dual<D>;
    S x[NX], u[NUMAX > 0 ? NUMAX : 1];
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        x[r] = dconst<D>(V[(zb + r) * B + b]);
#pragma unroll
        for (int d = 0; d < D; ++d) x[r].d[d] = (r == c0 + d) ? 1.0 : 0.0;
    }
#pragma unroll
    for (int i = 0; i < NUMAX; ++i) {
        const int dc = msk_udec<NM, FAM>(i, P.T, nu);
        u[i] = dconst<D>(dc >= 0 ? V[(zb + NX + dc) * B + b] : 0.0);
#pragma unroll
        for (int d = 0; d < D; ++d) u[i].d[d] = (dc >= 0 && NX + dc == c0 + d) ? 1.0 : 0.0;
    }
    double xn[NX];
    if (Gout && blockIdx.z == 0) {
#pragma unroll
        for (int r = 0; r < NX; ++r) xn[r] = V[(zb + nz + r) * B + b];
    }
    double lam[msk_hmed<FAM>() ? NM * msk_tmax<FAM>() : 1];
    msk_interval_lam<NM, FAM>(G, u, lam);
    msk_interval<NQ, NM, FAM, SCHEME>(P, G, k, x, u, lam);
    if (Gout && blockIdx.z == 0) {
#pragma unroll
        for (int r = 0; r < NX; ++r) Gout[((int64_t)k * P.ngk + r) * B + b] = x[r].v - xn[r];
    }
    if (J) {
        const int64_t jb = (int64_t)k * P.nnzk;
#pragma unroll
        for (int r = 0; r < NX; ++r)
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int col = c0 + d;
                if (col < nz) {
                    const int pos = G.jpos[r * kMskMaxZ + col];
                    if (pos >= 0) J[(jb + pos) * B + b] = x[r].d[d];
                }
            }
        if (blockIdx.z == 0 && !P.keepc) {
#pragma unroll
            for (int r = 0; r < NX; ++r) J[(jb + G.jneg[r]) * B + b] = -1.0;
        }
    }
}

// ---- g + J_g, structured (three launches) -------------------------------------------------------------------
// The muscle ODEs touch the skeleton only through mult_m(q, qdot) (Hill multiplier) and the forces F_m, and the
// skeleton is linear in F and in the residual torque: qdd = a(q, qdot) + sum_m B_m(q) F_m + M^-1 tau.  So every
// RK stage's RHS Jacobian is assembled from one Dual<2 nq> pass of the skeleton over (q, qdot) — independent of
// how many Jacobian columns are wanted — the values of B_m = -M^-1 J_L[m]^T and M^-1, and the analytic partials
// of the muscle ODEs (ding2003.py:254-311, ding2003_with_fatigue.py:197-240, ding2007.py:172-188).
//   k_msk_values     thread = (instance, interval): the value recursion (g), every stage input stored (XS);
//   k_msk_stagecoef_par  thread = (instance, interval, stage): per RK stage (skeleton in Dual<nq> for the q-only
//                    part, Dual<2 nq> for the velocity-dependent part), those NC coefficients, stored
//                    element-major over the batch in a scratch buffer;
//   k_msk_tangents   thread = (instance, interval, Jacobian column): the RK recursion of one tangent column
//                    through the stored stage Jacobians (~100 FMAs per stage); a block holds 256 consecutive
//                    instances of one column (coalesced loads and J stores), XCD-aware block numbering.

template <int NQ, int NM>
constexpr int msk_ncoef() {
    return NM * (6 + 2 * NQ) + 3 * NQ * NQ + NQ * NM;
}

// dF'/d(cn, F, A, Tau1, Km, pw) (times the Hill multiplier) and base = A_eff s - F / (tau1 + tau2 s).
template <int FAM>
__device__ __forceinline__ void msk_muscle_coef(const MskMuscleConst& C, const double* xm, double pw, double mult,
                                                double* c, double& base) {
    constexpr bool FAT = (FAM & 1) != 0, PW = msk_pw<FAM>();
    const double cn = xm[0], F = xm[1];
    double A = C.a_force, tau1 = C.tau1_rest, km = C.km_rest;
    if constexpr (FAT) {
        A = xm[2];
        tau1 = xm[3];
        km = xm[4];
    }
    double E = 1.0, dE = 0.0;
    if constexpr (PW) {
        const double e = exp(-(pw - C.pd0) * C.inv_pdt);
        E = 1.0 - e;
        dE = e * C.inv_pdt;
    }
    const double Aeff = A * E;
    const double d1 = km + cn, s = cn / d1, den = tau1 + C.tau2 * s, iden = 1.0 / den;
    base = Aeff * s - F * iden;
    const double dbs = Aeff + F * C.tau2 * iden * iden;  // d base / d s
    const double id1 = 1.0 / (d1 * d1);
    c[0] = mult * dbs * km * id1;
    c[1] = -mult * iden;
    c[2] = FAT ? mult * s * E : 0.0;
    c[3] = FAT ? mult * F * iden * iden : 0.0;
    c[4] = FAT ? -mult * dbs * cn * id1 : 0.0;
    c[5] = PW ? mult * s * A * dE : 0.0;
}

// M^-1 (symmetric positive definite, NQ <= 4: Gauss-Jordan without pivoting)
template <int NQ>
__device__ __forceinline__ void msk_spd_inverse(const double (*Mv)[NQ], double (*Mi)[NQ]) {
    if constexpr (NQ == 1) {
        Mi[0][0] = 1.0 / Mv[0][0];
    } else if constexpr (NQ == 2) {
        const double id = 1.0 / (Mv[0][0] * Mv[1][1] - Mv[1][0] * Mv[1][0]);
        Mi[0][0] = Mv[1][1] * id, Mi[1][1] = Mv[0][0] * id, Mi[0][1] = Mi[1][0] = -Mv[1][0] * id;
    } else {
        double a[NQ][NQ];
#pragma unroll
        for (int i = 0; i < NQ; ++i)
#pragma unroll
            for (int k = 0; k < NQ; ++k) a[i][k] = Mv[i][k], Mi[i][k] = i == k ? 1.0 : 0.0;
#pragma unroll
        for (int p = 0; p < NQ; ++p) {
            const double ip = 1.0 / a[p][p];
#pragma unroll
            for (int k = 0; k < NQ; ++k) a[p][k] *= ip, Mi[p][k] *= ip;
#pragma unroll
            for (int i = 0; i < NQ; ++i)
                if (i != p) {
                    const double fi = a[i][p];
#pragma unroll
                    for (int k = 0; k < NQ; ++k) a[i][k] -= fi * a[p][k], Mi[i][k] -= fi * Mi[p][k];
                }
        }
    }
}

// One RK stage: the RHS value f(xs, u) and the stage coefficients written to Ws[c * B].
template <int NQ, int NM, int FAM>
__device__ __forceinline__ void msk_stage(const MskGeom& G, int residual, const double* cs, const double* cs1,
                                          const double* xs, const double* u, double* f, double* __restrict__ Ws,
                                          int64_t B) {
    constexpr int NXM = msk_nxm<FAM>(), XQ = NM * NXM, XQD = XQ + NQ, ND = 2 * NQ;
    constexpr bool FAT = (FAM & 1) != 0, PW = msk_pw<FAM>();
    constexpr int NUI = msk_nui<NM, FAM>(), OM = 6 + ND, ODQ = NM * OM, OB = ODQ + NQ * ND, OMI = OB + NQ * NM;
    using S = Dual<ND>;
    Dual<NQ> q[NQ];  // q-only quantities carry the nq q-directions, the rest all 2 nq (msk_skeleton)
    S qd[NQ], F[NM], taur[NQ], mult[NM], qdd[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
        q[k] = dconst<NQ>(xs[XQ + k]);
        qd[k] = dconst<ND>(xs[XQD + k]);
        q[k].d[k] = 1.0;
        qd[k].d[NQ + k] = 1.0;
        taur[k] = dconst<ND>(residual ? u[NUI + k] : 0.0);
    }
#pragma unroll
    for (int mu = 0; mu < NM; ++mu) F[mu] = dconst<ND>(xs[mu * NXM + 1]);
    double Mv[NQ][NQ], JLv[NM][NQ];
    msk_skeleton<NQ, NM>(G, q, qd, F, taur, mult, qdd, Mv, JLv);
#pragma unroll
    for (int mu = 0; mu < NM; ++mu) {
        const MskMuscleConst& C = G.mc[mu];
        const double* xm = xs + mu * NXM;
        double c[6], base, pw = 0.0;
        if constexpr (PW) pw = u[mu];  // (a plain ternary would still index u out of range for NM > NQ)
        msk_muscle_coef<FAM>(C, xm, pw, mult[mu].v, c, base);
        f[mu * NXM] = (cs[mu] - xm[0]) * C.inv_tauc;
        f[mu * NXM + 1] = base * mult[mu].v;
        if constexpr (FAT) {
            if (cs1) f[mu * NXM] = f[mu * NXM] + (xm[4] - C.km_rest) * (cs1[mu] * C.inv_tauc);
            f[mu * NXM + 2] = C.alpha_a * xm[1] - (xm[2] - C.a_fat_rest) * C.inv_tau_fat;
            f[mu * NXM + 3] = C.alpha_tau1 * xm[1] - (xm[3] - C.tau1_rest) * C.inv_tau_fat;
            f[mu * NXM + 4] = C.alpha_km * xm[1] - (xm[4] - C.km_rest) * C.inv_tau_fat;
        }
#pragma unroll
        for (int e = 0; e < 6; ++e) Ws[(mu * OM + e) * B] = c[e];
#pragma unroll
        for (int d = 0; d < ND; ++d) Ws[(mu * OM + 6 + d) * B] = base * mult[mu].d[d];
    }
    double Mi[NQ][NQ];
    msk_spd_inverse<NQ>(Mv, Mi);
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        f[XQ + i] = xs[XQD + i];
        f[XQD + i] = qdd[i].v;
#pragma unroll
        for (int d = 0; d < ND; ++d) Ws[(ODQ + i * ND + d) * B] = qdd[i].d[d];
#pragma unroll
        for (int mu = 0; mu < NM; ++mu) {
            double bsum = 0.0;
#pragma unroll
            for (int k = 0; k < NQ; ++k) bsum += Mi[i][k] * JLv[mu][k];
            Ws[(OB + i * NM + mu) * B] = -bsum;
        }
#pragma unroll
        for (int k = 0; k < NQ; ++k) Ws[(OMI + i * NQ + k) * B] = Mi[i][k];
    }
}

// msk_stage split by derivative direction (k_msk_stagecoef_split): HALF 0 carries the nq q-directions through
// everything (SQ = SV = Dual<nq>) and writes the coefficients that need them (the muscle coefficients, the q half of
// d(base mult) and d qdd, -M^-1 J_L, M^-1); HALF 1 carries the nq qdot-directions only through the velocity-dependent
// part (SQ = double: the frames, geometry and M are plain values) and writes the qdot half.  Each direction is the same
// chain-rule expression as in msk_stage's Dual<2 nq> (per-direction arithmetic does not depend on how many directions
// travel together), at about 3/5 of its registers.
template <int NQ, int NM, int FAM, int HALF>
__device__ __forceinline__ void msk_stage_half(const MskGeom& G, int residual, const double* xs, const double* u,
                                               double* __restrict__ Ws, int64_t B) {
    constexpr int NXM = msk_nxm<FAM>(), XQ = NM * NXM, XQD = XQ + NQ, ND = 2 * NQ;
    constexpr int NUI = msk_nui<NM, FAM>(), OM = 6 + ND, ODQ = NM * OM, OB = ODQ + NQ * ND, OMI = OB + NQ * NM;
    constexpr bool PW = msk_pw<FAM>();
    using SV = Dual<NQ>;
    using SQ = typename std::conditional<HALF == 0, Dual<NQ>, double>::type;
    SQ q[NQ];
    SV qd[NQ], F[NM], taur[NQ], mult[NM], qdd[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
        if constexpr (HALF == 0) {
            q[k] = dconst<NQ>(xs[XQ + k]);
            q[k].d[k] = 1.0;
            qd[k] = dconst<NQ>(xs[XQD + k]);
        } else {
            q[k] = xs[XQ + k];
            qd[k] = dconst<NQ>(xs[XQD + k]);
            qd[k].d[k] = 1.0;
        }
        taur[k] = dconst<NQ>(residual ? u[NUI + k] : 0.0);
    }
#pragma unroll
    for (int mu = 0; mu < NM; ++mu) F[mu] = dconst<NQ>(xs[mu * NXM + 1]);
    double Mv[NQ][NQ], JLv[NM][NQ];
    msk_skeleton<NQ, NM>(G, q, qd, F, taur, mult, qdd, Mv, JLv);
    constexpr int D0 = HALF == 0 ? 0 : NQ;  // the directions' slots among msk_stage's 2 nq
#pragma unroll
    for (int mu = 0; mu < NM; ++mu) {
        const MskMuscleConst& C = G.mc[mu];
        const double* xm = xs + mu * NXM;
        double c[6], base, pw = 0.0;
        if constexpr (PW) pw = u[mu];
        msk_muscle_coef<FAM>(C, xm, pw, mult[mu].v, c, base);
        if constexpr (HALF == 0) {
#pragma unroll
            for (int e = 0; e < 6; ++e) Ws[(mu * OM + e) * B] = c[e];
        }
#pragma unroll
        for (int d = 0; d < NQ; ++d) Ws[(mu * OM + 6 + D0 + d) * B] = base * mult[mu].d[d];
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i)
#pragma unroll
        for (int d = 0; d < NQ; ++d) Ws[(ODQ + i * ND + D0 + d) * B] = qdd[i].d[d];
    if constexpr (HALF == 0) {
        double Mi[NQ][NQ];
        msk_spd_inverse<NQ>(Mv, Mi);
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
#pragma unroll
            for (int mu = 0; mu < NM; ++mu) {
                double bsum = 0.0;
#pragma unroll
                for (int k = 0; k < NQ; ++k) bsum += Mi[i][k] * JLv[mu][k];
                Ws[(OB + i * NM + mu) * B] = -bsum;
            }
#pragma unroll
            for (int k = 0; k < NQ; ++k) Ws[(OMI + i * NQ + k) * B] = Mi[i][k];
        }
    }
}

// tk = (df/dx, df/du)(stage) . (t, tu) for one tangent column, from the stored stage coefficients.
// dcs: Hmed, the stage's d cs_mu / d(column) (zero unless the column is one of the muscle's intensities).
template <int NQ, int NM, int FAM>
// cs1: legacy calcium, the stage's d cs / d Km (nullptr: off)
__device__ __forceinline__ void msk_tangent(const MskGeom& G, int residual, const double* __restrict__ Ws, int64_t B,
                                            const double* t, const double* tu, const double* dcs, const double* cs1,
                                            double* tk) {
    constexpr int NXM = msk_nxm<FAM>(), XQ = NM * NXM, XQD = XQ + NQ, ND = 2 * NQ;
    constexpr bool FAT = (FAM & 1) != 0, PW = msk_pw<FAM>();
    constexpr int NUI = msk_nui<NM, FAM>(), OM = 6 + ND, ODQ = NM * OM, OB = ODQ + NQ * ND, OMI = OB + NQ * NM;
#pragma unroll
    for (int mu = 0; mu < NM; ++mu) {
        const MskMuscleConst& C = G.mc[mu];
        const int o = mu * NXM;
        const double* c = Ws + (int64_t)mu * OM * B;
        tk[o] = -C.inv_tauc * t[o];
        if constexpr (msk_hmed<FAM>()) tk[o] += C.inv_tauc * dcs[mu];
        if constexpr (FAT)
            if (cs1) tk[o] += (cs1[mu] * C.inv_tauc) * t[o + 4];
        double s = c[0] * t[o] + c[B] * t[o + 1];
        if constexpr (FAT) s += c[2 * B] * t[o + 2] + c[3 * B] * t[o + 3] + c[4 * B] * t[o + 4];
        if constexpr (PW) s += c[5 * B] * tu[mu];
#pragma unroll
        for (int e = 0; e < ND; ++e) s += c[(6 + e) * B] * t[XQ + e];
        tk[o + 1] = s;
        if constexpr (FAT) {
            tk[o + 2] = C.alpha_a * t[o + 1] - C.inv_tau_fat * t[o + 2];
            tk[o + 3] = C.alpha_tau1 * t[o + 1] - C.inv_tau_fat * t[o + 3];
            tk[o + 4] = C.alpha_km * t[o + 1] - C.inv_tau_fat * t[o + 4];
        }
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        tk[XQ + i] = t[XQD + i];
        double s = 0.0;
#pragma unroll
        for (int e = 0; e < ND; ++e) s += Ws[(ODQ + i * ND + e) * B] * t[XQ + e];
#pragma unroll
        for (int mu = 0; mu < NM; ++mu) s += Ws[(OB + i * NM + mu) * B] * t[mu * NXM + 1];
        if (residual) {
#pragma unroll
            for (int k = 0; k < NQ; ++k) s += Ws[(OMI + i * NQ + k) * B] * tu[NUI + k];
        }
        tk[XQD + i] = s;
    }
}

// Hmed: is z-column col one of muscle m's intensities (its slot i), and lambda'(I) there; the stage's d cs / d col
// is then coef[kq][m][i] lambda'(I) (cn_sum is linear in the lambdas, hmed2018.py:97-98)
struct MskICol {
    int m, i;
    double dlam;
};
template <int NM, int FAM>
__device__ __forceinline__ MskICol msk_icol(const MskParams& P, const MskGeom& G, const double* __restrict__ V,
                                            int64_t zb, int64_t b, bool valid, int col) {
    MskICol r{-1, 0, 0.0};
    if constexpr (msk_hmed<FAM>()) {
        const int d = col - P.nx;
        if (d >= 0 && d < NM * P.T) {
            r.m = d / P.T;
            r.i = d - r.m * P.T;
            double l0, l2;
            msk_lambda(G.mc[r.m], valid ? V[(zb + col) * P.B + b] : 0.0, l0, r.dlam, l2);
        }
    }
    return r;
}
template <int NM, int FAM>
__device__ __forceinline__ void msk_icol_dcs(const MskParams& P, const MskICol& ic, int64_t kq, double* dcs) {
    if constexpr (msk_hmed<FAM>()) {
        constexpr int TM = msk_tmax<FAM>();
#pragma unroll
        for (int mu = 0; mu < NM; ++mu) dcs[mu] = mu == ic.m ? P.cs[(kq * NM + mu) * TM + ic.i] * ic.dlam : 0.0;
    }
}

template <int NQ, int NM, int FAM, int SCHEME>
__global__ void __launch_bounds__(256) k_msk_tangents(const MskParams P, const MskGeom* __restrict__ GG,
                                                      const double* __restrict__ V, double* __restrict__ J,
                                                      int flat) {
    constexpr int NXM = msk_nxm<FAM>(), NX = NM * NXM + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    constexpr int NC = msk_ncoef<NQ, NM>();
    constexpr int ST = SCHEME == 4 ? 4 : (SCHEME == 2 ? 2 : 1);
    const int64_t B = P.B;
    const int nz = P.nz;
    // block = 256 consecutive instances x one column.  Workgroups are dispatched round-robin over the 8 XCDs
    // (blockIdx % 8), each with its own L2: the nz column blocks of one instance range are given ids of the same
    // residue, so they run on one XCD, together, and read the range's coefficients from that XCD's L2.  Small
    // batches (flat): thread = (instance, column), the columns of an instance side by side — at batch 1 the
    // per-column blocks left 255 of 256 lanes and 7 of 8 ranges idle (33 ms per call for the 1,500-interval
    // reaching task, 40 columns).
    int col;
    int64_t b;
    if (flat) {
        const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        col = (int)(e % nz);
        b = e / nz;
    } else {
        const unsigned L = blockIdx.x, slot = L >> 3;
        col = (int)(slot % (unsigned)nz);
        const int64_t range = (int64_t)(slot / (unsigned)nz) * 8 + (L & 7);
        b = range * blockDim.x + threadIdx.x;
    }
    if (b >= B) return;
    const int k = blockIdx.y;
    const MskGeom& G = *GG;
    const int residual = P.residual;
    const double h = P.h;
    const double* __restrict__ Wk = P.scratch + (int64_t)k * P.Q * NC * B + b;
    double tx[NX], tu[NUMAX];
#pragma unroll
    for (int r = 0; r < NX; ++r) tx[r] = r == col ? 1.0 : 0.0;
#pragma unroll
    for (int i = 0; i < NUMAX; ++i) {
        const int dc = msk_udec<NM, FAM>(i, P.T, P.nu);
        tu[i] = dc >= 0 && NX + dc == col ? 1.0 : 0.0;
    }
    const MskICol ic = msk_icol<NM, FAM>(P, G, V, (int64_t)k * nz, b, true, col);
    for (int j = 0; j < P.m; ++j) {
        double tacc[NX], txs[NX];
#pragma unroll
        for (int r = 0; r < NX; ++r) txs[r] = tx[r];
#pragma unroll
        for (int st = 0; st < ST; ++st) {
            double tk[NX], dcs[NM];
            msk_icol_dcs<NM, FAM>(P, ic, (int64_t)k * P.Q + j * ST + st, dcs);
            msk_tangent<NQ, NM, FAM>(G, residual, Wk + (int64_t)(j * ST + st) * NC * B, B, txs, tu, dcs,
                                     msk_cs1<NM>(P, (int64_t)k * P.Q + j * ST + st), tk);
            const double cst = (ST == 4 && st == 2) ? h : 0.5 * h;
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                if (ST == 4) {
                    if (st == 0) tacc[r] = tk[r];
                    else if (st < 3) tacc[r] = tacc[r] + 2.0 * tk[r];
                }
                if (st + 1 < ST) txs[r] = tx[r] + cst * tk[r];
                else tx[r] = ST == 4 ? tx[r] + (h / 6.0) * (tacc[r] + tk[r]) : tx[r] + h * tk[r];
            }
        }
    }
    const int64_t jb = (int64_t)k * P.nnzk;
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        const int pos = G.jpos[r * kMskMaxZ + col];
        if (pos >= 0) J[(jb + pos) * B + b] = tx[r];
    }
    if (col == 0 && !P.keepc) {
#pragma unroll
        for (int r = 0; r < NX; ++r) J[(jb + G.jneg[r]) * B + b] = -1.0;
    }
}

// k_msk_tangents with the stage coefficients staged in LDS: block = TW instances x nz columns (nz <= 16, a wave
// holds 64 / TW columns of TW instances), so each coefficient is read from L2 once per block instead of once per
// column.  Per RK sub-step the block loads the ST stages' coefficients of its TW instances (ST * NC * TW * 8 B),
// then every thread carries its column through them.  A column takes ~200 VGPRs (2 waves per SIMD).  cfg 5 at
// B = 65536: TW = 32 0.66 ms, TW = 16 0.70 ms; 0.96 ms before the staging loads were issued all at once.  A block
// runs kpb consecutive intervals with the next sub-step's coefficients prefetched during the current one (below).
constexpr int kMskLdsCols = 16;
constexpr int kMskLdsLoads = 16;  // coefficient loads in flight per thread while staging
// J_g stores of the tangent kernel: non-temporal, as the shooting kernel's output stream (cfg 5: 1.533 / 1.535 ->
// 1.529 / 1.526 ms per g + J_g, alternating builds, profiles/round3/msk_waits/nt_j_ab.jsonl)
__device__ __forceinline__ void msk_st_j(double* p, double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
#ifndef CFX_MSK_TW
#define CFX_MSK_TW 32
#endif
constexpr int kMskTangentInstances = CFX_MSK_TW;  // TW: instances per k_msk_tangents_lds block (16 or 32)

// Default intervals per k_msk_tangents_lds block: as many as keep >= 4,096 blocks (16 per CU) in flight.
inline int msk_default_kpb(int64_t B, int N) {
    const int64_t nbx = (B + kMskTangentInstances - 1) / kMskTangentInstances;
    const int64_t kpb = nbx * N / 4096;
    return (int)(kpb < 1 ? 1 : (kpb > N ? N : kpb));
}

template <int NQ, int NM, int FAM, int SCHEME, int TW>
__global__ void __launch_bounds__(32 * kMskLdsCols) k_msk_tangents_lds(const MskParams P, const MskGeom* __restrict__ GG,
                                                                     const double* __restrict__ V,
                                                                     double* __restrict__ J, int kpb) {
    constexpr int NXM = msk_nxm<FAM>(), NX = NM * NXM + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    constexpr int NC = msk_ncoef<NQ, NM>();
    constexpr int ST = SCHEME == 4 ? 4 : (SCHEME == 2 ? 2 : 1);
    constexpr int NE = ST * NC * TW;  // coefficients of one sub-step of the block's TW instances
    extern __shared__ double sW[];    // [2][ST][NC][TW] (two buffers when B is even)
    const int64_t B = P.B;
    const int nz = P.nz, lane = threadIdx.x % TW, col = threadIdx.x / TW, nthr = TW * nz;
    const int64_t b0 = (int64_t)blockIdx.x * TW, b = b0 + lane;
    const int k0 = blockIdx.y * kpb, k1 = min(P.N, k0 + kpb);
    const MskGeom& G = *GG;
    const int residual = P.residual;
    const double h = P.h;
    // Several intervals per block (kpb) with the coefficients double-buffered in LDS: while a sub-step computes from
    // one buffer, the next (interval, sub-step)'s coefficients stream into the other by direct-to-LDS loads
    // (global_load_lds_dwordx4: lane L of a wave moves 16 B to M0 + 16 L, so one wave instruction fills four
    // TW-double rows), so only the block's first staging waits for HBM and no registers hold the prefetch.  Needs
    // 16-byte rows (B even); otherwise the sub-steps stage through registers one at a time.
    static_assert(TW == 16 || TW == 32, "a TW / 2-lane part of a wave moves one TW-double row");
    constexpr int RPW = 128 / TW;  // rows of TW doubles per wave instruction (64 lanes x 16 B)
    const bool async = (B % 2) == 0;
    const int wave = threadIdx.x / 64, nwave = nthr / 64, L = threadIdx.x % 64;  // full waves only (nz odd: one half)
    auto issue = [&](int kk, int j, int buf) {
        const double* __restrict__ Wk = P.scratch + (int64_t)kk * P.Q * NC * B + (int64_t)j * ST * NC * B;
        double* base = sW + buf * NE;
        for (int c = wave; wave < nwave && c * RPW * TW < NE; c += nwave) {  // chunk c: rows RPW c .. RPW c + RPW - 1
            const int row = RPW * c + L / (TW / 2), l = (L % (TW / 2)) * 2;
            if (row * TW < NE && b0 + l < B)
                __builtin_amdgcn_global_load_lds(Wk + (int64_t)row * B + b0 + l,
                                                 (__attribute__((address_space(3))) void*)(base + c * RPW * TW), 16, 0, 0);
        }
    };
    int buf = 0;
    if (async && k0 < k1) issue(k0, 0, 0);
    for (int k = k0; k < k1; ++k) {
        const double* __restrict__ Wk = P.scratch + (int64_t)k * P.Q * NC * B;
        double tx[NX], tu[NUMAX];
#pragma unroll
        for (int r = 0; r < NX; ++r) tx[r] = r == col ? 1.0 : 0.0;
#pragma unroll
        for (int i = 0; i < NUMAX; ++i) {
            const int dc = msk_udec<NM, FAM>(i, P.T, P.nu);
            tu[i] = dc >= 0 && NX + dc == col ? 1.0 : 0.0;
        }
        const MskICol ic = msk_icol<NM, FAM>(P, G, V, (int64_t)k * nz, b, b < B, col);
        for (int j = 0; j < P.m; ++j) {
            const double* sWb = sW;
            if (async) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's direct-to-LDS loads have landed
                __syncthreads();  // every wave's have, and the other buffer's readers are done
                const bool last = j + 1 == P.m;
                if (!last || k + 1 < k1) issue(last ? k + 1 : k, last ? 0 : j + 1, buf ^ 1);
                sWb = sW + buf * NE;
                buf ^= 1;
            } else {
                __syncthreads();  // the previous sub-step's coefficients are consumed
                // all of a thread's loads are issued before the first LDS store, so the block waits for one HBM round
                // trip per sub-step rather than one per element
                for (int e0 = threadIdx.x; e0 < NE; e0 += kMskLdsLoads * nthr) {
                    double tmp[kMskLdsLoads];
#pragma unroll
                    for (int i = 0; i < kMskLdsLoads; ++i) {
                        const int e = e0 + i * nthr, l = e % TW, sc = e / TW;  // sc = st * NC + c
                        const int64_t bb = b0 + l;
                        tmp[i] = (e < NE && bb < B) ? Wk[((int64_t)j * ST * NC + sc) * B + bb] : 0.0;
                    }
#pragma unroll
                    for (int i = 0; i < kMskLdsLoads; ++i)
                        if (e0 + i * nthr < NE) sW[e0 + i * nthr] = tmp[i];
                }
                __syncthreads();
            }
            double tacc[NX], txs[NX];
#pragma unroll
            for (int r = 0; r < NX; ++r) txs[r] = tx[r];
#pragma unroll
            for (int st = 0; st < ST; ++st) {
                double tk[NX], dcs[NM];
                msk_icol_dcs<NM, FAM>(P, ic, (int64_t)k * P.Q + j * ST + st, dcs);
                msk_tangent<NQ, NM, FAM>(G, residual, sWb + st * NC * TW + lane, TW, txs, tu, dcs,
                                         msk_cs1<NM>(P, (int64_t)k * P.Q + j * ST + st), tk);
                const double cst = (ST == 4 && st == 2) ? h : 0.5 * h;
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    if (ST == 4) {
                        if (st == 0) tacc[r] = tk[r];
                        else if (st < 3) tacc[r] = tacc[r] + 2.0 * tk[r];
                    }
                    if (st + 1 < ST) txs[r] = tx[r] + cst * tk[r];
                    else tx[r] = ST == 4 ? tx[r] + (h / 6.0) * (tacc[r] + tk[r]) : tx[r] + h * tk[r];
                }
            }
        }
        if (b < B) {
            const int64_t jb = (int64_t)k * P.nnzk;
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                const int pos = G.jpos[r * kMskMaxZ + col];
                if (pos >= 0) msk_st_j(J + (jb + pos) * B + b, tx[r]);
            }
            if (col == 0 && !P.keepc) {
#pragma unroll
                for (int r = 0; r < NX; ++r) msk_st_j(J + (jb + G.jneg[r]) * B + b, -1.0);
            }
        }
    }
}

// ---- Lagrangian Hessian by stages ------------------------------------------------------------------------------
// lambda^T Phi_m(z) is a composition whose only nonlinear nodes are the RK stage evaluations k_s = f(Y_s, u); every
// other operation is linear in (z, k).  Its Hessian is therefore  sum_s mu_s^T f''(Y_s, u)[dY_s/dz, dY_s/dz],
// mu_s = d(lambda^T Phi)/dk_s.  Five launches: stage values and coefficients (as for g + J_g, or re-used), stage
// tangents T_s = dY_s/dz (k_msk_htan, thread per column), stage adjoints mu_s (k_msk_hadj, backward sweep), the
// Y-space Hessians G_s = d^2(mu_s^T f)/dY^2 (k_msk_hpair, thread per stage and coordinate pair, Jet<2>) and the
// projection H = sum_s T_s^T G_s T_s (k_msk_hproj, thread per Hessian entry).  Every stage is its own thread, so
// at batch 1 the latency is one Jet<2> RHS rather than m * ST of them in sequence.

// explicit Butcher tableaux of RK1 / RK2 (midpoint) / RK4: weights b_s and sub-diagonal a_{s,s-1}
template <int ST>
__device__ __forceinline__ double rk_b(int s) {
    return ST == 1 ? 1.0 : (ST == 2 ? (s == 1 ? 1.0 : 0.0) : ((s == 0 || s == 3) ? 1.0 / 6.0 : 1.0 / 3.0));
}
template <int ST>
__device__ __forceinline__ double rk_a(int s) {
    return (ST == 4 && s == 3) ? 1.0 : 0.5;
}

// a = (df/dx)^T w at the stage whose coefficients are Ws (the transpose of msk_tangent's state part)
template <int NQ, int NM, int FAM>
__device__ __forceinline__ void msk_tangent_T(const MskGeom& G, const double* __restrict__ Ws, int64_t B,
                                              const double* cs1, const double* w, double* a) {
    constexpr int NXM = msk_nxm<FAM>(), XQ = NM * NXM, XQD = XQ + NQ, ND = 2 * NQ, NX = XQ + 2 * NQ;
    constexpr bool FAT = (FAM & 1) != 0;
    constexpr int OM = 6 + ND, ODQ = NM * OM, OB = ODQ + NQ * ND;
#pragma unroll
    for (int r = 0; r < NX; ++r) a[r] = 0.0;
#pragma unroll
    for (int mu = 0; mu < NM; ++mu) {
        const MskMuscleConst& C = G.mc[mu];
        const int o = mu * NXM;
        const double* c = Ws + (int64_t)mu * OM * B;
        const double w1 = w[o + 1];
        a[o] += c[0] * w1 - C.inv_tauc * w[o];
        a[o + 1] += c[B] * w1;
        if constexpr (FAT) {
            a[o + 1] += C.alpha_a * w[o + 2] + C.alpha_tau1 * w[o + 3] + C.alpha_km * w[o + 4];
            a[o + 2] += c[2 * B] * w1 - C.inv_tau_fat * w[o + 2];
            a[o + 3] += c[3 * B] * w1 - C.inv_tau_fat * w[o + 3];
            a[o + 4] += c[4 * B] * w1 - C.inv_tau_fat * w[o + 4];
            if (cs1) a[o + 4] += (cs1[mu] * C.inv_tauc) * w[o];
        }
#pragma unroll
        for (int e = 0; e < ND; ++e) a[XQ + e] += c[(6 + e) * B] * w1;
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        a[XQD + i] += w[XQ + i];
        const double wi = w[XQD + i];
#pragma unroll
        for (int e = 0; e < ND; ++e) a[XQ + e] += Ws[(ODQ + i * ND + e) * B] * wi;
#pragma unroll
        for (int mu = 0; mu < NM; ++mu) a[mu * NXM + 1] += Ws[(OB + i * NM + mu) * B] * wi;
    }
}

// stage input tangents TS[k][q][r][col][b] = dY_q[r]/dz[col] (thread = instance, interval, column)
template <int NQ, int NM, int FAM, int SCHEME>
__global__ void __launch_bounds__(256) k_msk_htan(const MskParams P, const MskGeom* __restrict__ GG,
                                                  const double* __restrict__ V, double* __restrict__ TS) {
    constexpr int NXM = msk_nxm<FAM>(), NX = NM * NXM + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    constexpr int NC = msk_ncoef<NQ, NM>();
    constexpr int ST = SCHEME == 4 ? 4 : (SCHEME == 2 ? 2 : 1);
    const int64_t B = P.B;
    const int nz = P.nz, Q = P.Q;
    // flat item index, instance fastest (coalesced for large B; at batch 1 the items of a wave are distinct
    // columns and intervals, so the launch is a few waves rather than N * nz single-lane ones)
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= B * P.N * nz) return;
    const int64_t b = item % B, rest = item / B;
    const int col = (int)(rest % nz), k = (int)(rest / nz);
    const MskGeom& G = *GG;
    const double h = P.h;
    const double* __restrict__ Wk = P.scratch + (int64_t)k * Q * NC * B + b;
    double tx[NX], tu[NUMAX];
#pragma unroll
    for (int r = 0; r < NX; ++r) tx[r] = r == col ? 1.0 : 0.0;
#pragma unroll
    for (int i = 0; i < NUMAX; ++i) {
        const int dc = msk_udec<NM, FAM>(i, P.T, P.nu);
        tu[i] = dc >= 0 && NX + dc == col ? 1.0 : 0.0;
    }
    const MskICol ic = msk_icol<NM, FAM>(P, G, V, (int64_t)k * nz, b, true, col);
    for (int j = 0; j < P.m; ++j) {
        double tacc[NX], txs[NX];
#pragma unroll
        for (int r = 0; r < NX; ++r) txs[r] = tx[r];
#pragma unroll
        for (int st = 0; st < ST; ++st) {
            const int slot = j * ST + st;
            double* __restrict__ ts = TS + (((int64_t)k * Q + slot) * NX * nz + col) * B + b;
#pragma unroll
            for (int r = 0; r < NX; ++r) ts[(int64_t)r * nz * B] = txs[r];
            double tk[NX], dcs[NM];
            msk_icol_dcs<NM, FAM>(P, ic, (int64_t)k * Q + slot, dcs);
            msk_tangent<NQ, NM, FAM>(G, P.residual, Wk + (int64_t)slot * NC * B, B, txs, tu, dcs,
                                     msk_cs1<NM>(P, (int64_t)k * Q + slot), tk);
            const double cst = (ST == 4 && st == 2) ? h : 0.5 * h;
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                if (ST == 4) {
                    if (st == 0) tacc[r] = tk[r];
                    else if (st < 3) tacc[r] = tacc[r] + 2.0 * tk[r];
                }
                if (st + 1 < ST) txs[r] = tx[r] + cst * tk[r];
                else tx[r] = ST == 4 ? tx[r] + (h / 6.0) * (tacc[r] + tk[r]) : tx[r] + h * tk[r];
            }
        }
    }
}

// stage adjoints MU[k][q][r][b] = d(lambda_k^T Phi)/dk_q[r] by the reverse sweep of the RK sub-steps
template <int NQ, int NM, int FAM, int SCHEME>
__global__ void __launch_bounds__(256) k_msk_hadj(const MskParams P, const MskGeom* __restrict__ GG,
                                                  const double* __restrict__ LAM, double* __restrict__ MU) {
    constexpr int NXM = msk_nxm<FAM>(), NX = NM * NXM + 2 * NQ;
    constexpr int NC = msk_ncoef<NQ, NM>();
    constexpr int ST = SCHEME == 4 ? 4 : (SCHEME == 2 ? 2 : 1);
    const int64_t B = P.B;
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= B * P.N) return;
    const int64_t b = item % B;
    const int k = (int)(item / B), Q = P.Q;
    const MskGeom& G = *GG;
    const double h = P.h;
    const double* __restrict__ Wk = P.scratch + (int64_t)k * Q * NC * B + b;
    double xb[NX];
#pragma unroll
    for (int r = 0; r < NX; ++r) xb[r] = LAM[((int64_t)k * P.ngk + r) * B + b];
    for (int j = P.m - 1; j >= 0; --j) {
        double xn[NX], yb[NX];
#pragma unroll
        for (int r = 0; r < NX; ++r) xn[r] = xb[r], yb[r] = 0.0;
#pragma unroll
        for (int st = ST - 1; st >= 0; --st) {
            const int slot = j * ST + st;
            const double wb = h * rk_b<ST>(st), wa = st + 1 < ST ? h * rk_a<ST>(st + 1) : 0.0;
            double mu[NX];
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                mu[r] = wb * xb[r] + wa * yb[r];
                MU[(((int64_t)k * Q + slot) * NX + r) * B + b] = mu[r];
            }
            msk_tangent_T<NQ, NM, FAM>(G, Wk + (int64_t)slot * NC * B, B, msk_cs1<NM>(P, (int64_t)k * Q + slot), mu, yb);
#pragma unroll
            for (int r = 0; r < NX; ++r) xn[r] += yb[r];
        }
#pragma unroll
        for (int r = 0; r < NX; ++r) xb[r] = xn[r];
    }
}

// GQ[k][q][t][b] = d^2(mu_q^T f)/dY_I dY_J at stage q for coordinate pair t = (I, J) of (x, u); tasks holds
// (I, J, t) triples of the structurally non-zero pairs (cfx_msk_create), in three groups launched apart (VAR):
//   0  neither coordinate is a q: the frames, muscle geometry and mass matrix are plain values (their derivatives in
//      both directions vanish);
//   1  I is a q, J not: they carry the I direction only (Dual<1>, promoted with zero second derivatives — the frames
//      depend on q alone, so their d2/dI dJ and d2/dJ2 vanish and d2/dI2, which does, is not the entry asked for);
//   2  both are q: Jet<2> throughout.
// Each entry is the same chain-rule sum as with Jet<2> frames (the dropped terms are exact zeros); the six-muscle arm's
// Jet<2> frames spilled 235 registers per thread.
template <int NQ, int NM, int FAM, int VAR>
__global__ void __launch_bounds__(256) k_msk_hpair(const MskParams P, const MskGeom* __restrict__ GG,
                                                   const int16_t* __restrict__ tasks, int ntasks, int npair,
                                                   const double* __restrict__ V, const double* __restrict__ XS,
                                                   const double* __restrict__ MU, double* __restrict__ GQ) {
    constexpr int NX = NM * msk_nxm<FAM>() + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    using S = Jet<2>;
    const int64_t B = P.B;
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= B * P.N * P.Q * ntasks) return;
    const int64_t b = item % B, rest = item / B;
    const int p = (int)(rest % ntasks), kq = (int)(rest / ntasks), k = kq / P.Q;
    const int I = tasks[3 * p], J = tasks[3 * p + 1], t = tasks[3 * p + 2];
    const MskGeom& G = *GG;
    const int nu = P.nu;
    const int64_t zb = (int64_t)k * P.nz;
    // pairs inside one muscle's variables (its states and pulse width): the muscle's F' = base(Cn, F, A, Tau1, Km,
    // pw) * mult(q, qdot) is the only non-linear term they share, and mult = -c1 (tau1 + tau2 s) is read back
    // from the stage coefficients, so no skeleton is evaluated (42 of cfg 5's 100 pairs)
    constexpr int NXM = msk_nxm<FAM>(), NPW = msk_pw<FAM>() ? NM : 0, NC = msk_ncoef<NQ, NM>();
    constexpr bool FAT = (FAM & 1) != 0;
    if constexpr (msk_hmed<FAM>()) {
        // intensity pairs: cs is a sum of separate lambda(I_i), entering cn_dot linearly, so the only second
        // derivative is d2/dI_i^2 = coef_i lambda''(I_i) / tau_c on the muscle's Cn row (the host lists no other)
        const int dI = I - NX, dJ = J - NX;
        if (dI >= 0 && dI < NM * P.T) {
            double val = 0.0;
            if (dJ == dI) {
                const int m = dI / P.T, i = dI - m * P.T;
                double l0, l1, l2;
                msk_lambda(G.mc[m], V[(zb + I) * B + b], l0, l1, l2);
                const double muc = MU[((int64_t)kq * NX + m * NXM) * B + b];
                val = muc * G.mc[m].inv_tauc * P.cs[((int64_t)kq * NM + m) * msk_tmax<FAM>() + i] * l2;
            }
            GQ[((int64_t)kq * npair + t) * B + b] = val;
            return;
        }
    }
    auto owner = [](int e) { return e < NM * NXM ? e / NXM : ((e >= NX && e < NX + NPW) ? e - NX : -1); };
    const int mI = owner(I), mJ = owner(J);
    if (VAR == 0 && mI >= 0 && mI == mJ) {
        const int mu = mI, o = mu * NXM;
        const MskMuscleConst& C = G.mc[mu];
        auto seed = [&](int e, double v) {
            S r = jconst<2>(v);
            r.g[0] = e == I ? 1.0 : 0.0;
            r.g[1] = (I != J && e == J) ? 1.0 : 0.0;
            return r;
        };
        double xv[NXM];
#pragma unroll
        for (int i = 0; i < NXM; ++i) xv[i] = XS[((int64_t)kq * NX + o + i) * B + b];
        const S cn = seed(o, xv[0]), F = seed(o + 1, xv[1]);
        S A = jconst<2>(C.a_force), tau1 = jconst<2>(C.tau1_rest), km = jconst<2>(C.km_rest);
        if constexpr (FAT) {
            A = seed(o + 2, xv[2]);
            tau1 = seed(o + 3, xv[3]);
            km = seed(o + 4, xv[4]);
        }
        if constexpr (NPW > 0) {
            const S pw = seed(NX + mu, V[(zb + NX + mu) * B + b]);
            A = A * (1.0 - mexp(-(pw - C.pd0) * C.inv_pdt));
        }
        const S sj = cn / (km + cn);
        const S base = A * sj - F / (tau1 + C.tau2 * sj);
        const double c1 = P.scratch[((int64_t)kq * NC + mu * (6 + 2 * NQ) + 1) * B + b];
        const double tau1v = FAT ? xv[3] : C.tau1_rest, kmv = FAT ? xv[4] : C.km_rest;
        const double mult = -c1 * (tau1v + C.tau2 * (xv[0] / (kmv + xv[0])));
        const double muF = MU[((int64_t)kq * NX + o + 1) * B + b];
        GQ[((int64_t)kq * npair + t) * B + b] = muF * mult * base.h[I == J ? 0 : 1];
        return;
    }
    S x[NX], u[NUMAX];
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        x[r] = jconst<2>(XS[((int64_t)kq * NX + r) * B + b]);
        x[r].g[0] = r == I ? 1.0 : 0.0;
        x[r].g[1] = (I != J && r == J) ? 1.0 : 0.0;
    }
#pragma unroll
    for (int i = 0; i < NUMAX; ++i) {
        const int dc = msk_udec<NM, FAM>(i, P.T, nu);
        u[i] = jconst<2>(dc >= 0 ? V[(zb + NX + dc) * B + b] : 0.0);
        u[i].g[0] = dc >= 0 && NX + dc == I ? 1.0 : 0.0;
        u[i].g[1] = (I != J && dc >= 0 && NX + dc == J) ? 1.0 : 0.0;
    }
    S f[NX];
    double csl[NM];  // cs enters cn_dot linearly: its value does not reach a second derivative
    if constexpr (msk_hmed<FAM>()) {
#pragma unroll
        for (int mu = 0; mu < NM; ++mu) csl[mu] = 0.0;
    } else {
        msk_stage_cs<NM, FAM>(P.cs, kq, nullptr, csl);
    }
    if constexpr (VAR == 2) {
        msk_rhs<NQ, NM, FAM>(G, P.residual, csl, msk_cs1<NM>(P, kq), x, u, f);
    } else if constexpr (VAR == 1) {
        constexpr int XQ = NM * NXM;
        Dual<1> q[NQ];
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            q[k] = dconst<1>(x[XQ + k].v);
            q[k].d[0] = XQ + k == I ? 1.0 : 0.0;
        }
        msk_rhs_q<NQ, NM, FAM>(G, P.residual, csl, msk_cs1<NM>(P, kq), x, q, u, f);
    } else {
        constexpr int XQ = NM * NXM;
        double q[NQ];
#pragma unroll
        for (int k = 0; k < NQ; ++k) q[k] = x[XQ + k].v;
        msk_rhs_q<NQ, NM, FAM>(G, P.residual, csl, msk_cs1<NM>(P, kq), x, q, u, f);
    }
    const int hi = I == J ? 0 : 1;  // Jet<2> second-order slots: (0,0), (1,0), (1,1)
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < NX; ++r) acc += MU[((int64_t)kq * NX + r) * B + b] * f[r].h[hi];
    GQ[((int64_t)kq * npair + t) * B + b] = acc;
}

// H[k][:, a] = sum_q T_q^T (G_q T_q[:, a]) for the rows >= a (thread = instance, interval, column a): each thread
// reads the stage's pair Hessians once and the tangent columns it needs, instead of one thread per entry
// re-reading both (3.5x fewer loads).  T_q's control rows are the identity.
template <int NQ, int NM, int FAM>
__global__ void __launch_bounds__(256) k_msk_hproj(const MskParams P, const double* __restrict__ TS,
                                                   const double* __restrict__ GQ, int ntasks, double* __restrict__ H) {
    constexpr int NX = NM * msk_nxm<FAM>() + 2 * NQ;
    constexpr int NZ = NX + (msk_pw<FAM>() ? NM : 0) + NQ;  // upper bound of nz
    const int64_t B = P.B;
    const int nz = P.nz, Q = P.Q;
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= B * P.N * nz) return;
    const int64_t b = item % B, rest = item / B;
    const int a = (int)(rest % nz), k = (int)(rest / nz);
    double out[NZ];
#pragma unroll
    for (int i = 0; i < NZ; ++i) out[i] = 0.0;
    for (int q = 0; q < Q; ++q) {
        const int64_t kq = (int64_t)k * Q + q;
        const double* __restrict__ ts = TS + kq * NX * nz * B + b;  // [r][col][b]
        double ta[NZ], w[NZ];
#pragma unroll
        for (int I = 0; I < NX; ++I) ta[I] = ts[((int64_t)I * nz + a) * B];
#pragma unroll
        for (int I = NX; I < NZ; ++I) ta[I] = I == a ? 1.0 : 0.0;
#pragma unroll
        for (int I = 0; I < NZ; ++I) w[I] = 0.0;
        const double* __restrict__ gq = GQ + kq * ntasks * B + b;
#pragma unroll
        for (int I = 0; I < NZ; ++I)
#pragma unroll
            for (int J = I; J < NZ; ++J) {
                if (J >= nz) continue;
                const int t = I * nz - I * (I - 1) / 2 + (J - I);  // lexicographic (I <= J) task order
                const double g = gq[(int64_t)t * B];
                w[I] += g * ta[J];
                if (J != I) w[J] += g * ta[I];
            }
#pragma unroll
        for (int c = 0; c < NZ; ++c) {
            if (c < a || c >= nz) continue;
            double sacc = 0.0;  // w[c] for the control rows (T_q's identity), picked without a run-time register index
#pragma unroll
            for (int e = NX; e < NZ; ++e) sacc = e == c ? w[e] : sacc;
#pragma unroll
            for (int I = 0; I < NX; ++I) sacc += ts[((int64_t)I * nz + c) * B] * w[I];
            out[c] += sacc;
        }
    }
    const int64_t hb = (int64_t)k * P.nhk;
#pragma unroll
    for (int c = 0; c < NZ; ++c)
        if (c >= a && c < nz) H[(hb + c * (c + 1) / 2 + a) * B + b] = out[c];
}

// ---- every stage in its own thread ----------------------------------------------------------------------------
// A fused kernel running the m * ST dependent stage evaluations (Dual skeleton) of an interval in one thread was
// latency-bound at batch 1 (~0.5 ms for cfg 5 at RK4 x 5).  Split: k_msk_values runs the plain-double recursion (the
// g values) and stores every stage input XS, then k_msk_stagecoef_par evaluates each stage's coefficients in its own
// thread, so the latency is one double recursion plus one Dual stage.  Small batches also split the Hessian
// projection: k_msk_hproj_stage gives every (stage, column) its own thread and k_msk_hproj_sum adds the stages up in
// the order k_msk_hproj does.
// Small batches (msk_values_grid: B below one block) take a flat grid, thread = (interval, instance) with the instances
// fastest, so a wavefront carries 64 intervals instead of one live lane per block (the reaching task at batch 1: 1,500
// single-lane blocks); every thread runs the same code on the same data either way.
template <int NQ, int NM, int FAM, int SCHEME>
__global__ void __launch_bounds__(256) k_msk_values(const MskParams P, const MskGeom* __restrict__ GG,
                                                    const double* __restrict__ V, double* __restrict__ Gout,
                                                    double* __restrict__ XS) {
    constexpr int NXM = msk_nxm<FAM>(), NX = NM * NXM + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    constexpr int ST = SCHEME == 4 ? 4 : (SCHEME == 2 ? 2 : 1);
    const int64_t B = P.B;
    const bool flat = gridDim.y == 1 && P.N > 1;  // (msk_values_grid)
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t b = flat ? e % B : e;
    const int k = flat ? (int)(e / B) : (int)blockIdx.y;
    if (b >= B || k >= P.N) return;
    const MskGeom& G = *GG;
    const int nz = P.nz, nu = P.nu, Q = P.Q, residual = P.residual;
    const int64_t zb = (int64_t)k * nz;
    const double h = P.h;
    double x[NX], u[NUMAX];
#pragma unroll
    for (int r = 0; r < NX; ++r) x[r] = V[(zb + r) * B + b];
#pragma unroll
    for (int i = 0; i < NUMAX; ++i) {
        const int dc = msk_udec<NM, FAM>(i, P.T, nu);
        u[i] = dc >= 0 ? V[(zb + NX + dc) * B + b] : 0.0;
    }
    double lam[msk_hmed<FAM>() ? NM * msk_tmax<FAM>() : 1];
    msk_interval_lam<NM, FAM>(G, u, lam);
    for (int j = 0; j < P.m; ++j) {
        double acc[NX], xs[NX];
#pragma unroll
        for (int r = 0; r < NX; ++r) xs[r] = x[r];
#pragma unroll
        for (int st = 0; st < ST; ++st) {
            const int64_t kq = (int64_t)k * Q + j * ST + st;
            if (XS) {  // (null: g only)
#pragma unroll
                for (int r = 0; r < NX; ++r) XS[(kq * NX + r) * B + b] = xs[r];
            }
            double f[NX], csl[NM];
            msk_stage_cs<NM, FAM>(P.cs, kq, lam, csl);
            msk_rhs<NQ, NM, FAM>(G, residual, csl, msk_cs1<NM>(P, kq), xs, u, f);
            const double cst = (ST == 4 && st == 2) ? h : 0.5 * h;
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                if (ST == 4) {
                    if (st == 0) acc[r] = f[r];
                    else if (st < 3) acc[r] = acc[r] + 2.0 * f[r];
                }
                if (st + 1 < ST) xs[r] = x[r] + cst * f[r];
                else x[r] = ST == 4 ? x[r] + (h / 6.0) * (acc[r] + f[r]) : x[r] + h * f[r];
            }
        }
    }
    if (Gout) {
#pragma unroll
        for (int r = 0; r < NX; ++r) Gout[((int64_t)k * P.ngk + r) * B + b] = x[r] - V[(zb + nz + r) * B + b];
    }
}

// stage coefficients from the stored stage inputs (thread = instance, interval, stage).  Occupancy is what the
// 334-register allocation gives (one wave per SIMD); forcing two (amdgpu_waves_per_eu(2, 2), <= 256 registers) ran
// 0.70 -> 0.81 ms at cfg 5 (profiles/round3/msk_w2).
template <int NQ, int NM, int FAM>
__global__ void __launch_bounds__(256) k_msk_stagecoef_par(const MskParams P, const MskGeom* __restrict__ GG,
                                                           const double* __restrict__ V, const double* __restrict__ XS) {
    constexpr int NXM = msk_nxm<FAM>(), NX = NM * NXM + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    constexpr int NC = msk_ncoef<NQ, NM>();
    const int64_t B = P.B;
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= B * P.N * P.Q) return;
    const int64_t b = item % B, kq = item / B;
    const int k = (int)(kq / P.Q);
    const MskGeom& G = *GG;
    const int nu = P.nu;
    const int64_t zb = (int64_t)k * P.nz;
    double xs[NX], u[NUMAX], f[NX], csl[NM];
#pragma unroll
    for (int r = 0; r < NX; ++r) xs[r] = XS[(kq * NX + r) * B + b];
#pragma unroll
    for (int i = 0; i < NUMAX; ++i) {
        const int dc = msk_udec<NM, FAM>(i, P.T, nu);
        u[i] = dc >= 0 ? V[(zb + NX + dc) * B + b] : 0.0;
    }
    // f is not used here, and cs enters only f: the Hmed sums are not formed
    if constexpr (msk_hmed<FAM>()) {
#pragma unroll
        for (int mu = 0; mu < NM; ++mu) csl[mu] = 0.0;
    } else {
        msk_stage_cs<NM, FAM>(P.cs, kq, nullptr, csl);
    }
    msk_stage<NQ, NM, FAM>(G, P.residual, csl, msk_cs1<NM>(P, kq), xs, u, f, P.scratch + kq * NC * B + b, B);
}

// k_msk_stagecoef_par with the derivative directions split over two threads (blockIdx.y: 0 the q-directions, 1 the
// qdot-directions; msk_stage_half): the same coefficients, each from the same expression, at fewer registers per
// thread.  The stage's calcium sum enters f only, which neither half forms.
#ifndef CFX_MSK_SPLIT_WAVES
#define CFX_MSK_SPLIT_WAVES 2  // waves per SIMD the split kernel is compiled for (the q half takes 272 registers free)
#endif
template <int NQ, int NM, int FAM>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CFX_MSK_SPLIT_WAVES, CFX_MSK_SPLIT_WAVES)))
k_msk_stagecoef_split(const MskParams P, const MskGeom* __restrict__ GG,
                                                             const double* __restrict__ V,
                                                             const double* __restrict__ XS) {
    constexpr int NXM = msk_nxm<FAM>(), NX = NM * NXM + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    constexpr int NC = msk_ncoef<NQ, NM>();
    const int64_t B = P.B;
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= B * P.N * P.Q) return;
    const int64_t b = item % B, kq = item / B;
    const int k = (int)(kq / P.Q);
    const MskGeom& G = *GG;
    const int64_t zb = (int64_t)k * P.nz;
    double xs[NX], u[NUMAX];
#pragma unroll
    for (int r = 0; r < NX; ++r) xs[r] = XS[(kq * NX + r) * B + b];
#pragma unroll
    for (int i = 0; i < NUMAX; ++i) {
        const int dc = msk_udec<NM, FAM>(i, P.T, P.nu);
        u[i] = dc >= 0 ? V[(zb + NX + dc) * B + b] : 0.0;
    }
    double* Ws = P.scratch + kq * NC * B + b;
    if (blockIdx.y == 0) msk_stage_half<NQ, NM, FAM, 0>(G, P.residual, xs, u, Ws, B);
    else msk_stage_half<NQ, NM, FAM, 1>(G, P.residual, xs, u, Ws, B);
}

// g + J_g's stage coefficients and tangent columns in one launch (k_msk_stagecoef_par followed by k_msk_tangents_lds,
// without the coefficients' round trip through HBM: 1.1 GB written and 0.76 GB read back per cfg-5 call at B = 65,536,
// and the tangent blocks' waits at every hand-off).  Block = TW instances x ki consecutive intervals, 256 threads:
//   phase A: thread = (instance, interval, stage) task, msk_stage from the stage inputs XS into LDS sW[ki][Q][NC][TW]
//            (the stage kernel's expression, so the coefficients are the same numbers);
//   phase B: thread = (instance, CPT columns), the RK recursion of each column through the LDS coefficients — every
//            coefficient read from LDS once per stage for all the thread's columns (they share the instance).
// The stage body sets the register allocation (one wave per SIMD, as the stage kernel runs), so a 256-thread block
// covers TW x nz <= 16 TW (instance, column) pairs with CPT = TW / 16 columns per thread: TW = 32 where one interval's
// coefficients fit in LDS at 32 instances, else TW = 16 (RK4 x 5: 20 stages x 36 coefficients x 32 x 8 B = 184 KB).
// keep: the coefficients are also stored to P.scratch (the interior point's Hessian at the same point reuses them,
// cfx_api.hip msk_stash).
constexpr int kMskFusedThreads = 256;
constexpr size_t kMskFusedMaxLds = 160 * 1024;

template <int NQ, int NM, int FAM>
__device__ __forceinline__ void msk_stage_task(const MskParams& P, const MskGeom& G, const double* __restrict__ V,
                                               const double* __restrict__ XS, int64_t b, int64_t kq,
                                               double* __restrict__ Ws, int64_t ws) {
    constexpr int NXM = msk_nxm<FAM>(), NX = NM * NXM + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    const int64_t B = P.B;
    const int k = (int)(kq / P.Q);
    const int64_t zb = (int64_t)k * P.nz;
    double xs[NX], u[NUMAX], f[NX], csl[NM];
#pragma unroll
    for (int r = 0; r < NX; ++r) xs[r] = XS[(kq * NX + r) * B + b];
#pragma unroll
    for (int i = 0; i < NUMAX; ++i) {
        const int dc = msk_udec<NM, FAM>(i, P.T, P.nu);
        u[i] = dc >= 0 ? V[(zb + NX + dc) * B + b] : 0.0;
    }
    if constexpr (msk_hmed<FAM>()) {  // cs enters f only, which is not used here
#pragma unroll
        for (int mu = 0; mu < NM; ++mu) csl[mu] = 0.0;
    } else {
        msk_stage_cs<NM, FAM>(P.cs, kq, nullptr, csl);
    }
    msk_stage<NQ, NM, FAM>(G, P.residual, csl, msk_cs1<NM>(P, kq), xs, u, f, Ws, ws);
}

template <int NQ, int NM, int FAM, int SCHEME, int TW>
__global__ void __launch_bounds__(kMskFusedThreads) k_msk_stage_tangents(const MskParams P, const MskGeom* __restrict__ GG,
                                                                        const double* __restrict__ V,
                                                                        const double* __restrict__ XS,
                                                                        double* __restrict__ J, int ki, int keep) {
    constexpr int NXM = msk_nxm<FAM>(), NX = NM * NXM + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    constexpr int NC = msk_ncoef<NQ, NM>();
    constexpr int ST = SCHEME == 4 ? 4 : (SCHEME == 2 ? 2 : 1);
    constexpr int CPT = TW * kMskLdsCols / kMskFusedThreads;
    static_assert(CPT >= 1 && TW * kMskLdsCols == CPT * kMskFusedThreads, "phase B: CPT columns per thread");
    extern __shared__ double sW[];  // [ki][Q][NC][TW]
    const int64_t B = P.B;
    const int nz = P.nz, Q = P.Q;
    const int64_t b0 = (int64_t)blockIdx.x * TW;
    const int k0 = blockIdx.y * ki, nk = min(ki, P.N - k0);
    const MskGeom& G = *GG;
    // phase A: the block's stage coefficients (lanes past the batch end leave their slots unset; their columns are
    // carried through them below but never stored)
    const int ntask = TW * nk * Q;
    for (int t = threadIdx.x; t < ntask; t += kMskFusedThreads) {
        const int l = t % TW, kql = t / TW;  // kql = local interval * Q + stage
        const int64_t b = b0 + l;
        if (b < B) msk_stage_task<NQ, NM, FAM>(P, G, V, XS, b, (int64_t)k0 * Q + kql, sW + kql * NC * TW + l, TW);
    }
    __syncthreads();
    if (keep) {
        const int ne = nk * Q * NC * TW;
        double* __restrict__ Wg = P.scratch + (int64_t)k0 * Q * NC * B + b0;
        for (int e = threadIdx.x; e < ne; e += kMskFusedThreads) {
            const int l = e % TW, row = e / TW;
            if (b0 + l < B) Wg[(int64_t)row * B + l] = sW[e];
        }
    }
    // phase B: thread = instance lane, columns col0 + g (kMskFusedThreads / TW)
    const int lane = threadIdx.x % TW, col0 = threadIdx.x / TW;
    constexpr int CSTEP = kMskFusedThreads / TW;
    const int64_t b = b0 + lane;
    const int residual = P.residual;
    const double h = P.h;
    for (int kl = 0; kl < nk; ++kl) {
        const int k = k0 + kl;
        double tx[CPT][NX], tu[CPT][NUMAX];
        MskICol ic[CPT];
#pragma unroll
        for (int g = 0; g < CPT; ++g) {
            const int col = col0 + g * CSTEP;
#pragma unroll
            for (int r = 0; r < NX; ++r) tx[g][r] = r == col ? 1.0 : 0.0;
#pragma unroll
            for (int i = 0; i < NUMAX; ++i) {
                const int dc = msk_udec<NM, FAM>(i, P.T, P.nu);
                tu[g][i] = dc >= 0 && NX + dc == col ? 1.0 : 0.0;
            }
            ic[g] = msk_icol<NM, FAM>(P, G, V, (int64_t)k * nz, b, b < B && col < nz, col);
        }
        for (int j = 0; j < P.m; ++j) {
            double tacc[CPT][NX], txs[CPT][NX];
#pragma unroll
            for (int g = 0; g < CPT; ++g)
#pragma unroll
                for (int r = 0; r < NX; ++r) txs[g][r] = tx[g][r];
#pragma unroll
            for (int st = 0; st < ST; ++st) {
                const int64_t kq = (int64_t)k * Q + j * ST + st;
                const double* __restrict__ sWb = sW + (kl * Q + j * ST + st) * NC * TW + lane;
                double cw[NC];  // the stage's coefficients of this instance, read once for the CPT columns
#pragma unroll
                for (int c = 0; c < NC; ++c) cw[c] = sWb[c * TW];
                const double* cs1 = msk_cs1<NM>(P, kq);
                const double cst = (ST == 4 && st == 2) ? h : 0.5 * h;
#pragma unroll
                for (int g = 0; g < CPT; ++g) {
                    double tk[NX], dcs[NM];
                    msk_icol_dcs<NM, FAM>(P, ic[g], kq, dcs);
                    msk_tangent<NQ, NM, FAM>(G, residual, cw, 1, txs[g], tu[g], dcs, cs1, tk);
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        if (ST == 4) {
                            if (st == 0) tacc[g][r] = tk[r];
                            else if (st < 3) tacc[g][r] = tacc[g][r] + 2.0 * tk[r];
                        }
                        if (st + 1 < ST) txs[g][r] = tx[g][r] + cst * tk[r];
                        else tx[g][r] = ST == 4 ? tx[g][r] + (h / 6.0) * (tacc[g][r] + tk[r]) : tx[g][r] + h * tk[r];
                    }
                }
            }
        }
        if (b < B) {
            const int64_t jb = (int64_t)k * P.nnzk;
#pragma unroll
            for (int g = 0; g < CPT; ++g) {
                const int col = col0 + g * CSTEP;
                if (col >= nz) continue;
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    const int pos = G.jpos[r * kMskMaxZ + col];
                    if (pos >= 0) msk_st_j(J + (jb + pos) * B + b, tx[g][r]);
                }
                if (col == 0 && !P.keepc) {
#pragma unroll
                    for (int r = 0; r < NX; ++r) msk_st_j(J + (jb + G.jneg[r]) * B + b, -1.0);
                }
            }
        }
    }
}

// intervals per k_msk_stage_tangents block: enough (instance, interval, stage) tasks to fill the block once, within
// the LDS; 0 when even one interval's coefficients do not fit (the unfused path then runs)
inline int msk_fused_ki(int N, int Q, int NC, int TW) {
    const size_t per = (size_t)Q * NC * TW * sizeof(double);
    if (per > kMskFusedMaxLds) return 0;
    int ki = std::max(1, kMskFusedThreads / (TW * Q));
    ki = std::min(ki, N);
    while (ki > 1 && (size_t)ki * per > kMskFusedMaxLds) --ki;
    while (ki > 1 && N % ki != 0 && (N + ki - 1) / ki == (N + ki - 2) / (ki - 1)) --ki;  // same groups, fewer idle
    return ki;
}

// one stage's term T_q^T (G_q T_q[:, a]) of k_msk_hproj (thread = instance, column a, interval-stage kq)
template <int NQ, int NM, int FAM>
__global__ void __launch_bounds__(256) k_msk_hproj_stage(const MskParams P, const double* __restrict__ TS,
                                                         const double* __restrict__ GQ, int ntasks,
                                                         double* __restrict__ HQ) {
    constexpr int NX = NM * msk_nxm<FAM>() + 2 * NQ;
    constexpr int NZ = NX + (msk_pw<FAM>() ? NM : 0) + NQ;
    const int64_t B = P.B;
    const int nz = P.nz;
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= B * P.N * P.Q * nz) return;
    const int64_t b = item % B, rest = item / B;
    const int a = (int)(rest % nz);
    const int64_t kq = rest / nz;
    const double* __restrict__ ts = TS + kq * NX * nz * B + b;
    double ta[NZ], w[NZ];
#pragma unroll
    for (int I = 0; I < NX; ++I) ta[I] = ts[((int64_t)I * nz + a) * B];
#pragma unroll
    for (int I = NX; I < NZ; ++I) ta[I] = I == a ? 1.0 : 0.0;
#pragma unroll
    for (int I = 0; I < NZ; ++I) w[I] = 0.0;
    const double* __restrict__ gq = GQ + kq * ntasks * B + b;
#pragma unroll
    for (int I = 0; I < NZ; ++I)
#pragma unroll
        for (int J = I; J < NZ; ++J) {
            if (J >= nz) continue;
            const int t = I * nz - I * (I - 1) / 2 + (J - I);
            const double g = gq[(int64_t)t * B];
            w[I] += g * ta[J];
            if (J != I) w[J] += g * ta[I];
        }
    double* __restrict__ hq = HQ + kq * P.nhk * B + b;
#pragma unroll
    for (int c = 0; c < NZ; ++c) {
        if (c < a || c >= nz) continue;
        double sacc = 0.0;  // w[c] for the control rows, picked without a run-time register index
#pragma unroll
        for (int e = NX; e < NZ; ++e) sacc = e == c ? w[e] : sacc;
#pragma unroll
        for (int I = 0; I < NX; ++I) sacc += ts[((int64_t)I * nz + c) * B] * w[I];
        hq[(int64_t)(c * (c + 1) / 2 + a) * B] = sacc;
    }
}

// k_msk_hproj_stage with each stage's pair Hessian G_q and tangents T_q staged in LDS: a block takes kMskHpS
// consecutive stages of one instance, thread = (stage slot, column a).  Every column of a stage read the stage's G_q and
// T_q from the cache on its own (~1,500 loads a thread; 452 us per call for the reaching task at batch 1); here they are
// read from HBM once per stage (193 us).  The same sums in the same order as k_msk_hproj_stage; the entries agree to
// rounding (the compiler forms the two kernels' multiply-adds differently), and the chaotic reaching solve follows
// another path.
constexpr int kMskHpS = 3;  // stages per block (LDS: 3 x (nz (nz + 1) / 2 + NX nz) doubles, 52 KB at nz = 40)
inline size_t msk_hproj_lds(int nx, int nz) { return (size_t)kMskHpS * ((size_t)nz * (nz + 1) / 2 + (size_t)nx * nz) * 8; }
template <int NQ, int NM, int FAM>
__global__ void __launch_bounds__(kMskHpS * kMskMaxZ) k_msk_hproj_stage_lds(const MskParams P, const double* __restrict__ TS,
                                                                            const double* __restrict__ GQ, int ntasks,
                                                                            double* __restrict__ HQ) {
    constexpr int NX = NM * msk_nxm<FAM>() + 2 * NQ;
    constexpr int NZ = NX + (msk_pw<FAM>() ? NM : 0) + NQ;
    extern __shared__ double sh[];  // [kMskHpS][ntasks] G, then [kMskHpS][NX nz] T
    const int64_t B = P.B;
    const int nz = P.nz;
    const int64_t b = blockIdx.y;
    const int64_t nkq = (int64_t)P.N * P.Q, kq0 = (int64_t)blockIdx.x * kMskHpS;
    const int ns = (int)min((int64_t)kMskHpS, nkq - kq0);
    double* sG = sh;
    double* sT = sh + kMskHpS * ntasks;
    const int nt = NX * nz;
    for (int e = threadIdx.x; e < ns * ntasks; e += blockDim.x) {
        const int sl = e / ntasks, t = e - sl * ntasks;
        sG[e] = GQ[((kq0 + sl) * ntasks + t) * B + b];
    }
    for (int e = threadIdx.x; e < ns * nt; e += blockDim.x) {
        const int sl = e / nt, t = e - sl * nt;
        sT[e] = TS[((kq0 + sl) * nt + t) * B + b];
    }
    __syncthreads();
    const int sl = threadIdx.x / nz, a = threadIdx.x - sl * nz;
    if (sl >= ns) return;
    const int64_t kq = kq0 + sl;
    const double* ts = sT + sl * nt;
    const double* gq = sG + sl * ntasks;
    double ta[NZ], w[NZ];
#pragma unroll
    for (int I = 0; I < NX; ++I) ta[I] = ts[I * nz + a];
#pragma unroll
    for (int I = NX; I < NZ; ++I) ta[I] = I == a ? 1.0 : 0.0;
#pragma unroll
    for (int I = 0; I < NZ; ++I) w[I] = 0.0;
#pragma unroll
    for (int I = 0; I < NZ; ++I)
#pragma unroll
        for (int J = I; J < NZ; ++J) {
            if (J >= nz) continue;
            const int t = I * nz - I * (I - 1) / 2 + (J - I);
            const double g = gq[t];
            w[I] += g * ta[J];
            if (J != I) w[J] += g * ta[I];
        }
    double* __restrict__ hq = HQ + kq * P.nhk * B + b;
#pragma unroll
    for (int c = 0; c < NZ; ++c) {
        if (c < a || c >= nz) continue;
        double sacc = 0.0;
#pragma unroll
        for (int e = NX; e < NZ; ++e) sacc = e == c ? w[e] : sacc;
#pragma unroll
        for (int I = 0; I < NX; ++I) sacc += ts[I * nz + c] * w[I];
        hq[(int64_t)(c * (c + 1) / 2 + a) * B] = sacc;
    }
}

// H[k][e] = sum over the interval's stages of HQ, in stage order (thread = instance, entry, interval)
static __global__ void __launch_bounds__(256) k_msk_hproj_sum(const MskParams P, const double* __restrict__ HQ,
                                                       double* __restrict__ H) {
    const int64_t B = P.B;
    const int nhk = P.nhk, Q = P.Q;
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= B * P.N * nhk) return;
    const int64_t b = item % B, rest = item / B;
    const int e = (int)(rest % nhk);
    const int64_t k = rest / nhk;
    double s = 0.0;
    for (int q = 0; q < Q; ++q) s += HQ[(((k * Q + q) * nhk) + e) * B + b];
    H[(k * nhk + e) * B + b] = s;
}

// ---- single shooting (IVP): thread = instance, every sub-step written -------------------------------------
template <int NQ, int NM, int FAM, int SCHEME>
__global__ void __launch_bounds__(256) k_msk_ivp(const MskParams P, const MskGeom* __restrict__ GG,
                                                 const double* __restrict__ X0, const double* __restrict__ U,
                                                 double* __restrict__ TR) {
    constexpr int NX = NM * msk_nxm<FAM>() + 2 * NQ;
    constexpr int NUMAX = msk_numax<NQ, NM, FAM>();
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const MskGeom& G = *GG;
    double x[NX], u[NUMAX > 0 ? NUMAX : 1];
    double lam[msk_hmed<FAM>() ? NM * msk_tmax<FAM>() : 1];
#pragma unroll
    for (int r = 0; r < NX; ++r) x[r] = X0 ? X0[(int64_t)r * B + b] : P.rest[r];
    int64_t row = 0;
#pragma unroll
    for (int r = 0; r < NX; ++r) TR[(row * NX + r) * B + b] = x[r];
    MskParams P1 = P;
    P1.m = 1;
    for (int k = 0; k < P.N; ++k) {
#pragma unroll
        for (int i = 0; i < NUMAX; ++i) {
            const int dc = msk_udec<NM, FAM>(i, P.T, P.nu);
            u[i] = dc >= 0 ? U[((int64_t)k * P.nu + dc) * B + b] : 0.0;
        }
        msk_interval_lam<NM, FAM>(G, u, lam);
        for (int j = 0; j < P.m; ++j) {
            MskParams Pj = P1;
            Pj.cs = P.cs + (int64_t)j * (P.Q / P.m) * msk_cs_stride<NM, FAM>();  // sub-step j's stages inside interval k
            if (P.cs1) Pj.cs1 = P.cs1 + (int64_t)j * (P.Q / P.m) * NM;
            msk_interval<NQ, NM, FAM, SCHEME>(Pj, G, k, x, u, lam);
            ++row;
#pragma unroll
            for (int r = 0; r < NX; ++r) TR[(row * NX + r) * B + b] = x[r];
        }
    }
}

// ---- Hmed sliding-window rows (CustomConstraint.pulse_intensity_sliding_window_constraint, custom_constraints.py:
// 102-119): row (k, s) = u_k[s] - (parameter sl_param[k][s], or I_min where the window reaches before the first
// pulse); J entries +1 (and -1 on the parameter) at sl_joff.  thread = (instance, row)
static __global__ void __launch_bounds__(256) k_msk_slide(const MskParams P, int ns, const int32_t* __restrict__ sl_param,
                                                   const int32_t* __restrict__ sl_joff, const double* __restrict__ imin,
                                                   int64_t p_off, const double* __restrict__ V,
                                                   double* __restrict__ Gout, double* __restrict__ J) {
    const int64_t B = P.B;
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= B * P.N * ns) return;
    const int64_t b = item % B, rest = item / B;
    const int s = (int)(rest % ns);
    const int64_t k = rest / ns;
    const int64_t r = k * ns + s;
    const int pi = sl_param[r];
    if (Gout) {
        const double u = V[(k * P.nz + P.nx + s) * B + b];
        const double w = pi >= 0 ? V[(p_off + pi) * B + b] : imin[s / P.T];
        Gout[(k * P.ngk + P.nx + s) * B + b] = u - w;
    }
    if (J) {
        J[(int64_t)sl_joff[r] * B + b] = 1.0;
        if (pi >= 0) J[((int64_t)sl_joff[r] + 1) * B + b] = -1.0;
    }
}

// ---- marker superimposition rows (bioptim ConstraintFcn.SUPERIMPOSE_MARKERS, cfx_msk_marker_pair) ------------
// Row r of a pair: world axis axis[r] of marker(second) - marker(first) at q_node.  A marker fixed in dof frame f
// moves with q_0 .. q_f, so a pair depends on its first nd = max(frame) + 1 dofs: nd J_g entries per row (dof order,
// from jo), and the Hessian entries of the q_node pairs (i, j <= i < nd) at hoff (packed as Jet<NQ>::h).
struct MskMarker {
    int32_t node, nrow, nd, row0, jo;
    int32_t axis[3];
    int32_t frame[2];
    int32_t hoff[kMskMaxQ * (kMskMaxQ + 1) / 2];
    double pos[2][3];
};

template <int NQ, class S>
MSK_HD void msk_marker_diff(const MskGeom& G, const MskMarker& c, const S* q, S* d) {
    S R[NQ][9], o[NQ][3], z[NQ][3];
    msk_frames<NQ>(G, q, R, o, z);
    S P0[3], P1[3], dP[NQ][3];
    msk_point<NQ>(R, o, z, c.frame[0], c.pos[0], P0, dP);
    msk_point<NQ>(R, o, z, c.frame[1], c.pos[1], P1, dP);
#pragma unroll
    for (int a = 0; a < 3; ++a) d[a] = P1[a] - P0[a];
}
template <class S>
MSK_HD const S& msk_axis(const S* d, int a) {  // wave-uniform a: a select, not a dynamically indexed array
    return a == 0 ? d[0] : a == 1 ? d[1] : d[2];
}

// thread = instance, every pair in order (a few rows each; one thread per instance keeps the += of pairs that share
// a node race-free).  LAM == nullptr: the rows into Gout (nullable) and their J_g values into J (nullable);
// otherwise sum_r lambda_r d^2 row_r / dq^2 is added to H (after the dynamics' Hessian launch, same stream).
template <int NQ>
__global__ void __launch_bounds__(256) k_msk_markers(const MskParams P, const MskGeom* __restrict__ GG, int n,
                                                     const MskMarker* __restrict__ mk, int qoff,
                                                     const double* __restrict__ V, double* __restrict__ Gout,
                                                     double* __restrict__ J, const double* __restrict__ LAM,
                                                     double* __restrict__ H) {
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const MskGeom& G = *GG;
    for (int i = 0; i < n; ++i) {
        const MskMarker& c = mk[i];
        const int64_t qb = (int64_t)c.node * P.nz + qoff;
        if (LAM) {
            Jet<NQ> q[NQ], d[3];
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                q[j] = jconst<NQ>(V[(qb + j) * B + b]);
                q[j].g[j] = 1.0;
            }
            msk_marker_diff<NQ>(G, c, q, d);
            for (int r = 0; r < c.nrow; ++r) {
                const double lam = LAM[(int64_t)(c.row0 + r) * B + b];
                const Jet<NQ>& e = msk_axis(d, c.axis[r]);
#pragma unroll
                for (int t = 0; t < Jet<NQ>::H; ++t)
                    if (c.hoff[t] >= 0) H[(int64_t)c.hoff[t] * B + b] += lam * e.h[t];
            }
        } else if (J) {
            Dual<NQ> q[NQ], d[3];
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                q[j] = dconst<NQ>(V[(qb + j) * B + b]);
                q[j].d[j] = 1.0;
            }
            msk_marker_diff<NQ>(G, c, q, d);
            for (int r = 0; r < c.nrow; ++r) {
                const Dual<NQ>& e = msk_axis(d, c.axis[r]);
                if (Gout) Gout[(int64_t)(c.row0 + r) * B + b] = e.v;
#pragma unroll
                for (int j = 0; j < NQ; ++j)
                    if (j < c.nd) J[(int64_t)(c.jo + r * c.nd + j) * B + b] = e.d[j];
            }
        } else if (Gout) {
            double q[NQ], d[3];
#pragma unroll
            for (int j = 0; j < NQ; ++j) q[j] = V[(qb + j) * B + b];
            msk_marker_diff<NQ>(G, c, q, d);
            for (int r = 0; r < c.nrow; ++r) Gout[(int64_t)(c.row0 + r) * B + b] = msk_axis(d, c.axis[r]);
        }
    }
}

// ---- objective: quadratic tracking terms and the fatigue ratio term; thread = instance ---------------------
struct MskObjective {
    int32_t kind;  // 0 Lagrange quadratic, 1 Mayer quadratic, 2 Mayer inverse square  w (c / z)^2
    int32_t var_kind, var_index, node_first, node_last, target_off;
    double w_eff, target_value;
};

static __global__ void __launch_bounds__(256) k_msk_objective(const MskParams P, int n_obj, const MskObjective* __restrict__ obj,
                                                       const double* __restrict__ targets, const double* __restrict__ V,
                                                       double* __restrict__ F, double* __restrict__ GRAD,
                                                       const double* __restrict__ obj_factor, double* __restrict__ H,
                                                       const int32_t* __restrict__ hdiag) {
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double f = 0.0;
    const double s = H ? obj_factor[b] : 0.0;
    for (int t = 0; t < n_obj; ++t) {
        const MskObjective o = obj[t];
        for (int k = o.node_first; k <= o.node_last; ++k) {
            const int e = (o.var_kind == 0 ? 0 : P.nx) + o.var_index;
            const int64_t off = (int64_t)k * P.nz + e;
            const double z = V[off * B + b];
            double val, g1, g2;
            if (o.kind == 2) {
                const double r = o.target_value / z;
                val = o.w_eff * r * r;
                g1 = -2.0 * val / z;
                g2 = 6.0 * val / (z * z);
            } else {
                const double tgt = o.target_off >= 0 ? targets[o.target_off + k] : o.target_value;
                const double d = z - tgt;
                val = o.w_eff * d * d;
                g1 = 2.0 * o.w_eff * d;
                g2 = 2.0 * o.w_eff;
            }
            f += val;
            if (GRAD) GRAD[off * B + b] += g1;
            if (H) H[(int64_t)hdiag[k * P.nz + e] * B + b] += s * g2;
        }
    }
    if (F) F[b] = f;
}

}  // namespace cfx
