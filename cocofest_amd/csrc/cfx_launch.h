// cfx_launch.h — host-side launchers of the templated kernels (instantiated per model family in
// cfx_inst_ding.hip / cfx_inst_hmed.hip so the builds run in parallel).
#pragma once

#include <hip/hip_runtime.h>

#include "cfx_hessian.h"
#include "cfx_kernels.h"

namespace cfx {

#ifndef HMED_DIRS
#define HMED_DIRS 12  // Jacobian directions per lane for Hmed2018 (nx = 2), see dirs_of
#endif

// Jacobian directions carried per lane (nz = nx + nu).  The Ding families carry all of them in one lane.
// Hmed carries nx + T directions: as many per lane as the RK stage arrays (2 / 3 / 5 arrays of nx x D doubles
// for RK1 / RK2 / RK4) fit in ~160 VGPRs, so the value recursion is repeated over as few chunks as possible.
constexpr int dirs_of(int model, int scheme = 1, int tmax = 4) {
    if (model == M_D03) return 2;
    if (model == M_D03F) return 5;
    if (model == M_D07) return 3;
    if (model == M_D07F) return 6;
    const int all = (model == M_H18 ? 2 : 5) + tmax;
    const int d = model == M_H18 ? HMED_DIRS : 5;
    return all < d ? all : d;
}

// Direction chunks per lane group for a problem with nz directions.
inline int nchunk_of(int model, int scheme, int tmax, int nz) {
    const int d = dirs_of(model, scheme, tmax);
    return (nz + d - 1) / d;
}

// Smallest supported register-resident truncation bucket >= T (Hmed only).
inline int tmax_bucket(int T) { return T <= 4 ? 4 : T <= 8 ? 8 : T <= 16 ? 16 : 32; }

hipError_t launch_shooting_ding(int model, int scheme, bool derivs, int ni, const KParams& P, const double* V,
                                double* G, double* J, hipStream_t s);
hipError_t launch_shooting_hmed(int model, int scheme, bool derivs, int tmax, const KParams& P, const double* V,
                                double* G, double* J, hipStream_t s);
hipError_t launch_ivp_ding(int model, int scheme, const KParams& P, const double* X0, const double* U, double* TR,
                           hipStream_t s);
hipError_t launch_ivp_hmed(int model, int scheme, int tmax, const KParams& P, const double* X0, const double* U,
                           double* TR, hipStream_t s);

constexpr int kBlock = 256;

// Hessian jets: slots per lane (DJ), and whether the directions are split in block-pair tasks of DJ/2 each.
// Chosen so the RK4 stage arrays of Jet<DJ> stay in VGPRs (5 states x 4 arrays x Jet<2> = 240 registers).
constexpr int hjet_of(int model) {
    return model == M_D03 ? 2 : model == M_D07 ? 3 : model == M_H18 ? 4 : 2;
}
constexpr bool hsplit_of(int model) { return model != M_D03 && model != M_D07; }

// G, J (both or neither): the same launch writes g and J_g too (cfx_eval_all_h)
hipError_t launch_hessian(int model, int scheme, int tmax, const KParams& P, const HTask* tasks, int ntasks, int bs,
                          const double* V, const double* LAM, double* H, double* G, double* J, hipStream_t s);

// direct collocation (cfx_colloc.h, instantiated in cfx_inst_colloc.hip)
// ni: adjacent instances per lane (1 or 2; the Ding families, degrees 1..5).  launch_colloc_hess with G, J (both or
// neither): the same launch writes g and J_g too (cfx_eval_all_h)
hipError_t launch_colloc(int model, int tmax, int ni, const KParams& P, const double* V, double* G, double* J,
                         hipStream_t s);
hipError_t launch_colloc_hess(int model, int tmax, const KParams& P, const HTask* tasks, int ntasks, int bs,
                              const double* V, const double* LAM, double* H, double* G, double* J, hipStream_t s);

template <int MODEL, int SCHEME, int DJ, int TMAX>
hipError_t launch_hessian_t(const KParams& P, const HTask* tasks, int ntasks, int bs, const double* V,
                            const double* LAM, double* H, double* G, double* J, hipStream_t s) {
    dim3 grid((unsigned)((P.B + kBlock - 1) / kBlock), (unsigned)P.N, (unsigned)ntasks);
    if (G && J)
        hipLaunchKernelGGL((k_hessian<MODEL, SCHEME, DJ, TMAX, true>), grid, dim3(kBlock), 0, s, P, tasks, bs, V, LAM, H,
                           G, J);
    else
        hipLaunchKernelGGL((k_hessian<MODEL, SCHEME, DJ, TMAX, false>), grid, dim3(kBlock), 0, s, P, tasks, bs, V, LAM,
                           H, (double*)nullptr, (double*)nullptr);
    return hipGetLastError();
}

template <int MODEL, int SCHEME, int D, int TMAX, int NI>
hipError_t launch_shooting_t(const KParams& P, const double* V, double* G, double* J, hipStream_t s) {
    const int nz = P.nz;
    const int nchunk = D > 0 ? (nz + D - 1) / D : 1;
    const int64_t per_block = (int64_t)kBlock * NI;  // NI adjacent instances per lane
    const unsigned nbi = (unsigned)((P.B + per_block - 1) / per_block), nbk = (unsigned)((P.N + P.kpt - 1) / P.kpt);
    if (!P.ifast || nbi <= (unsigned)kMaxGridY) {
        dim3 grid(P.ifast ? nbk : nbi, P.ifast ? nbi : nbk, (unsigned)nchunk);
        hipLaunchKernelGGL((k_shooting<MODEL, SCHEME, D, TMAX, NI>), grid, dim3(kBlock), 0, s, P, V, G, J);
    } else {
        // the intervals-fast order was chosen for the handle's instances per lane; this launch runs fewer (an
        // unaligned buffer) and its instance blocks no longer fit grid.y: instance blocks on grid.x instead
        KParams Q = P;
        Q.ifast = 0;
        hipLaunchKernelGGL((k_shooting<MODEL, SCHEME, D, TMAX, NI>), dim3(nbi, nbk, (unsigned)nchunk), dim3(kBlock), 0,
                           s, Q, V, G, J);
    }
    return hipGetLastError();
}

template <int MODEL, int SCHEME, int TMAX>
hipError_t launch_ivp_t(const KParams& P, const double* X0, const double* U, double* TR, hipStream_t s) {
    dim3 grid((unsigned)((P.B + kBlock - 1) / kBlock));
    hipLaunchKernelGGL((k_ivp<MODEL, SCHEME, TMAX>), grid, dim3(kBlock), 0, s, P, X0, U, TR);
    return hipGetLastError();
}

}  // namespace cfx
