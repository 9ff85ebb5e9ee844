// cfx_launch.h — host-side launchers of the templated kernels (instantiated per model family in
// cfx_inst_ding.hip / cfx_inst_hmed.hip so the builds run in parallel).
#pragma once

#include <hip/hip_runtime.h>

#include "cfx_hessian.h"
#include "cfx_kernels.h"

namespace cfx {

// Jacobian directions carried per lane, per model (nz = nx + nu).  Hmed splits its nx + T directions
// into chunks of 4 (nx = 2) or 5 (nx = 5); the others carry all directions in one lane.
constexpr int dirs_of(int model) {
    return model == M_D03 ? 2 : model == M_D03F ? 5 : model == M_D07 ? 3 : model == M_D07F ? 6 : model == M_H18 ? 4 : 5;
}

// Direction chunks per lane group for a problem with nz directions.
inline int nchunk_of(int model, int nz) { return (nz + dirs_of(model) - 1) / dirs_of(model); }

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

hipError_t launch_hessian(int model, int scheme, int tmax, const KParams& P, const HTask* tasks, int ntasks, int bs,
                          const double* V, const double* LAM, double* H, hipStream_t s);

// direct collocation (cfx_colloc.h, instantiated in cfx_inst_colloc.hip)
hipError_t launch_colloc(int model, int tmax, const KParams& P, const double* V, double* G, double* J,
                         hipStream_t s);
hipError_t launch_colloc_hess(int model, int tmax, const KParams& P, const HTask* tasks, int ntasks, int bs,
                              const double* V, const double* LAM, double* H, hipStream_t s);

template <int MODEL, int SCHEME, int DJ, int TMAX>
hipError_t launch_hessian_t(const KParams& P, const HTask* tasks, int ntasks, int bs, const double* V,
                            const double* LAM, double* H, hipStream_t s) {
    dim3 grid((unsigned)((P.B + kBlock - 1) / kBlock), (unsigned)P.N, (unsigned)ntasks);
    hipLaunchKernelGGL((k_hessian<MODEL, SCHEME, DJ, TMAX>), grid, dim3(kBlock), 0, s, P, tasks, bs, V, LAM, H);
    return hipGetLastError();
}

template <int MODEL, int SCHEME, int D, int TMAX, int NI>
hipError_t launch_shooting_t(const KParams& P, const double* V, double* G, double* J, hipStream_t s) {
    const int nz = P.nz;
    const int nchunk = D > 0 ? (nz + D - 1) / D : 1;
    const int64_t per_block = (int64_t)kBlock * NI;  // NI adjacent instances per lane
    dim3 grid((unsigned)((P.B + per_block - 1) / per_block), (unsigned)((P.N + P.kpt - 1) / P.kpt), (unsigned)nchunk);
    hipLaunchKernelGGL((k_shooting<MODEL, SCHEME, D, TMAX, NI>), grid, dim3(kBlock), 0, s, P, V, G, J);
    return hipGetLastError();
}

template <int MODEL, int SCHEME, int TMAX>
hipError_t launch_ivp_t(const KParams& P, const double* X0, const double* U, double* TR, hipStream_t s) {
    dim3 grid((unsigned)((P.B + kBlock - 1) / kBlock));
    hipLaunchKernelGGL((k_ivp<MODEL, SCHEME, TMAX>), grid, dim3(kBlock), 0, s, P, X0, U, TR);
    return hipGetLastError();
}

}  // namespace cfx
