// cfx_msk_launch.h — host-side entry points of the musculoskeletal kernels (instantiated in cfx_inst_msk.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "cfx_msk.h"

namespace cfx {

// Supported shapes: is (n_dof, n_muscles, family, scheme) compiled in?
bool msk_supported(int nq, int nm, int fam, int scheme);

// Structural dependency masks of the nx end states of one interval over z = (x_k, u_k) (host, Dep arithmetic).
void msk_dep_pattern(int nq, int nm, int fam, int scheme, const MskParams& P, const MskGeom& G, uint64_t* dep);

// Per-stage Jacobian coefficients of k_msk_stagecoef_par (msk_ncoef in cfx_msk.h).
inline int msk_ncoef_host(int nq, int nm) { return nm * (6 + 2 * nq) + 3 * nq * nq + nq * nm; }

// Batches up to this size split the Hessian projection by stage (k_msk_hproj_stage + k_msk_hproj_sum): at a few
// instances the launch is latency-bound, and a thread per stage cuts the chain.
constexpr int64_t kMskSmallBatch = 256;

// Work buffer of launch_msk_shooting / launch_msk_hessian (doubles): stage coefficients, stage values XS (their
// first two regions are what g + J_g needs), stage tangents TS, stage adjoints MU, the Y-space pair Hessians GQ
// and, for small batches, the per-stage Hessian terms HQ of every (instance, interval, stage).
inline size_t msk_shoot_work_host(int nq, int nm, int nx, int64_t B, int N, int Q) {
    return (size_t)B * N * Q * ((size_t)msk_ncoef_host(nq, nm) + nx);
}
inline size_t msk_hess_work_host(int nq, int nm, int nx, int nz, int ntasks, int64_t B, int N, int Q) {
    const size_t hq = B <= kMskSmallBatch ? (size_t)nz * (nz + 1) / 2 : 0;
    return (size_t)B * N * Q * ((size_t)msk_ncoef_host(nq, nm) + nx + (size_t)nx * nz + nx + ntasks + hq);
}

// g (+ J_g when J != nullptr; P.scratch then points at a msk_shoot_work_host buffer, whose XS region keeps the stage
// values, so that a launch_msk_hessian at the same point can skip the recursion: reuse).  keep_xs: a Hessian at this
// point will reuse the stage data, so the fused stage/tangent kernel stores the coefficients too.
hipError_t launch_msk_shooting(int nq, int nm, int fam, int scheme, const MskParams& P, const MskGeom* G,
                               const double* V, double* Gout, double* J, bool keep_xs, hipStream_t s);
hipError_t launch_msk_hessian(int nq, int nm, int fam, int scheme, const MskParams& P, const MskGeom* G,
                              const int16_t* tasks, int ntasks, const double* V, const double* LAM, double* H,
                              double* work, bool reuse, hipStream_t s);
hipError_t launch_msk_ivp(int nq, int nm, int fam, int scheme, const MskParams& P, const MskGeom* G,
                          const double* X0, const double* U, double* TR, hipStream_t s);

}  // namespace cfx
