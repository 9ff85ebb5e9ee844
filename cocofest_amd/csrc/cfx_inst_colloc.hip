// Direct-collocation kernel instantiations (all models; Hmed truncation buckets as in cfx_inst_hmed.hip).
#include "cfx_colloc.h"
#include "cfx_launch.h"

namespace cfx {

template <int MODEL, int TMAX, int DEG>
static hipError_t colloc_deg(const KParams& P, const double* V, double* G, double* J, hipStream_t s) {
    dim3 grid((unsigned)((P.B + kBlock - 1) / kBlock), (unsigned)P.N);
    hipLaunchKernelGGL((k_colloc<MODEL, TMAX, DEG>), grid, dim3(kBlock), 0, s, P, V, G, J);
    return hipGetLastError();
}

// degrees 1..5 (bioptim's default is 4) with register-resident states; any other degree runs the generic kernel
template <int MODEL, int TMAX>
static hipError_t colloc_t(const KParams& P, const double* V, double* G, double* J, hipStream_t s) {
    switch (P.deg) {
        case 1: return colloc_deg<MODEL, TMAX, 1>(P, V, G, J, s);
        case 2: return colloc_deg<MODEL, TMAX, 2>(P, V, G, J, s);
        case 3: return colloc_deg<MODEL, TMAX, 3>(P, V, G, J, s);
        case 4: return colloc_deg<MODEL, TMAX, 4>(P, V, G, J, s);
        case 5: return colloc_deg<MODEL, TMAX, 5>(P, V, G, J, s);
        default: return colloc_deg<MODEL, TMAX, 0>(P, V, G, J, s);
    }
}

template <int MODEL, int TMAX>
static hipError_t colloc_hess_t(const KParams& P, const HTask* tasks, int ntasks, int bs, const double* V,
                                const double* LAM, double* H, hipStream_t s) {
    dim3 grid((unsigned)((P.B + kBlock - 1) / kBlock), (unsigned)P.N, (unsigned)ntasks);
    hipLaunchKernelGGL((k_colloc_hess<MODEL, hjet_of(MODEL), TMAX>), grid, dim3(kBlock), 0, s, P, tasks, bs, V, LAM, H);
    return hipGetLastError();
}

template <int MODEL>
static hipError_t colloc_hmed(int tmax, const KParams& P, const double* V, double* G, double* J, hipStream_t s) {
    switch (tmax) {
        case 4: return colloc_t<MODEL, 4>(P, V, G, J, s);
        case 8: return colloc_t<MODEL, 8>(P, V, G, J, s);
        case 16: return colloc_t<MODEL, 16>(P, V, G, J, s);
        case 32: return colloc_t<MODEL, 32>(P, V, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

template <int MODEL>
static hipError_t colloc_hess_hmed(int tmax, const KParams& P, const HTask* tasks, int ntasks, int bs,
                                   const double* V, const double* LAM, double* H, hipStream_t s) {
    switch (tmax) {
        case 4: return colloc_hess_t<MODEL, 4>(P, tasks, ntasks, bs, V, LAM, H, s);
        case 8: return colloc_hess_t<MODEL, 8>(P, tasks, ntasks, bs, V, LAM, H, s);
        case 16: return colloc_hess_t<MODEL, 16>(P, tasks, ntasks, bs, V, LAM, H, s);
        case 32: return colloc_hess_t<MODEL, 32>(P, tasks, ntasks, bs, V, LAM, H, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_colloc(int model, int tmax, const KParams& P, const double* V, double* G, double* J,
                         hipStream_t s) {
    switch (model) {
        case M_D03: return colloc_t<M_D03, 1>(P, V, G, J, s);
        case M_D03F: return colloc_t<M_D03F, 1>(P, V, G, J, s);
        case M_D07: return colloc_t<M_D07, 1>(P, V, G, J, s);
        case M_D07F: return colloc_t<M_D07F, 1>(P, V, G, J, s);
        case M_H18: return colloc_hmed<M_H18>(tmax, P, V, G, J, s);
        case M_H18F: return colloc_hmed<M_H18F>(tmax, P, V, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_colloc_hess(int model, int tmax, const KParams& P, const HTask* tasks, int ntasks, int bs,
                              const double* V, const double* LAM, double* H, hipStream_t s) {
    switch (model) {
        case M_D03: return colloc_hess_t<M_D03, 1>(P, tasks, ntasks, bs, V, LAM, H, s);
        case M_D03F: return colloc_hess_t<M_D03F, 1>(P, tasks, ntasks, bs, V, LAM, H, s);
        case M_D07: return colloc_hess_t<M_D07, 1>(P, tasks, ntasks, bs, V, LAM, H, s);
        case M_D07F: return colloc_hess_t<M_D07F, 1>(P, tasks, ntasks, bs, V, LAM, H, s);
        case M_H18: return colloc_hess_hmed<M_H18>(tmax, P, tasks, ntasks, bs, V, LAM, H, s);
        case M_H18F: return colloc_hess_hmed<M_H18F>(tmax, P, tasks, ntasks, bs, V, LAM, H, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace cfx
