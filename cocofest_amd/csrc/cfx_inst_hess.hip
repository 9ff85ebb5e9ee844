// Lagrangian-Hessian kernel instantiations (all models; Hmed truncation buckets as in cfx_inst_hmed.hip).
#include "cfx_launch.h"

namespace cfx {

template <int MODEL, int TMAX>
static hipError_t hess_scheme(int scheme, const KParams& P, const HTask* tasks, int ntasks, int bs, const double* V,
                              const double* LAM, double* H, double* G, double* J, hipStream_t s) {
    constexpr int DJ = hjet_of(MODEL);
    switch (scheme) {
        case 1: return launch_hessian_t<MODEL, 1, DJ, TMAX>(P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case 2: return launch_hessian_t<MODEL, 2, DJ, TMAX>(P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case 4: return launch_hessian_t<MODEL, 4, DJ, TMAX>(P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

template <int MODEL>
static hipError_t hess_hmed(int scheme, int tmax, const KParams& P, const HTask* tasks, int ntasks, int bs,
                            const double* V, const double* LAM, double* H, double* G, double* J, hipStream_t s) {
    switch (tmax) {
        case 4: return hess_scheme<MODEL, 4>(scheme, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case 8: return hess_scheme<MODEL, 8>(scheme, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case 16: return hess_scheme<MODEL, 16>(scheme, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case 32: return hess_scheme<MODEL, 32>(scheme, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_hessian(int model, int scheme, int tmax, const KParams& P, const HTask* tasks, int ntasks, int bs,
                          const double* V, const double* LAM, double* H, double* G, double* J, hipStream_t s) {
    switch (model) {
        case M_D03: return hess_scheme<M_D03, 1>(scheme, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case M_D03F: return hess_scheme<M_D03F, 1>(scheme, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case M_D07: return hess_scheme<M_D07, 1>(scheme, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case M_D07F: return hess_scheme<M_D07F, 1>(scheme, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case M_H18: return hess_hmed<M_H18>(scheme, tmax, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case M_H18F: return hess_hmed<M_H18F>(scheme, tmax, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace cfx
