// Direct-collocation kernel instantiations (all models; Hmed truncation buckets as in cfx_inst_hmed.hip).
#include "cfx_colloc.h"
#include "cfx_launch.h"

#include <cstdlib>
#include <cstring>

namespace cfx {

// grid as the shooting launch: interval chunks of P.kpt intervals on grid.x when P.ifast (the chunks of one instance
// block, which write one region of each 64-instance output tile, dispatched together), instance blocks on grid.y
// CFX_COLLOC_STORE (probe of the bench's instantiation only, read once per process): "plain" — ordinary instead of
// non-temporal output stores; "w4" / "w4plain" — the kernel held to 4 waves per SIMD.  Returns bit 0 plain, bit 1 w4
static int colloc_variant() {
    static const int v = [] {
        const char* e = getenv("CFX_COLLOC_STORE");
        if (!e) return 0;
        return (strstr(e, "plain") ? 1 : 0) | (strncmp(e, "w4", 2) == 0 ? 2 : 0);
    }();
    return v;
}

template <int MODEL, int TMAX, int DEG, int NI>
static hipError_t colloc_deg(const KParams& P, const double* V, double* G, double* J, hipStream_t s) {
    const int64_t per_block = (int64_t)kBlock * NI;
    const unsigned nbi = (unsigned)((P.B + per_block - 1) / per_block), nbk = (unsigned)((P.N + P.kpt - 1) / P.kpt);
    KParams Q = P;
    if (nbi > (unsigned)kMaxGridY) Q.ifast = 0;  // instance blocks must fit grid.y in the intervals-fast order
    dim3 grid(Q.ifast ? nbk : nbi, Q.ifast ? nbi : nbk);
    if constexpr (MODEL == M_D03 && DEG == 4 && NI == 2) {
        switch (colloc_variant()) {
            case 1: hipLaunchKernelGGL((k_colloc<MODEL, TMAX, DEG, NI, true>), grid, dim3(kBlock), 0, s, Q, V, G, J);
                    return hipGetLastError();
            case 2: hipLaunchKernelGGL((k_colloc_w4<MODEL, TMAX, DEG, NI, false>), grid, dim3(kBlock), 0, s, Q, V, G, J);
                    return hipGetLastError();
            case 3: hipLaunchKernelGGL((k_colloc_w4<MODEL, TMAX, DEG, NI, true>), grid, dim3(kBlock), 0, s, Q, V, G, J);
                    return hipGetLastError();
            default: break;
        }
        // the bench's shape: one kernel name per layout and J_g form (traces attribute each launch)
        if (J) {
            if (Q.tiled)
                hipLaunchKernelGGL((Q.keepc ? k_colloc_tiles_keepj<MODEL, TMAX, DEG, NI> : k_colloc_tiles<MODEL, TMAX, DEG, NI>),
                                   grid, dim3(kBlock), 0, s, Q, V, G, J);
            else
                hipLaunchKernelGGL((Q.keepc ? k_colloc_soa_keepj<MODEL, TMAX, DEG, NI> : k_colloc_soa<MODEL, TMAX, DEG, NI>),
                                   grid, dim3(kBlock), 0, s, Q, V, G, J);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((k_colloc<MODEL, TMAX, DEG, NI>), grid, dim3(kBlock), 0, s, Q, V, G, J);
    return hipGetLastError();
}

// degrees 1..5 (bioptim's default is 4) with register-resident states, one or two instances per lane; any other
// degree runs the generic kernel
template <int MODEL, int TMAX>
static hipError_t colloc_t(const KParams& P, int ni, const double* V, double* G, double* J, hipStream_t s) {
    if (ni == 2 && !is_int(MODEL)) {
        switch (P.deg) {
            case 1: return colloc_deg<MODEL, TMAX, 1, 2>(P, V, G, J, s);
            case 2: return colloc_deg<MODEL, TMAX, 2, 2>(P, V, G, J, s);
            case 3: return colloc_deg<MODEL, TMAX, 3, 2>(P, V, G, J, s);
            case 4: return colloc_deg<MODEL, TMAX, 4, 2>(P, V, G, J, s);
            case 5: return colloc_deg<MODEL, TMAX, 5, 2>(P, V, G, J, s);
            default: break;
        }
    }
    switch (P.deg) {
        case 1: return colloc_deg<MODEL, TMAX, 1, 1>(P, V, G, J, s);
        case 2: return colloc_deg<MODEL, TMAX, 2, 1>(P, V, G, J, s);
        case 3: return colloc_deg<MODEL, TMAX, 3, 1>(P, V, G, J, s);
        case 4: return colloc_deg<MODEL, TMAX, 4, 1>(P, V, G, J, s);
        case 5: return colloc_deg<MODEL, TMAX, 5, 1>(P, V, G, J, s);
        default: return colloc_deg<MODEL, TMAX, 0, 1>(P, V, G, J, s);
    }
}

template <int MODEL, int TMAX>
static hipError_t colloc_hess_t(const KParams& P, const HTask* tasks, int ntasks, int bs, const double* V,
                                const double* LAM, double* H, double* G, double* J, hipStream_t s) {
    dim3 grid((unsigned)((P.B + kBlock - 1) / kBlock), (unsigned)P.N, (unsigned)ntasks);
    if (G && J)
        hipLaunchKernelGGL((k_colloc_hess<MODEL, hjet_of(MODEL), TMAX, true>), grid, dim3(kBlock), 0, s, P, tasks, bs,
                           V, LAM, H, G, J);
    else
        hipLaunchKernelGGL((k_colloc_hess<MODEL, hjet_of(MODEL), TMAX, false>), grid, dim3(kBlock), 0, s, P, tasks, bs,
                           V, LAM, H, (double*)nullptr, (double*)nullptr);
    return hipGetLastError();
}

template <int MODEL>
static hipError_t colloc_hmed(int tmax, const KParams& P, const double* V, double* G, double* J, hipStream_t s) {
    switch (tmax) {
        case 4: return colloc_t<MODEL, 4>(P, 1, V, G, J, s);
        case 8: return colloc_t<MODEL, 8>(P, 1, V, G, J, s);
        case 16: return colloc_t<MODEL, 16>(P, 1, V, G, J, s);
        case 32: return colloc_t<MODEL, 32>(P, 1, V, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

template <int MODEL>
static hipError_t colloc_hess_hmed(int tmax, const KParams& P, const HTask* tasks, int ntasks, int bs,
                                   const double* V, const double* LAM, double* H, double* G, double* J, hipStream_t s) {
    switch (tmax) {
        case 4: return colloc_hess_t<MODEL, 4>(P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case 8: return colloc_hess_t<MODEL, 8>(P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case 16: return colloc_hess_t<MODEL, 16>(P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case 32: return colloc_hess_t<MODEL, 32>(P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_colloc(int model, int tmax, int ni, const KParams& P, const double* V, double* G, double* J,
                         hipStream_t s) {
    switch (model) {
        case M_D03: return colloc_t<M_D03, 1>(P, ni, V, G, J, s);
        case M_D03F: return colloc_t<M_D03F, 1>(P, ni, V, G, J, s);
        case M_D07: return colloc_t<M_D07, 1>(P, ni, V, G, J, s);
        case M_D07F: return colloc_t<M_D07F, 1>(P, ni, V, G, J, s);
        case M_H18: return colloc_hmed<M_H18>(tmax, P, V, G, J, s);
        case M_H18F: return colloc_hmed<M_H18F>(tmax, P, V, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_colloc_hess(int model, int tmax, const KParams& P, const HTask* tasks, int ntasks, int bs,
                              const double* V, const double* LAM, double* H, double* G, double* J, hipStream_t s) {
    switch (model) {
        case M_D03: return colloc_hess_t<M_D03, 1>(P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case M_D03F: return colloc_hess_t<M_D03F, 1>(P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case M_D07: return colloc_hess_t<M_D07, 1>(P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case M_D07F: return colloc_hess_t<M_D07F, 1>(P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case M_H18: return colloc_hess_hmed<M_H18>(tmax, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        case M_H18F: return colloc_hess_hmed<M_H18F>(tmax, P, tasks, ntasks, bs, V, LAM, H, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace cfx
