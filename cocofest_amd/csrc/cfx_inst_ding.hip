// Kernel instantiations for the Ding2003 / Ding2007 families (with and without fatigue).
#include "cfx_launch.h"

namespace cfx {

template <int MODEL, int NI>
static hipError_t shooting_ni(int scheme, bool derivs, const KParams& P, const double* V, double* G, double* J,
                              hipStream_t s) {
    constexpr int D = dirs_of(MODEL);
    switch (scheme) {
        case 1:
            return derivs ? launch_shooting_t<MODEL, 1, D, 1, NI>(P, V, G, J, s)
                          : launch_shooting_t<MODEL, 1, 0, 1, NI>(P, V, G, J, s);
        case 2:
            return derivs ? launch_shooting_t<MODEL, 2, D, 1, NI>(P, V, G, J, s)
                          : launch_shooting_t<MODEL, 2, 0, 1, NI>(P, V, G, J, s);
        case 4:
            return derivs ? launch_shooting_t<MODEL, 4, D, 1, NI>(P, V, G, J, s)
                          : launch_shooting_t<MODEL, 4, 0, 1, NI>(P, V, G, J, s);
        default:
            return hipErrorInvalidValue;
    }
}

// ni: instances integrated side by side per thread (1, 2 or 4)
template <int MODEL>
static hipError_t shooting_model(int scheme, bool derivs, int ni, const KParams& P, const double* V, double* G,
                                 double* J, hipStream_t s) {
    switch (ni) {
        case 1: return shooting_ni<MODEL, 1>(scheme, derivs, P, V, G, J, s);
        case 2: return shooting_ni<MODEL, 2>(scheme, derivs, P, V, G, J, s);
        case 4: return shooting_ni<MODEL, 4>(scheme, derivs, P, V, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_shooting_ding(int model, int scheme, bool derivs, int ni, const KParams& P, const double* V,
                                double* G, double* J, hipStream_t s) {
    switch (model) {
        case M_D03: return shooting_model<M_D03>(scheme, derivs, ni, P, V, G, J, s);
        case M_D03F: return shooting_model<M_D03F>(scheme, derivs, ni, P, V, G, J, s);
        case M_D07: return shooting_model<M_D07>(scheme, derivs, ni, P, V, G, J, s);
        case M_D07F: return shooting_model<M_D07F>(scheme, derivs, ni, P, V, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

template <int MODEL>
static hipError_t ivp_model(int scheme, const KParams& P, const double* X0, const double* U, double* TR, hipStream_t s) {
    switch (scheme) {
        case 1: return launch_ivp_t<MODEL, 1, 1>(P, X0, U, TR, s);
        case 2: return launch_ivp_t<MODEL, 2, 1>(P, X0, U, TR, s);
        case 4: return launch_ivp_t<MODEL, 4, 1>(P, X0, U, TR, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_ivp_ding(int model, int scheme, const KParams& P, const double* X0, const double* U, double* TR,
                           hipStream_t s) {
    switch (model) {
        case M_D03: return ivp_model<M_D03>(scheme, P, X0, U, TR, s);
        case M_D03F: return ivp_model<M_D03F>(scheme, P, X0, U, TR, s);
        case M_D07: return ivp_model<M_D07>(scheme, P, X0, U, TR, s);
        case M_D07F: return ivp_model<M_D07F>(scheme, P, X0, U, TR, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace cfx
