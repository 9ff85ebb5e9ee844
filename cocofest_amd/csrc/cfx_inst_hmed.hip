// Kernel instantiations for the Hmed2018 family; the truncation T lives in a register-resident
// bucket TMAX in {4, 8, 16, 32} (coefficients and lambdas zero-padded past T).
#include "cfx_launch.h"

namespace cfx {

template <int MODEL, int TMAX>
static hipError_t shooting_t(int scheme, bool derivs, const KParams& P, const double* V, double* G, double* J,
                             hipStream_t s) {
    switch (scheme) {
        case 1:
            return derivs ? launch_shooting_t<MODEL, 1, dirs_of(MODEL, 1, TMAX), TMAX, 1>(P, V, G, J, s)
                          : launch_shooting_t<MODEL, 1, 0, TMAX, 1>(P, V, G, J, s);
        case 2:
            return derivs ? launch_shooting_t<MODEL, 2, dirs_of(MODEL, 2, TMAX), TMAX, 1>(P, V, G, J, s)
                          : launch_shooting_t<MODEL, 2, 0, TMAX, 1>(P, V, G, J, s);
        case 4:
            return derivs ? launch_shooting_t<MODEL, 4, dirs_of(MODEL, 4, TMAX), TMAX, 1>(P, V, G, J, s)
                          : launch_shooting_t<MODEL, 4, 0, TMAX, 1>(P, V, G, J, s);
        default:
            return hipErrorInvalidValue;
    }
}

template <int MODEL>
static hipError_t shooting_model(int scheme, bool derivs, int tmax, const KParams& P, const double* V, double* G,
                                 double* J, hipStream_t s) {
    switch (tmax) {
        case 4: return shooting_t<MODEL, 4>(scheme, derivs, P, V, G, J, s);
        case 8: return shooting_t<MODEL, 8>(scheme, derivs, P, V, G, J, s);
        case 16: return shooting_t<MODEL, 16>(scheme, derivs, P, V, G, J, s);
        case 32: return shooting_t<MODEL, 32>(scheme, derivs, P, V, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_shooting_hmed(int model, int scheme, bool derivs, int tmax, const KParams& P, const double* V,
                                double* G, double* J, hipStream_t s) {
    switch (model) {
        case M_H18: return shooting_model<M_H18>(scheme, derivs, tmax, P, V, G, J, s);
        case M_H18F: return shooting_model<M_H18F>(scheme, derivs, tmax, P, V, G, J, s);
        default: return hipErrorInvalidValue;
    }
}

template <int MODEL, int TMAX>
static hipError_t ivp_t(int scheme, const KParams& P, const double* X0, const double* U, double* TR, hipStream_t s) {
    switch (scheme) {
        case 1: return launch_ivp_t<MODEL, 1, TMAX>(P, X0, U, TR, s);
        case 2: return launch_ivp_t<MODEL, 2, TMAX>(P, X0, U, TR, s);
        case 4: return launch_ivp_t<MODEL, 4, TMAX>(P, X0, U, TR, s);
        default: return hipErrorInvalidValue;
    }
}

template <int MODEL>
static hipError_t ivp_model(int scheme, int tmax, const KParams& P, const double* X0, const double* U, double* TR,
                            hipStream_t s) {
    switch (tmax) {
        case 4: return ivp_t<MODEL, 4>(scheme, P, X0, U, TR, s);
        case 8: return ivp_t<MODEL, 8>(scheme, P, X0, U, TR, s);
        case 16: return ivp_t<MODEL, 16>(scheme, P, X0, U, TR, s);
        case 32: return ivp_t<MODEL, 32>(scheme, P, X0, U, TR, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_ivp_hmed(int model, int scheme, int tmax, const KParams& P, const double* X0, const double* U,
                           double* TR, hipStream_t s) {
    switch (model) {
        case M_H18: return ivp_model<M_H18>(scheme, tmax, P, X0, U, TR, s);
        case M_H18F: return ivp_model<M_H18F>(scheme, tmax, P, X0, U, TR, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace cfx
