// cfx_internal.h — library-internal accessors shared between the translation units of libcfx (not part of the
// C ABI in include/cfx.h).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/cfx.h"

// last failure of a handle-free call on this thread (cfx_last_error(NULL))
extern thread_local std::string g_create_error;

// batch, layout, device and launch stream of a handle (cfx_api.hip)
int cfx_internal_info(const cfx_handle* h, int64_t* batch, int* layout, int* device, hipStream_t* stream);

// batched band LU helpers (cfx_band.hip): does the one-wavefront register placement apply; parallel right-hand
// sides (one wavefront each) with the factors of cfx_band_lu over batch = instances x parts systems: system q
// of instance b has its column c < nx at X + b x_inst + q x_part + c x_rhs, plus (Y != NULL) one at
// Y + b y_inst + q y_part
int cfx_band_reg_ok(int64_t n, int32_t kl, int32_t ku);
int cfx_band_solve_multi(int64_t n, int32_t kl, int32_t ku, int64_t batch, int32_t parts, const double* ab,
                         const int32_t* ipiv, double* X, int64_t x_inst, int64_t x_part, int64_t x_rhs, int32_t nx,
                         double* Y, int64_t y_inst, int64_t y_part, void* stream);

// MSK handles: keep the stage values / coefficients of every cfx_eval_all with J_g (on = 1; 0 switches it off); a
// following cfx_eval_h re-uses them only when the caller has declared, with on = 2 right before it, that the point
// is the one of that eval_all (cfx_ipm_solve, which does not move K.vx in between).  Any other eval_h recomputes.
int cfx_internal_msk_stash(cfx_handle* h, int on);

// block-tridiagonal (stage chain) factorisation and solves by block cyclic reduction (cfx_chain.hip): node size sp
// (a multiple of 16, <= 128); D / L / U [M][sp][sp] per instance at `stride`, work Cl / Cr at `wstride`; right-hand
// side c of instance b at R + b r_inst + c r_rhs (node k at + k sp), scratch T of the same shape
int cfx_chain_sp_ok(int32_t sp);
int cfx_chain_factor_s(int64_t batch, int32_t M, int32_t sp, double* D, double* L, double* U, int64_t stride,
                       double* Cl, double* Cr, int64_t wstride, int32_t* info, void* stream);
int cfx_chain_solve_s(int64_t batch, int32_t M, int32_t sp, const double* D, const double* L, const double* U,
                      int64_t stride, const double* Cl, const double* Cr, int64_t wstride, int32_t nrhs, double* R,
                      int64_t r_inst, int64_t r_rhs, double* T, int64_t t_inst, int64_t t_rhs, void* stream);
// negative eigenvalues of the symmetric block-tridiagonal matrix factored by cfx_chain_factor_s (its D slots), added
// to neg[b] (zero pivots add 1 << 20)
int cfx_chain_inertia_s(int64_t batch, int32_t M, int32_t sp, const double* D, int64_t stride, int32_t* neg,
                        void* stream);
