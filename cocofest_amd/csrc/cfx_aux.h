// cfx_aux.h — small kernels around the shooting kernel: objective value/gradient, the Hmed
// sliding-window rows, AoS <-> SoA transposes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cfx_kernels.h"

namespace cfx {

// One quadratic tracking term (fes_ocp.py:531-569): w_eff * (z_k - target_k)^2 for k in [k0, k1],
// w_eff = weight * dt (Lagrange) or weight (Mayer).
struct DevObjective {
    int32_t var_kind;   // 0 state, 1 control
    int32_t var_index;
    int32_t node_first, node_last;
    int32_t target_off; // offset into the targets array, -1: scalar target
    int32_t pad_;
    double w_eff;
    double target_value;
};

// Objective value and gradient, one thread per instance.  GRAD must be zeroed beforehand.
__global__ void __launch_bounds__(256) k_objective(const KParams P, int n_obj, const DevObjective* __restrict__ obj,
                                                   const double* __restrict__ targets, const double* __restrict__ V,
                                                   double* __restrict__ F, double* __restrict__ GRAD) {
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int64_t ES = lay_stride(P), vb = lay_base(P, P.nv_tot, b);  // V and GRAD share the layout
    double f = 0.0;
    for (int t = 0; t < n_obj; ++t) {
        const DevObjective o = obj[t];
        for (int k = o.node_first; k <= o.node_last; ++k) {
            const int64_t off = (int64_t)k * P.nz + (o.var_kind == 0 ? 0 : P.uoff) + o.var_index;
            const double z = V[vb + off * ES];
            const double tgt = o.target_off >= 0 ? targets[o.target_off + k] : o.target_value;
            const double d = z - tgt;
            f += o.w_eff * d * d;
            if (GRAD) GRAD[vb + off * ES] += 2.0 * o.w_eff * d;
        }
    }
    if (F) F[b] = f;
}

// Objective Hessian diagonal contributions added into the Lagrangian Hessian values.
__global__ void __launch_bounds__(256) k_objective_hess(const KParams P, int n_obj, const DevObjective* __restrict__ obj,
                                                        const double* __restrict__ obj_factor,
                                                        double* __restrict__ H) {
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const double s = obj_factor[b];
    const int64_t ES = lay_stride(P), hb = lay_base(P, P.nh_tot, b);
    for (int t = 0; t < n_obj; ++t) {
        const DevObjective o = obj[t];
        const int e = (o.var_kind == 0 ? 0 : P.nx) + o.var_index;  // element of (x_k, u_k)
        for (int k = o.node_first; k <= o.node_last; ++k) {
            const int64_t hoff = P.hdiag[k * (P.nx + P.nu) + e];
            H[hb + hoff * ES] += 2.0 * o.w_eff * s;
        }
    }
}

// Small batches (latency-bound: the interior point at batch 1): one block per instance, a thread per node.
// Every term of a node is handled by that node's thread, so no two threads touch one gradient or Hessian entry;
// the block zeroes its own gradient first (no separate memset), f is a block sum in a fixed order.
constexpr int64_t kObjBlockMaxB = 2048;

__device__ inline double block_sum256(double v, double* sh) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    return sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ void __launch_bounds__(256) k_objective_blk(const KParams P, int n_obj, const DevObjective* __restrict__ obj,
                                                       const double* __restrict__ targets,
                                                       const double* __restrict__ V, double* __restrict__ F,
                                                       double* __restrict__ GRAD) {
    __shared__ double sh[4];
    const int64_t b = blockIdx.x;
    const int64_t ES = lay_stride(P), vb = lay_base(P, P.nv_tot, b);
    if (GRAD) {
        for (int64_t e = threadIdx.x; e < P.nv_tot; e += 256) GRAD[vb + e * ES] = 0.0;
        __syncthreads();
    }
    double f = 0.0;
    for (int k = threadIdx.x; k <= P.N; k += 256)
        for (int t = 0; t < n_obj; ++t) {
            const DevObjective o = obj[t];
            if (k < o.node_first || k > o.node_last) continue;
            const int64_t off = (int64_t)k * P.nz + (o.var_kind == 0 ? 0 : P.uoff) + o.var_index;
            const double d = V[vb + off * ES] - (o.target_off >= 0 ? targets[o.target_off + k] : o.target_value);
            f += o.w_eff * d * d;
            if (GRAD) GRAD[vb + off * ES] += 2.0 * o.w_eff * d;
        }
    f = block_sum256(f, sh);
    if (F && threadIdx.x == 0) F[b] = f;
}

__global__ void __launch_bounds__(256) k_objective_hess_blk(const KParams P, int n_obj,
                                                            const DevObjective* __restrict__ obj,
                                                            const double* __restrict__ obj_factor,
                                                            double* __restrict__ H) {
    const int64_t b = blockIdx.x;
    const double s = obj_factor[b];
    const int64_t ES = lay_stride(P), hb = lay_base(P, P.nh_tot, b);
    for (int k = threadIdx.x; k <= P.N; k += 256)
        for (int t = 0; t < n_obj; ++t) {
            const DevObjective o = obj[t];
            if (k < o.node_first || k > o.node_last) continue;
            const int e = (o.var_kind == 0 ? 0 : P.nx) + o.var_index;
            H[hb + (int64_t)P.hdiag[k * (P.nx + P.nu) + e] * ES] += 2.0 * o.w_eff * s;
        }
}

// Hmed sliding-window rows (custom_constraints.py:102-119): g = u_k[j] - window_k(p)[j], J = +1 / -1.
// slot (k, j): param index or -1 for the intensity-floor padding; joff = J offset of its +1 entry.
// Thread = (instance, slot): its two loads precede its stores (a per-instance loop over the slots would issue
// every load behind the previous slot's stores, which vmcnt serialises).
__global__ void __launch_bounds__(256) k_slide(const KParams P, const int32_t* __restrict__ sl_param,
                                               const int32_t* __restrict__ sl_joff, double floor_value,
                                               const double* __restrict__ V, double* __restrict__ G,
                                               double* __restrict__ J) {
    const int64_t B = P.B;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int64_t p_off = (int64_t)P.N * P.nz + P.nx;
    const int g_off = P.ngk - P.n_slide;  // the window rows follow the interval's dynamics rows
    const int64_t ES = lay_stride(P), vb = lay_base(P, P.nv_tot, b), gb = lay_base(P, P.ng_tot, b),
                  jb = lay_base(P, P.nnz_tot, b);
    // slot = k * T + j; grid.y is capped at 65535, so the slots are strided over it
    for (int slot = blockIdx.y; slot < P.N * P.T; slot += gridDim.y) {
        const int k = slot / P.T, j = slot - k * P.T;
        const int pi = sl_param[slot];
        if (G) {
            const double u = V[vb + ((int64_t)k * P.nz + P.uoff + j) * ES];
            const double w = pi >= 0 ? V[vb + (p_off + pi) * ES] : floor_value;
            G[gb + ((int64_t)k * P.ngk + g_off + j) * ES] = u - w;
        }
        if (J) {
            const int64_t jo = sl_joff[slot];
            J[jb + jo * ES] = 1.0;
            if (pi >= 0) J[jb + (jo + 1) * ES] = -1.0;
        }
    }
}

// dst[e * B + b] = src[b * len + e]  (AoS -> SoA) through a 64x64 LDS tile; 256 threads.
__global__ void __launch_bounds__(256) k_aos_to_soa(const double* __restrict__ src, double* __restrict__ dst,
                                                    int64_t B, int64_t len) {
    __shared__ double tile[64][65];
    const int64_t b0 = (int64_t)blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int64_t e0 = (int64_t)blockIdx.y * 64; e0 < len; e0 += (int64_t)gridDim.y * 64) {
        for (int r = ty; r < 64; r += 4) {  // read rows b, columns e (coalesced in e)
            const int64_t b = b0 + r, e = e0 + tx;
            if (b < B && e < len) tile[r][tx] = src[b * len + e];
        }
        __syncthreads();
        for (int r = ty; r < 64; r += 4) {  // write rows e, columns b (coalesced in b)
            const int64_t e = e0 + r, b = b0 + tx;
            if (b < B && e < len) dst[e * B + b] = tile[tx][r];
        }
        __syncthreads();
    }
}

// dst[b * len + e] = src[e * B + b]  (SoA -> AoS)
__global__ void __launch_bounds__(256) k_soa_to_aos(const double* __restrict__ src, double* __restrict__ dst,
                                                    int64_t B, int64_t len) {
    __shared__ double tile[64][65];
    const int64_t b0 = (int64_t)blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int64_t e0 = (int64_t)blockIdx.y * 64; e0 < len; e0 += (int64_t)gridDim.y * 64) {
        for (int r = ty; r < 64; r += 4) {
            const int64_t e = e0 + r, b = b0 + tx;
            if (b < B && e < len) tile[r][tx] = src[e * B + b];
        }
        __syncthreads();
        for (int r = ty; r < 64; r += 4) {
            const int64_t b = b0 + r, e = e0 + tx;
            if (b < B && e < len) dst[b * len + e] = tile[tx][r];
        }
        __syncthreads();
    }
}

}  // namespace cfx
