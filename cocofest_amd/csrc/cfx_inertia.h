// cfx_inertia.h — the inertia of a small symmetric matrix in LDS, for the interior point's inertia correction.
//
// Ipopt decides its Hessian regularisation from the inertia MUMPS reports with the KKT factorisation (the number of
// negative eigenvalues must equal the number of constraints; IpPDFullSpaceSolver / IpPDPerturbationHandler).  The
// stage-chain factorisation (cfx_chain.hip) is a sequence of block eliminations, each a congruence of the symmetric
// KKT matrix, so by Sylvester's law and Haynsworth's inertia additivity the KKT matrix's inertia is the sum of the
// inertias of its pivot blocks (and of the border's Schur complement).  Each of those is counted here by a
// Bunch-Kaufman LDL^T (symmetric pivoting, 1 x 1 and 2 x 2 pivots, alpha = (1 + sqrt 17) / 8): the inertia of the
// block-diagonal factor is the matrix's.
#pragma once

#include <hip/hip_runtime.h>

namespace cfx_inertia {

// The largest of the 64 lanes' non-negative candidates v (each with its row idx), ties to the lowest row; every lane
// gets both.  Two DPP reductions (the maximum, then the lowest row holding it) instead of a shuffle butterfly of
// pairs (__shfl_xor is an LDS permute per step).  A NaN candidate never wins (as `v > best` comparisons).
#define CFX_INERTIA_DPP(x, OP, ID, CTRL, RM, BM)                                                                  \
    do {                                                                                                         \
        const int slo_ = __builtin_amdgcn_update_dpp(__double2loint(ID), __double2loint(x), CTRL, RM, BM, false);  \
        const int shi_ = __builtin_amdgcn_update_dpp(__double2hiint(ID), __double2hiint(x), CTRL, RM, BM, false);  \
        x = OP(x, __hiloint2double(shi_, slo_));                                                                  \
    } while (0)
__device__ __forceinline__ double inertia_wave_max(double x) {
    CFX_INERTIA_DPP(x, fmax, -1.0, 0x111, 0xf, 0xf);
    CFX_INERTIA_DPP(x, fmax, -1.0, 0x112, 0xf, 0xf);
    CFX_INERTIA_DPP(x, fmax, -1.0, 0x114, 0xf, 0xf);
    CFX_INERTIA_DPP(x, fmax, -1.0, 0x118, 0xf, 0xf);
    CFX_INERTIA_DPP(x, fmax, -1.0, 0x142, 0xa, 0xf);
    CFX_INERTIA_DPP(x, fmax, -1.0, 0x143, 0xc, 0xf);
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), 63), __builtin_amdgcn_readlane(__double2loint(x), 63));
}
__device__ __forceinline__ void wave_argmax(double& v, int& idx) {
    const double best = inertia_wave_max(v == v ? v : -1.0);
    double r = (v == best) ? (double)idx : 1e9;  // rows are small integers: exact in a double
    CFX_INERTIA_DPP(r, fmin, 1e9, 0x111, 0xf, 0xf);
    CFX_INERTIA_DPP(r, fmin, 1e9, 0x112, 0xf, 0xf);
    CFX_INERTIA_DPP(r, fmin, 1e9, 0x114, 0xf, 0xf);
    CFX_INERTIA_DPP(r, fmin, 1e9, 0x118, 0xf, 0xf);
    CFX_INERTIA_DPP(r, fmin, 1e9, 0x142, 0xa, 0xf);
    CFX_INERTIA_DPP(r, fmin, 1e9, 0x143, 0xc, 0xf);
    const double rr = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(r), 63), __builtin_amdgcn_readlane(__double2loint(r), 63));
    v = best;
    idx = (int)rr;
}

// Negative eigenvalues of the symmetric n x n matrix A (LDS, row stride ld, n <= 128; destroyed), by the whole
// workgroup (every thread must call it; blockDim.x a multiple of 64).  Returns the count in every thread; a zero 1 x 1
// pivot (a singular matrix) adds kZeroPivot so that no count of a singular matrix equals a valid one.
constexpr int kZeroPivot = 1 << 20;
__device__ __forceinline__ int sym_neg_count(double* A, int ld, int n) {
    __shared__ int ctl[3];  // pivot size s, pivot row, running count
    const int t = threadIdx.x, nt = blockDim.x;
    const double alpha = 0.6403882032022076;  // (1 + sqrt(17)) / 8
    if (t == 0) ctl[2] = 0;
    int k = 0;
#pragma unroll 1
    while (k < n) {
        if (t < 64) {  // pivot choice (wave 0)
            const double akk = A[k * ld + k];
            double lam = -1.0;
            int r = n;
            for (int i = k + 1 + t; i < n; i += 64) {
                const double v = fabs(A[i * ld + k]);
                if (v > lam) lam = v, r = i;
            }
            wave_argmax(lam, r);
            int s = 1, piv = k;
            if (lam > 0.0 && fabs(akk) < alpha * lam) {
                double sig = -1.0;
                int c = n;
                for (int j = k + t; j < n; j += 64) {
                    const double v = j == r ? -1.0 : fabs(A[r * ld + j]);
                    if (v > sig) sig = v, c = j;
                }
                wave_argmax(sig, c);
                if (fabs(akk) * sig >= alpha * lam * lam) {
                    s = 1, piv = k;
                } else if (fabs(A[r * ld + r]) >= alpha * sig) {
                    s = 1, piv = r;
                } else {
                    s = 2, piv = r;
                }
            }
            if (t == 0) ctl[0] = s, ctl[1] = piv;
        }
        __syncthreads();
        const int s = ctl[0], piv = ctl[1], tg = k + s - 1;  // row / column piv moves to tg
        if (piv != tg) {  // symmetric interchange: rows, then columns (of the trailing part)
            for (int j = k + t; j < n; j += nt) {
                const double a = A[tg * ld + j];
                A[tg * ld + j] = A[piv * ld + j];
                A[piv * ld + j] = a;
            }
            __syncthreads();
            for (int i = k + t; i < n; i += nt) {
                const double a = A[i * ld + tg];
                A[i * ld + tg] = A[i * ld + piv];
                A[i * ld + piv] = a;
            }
            __syncthreads();
        }
        // the trailing update: thread (ty, tx) of a 16 x 16 grid (nt = 256) takes rows k + s + ty + 16 u and columns
        // k + s + tx + 16 w, so no element index is divided (generic blocks: one element per thread and stride)
        const int k0 = k + s, m = n - k0;
        const bool grid16 = nt == 256;
        const int tx = t & 15, ty = t >> 4;
        if (s == 1) {
            const double d = A[k * ld + k];
            if (t == 0) ctl[2] += d < 0.0 ? 1 : (d == 0.0 ? kZeroPivot : 0);
            if (d != 0.0) {
                const double inv = 1.0 / d;
                if (grid16) {
                    for (int i = k0 + ty; i < n; i += 16) {
                        const double f = -A[i * ld + k] * inv;
                        for (int j = k0 + tx; j < n; j += 16) A[i * ld + j] = fma(f, A[k * ld + j], A[i * ld + j]);
                    }
                } else {
                    for (int e = t; e < m * m; e += nt) {
                        const int i = k0 + e / m, j = k0 + e % m;
                        A[i * ld + j] = fma(-A[i * ld + k] * inv, A[k * ld + j], A[i * ld + j]);
                    }
                }
            }
        } else {
            const double a = A[k * ld + k], b = A[(k + 1) * ld + k], c = A[(k + 1) * ld + k + 1];
            const double det = a * c - b * b;
            if (t == 0) ctl[2] += det < 0.0 ? 1 : (det == 0.0 ? kZeroPivot : (a + c < 0.0 ? 2 : 0));
            if (det != 0.0) {
                const double id = 1.0 / det;
                auto upd = [&](int i, int j, double w0, double w1) {
                    A[i * ld + j] -= w0 * A[k * ld + j] + w1 * A[(k + 1) * ld + j];
                };
                if (grid16) {
                    for (int i = k0 + ty; i < n; i += 16) {
                        const double li0 = A[i * ld + k], li1 = A[i * ld + k + 1];
                        const double w0 = (c * li0 - b * li1) * id, w1 = (a * li1 - b * li0) * id;  // [li0 li1] E^-1
                        for (int j = k0 + tx; j < n; j += 16) upd(i, j, w0, w1);
                    }
                } else {
                    for (int e = t; e < m * m; e += nt) {
                        const int i = k0 + e / m, j = k0 + e % m;
                        const double li0 = A[i * ld + k], li1 = A[i * ld + k + 1];
                        upd(i, j, (c * li0 - b * li1) * id, (a * li1 - b * li0) * id);
                    }
                }
            }
        }
        __syncthreads();
        k += s;
    }
    return ctl[2];
}

}  // namespace cfx_inertia
