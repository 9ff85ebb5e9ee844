// cfx_band.hip — batched banded LU with partial pivoting (LAPACK dgbtrf/dgbtrs semantics) for the
// interior-point Newton (KKT) systems on gfx950.
//
// The KKT matrix of a multiple-shooting transcription, ordered stage by stage (x_k, u_k, then the rows of
// g_k), is banded with a half-bandwidth of a few times nx + nu (Ding: 5-12, Hmed with its sliding-window
// rows: up to ~80), against 100-600 unknowns.  A dense LU per instance (O(n^3)) spends almost all of its
// time on zeros; the band LU is O(n kl (kl + ku)).  One workgroup of ONE wave factors one instance; each
// column step is a pivot search (wave argmax), a row swap, a scale and a rank-1 update spread over the 64
// lanes.  Batches of >= 128 instances use the windowed kernels below (a few KiB of LDS per instance, tens
// of instances per CU); small batches keep the whole band (n x (2 kl + ku + 1) doubles, <= 160 KiB) and
// the right-hand sides in LDS; bands too large for either run on the global-memory copy (L2-resident).
//
// Storage (per instance, instance-major): ab[b][j][r] = A(i, j) at r = kl + ku + i - j (LAPACK band
// storage, column j contiguous); rows r < kl hold the fill-in of U and are zeroed by the factorisation.
// rhs[b][c][i], ipiv[b][i] (0-based row interchanged with i), info[b] (0, or j + 1 for the first zero
// pivot, as LAPACK).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "../../include/cfx.h"

extern thread_local std::string g_create_error;

namespace cfx {

constexpr int kBandLds = 160 * 1024;

struct Band {
    double* a;
    int ldab, kv;
    __device__ double& operator()(int i, int j) const { return a[(int64_t)j * ldab + kv + i - j]; }
};

template <bool LDS>
__global__ void __launch_bounds__(64) k_band_lu(int n, int kl, int ku, int nrhs, double* __restrict__ AB,
                                                int32_t* __restrict__ IPIV, double* __restrict__ RHS,
                                                int32_t* __restrict__ INFO, int factor) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku;
    const int64_t na = (int64_t)n * ldab, nr = (int64_t)n * nrhs;
    double* ga = AB + b * na;
    double* gr = RHS ? RHS + b * nr : nullptr;
    int32_t* gp = IPIV + b * n;
    double* a = LDS ? smem : ga;
    double* r = LDS ? smem + na : gr;
    int32_t* piv = LDS ? reinterpret_cast<int32_t*>(smem + na + nr) : gp;
    if constexpr (LDS) {
        for (int64_t t = lane; t < na; t += 64) a[t] = (factor && (t % ldab) < kl) ? 0.0 : ga[t];
        for (int64_t t = lane; t < nr; t += 64) r[t] = gr[t];
        if (!factor)
            for (int t = lane; t < n; t += 64) piv[t] = gp[t];
    } else if (factor) {
        for (int64_t t = lane; t < na; t += 64)
            if ((t % ldab) < kl) a[t] = 0.0;
    }
    __syncthreads();
    const Band A{a, ldab, kv};

    if (factor) {
        int info = 0, ju = 0;
        for (int j = 0; j < n; ++j) {
            const int km = min(kl, n - 1 - j);
            double av = -1.0;
            int ai = 0;
            for (int i = lane; i <= km; i += 64) {
                const double v = fabs(A(j + i, j));
                if (v > av) {
                    av = v;
                    ai = i;
                }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {  // argmax over the wave, first index on ties (idamax)
                const double ov = __shfl_xor(av, off);
                const int oi = __shfl_xor(ai, off);
                if (ov > av || (ov == av && oi < ai)) {
                    av = ov;
                    ai = oi;
                }
            }
            const int p = ai;
            if (lane == 0) piv[j] = j + p;
            const double pv = A(j + p, j);
            if (pv != 0.0) {
                ju = max(ju, min(j + ku + p, n - 1));
                if (p != 0) {
                    for (int c = j + lane; c <= ju; c += 64) {
                        const double t = A(j, c);
                        A(j, c) = A(j + p, c);
                        A(j + p, c) = t;
                    }
                    __syncthreads();
                }
                const double inv = 1.0 / pv;
                for (int i = 1 + lane; i <= km; i += 64) A(j + i, j) *= inv;
                __syncthreads();
                if (km > 0) {
                    const int total = (ju - j) * km;
                    for (int t = lane; t < total; t += 64) {
                        const int c = j + 1 + t / km, i = 1 + t % km;
                        A(j + i, c) -= A(j + i, j) * A(j, c);
                    }
                    __syncthreads();
                }
            } else if (info == 0) {
                info = j + 1;
            }
        }
        if (lane == 0) INFO[b] = info;
    }

    for (int c = 0; c < nrhs; ++c) {
        double* x = r + (int64_t)c * n;
        for (int j = 0; j < n - 1 && kl > 0; ++j) {  // L solve with the row interchanges
            const int km = min(kl, n - 1 - j), l = piv[j];
            if (l != j) {
                if (lane == 0) {
                    const double t = x[l];
                    x[l] = x[j];
                    x[j] = t;
                }
                __syncthreads();
            }
            const double xj = x[j];
            for (int i = 1 + lane; i <= km; i += 64) x[j + i] -= A(j + i, j) * xj;
            __syncthreads();
        }
        for (int j = n - 1; j >= 0; --j) {  // U solve, bandwidth kl + ku
            const double xj = x[j] / A(j, j);
            __syncthreads();
            if (lane == 0) x[j] = xj;
            for (int i = max(0, j - kv) + lane; i < j; i += 64) x[i] -= A(i, j) * xj;
            __syncthreads();
        }
    }

    if constexpr (LDS) {
        if (factor) {
            for (int64_t t = lane; t < na; t += 64) ga[t] = a[t];
            for (int t = lane; t < n; t += 64) gp[t] = piv[t];
        }
        for (int64_t t = lane; t < nr; t += 64) gr[t] = r[t];
    }
}

// ---------------------------------------------------------------------------------------------------
// Windowed variant (the default): the factorisation at column j only touches columns j .. j + kl + ku, so
// LDS holds a circular window of kl + ku + 2 band columns instead of the whole band.  Column j + kl + ku + 1
// enters as column j leaves (written back to HBM with one coalesced store); pivots and multipliers are
// applied to the right-hand sides on the fly; back (and, for cfx_band_lu_solve, forward) substitution
// streams the stored columns through LDS in chunks of kChunk columns (one contiguous load per chunk).
// The LDS footprint is a few KiB per instance instead of n (2 kl + ku + 1) doubles, so tens of instances
// share a CU and hide each other's latency.
// ---------------------------------------------------------------------------------------------------
constexpr int kChunk = 32;

struct Win {
    double* w;
    int ldab, kv, wc;
    __device__ double& operator()(int i, int j) const { return w[(j % wc) * ldab + kv + i - j]; }
};

__device__ inline void load_column(const double* ga, double* dst, int j, int ldab, int kl, int lane, bool zero_fill) {
    for (int r = lane; r < ldab; r += 64) dst[r] = (zero_fill && r < kl) ? 0.0 : ga[(int64_t)j * ldab + r];
}

// Stream the stored columns [lo, hi] of one instance into LDS (contiguous in the instance-major layout).
__device__ inline void load_chunk(const double* ga, double* cb, int lo, int hi, int ldab, int lane) {
    const int64_t base = (int64_t)lo * ldab, cnt = (int64_t)(hi - lo + 1) * ldab;
    for (int64_t t = lane; t < cnt; t += 64) cb[t] = ga[base + t];
}

// Back substitution x <- U^-1 x for one right-hand side in LDS, U columns streamed from HBM.
__device__ inline void back_substitute(const double* ga, double* cb, double* x, int n, int ldab, int kv, int lane) {
    for (int hi = n - 1; hi >= 0; hi -= kChunk) {
        const int lo = max(0, hi - kChunk + 1);
        __syncthreads();
        load_chunk(ga, cb, lo, hi, ldab, lane);
        __syncthreads();
        for (int j = hi; j >= lo; --j) {
            const double* col = cb + (int64_t)(j - lo) * ldab;  // A(i, j) at col[kv + i - j]
            const double xj = x[j] / col[kv];
            __syncthreads();
            if (lane == 0) x[j] = xj;
            for (int i = max(0, j - kv) + lane; i < j; i += 64) x[i] -= col[kv + i - j] * xj;
            __syncthreads();
        }
    }
}

__global__ void __launch_bounds__(64) k_band_lu_win(int n, int kl, int ku, int nrhs, double* __restrict__ AB,
                                                    int32_t* __restrict__ IPIV, double* __restrict__ RHS,
                                                    int32_t* __restrict__ INFO) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku, wc = kv + 2;
    double* ga = AB + b * (int64_t)n * ldab;
    int32_t* gp = IPIV + b * n;
    double* win = smem;
    double* x = win + (int64_t)wc * ldab;
    double* cb = x + (int64_t)n * nrhs;
    const Win A{win, ldab, kv, wc};
    double* gr = nrhs > 0 ? RHS + b * (int64_t)n * nrhs : nullptr;
    for (int64_t t = lane; t < (int64_t)n * nrhs; t += 64) x[t] = gr[t];
    for (int c = 0; c <= min(kv, n - 1); ++c) load_column(ga, win + (c % wc) * ldab, c, ldab, kl, lane, true);
    __syncthreads();

    int info = 0, ju = 0;
    for (int j = 0; j < n; ++j) {
        const int km = min(kl, n - 1 - j);
        double av = -1.0;
        int ai = 0;
        for (int i = lane; i <= km; i += 64) {
            const double v = fabs(A(j + i, j));
            if (v > av) {
                av = v;
                ai = i;
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {  // argmax over the wave, first index on ties (idamax)
            const double ov = __shfl_xor(av, off);
            const int oi = __shfl_xor(ai, off);
            if (ov > av || (ov == av && oi < ai)) {
                av = ov;
                ai = oi;
            }
        }
        const int p = ai;
        if (lane == 0) gp[j] = j + p;
        const double pv = A(j + p, j);
        if (pv != 0.0) {
            ju = max(ju, min(j + ku + p, n - 1));
            if (p != 0) {
                for (int c = j + lane; c <= ju; c += 64) {
                    const double t = A(j, c);
                    A(j, c) = A(j + p, c);
                    A(j + p, c) = t;
                }
                for (int c = lane; c < nrhs; c += 64) {
                    const double t = x[(int64_t)c * n + j];
                    x[(int64_t)c * n + j] = x[(int64_t)c * n + j + p];
                    x[(int64_t)c * n + j + p] = t;
                }
            }
            __syncthreads();
            const double inv = 1.0 / pv;
            for (int i = 1 + lane; i <= km; i += 64) A(j + i, j) *= inv;
            __syncthreads();
            if (km > 0) {
                const int total = (ju - j) * km;
                for (int t = lane; t < total; t += 64) {
                    const int c = j + 1 + t / km, i = 1 + t % km;
                    A(j + i, c) -= A(j + i, j) * A(j, c);
                }
                for (int t = lane; t < km * nrhs; t += 64) {  // L solve of the right-hand sides, on the fly
                    const int c = t / km, i = 1 + t % km;
                    x[(int64_t)c * n + j + i] -= A(j + i, j) * x[(int64_t)c * n + j];
                }
            }
        } else if (info == 0) {
            info = j + 1;
        }
        __syncthreads();
        // column j is final: store it; column j + kv + 1 takes its slot's successor
        for (int r = lane; r < ldab; r += 64) ga[(int64_t)j * ldab + r] = win[(j % wc) * ldab + r];
        if (j + kv + 1 < n) load_column(ga, win + ((j + kv + 1) % wc) * ldab, j + kv + 1, ldab, kl, lane, true);
        __syncthreads();
    }
    if (lane == 0) INFO[b] = info;
    if (nrhs > 0) {
        __threadfence();  // the stored columns are re-read below
        for (int c = 0; c < nrhs; ++c) back_substitute(ga, cb, x + (int64_t)c * n, n, ldab, kv, lane);
        __syncthreads();
        for (int64_t t = lane; t < (int64_t)n * nrhs; t += 64) gr[t] = x[t];
    }
}

// Solve with stored factors: forward pass (pivots + L, columns streamed in increasing order), then back.
__global__ void __launch_bounds__(64) k_band_solve_win(int n, int kl, int ku, int nrhs, const double* __restrict__ AB,
                                                       const int32_t* __restrict__ IPIV, double* __restrict__ RHS) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku;
    const double* ga = AB + b * (int64_t)n * ldab;
    const int32_t* gp = IPIV + b * n;
    double* x = smem;
    double* cb = x + (int64_t)n * nrhs;
    int32_t* piv = reinterpret_cast<int32_t*>(cb + (int64_t)kChunk * ldab);
    double* gr = RHS + b * (int64_t)n * nrhs;
    for (int64_t t = lane; t < (int64_t)n * nrhs; t += 64) x[t] = gr[t];
    for (int t = lane; t < n; t += 64) piv[t] = gp[t];
    for (int lo = 0; lo < n - 1 && kl > 0; lo += kChunk) {
        const int hi = min(n - 2, lo + kChunk - 1);
        __syncthreads();
        load_chunk(ga, cb, lo, hi, ldab, lane);
        __syncthreads();
        for (int j = lo; j <= hi; ++j) {
            const double* col = cb + (int64_t)(j - lo) * ldab;
            const int km = min(kl, n - 1 - j), l = piv[j];
            if (l != j) {
                for (int c = lane; c < nrhs; c += 64) {
                    const double t = x[(int64_t)c * n + l];
                    x[(int64_t)c * n + l] = x[(int64_t)c * n + j];
                    x[(int64_t)c * n + j] = t;
                }
                __syncthreads();
            }
            for (int t = lane; t < km * nrhs; t += 64) {
                const int c = t / km, i = 1 + t % km;
                x[(int64_t)c * n + j + i] -= col[kv + i] * x[(int64_t)c * n + j];
            }
            __syncthreads();
        }
    }
    for (int c = 0; c < nrhs; ++c) back_substitute(ga, cb, x + (int64_t)c * n, n, ldab, kv, lane);
    __syncthreads();
    for (int64_t t = lane; t < (int64_t)n * nrhs; t += 64) gr[t] = x[t];
}

static int band_launch(int64_t n, int32_t kl, int32_t ku, int64_t batch, double* ab, int32_t* ipiv, int32_t* info,
                       int32_t nrhs, double* rhs, void* stream, int factor) {
    if (n < 1 || n > (1 << 24) || kl < 0 || ku < 0 || kl >= n || ku >= n || batch < 1 || batch > 0x7fffffff ||
        nrhs < 0 || !ab || !ipiv || (factor && !info) || (nrhs > 0 && !rhs)) {
        g_create_error = "cfx_band_lu: invalid argument";
        return CFX_EINVAL;
    }
    const int64_t ldab = 2 * (int64_t)kl + ku + 1;
    const hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    // windowed kernels when their LDS footprint is small (<= 32 KiB: >= 5 instances per CU) and the batch is
    // large enough for throughput to matter; a handful of instances is latency-bound and faster with the whole
    // band resident (no per-column HBM round trips)
    const size_t lds_win = factor ? (size_t)((kl + ku + 2) * ldab + n * nrhs + kChunk * ldab) * sizeof(double)
                                  : (size_t)(n * nrhs + kChunk * ldab) * sizeof(double) + (size_t)n * sizeof(int32_t);
    const size_t lds_full = (size_t)(n * ldab + n * nrhs) * sizeof(double) + (size_t)n * sizeof(int32_t);
    const bool small_batch = batch < 128 && lds_full <= (size_t)kBandLds;
    if (lds_win <= 32 * 1024 && !small_batch && !std::getenv("CFX_BAND_FULL")) {
        if (factor)
            hipLaunchKernelGGL(k_band_lu_win, dim3((unsigned)batch), dim3(64), lds_win, s, (int)n, kl, ku, nrhs, ab,
                               ipiv, rhs, info);
        else
            hipLaunchKernelGGL(k_band_solve_win, dim3((unsigned)batch), dim3(64), lds_win, s, (int)n, kl, ku, nrhs,
                               (const double*)ab, (const int32_t*)ipiv, rhs);
        e = hipGetLastError();
        if (e == hipSuccess) return CFX_OK;
        g_create_error = std::string("cfx_band_lu: ") + hipGetErrorString(e);
        return CFX_EHIP;
    }
    const size_t lds = lds_full;
    if (lds <= (size_t)kBandLds) {
        e = hipSuccess;
        if (lds > 65536)
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_band_lu<true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_band_lu<true>, dim3((unsigned)batch), dim3(64), lds, s, (int)n, kl, ku, nrhs, ab, ipiv,
                               rhs, info, factor);
            e = hipGetLastError();
            if (e == hipSuccess) return CFX_OK;
        }
        (void)hipGetLastError();
    }
    hipLaunchKernelGGL(k_band_lu<false>, dim3((unsigned)batch), dim3(64), 0, s, (int)n, kl, ku, nrhs, ab, ipiv, rhs,
                       info, factor);
    e = hipGetLastError();
    if (e != hipSuccess) {
        g_create_error = std::string("cfx_band_lu: ") + hipGetErrorString(e);
        return CFX_EHIP;
    }
    return CFX_OK;
}

}  // namespace cfx

extern "C" int cfx_band_lu(int64_t n, int32_t kl, int32_t ku, int64_t batch, double* ab, int32_t* ipiv, int32_t* info,
                           int32_t nrhs, double* rhs, void* stream) {
    return cfx::band_launch(n, kl, ku, batch, ab, ipiv, info, nrhs, rhs, stream, 1);
}

extern "C" int cfx_band_lu_solve(int64_t n, int32_t kl, int32_t ku, int64_t batch, const double* ab,
                                 const int32_t* ipiv, int32_t nrhs, double* rhs, void* stream) {
    if (nrhs < 1) {
        g_create_error = "cfx_band_lu_solve: nrhs < 1";
        return CFX_EINVAL;
    }
    return cfx::band_launch(n, kl, ku, batch, const_cast<double*>(ab), const_cast<int32_t*>(ipiv), nullptr, nrhs, rhs,
                            stream, 0);
}
