// cfx_band.hip — batched banded LU with partial pivoting (LAPACK dgbtrf/dgbtrs semantics) for the
// interior-point Newton (KKT) systems on gfx950.
//
// The KKT matrix of a multiple-shooting / collocation transcription, ordered stage by stage (x_k, u_k, then
// the rows of g_k), is banded: half-bandwidths of 5-50 for the Ding families, up to ~180 for Hmed with its
// sliding-window rows, against 100-5,000 unknowns.  A dense LU per instance (O(n^3)) spends almost all of
// its time on zeros; the band LU is O(n kl (kl + ku)).  One workgroup factors one instance; each column
// step is a pivot search (argmax), a row swap, a scale and a rank-1 update of the km x (ju - j) trailing
// block, spread over the workgroup's NT threads (64 for narrow bands, 256 / 1024 for wide ones).
//
// Three placements of the band:
//  * windowed (batches >= 128, or whenever the whole band does not fit LDS): the step at column j only
//    touches columns j .. j + kl + ku, so LDS holds a circular window of kl + ku + 2 columns; column j is
//    stored to HBM with one coalesced write as it leaves and column j + kl + ku + 1 is loaded; pivots and
//    multipliers are applied to the right-hand sides on the fly; the substitutions stream the stored
//    columns back through LDS in 32-column chunks.  A few KiB per instance: tens of instances per CU.
//  * resident (small batches): the whole band (n (2 kl + ku + 1) doubles, <= 160 KiB) in LDS — no HBM
//    round trips on the latency-bound path of a single solve.
//  * global: bands too wide for either run the resident code on the HBM copy (L2-resident).
//
// Storage (per instance, instance-major): ab[b][j][r] = A(i, j) at r = kl + ku + i - j (LAPACK band
// storage, column j contiguous); rows r < kl hold the fill-in of U and are zeroed by the factorisation.
// rhs[b][c][i], ipiv[b][i] (0-based row interchanged with i), info[b] (0, or j + 1 for the first zero
// pivot, as LAPACK).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "../../include/cfx.h"

extern thread_local std::string g_create_error;

namespace cfx {

constexpr int kBandLds = 160 * 1024;
constexpr int kChunk = 32;

// A(i, j) of a band stored column by column: whole band, or a circular window of wc columns.
struct Band {
    double* a;
    int ldab, kv;
    __device__ double& operator()(int i, int j) const { return a[(int64_t)j * ldab + kv + i - j]; }
};
struct Win {
    double* w;
    int ldab, kv, wc;
    __device__ double& operator()(int i, int j) const { return w[(j % wc) * ldab + kv + i - j]; }
};

// Row offset (0 .. km) of the largest |A(j + i, j)|, first index on ties (idamax), over the NT threads.
template <int NT, class Acc>
__device__ int pivot_row(const Acc& A, int j, int km, int* s_ctl, double* s_val) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    double av = -1.0;
    int ai = 0;
    for (int i = t; i <= km; i += NT) {
        const double v = fabs(A(j + i, j));
        if (v > av) {
            av = v;
            ai = i;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(av, off);
        const int oi = __shfl_xor(ai, off);
        if (ov > av || (ov == av && oi < ai)) {
            av = ov;
            ai = oi;
        }
    }
    if constexpr (NT == 64) {
        return ai;
    } else {
        if (lane == 0) {
            s_val[wave] = av;
            s_ctl[1 + wave] = ai;
        }
        __syncthreads();
        if (t == 0) {
            double bv = s_val[0];
            int bi = s_ctl[1];
            for (int w = 1; w < NT / 64; ++w)
                if (s_val[w] > bv || (s_val[w] == bv && s_ctl[1 + w] < bi)) {
                    bv = s_val[w];
                    bi = s_ctl[1 + w];
                }
            s_ctl[0] = bi;
        }
        __syncthreads();
        return s_ctl[0];
    }
}

// One column step of the factorisation (swap, scale, rank-1 update) and, when x != nullptr, the matching
// step of the L solve on the nrhs right-hand sides x[c * n + i].  Returns false for a zero pivot.
template <int NT, class Acc>
__device__ bool column_step(const Acc& A, int j, int n, int kl, int ku, int& ju, int p, double* x, int nrhs) {
    const int t = threadIdx.x;
    const int km = min(kl, n - 1 - j);
    const double pv = A(j + p, j);
    if (pv == 0.0) return false;
    ju = max(ju, min(j + ku + p, n - 1));
    if (p != 0) {
        for (int c = j + t; c <= ju; c += NT) {
            const double s = A(j, c);
            A(j, c) = A(j + p, c);
            A(j + p, c) = s;
        }
        if (x)
            for (int c = t; c < nrhs; c += NT) {
                const double s = x[(int64_t)c * n + j];
                x[(int64_t)c * n + j] = x[(int64_t)c * n + j + p];
                x[(int64_t)c * n + j + p] = s;
            }
        __syncthreads();
    }
    const double inv = 1.0 / pv;
    for (int i = 1 + t; i <= km; i += NT) A(j + i, j) *= inv;
    __syncthreads();
    if (km > 0) {
        const int total = (ju - j) * km;
        for (int q = t; q < total; q += NT) {
            const int c = j + 1 + q / km, i = 1 + q % km;
            A(j + i, c) -= A(j + i, j) * A(j, c);
        }
        if (x)
            for (int q = t; q < km * nrhs; q += NT) {
                const int c = q / km, i = 1 + q % km;
                x[(int64_t)c * n + j + i] -= A(j + i, j) * x[(int64_t)c * n + j];
            }
    }
    return true;
}

// ---------------------------------------------------------------------------------------------------
// resident / global placement
// ---------------------------------------------------------------------------------------------------
template <bool LDS, int NT>
__global__ void __launch_bounds__(NT) k_band_lu(int n, int kl, int ku, int nrhs, double* __restrict__ AB,
                                                int32_t* __restrict__ IPIV, double* __restrict__ RHS,
                                                int32_t* __restrict__ INFO, int factor) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    __shared__ __attribute__((aligned(16))) int s_ctl[4 + NT / 64];
    __shared__ __attribute__((aligned(16))) double s_val[NT / 64 + 1];
    const int t = threadIdx.x;
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
        for (int64_t q = t; q < na; q += NT) a[q] = (factor && (q % ldab) < kl) ? 0.0 : ga[q];
        for (int64_t q = t; q < nr; q += NT) r[q] = gr[q];
        if (!factor)
            for (int q = t; q < n; q += NT) piv[q] = gp[q];
    } else if (factor) {
        for (int64_t q = t; q < na; q += NT)
            if ((q % ldab) < kl) a[q] = 0.0;
    }
    __syncthreads();
    const Band A{a, ldab, kv};

    if (factor) {
        int info = 0, ju = 0;
        for (int j = 0; j < n; ++j) {
            const int p = pivot_row<NT>(A, j, min(kl, n - 1 - j), s_ctl, s_val);
            if (t == 0) piv[j] = j + p;
            if (!column_step<NT>(A, j, n, kl, ku, ju, p, nullptr, 0) && info == 0) info = j + 1;
            __syncthreads();
        }
        if (t == 0) INFO[b] = info;
    }

    for (int c = 0; c < nrhs; ++c) {
        double* x = r + (int64_t)c * n;
        for (int j = 0; j < n - 1 && kl > 0; ++j) {  // L solve with the row interchanges
            const int km = min(kl, n - 1 - j), l = piv[j];
            if (l != j) {
                if (t == 0) {
                    const double s = x[l];
                    x[l] = x[j];
                    x[j] = s;
                }
                __syncthreads();
            }
            const double xj = x[j];
            for (int i = 1 + t; i <= km; i += NT) x[j + i] -= A(j + i, j) * xj;
            __syncthreads();
        }
        for (int j = n - 1; j >= 0; --j) {  // U solve, bandwidth kl + ku
            const double xj = x[j] / A(j, j);
            __syncthreads();
            if (t == 0) x[j] = xj;
            for (int i = max(0, j - kv) + t; i < j; i += NT) x[i] -= A(i, j) * xj;
            __syncthreads();
        }
    }

    if constexpr (LDS) {
        if (factor) {
            for (int64_t q = t; q < na; q += NT) ga[q] = a[q];
            for (int q = t; q < n; q += NT) gp[q] = piv[q];
        }
        for (int64_t q = t; q < nr; q += NT) gr[q] = r[q];
    }
}

// ---------------------------------------------------------------------------------------------------
// windowed placement
// ---------------------------------------------------------------------------------------------------
template <int NT>
__device__ inline void load_column(const double* ga, double* dst, int j, int ldab, int kl, bool zero_fill) {
    for (int r = threadIdx.x; r < ldab; r += NT) dst[r] = (zero_fill && r < kl) ? 0.0 : ga[(int64_t)j * ldab + r];
}

// Stream the stored columns [lo, hi] of one instance into LDS (contiguous in the instance-major layout).
template <int NT>
__device__ inline void load_chunk(const double* ga, double* cb, int lo, int hi, int ldab) {
    const int64_t base = (int64_t)lo * ldab, cnt = (int64_t)(hi - lo + 1) * ldab;
    for (int64_t q = threadIdx.x; q < cnt; q += NT) cb[q] = ga[base + q];
}

// Back substitution x <- U^-1 x for one right-hand side in LDS, U columns streamed from HBM.
template <int NT>
__device__ inline void back_substitute(const double* ga, double* cb, double* x, int n, int ldab, int kv, int chunk) {
    const int t = threadIdx.x;
    for (int hi = n - 1; hi >= 0; hi -= chunk) {
        const int lo = max(0, hi - chunk + 1);
        __syncthreads();
        load_chunk<NT>(ga, cb, lo, hi, ldab);
        __syncthreads();
        for (int j = hi; j >= lo; --j) {
            const double* col = cb + (int64_t)(j - lo) * ldab;  // A(i, j) at col[kv + i - j]
            const double xj = x[j] / col[kv];
            __syncthreads();
            if (t == 0) x[j] = xj;
            for (int i = max(0, j - kv) + t; i < j; i += NT) x[i] -= col[kv + i - j] * xj;
            __syncthreads();
        }
    }
}

template <int NT>
__global__ void __launch_bounds__(NT) k_band_lu_win(int n, int kl, int ku, int nrhs, double* __restrict__ AB,
                                                    int32_t* __restrict__ IPIV, double* __restrict__ RHS,
                                                    int32_t* __restrict__ INFO, int chunk) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    __shared__ __attribute__((aligned(16))) int s_ctl[4 + NT / 64];
    __shared__ __attribute__((aligned(16))) double s_val[NT / 64 + 1];
    const int t = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku, wc = kv + 2;
    double* ga = AB + b * (int64_t)n * ldab;
    int32_t* gp = IPIV + b * n;
    double* win = smem;
    double* x = win + (int64_t)wc * ldab;
    double* cb = x + (int64_t)n * nrhs;
    const Win A{win, ldab, kv, wc};
    double* gr = nrhs > 0 ? RHS + b * (int64_t)n * nrhs : nullptr;
    for (int64_t q = t; q < (int64_t)n * nrhs; q += NT) x[q] = gr[q];
    for (int c = 0; c <= min(kv, n - 1); ++c) load_column<NT>(ga, win + (c % wc) * ldab, c, ldab, kl, true);
    __syncthreads();

    int info = 0, ju = 0;
    for (int j = 0; j < n; ++j) {
        const int p = pivot_row<NT>(A, j, min(kl, n - 1 - j), s_ctl, s_val);
        if (t == 0) gp[j] = j + p;
        if (!column_step<NT>(A, j, n, kl, ku, ju, p, nrhs > 0 ? x : nullptr, nrhs) && info == 0) info = j + 1;
        __syncthreads();
        // column j is final: store it; column j + kv + 1 takes the slot column j - 1 left
        for (int r = t; r < ldab; r += NT) ga[(int64_t)j * ldab + r] = win[(j % wc) * ldab + r];
        if (j + kv + 1 < n) load_column<NT>(ga, win + ((j + kv + 1) % wc) * ldab, j + kv + 1, ldab, kl, true);
        __syncthreads();
    }
    if (t == 0) INFO[b] = info;
    if (nrhs > 0) {
        __threadfence();  // the stored columns are re-read below
        for (int c = 0; c < nrhs; ++c) back_substitute<NT>(ga, cb, x + (int64_t)c * n, n, ldab, kv, chunk);
        __syncthreads();
        for (int64_t q = t; q < (int64_t)n * nrhs; q += NT) gr[q] = x[q];
    }
}

// Solve with stored factors: forward pass (pivots + L, columns streamed in increasing order), then back.
template <int NT>
__global__ void __launch_bounds__(NT) k_band_solve_win(int n, int kl, int ku, int nrhs, const double* __restrict__ AB,
                                                       const int32_t* __restrict__ IPIV, double* __restrict__ RHS,
                                                       int chunk) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int t = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku;
    const double* ga = AB + b * (int64_t)n * ldab;
    const int32_t* gp = IPIV + b * n;
    double* x = smem;
    double* cb = x + (int64_t)n * nrhs;
    int32_t* piv = reinterpret_cast<int32_t*>(cb + (int64_t)chunk * ldab);
    double* gr = RHS + b * (int64_t)n * nrhs;
    for (int64_t q = t; q < (int64_t)n * nrhs; q += NT) x[q] = gr[q];
    for (int q = t; q < n; q += NT) piv[q] = gp[q];
    for (int lo = 0; lo < n - 1 && kl > 0; lo += chunk) {
        const int hi = min(n - 2, lo + chunk - 1);
        __syncthreads();
        load_chunk<NT>(ga, cb, lo, hi, ldab);
        __syncthreads();
        for (int j = lo; j <= hi; ++j) {
            const double* col = cb + (int64_t)(j - lo) * ldab;
            const int km = min(kl, n - 1 - j), l = piv[j];
            if (l != j) {
                for (int c = t; c < nrhs; c += NT) {
                    const double s = x[(int64_t)c * n + l];
                    x[(int64_t)c * n + l] = x[(int64_t)c * n + j];
                    x[(int64_t)c * n + j] = s;
                }
                __syncthreads();
            }
            for (int q = t; q < km * nrhs; q += NT) {
                const int c = q / km, i = 1 + q % km;
                x[(int64_t)c * n + j + i] -= col[kv + i] * x[(int64_t)c * n + j];
            }
            __syncthreads();
        }
    }
    for (int c = 0; c < nrhs; ++c) back_substitute<NT>(ga, cb, x + (int64_t)c * n, n, ldab, kv, chunk);
    __syncthreads();
    for (int64_t q = t; q < (int64_t)n * nrhs; q += NT) gr[q] = x[q];
}

// ---------------------------------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------------------------------
template <class K>
static hipError_t allow_lds(K kernel, size_t bytes) {
    if (bytes <= 65536) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes);
}

template <int NT>
static hipError_t launch_nt(int placement, int64_t n, int32_t kl, int32_t ku, int64_t batch, double* ab,
                            int32_t* ipiv, int32_t* info, int32_t nrhs, double* rhs, hipStream_t s, int factor,
                            size_t lds, int chunk) {
    hipError_t e = hipSuccess;
    if (placement == 0) {  // windowed
        if (factor) {
            if ((e = allow_lds(&k_band_lu_win<NT>, lds)) != hipSuccess) return e;
            hipLaunchKernelGGL(k_band_lu_win<NT>, dim3((unsigned)batch), dim3(NT), lds, s, (int)n, kl, ku, nrhs, ab,
                               ipiv, rhs, info, chunk);
        } else {
            if ((e = allow_lds(&k_band_solve_win<NT>, lds)) != hipSuccess) return e;
            hipLaunchKernelGGL(k_band_solve_win<NT>, dim3((unsigned)batch), dim3(NT), lds, s, (int)n, kl, ku, nrhs,
                               (const double*)ab, (const int32_t*)ipiv, rhs, chunk);
        }
    } else if (placement == 1) {  // resident
        if ((e = allow_lds(&k_band_lu<true, NT>, lds)) != hipSuccess) return e;
        hipLaunchKernelGGL((k_band_lu<true, NT>), dim3((unsigned)batch), dim3(NT), lds, s, (int)n, kl, ku, nrhs, ab,
                           ipiv, rhs, info, factor);
    } else {  // global
        hipLaunchKernelGGL((k_band_lu<false, NT>), dim3((unsigned)batch), dim3(NT), 0, s, (int)n, kl, ku, nrhs, ab,
                           ipiv, rhs, info, factor);
    }
    return hipGetLastError();
}

static int band_launch(int64_t n, int32_t kl, int32_t ku, int64_t batch, double* ab, int32_t* ipiv, int32_t* info,
                       int32_t nrhs, double* rhs, void* stream, int factor) {
    if (n < 1 || n > (1 << 24) || kl < 0 || ku < 0 || kl >= n || ku >= n || batch < 1 || batch > 0x7fffffff ||
        nrhs < 0 || !ab || !ipiv || (factor && !info) || (nrhs > 0 && !rhs)) {
        g_create_error = "cfx_band_lu: invalid argument";
        return CFX_EINVAL;
    }
    const int64_t ldab = 2 * (int64_t)kl + ku + 1;
    // substitution chunk: kChunk columns, fewer when the window and the right-hand sides leave less LDS
    const int64_t fixed_win = factor ? ((kl + ku + 2) * ldab + n * nrhs) * (int64_t)sizeof(double)
                                     : n * nrhs * (int64_t)sizeof(double) + n * (int64_t)sizeof(int32_t);
    const int chunk = (int)std::max<int64_t>(1, std::min<int64_t>(kChunk, (kBandLds - fixed_win) / (ldab * 8)));
    const size_t lds_win = (size_t)(fixed_win + (int64_t)chunk * ldab * 8);
    const size_t lds_full = (size_t)(n * ldab + n * nrhs) * sizeof(double) + (size_t)n * sizeof(int32_t);
    // placement: small batches keep the whole band resident when it fits (latency-bound); otherwise the
    // window; bands too wide for both run on the global copy.  CFX_BAND_FULL forces resident / global.
    int placement;
    const bool force_full = std::getenv("CFX_BAND_FULL") != nullptr;
    if (!force_full && !(batch < 128 && lds_full <= (size_t)kBandLds) && lds_win <= (size_t)kBandLds && chunk >= 4)
        placement = 0;
    else
        placement = lds_full <= (size_t)kBandLds ? 1 : 2;
    const size_t lds = placement == 0 ? lds_win : (placement == 1 ? lds_full : 0);
    // threads per instance: enough lanes for the rank-1 update of the trailing km x (kl + ku) block
    const int64_t work = (int64_t)kl * (kl + ku);
    const hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    if (work <= 192)
        e = launch_nt<64>(placement, n, kl, ku, batch, ab, ipiv, info, nrhs, rhs, s, factor, lds, chunk);
    else if (work <= 2048)
        e = launch_nt<256>(placement, n, kl, ku, batch, ab, ipiv, info, nrhs, rhs, s, factor, lds, chunk);
    else
        e = launch_nt<1024>(placement, n, kl, ku, batch, ab, ipiv, info, nrhs, rhs, s, factor, lds, chunk);
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
