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
// Five placements of the band (the register and lane ones are described with their kernels below):
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
#include <map>
#include <mutex>
#include <string>
#include <type_traits>

#include "../../include/cfx.h"
#include "cfx_internal.h"

extern thread_local std::string g_create_error;

#define CFX_INLINE __attribute__((always_inline))  // lambdas over register arrays: never outlined

template <int A, int B, class F>
__device__ __forceinline__ void static_for(F&& f) {  // f(integral_constant<A>), ..., f(integral_constant<B - 1>)
    if constexpr (A < B) {
        f(std::integral_constant<int, A>{});
        static_for<A + 1, B>(f);
    }
}

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
// register placement: one wavefront per instance, the active window in VGPRs
// ---------------------------------------------------------------------------------------------------
// The step at column j touches rows j .. j + kl and columns j .. j + kv.  Lane c holds columns j + c + 64 k
// (k < KC) of that window, its rows in registers r[k][0 .. kl].  A step is: pivot search down lane 0's
// registers, a register swap in every lane (the pivot row index is wave-uniform), the multipliers
// broadcast with v_readlane and one FMA per row in every lane, the U row stored by the lanes that hold it,
// then the window slides: rows move up one register and columns one lane left (DPP wave_shl), and the next
// row of the original band, prefetched during the step, enters at the bottom.  No LDS and no barriers:
// the per-column latency of the shared-memory kernels above (LDS round trips + __syncthreads) is the whole
// cost of a single solve, and this is what removes it.  Bands with kl <= 63 and kv < 64 KC.
__device__ __forceinline__ double lane_read(double v, int l) {  // v on lane l (wave-uniform l)
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(unsigned)u, l);
    const int hi = __builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double from_next_lane(double v) {  // v on lane + 1, 0.0 on lane 63
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)u, 0x130, 0xf, 0xf, true);  // wave_shl:1
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), 0x130, 0xf, 0xf, true);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// lanes i <- i + 1 across the KC registers of a 64 KC-long vector (the last lane of register k takes the
// first lane of register k + 1)
template <int KC>
__device__ __forceinline__ void slide(double (&v)[KC]) {
    const int lane = threadIdx.x;
    static_for<0, KC>([&](auto K_) CFX_INLINE {
        constexpr int k = decltype(K_)::value;
        double s = from_next_lane(v[k]);
        if constexpr (k + 1 < KC) {
            const double head = lane_read(v[k + 1], 0);
            s = lane == 63 ? head : s;
        }
        v[k] = s;
    });
}

// Loads run D steps ahead of their use (a D-deep software pipeline, unrolled so that every prefetch keeps
// its own registers): the waitcnt before a use then only covers loads issued D steps earlier, never the
// stores of the steps in between.  Every prefetched element is one no earlier step writes.

// The window is padded to KLM = 8 NCH - 1 >= kl rows: rows j + kl + 1 .. j + KLM hold zeros in column j
// (outside the band, and no earlier step reaches them), so they are never chosen as pivots and take zero
// multipliers — the factors are exactly those of the kl-row window, and every register loop has a
// compile-time trip count (static_for: constant register indices from the front end on, so the window
// never leaves registers).  Rows past n are zeros as well.  The pivot row (a wave-uniform index) is
// swapped in by a chain of uniform branches, one taken.
// Write target of lanes with nothing to store (shared by every wave; its contents are meaningless).
// Store sinks of the register kernels (lanes with nothing to store write here, so no store sits under a branch):
// one slot per workgroup modulo kSinkSlots.  A single shared sink made every wavefront of a large batch store
// into the same few cache lines: at 4,096 instances the factorisation ran 15x slower per instance than alone.
constexpr int kSinkSlots = 2048;
constexpr int kSinkSlot = 64 * 5;  // doubles per slot: up to 3 x 64 doubles and 64 ints
__device__ double g_band_sink[kSinkSlots * kSinkSlot];
__device__ __forceinline__ double* block_sink() {
    return g_band_sink + (size_t)((blockIdx.x + (size_t)blockIdx.y * gridDim.x) % kSinkSlots) * kSinkSlot;
}


// rows 0 and p of the window (p wave-uniform): one uniform branch per row, kept apart by the volatile asm
// (neither if-converted to KLM selects per register nor merged)
template <int KLM, int KC>
__device__ __forceinline__ void swap_rows(double (&r)[KC][KLM + 1], int p) {
    static_for<1, KLM + 1>([&](auto I) CFX_INLINE {
        constexpr int i = decltype(I)::value;
        if (p == i) {
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                const double t = r[k][0];
                r[k][0] = r[k][i];
                r[k][i] = t;
            }
            asm volatile("; swap row %0" ::"i"(i));  // distinct tail per branch: the branches are neither
                                                     // if-converted nor sunk into one swap via a pointer
        }
    });
}
template <int L>
__device__ __forceinline__ int write_lane(int x, int old) {  // old with lane L replaced by the uniform x
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(old) : "s"(x), "i"(L));
    return old;
}
__device__ __forceinline__ int lo32(double v) { return (int)(unsigned)__double_as_longlong(v); }
__device__ __forceinline__ int hi32(double v) { return (int)(unsigned)((unsigned long long)__double_as_longlong(v) >> 32); }
__device__ __forceinline__ double from32(int lo, int hi) {
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// x <- U^-1 L^-1 P x for nrhs right-hand sides x[c * n + i] with the factors of k_band_lu*: forward pass
// with lane i holding x[j + i] (i <= kl), backward pass with lane i + 64 k holding x[j - i - 64 k] (<= kv).
// Same pipeline discipline as the factorisation: prefetches D steps ahead, consumed (and pinned) before the
// step's store, every lane storing (to the sink when it has nothing to store).
template <int KC, int D>
__device__ __forceinline__ void reg_solve(int n, int kl, int ku, int nrhs, const double* ab, const int32_t* piv,
                                          double* xs) {
    const int lane = threadIdx.x;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku;
    double* dsink = block_sink() + lane;
    for (int c = 0; c < nrhs; ++c) {
        double* x = xs + (int64_t)c * n;
        if (kl > 0) {
            // prefetches load unconditionally from clamped addresses and are masked at their use
            auto mult_ok = [&](int j) { return j < n && lane >= 1 && lane <= min(kl, n - 1 - j); };
            auto mult = [&](int j) { return ab[mult_ok(j) ? j * ldab + kv + lane : 0]; };  // L(j + lane, j)
            auto enter_ok = [&](int j) { return lane == kl && j + 1 + kl < n; };
            auto enter = [&](int j) { return x[enter_ok(j) ? j + 1 + kl : 0]; };
            auto pivot = [&](int j) { return piv[min(j, n - 1)]; };
            double xw = (lane <= kl && lane < n) ? x[lane] : 0.0;
            double lc[D], nx[D];
            int pj[D];
            static_for<0, D>([&](auto S_) CFX_INLINE {
                constexpr int s = decltype(S_)::value;
                lc[s] = mult(s);
                nx[s] = enter(s);
                pj[s] = pivot(s);
            });
            auto step = [&](int j, double& lcs, double& nxs, int& pjs, int jpre) CFX_INLINE {
                double lcv = mult_ok(j) ? lcs : 0.0, nxv = enter_ok(j) ? nxs : 0.0;
                int pjv = pjs;
                asm volatile("" : "+v"(lcv), "+v"(nxv), "+v"(pjv)::"memory");
                lcs = mult(jpre);
                nxs = enter(jpre);
                pjs = pivot(jpre);
                const int p = __builtin_amdgcn_readfirstlane(pjv) - j;
                if (p != 0) {
                    const double a = lane_read(xw, 0), b = lane_read(xw, p);
                    xw = lane == 0 ? b : (lane == p ? a : xw);
                }
                const double xj = lane_read(xw, 0);
                xw -= lcv * xj;
                *(lane == 0 ? x + j : dsink) = xj;
                xw = from_next_lane(xw);
                if (lane == kl) xw = nxv;
            };
            int j0 = 0;
            for (; j0 + D <= n - 1; j0 += D) {
                static_for<0, D>([&](auto S_) CFX_INLINE {
                    constexpr int s = decltype(S_)::value;
                    step(j0 + s, lc[s], nx[s], pj[s], j0 + s + D);
                });
            }
            static_for<0, D>([&](auto S_) CFX_INLINE {
                constexpr int s = decltype(S_)::value;
                if (j0 + s < n - 1) step(j0 + s, lc[s], nx[s], pj[s], n);
            });
            if (lane == 0) x[n - 1] = xw;
            __threadfence();  // the backward pass re-reads what this one stored
        }
        // U(j - i, j) on lane i = lane + 64 k <= min(kv, j) (i = 0: the diagonal)
        auto ucol_ok = [&](int j, int k) { return j >= 0 && lane + 64 * k <= min(kv, j); };
        auto ucol = [&](int j, int k) { return ab[ucol_ok(j, k) ? j * ldab + kv - lane - 64 * k : 0]; };
        auto enter_ok = [&](int j, int k) { return lane + 64 * k == kv && j - 1 - kv >= 0; };
        auto enter = [&](int j, int k) { return x[enter_ok(j, k) ? j - 1 - kv : 0]; };
        double xw[KC], uc[D][KC], nx[D][KC];
        static_for<0, KC>([&](auto K_) CFX_INLINE {
            constexpr int k = decltype(K_)::value;
            const int i = lane + 64 * k;
            xw[k] = (i <= kv && n - 1 - i >= 0) ? x[n - 1 - i] : 0.0;
#pragma unroll
            for (int s = 0; s < D; ++s) {
                uc[s][k] = ucol(n - 1 - s, k);
                nx[s][k] = enter(n - 1 - s, k);
            }
        });
        auto step = [&](int j, double (&ucs)[KC], double (&nxs)[KC], int jpre) CFX_INLINE {
            double ucv[KC], nxv[KC];
            static_for<0, KC>([&](auto K_) CFX_INLINE {
                constexpr int k = decltype(K_)::value;
                ucv[k] = ucol_ok(j, k) ? ucs[k] : 0.0;
                nxv[k] = enter_ok(j, k) ? nxs[k] : 0.0;
                asm volatile("" : "+v"(ucv[k]), "+v"(nxv[k])::"memory");
                ucs[k] = ucol(jpre, k);
                nxs[k] = enter(jpre, k);
            });
            const double xj = lane_read(xw[0], 0) / lane_read(ucv[0], 0);
            *(lane == 0 ? x + j : dsink) = xj;
            static_for<0, KC>([&](auto K_) CFX_INLINE {
                constexpr int k = decltype(K_)::value;
                xw[k] -= (k == 0 && lane == 0) ? 0.0 : ucv[k] * xj;
            });
            slide<KC>(xw);
            static_for<0, KC>([&](auto K_) CFX_INLINE {
                constexpr int k = decltype(K_)::value;
                if (lane + 64 * k == kv) xw[k] = nxv[k];
            });
        };
        int j0 = n - 1;
        for (; j0 - D + 1 >= 0; j0 -= D) {
            static_for<0, D>([&](auto S_) CFX_INLINE {
                constexpr int s = decltype(S_)::value;
                step(j0 - s, uc[s], nx[s], j0 - s - D);
            });
        }
        static_for<0, D>([&](auto S_) CFX_INLINE {
            constexpr int s = decltype(S_)::value;
            if (j0 - s >= 0) step(j0 - s, uc[s], nx[s], -1);
        });
    }
}

template <int NCH, int KC, int D>
__global__ void __launch_bounds__(64) k_band_lu_reg(int n, int kl, int ku, int nrhs, double* __restrict__ AB,
                                                    int32_t* __restrict__ IPIV, double* __restrict__ RHS,
                                                    int32_t* __restrict__ INFO) {
    constexpr int KLM = 8 * NCH - 1;
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku;  // n * ldab < 2^31 (checked at dispatch)
    double* ab = AB + b * (int64_t)n * ldab;
    int32_t* piv = IPIV + b * n;
    // lane constants: U(j, j + c) is ab[j ldab + cofs]; the entering row's element is ab[(j + 1) ldab + cofs
    // + KLM], inside the band for KLM - kl <= c <= KLM + ku
    int cofs[KC];
    bool uok[KC], eok[KC];
    static_for<0, KC>([&](auto K_) CFX_INLINE {
        constexpr int k = decltype(K_)::value;
        const int c = lane + 64 * k;
        cofs[k] = c * (ldab - 1) + kv;
        uok[k] = c <= kv;
        eok[k] = c >= KLM - kl && c <= KLM + ku;
    });
    auto entering_ok = [&](int j, int k) { return eok[k] && j + 1 + KLM < n && j + 1 + lane + 64 * k < n; };
    // prefetches load unconditionally (element 0 stands in outside the band) and are masked at their use
    auto fetch = [&](int j, int k) { return ab[entering_ok(j, k) ? (j + 1) * ldab + cofs[k] + KLM : 0]; };
    // every lane stores every step (lanes with nothing to store write the sink): no store sits under a
    // branch, so the compiler's vmcnt waits for a prefetch count the stores issued after it exactly
    double* const sinkb = block_sink();
    double* dsink = sinkb + lane;
    int32_t* isink = reinterpret_cast<int32_t*>(sinkb + 64 * (KC + 1)) + lane;

    double r[KC][KLM + 1];  // r[k][i]: row j + i of the window, column j + lane + 64 k
    static_for<0, KC>([&](auto K_) CFX_INLINE {
        constexpr int k = decltype(K_)::value;
        const int c = lane + 64 * k;
        static_for<0, KLM + 1>([&](auto I) CFX_INLINE {
            constexpr int i = decltype(I)::value;
            r[k][i] = (i < n && c < n && i - c <= kl && c - i <= ku) ? ab[c * ldab + kv + i - c] : 0.0;
        });
        // fill-in positions above the matrix, which no U row reaches (LAPACK zeroes them too)
        if (c < min(kv, n))
            for (int q = 0; q < min(kl, kv - c); ++q) ab[c * ldab + q] = 0.0;
    });
    double nxt[D][KC];  // row j + 1 + KLM enters the window after step j; fetched D steps ahead
    static_for<0, D>([&](auto S_) CFX_INLINE {
        constexpr int s = decltype(S_)::value;
        static_for<0, KC>([&](auto K_) CFX_INLINE { nxt[s][decltype(K_)::value] = fetch(s, decltype(K_)::value); });
    });
    int info = 0;

    auto step = [&](int j, double (&pre)[KC], int jpre) CFX_INLINE {
        // take the row that enters after this step and refill its slot (row of step jpre) before this
        // step's stores, so that the wait for a prefetch never covers stores just issued
        double ent[KC];
        static_for<0, KC>([&](auto K_) CFX_INLINE {
            constexpr int k = decltype(K_)::value;
            ent[k] = entering_ok(j, k) ? pre[k] : 0.0;
            asm volatile("" : "+v"(ent[k])::"memory");  // pinned here: not sunk past the stores below
            pre[k] = fetch(jpre, k);
        });
        // pivot: first largest |A(j + i, j)| on lane 0 (column j is its first register)
        double best = fabs(r[0][0]);
        int p = 0;
        static_for<1, KLM + 1>([&](auto I) CFX_INLINE {
            constexpr int i = decltype(I)::value;
            const double a = fabs(r[0][i]);
            p = a > best ? i : p;
            best = fmax(best, a);
        });
        p = __builtin_amdgcn_readfirstlane(p);
        *(lane == 0 ? piv + j : isink) = j + p;
        // u: the pivot row (row j of U); row p takes row j
        swap_rows<KLM, KC>(r, p);
        double u[KC];
        static_for<0, KC>([&](auto K_) CFX_INLINE {
            constexpr int k = decltype(K_)::value;
            u[k] = r[k][0];
            *(uok[k] && j + lane + 64 * k < n ? ab + j * ldab + cofs[k] : dsink + 64 * k) = u[k];
        });
        const double pivot = lane_read(u[0], 0);
        // multipliers (all zero for a zero pivot, whose column is zero: the stored column is unchanged)
        const double inv = pivot != 0.0 ? 1.0 / pivot : 0.0;
        if (pivot == 0.0 && info == 0) info = j + 1;
        int llo = 0, lhi = 0;  // lane i gathers L(j + i, j)
        static_for<1, KLM + 1>([&](auto I) CFX_INLINE {
            constexpr int i = decltype(I)::value;
            const double t = r[0][i] * inv;  // lane 0's value is L(j + i, j)
            const int tlo = __builtin_amdgcn_readlane(lo32(t), 0), thi = __builtin_amdgcn_readlane(hi32(t), 0);
            llo = write_lane<i>(tlo, llo);
            lhi = write_lane<i>(thi, lhi);
            const double l = from32(tlo, thi);
            static_for<0, KC>([&](auto K_) CFX_INLINE {
                constexpr int k = decltype(K_)::value;
                r[k][i] -= l * u[k];
            });
        });
        *(lane >= 1 && lane <= min(kl, n - 1 - j) ? ab + j * ldab + kv + lane : dsink + 64 * KC) = from32(llo, lhi);
        // slide the window down-right by one; the prefetched row enters at the bottom
        static_for<0, KLM>([&](auto I) CFX_INLINE {
            constexpr int i = decltype(I)::value;
            double row[KC];
            static_for<0, KC>([&](auto K_) CFX_INLINE {
                constexpr int k = decltype(K_)::value;
                row[k] = r[k][i + 1];
            });
            slide<KC>(row);
            static_for<0, KC>([&](auto K_) CFX_INLINE {
                constexpr int k = decltype(K_)::value;
                r[k][i] = row[k];
            });
        });
        static_for<0, KC>([&](auto K_) CFX_INLINE {
            constexpr int k = decltype(K_)::value;
            r[k][KLM] = ent[k];
        });
    };
    int j0 = 0;
    for (; j0 + D <= n; j0 += D) {
        static_for<0, D>([&](auto S_) CFX_INLINE {
            constexpr int s = decltype(S_)::value;
            step(j0 + s, nxt[s], j0 + s + D);
        });
    }
    static_for<0, D>([&](auto S_) CFX_INLINE {  // the last steps prefetch nothing (their rows are past n)
        constexpr int s = decltype(S_)::value;
        if (j0 + s < n) step(j0 + s, nxt[s], n);
    });
    if (lane == 0) INFO[b] = info;
    if (nrhs > 0) {
        __threadfence();  // the solve reads the factors stored above
        reg_solve<KC, D>(n, kl, ku, nrhs, ab, piv, RHS + b * (int64_t)n * nrhs);
    }
}

template <int KC, int D>
__global__ void __launch_bounds__(64) k_band_solve_reg(int n, int kl, int ku, int nrhs, const double* __restrict__ AB,
                                                       const int32_t* __restrict__ IPIV, double* __restrict__ RHS) {
    const int64_t b = blockIdx.x;
    reg_solve<KC, D>(n, kl, ku, nrhs, AB + b * (int64_t)n * (2 * kl + ku + 1), IPIV + b * n,
                     RHS + b * (int64_t)n * nrhs);
}

// Right-hand sides solved in parallel, one wavefront each (grid (batch, nx + (Y ? 1 : 0))).  The batch index
// bb = b parts + q addresses system q of instance b (factors at bb); its column c < nx is at X + b x_inst +
// q x_part + c x_rhs, the extra one at Y + b y_inst + q y_part.  For the bordered / dissected KKT solves of the
// interior point (cfx_ipm.hip), where the border's columns are as many right-hand sides.
template <int KC, int D>
__global__ void __launch_bounds__(64) k_band_solve_reg_multi(int n, int kl, int ku, const double* __restrict__ AB,
                                                             const int32_t* __restrict__ IPIV, int parts, double* X,
                                                             int64_t x_inst, int64_t x_part, int64_t x_rhs, int nx,
                                                             double* Y, int64_t y_inst, int64_t y_part) {
    const int64_t bb = blockIdx.x;
    const int64_t b = bb / parts, q = bb - (bb / parts) * parts;
    const int c = blockIdx.y;
    double* xs = c < nx ? X + b * x_inst + q * x_part + (int64_t)c * x_rhs : Y + b * y_inst + q * y_part;
    reg_solve<KC, D>(n, kl, ku, 1, AB + bb * (int64_t)n * (2 * kl + ku + 1), IPIV + bb * n, xs);
}

// ---------------------------------------------------------------------------------------------------
// grouped register placement: four instances per wavefront, 16 lanes each (narrow bands, large batches)
// ---------------------------------------------------------------------------------------------------
// The register kernel above gives each instance a whole wavefront, but a band with kl <= 7 and ku <= 8 keeps
// only the 8 + ku <= 16 lanes of its window busy: for the cfg-2 / cfg-3 KKT bands (kl = ku = 5..6) 50 of the 64
// lanes idle, and once the batch fills the chip the waves queue for the SIMDs.  Here a 16-lane row of the wave
// owns one instance (instance 4 blockIdx + lane / 16) and runs the same column step on its window, with the
// cross-lane operations kept inside the row: the group's lane 0 is broadcast with DPP row_newbcast:0, the window
// slides with DPP row_shl:1 (lane 15 of each row takes 0, as lane 63 does above), the pivot row (now different in
// each group) is swapped in by selects, and the multipliers are gathered into lanes 1 .. kl by selects.  Same
// storage, pivots, zero-pivot convention and D-step prefetch discipline as the one-instance kernel.
__device__ __forceinline__ int g16_first_i(int v) { return __builtin_amdgcn_mov_dpp(v, 0x150, 0xf, 0xf, false); }
__device__ __forceinline__ double g16_first(double v) {  // the group's lane 0 value (row_newbcast:0)
    return from32(g16_first_i(lo32(v)), g16_first_i(hi32(v)));
}
__device__ __forceinline__ double g16_next(double v) {  // v on group lane + 1, 0.0 on group lane 15 (row_shl:1)
    return from32(__builtin_amdgcn_mov_dpp(lo32(v), 0x101, 0xf, 0xf, true),
                  __builtin_amdgcn_mov_dpp(hi32(v), 0x101, 0xf, 0xf, true));
}
__device__ __forceinline__ double g16_read(double v, int src) {  // v on lane src (any lane; ds_bpermute)
    return from32(__builtin_amdgcn_ds_bpermute(src << 2, lo32(v)), __builtin_amdgcn_ds_bpermute(src << 2, hi32(v)));
}
constexpr int kG16Klm = 7;  // window rows (kl <= 7); columns 8 + ku <= 16

// x <- U^-1 L^-1 P x for nrhs right-hand sides, one instance per 16-lane group (factors of k_band_lu_reg16 or of
// any placement: same storage)
template <int D>
__device__ __forceinline__ void reg16_solve(int n, int kl, int ku, int nrhs, const double* ab, const int32_t* piv,
                                            double* xs, bool valid) {
    const int gl = threadIdx.x & 15, base = threadIdx.x & 48;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku;
    double* dsink = block_sink() + threadIdx.x;
    for (int c = 0; c < nrhs; ++c) {
        double* x = xs + (int64_t)c * n;
        if (kl > 0) {
            auto mult_ok = [&](int j) { return j < n && gl >= 1 && gl <= min(kl, n - 1 - j); };
            auto mult = [&](int j) { return ab[mult_ok(j) ? j * ldab + kv + gl : 0]; };
            auto enter_ok = [&](int j) { return gl == kl && j + 1 + kl < n; };
            auto enter = [&](int j) { return x[enter_ok(j) ? j + 1 + kl : 0]; };
            auto pivot = [&](int j) { return piv[min(j, n - 1)]; };
            double xw = (gl <= kl && gl < n) ? x[gl] : 0.0;
            double lc[D], nx[D];
            int pj[D];
            static_for<0, D>([&](auto S_) CFX_INLINE {
                constexpr int s = decltype(S_)::value;
                lc[s] = mult(s);
                nx[s] = enter(s);
                pj[s] = pivot(s);
            });
            auto step = [&](int j, double& lcs, double& nxs, int& pjs, int jpre) CFX_INLINE {
                double lcv = mult_ok(j) ? lcs : 0.0, nxv = enter_ok(j) ? nxs : 0.0;
                int pjv = pjs;
                asm volatile("" : "+v"(lcv), "+v"(nxv), "+v"(pjv)::"memory");
                lcs = mult(jpre);
                nxs = enter(jpre);
                pjs = pivot(jpre);
                const int p = pjv - j;  // the same in the group's lanes
                const double a = g16_first(xw), bq = g16_read(xw, base + p);
                xw = gl == 0 ? bq : (gl == p ? a : xw);
                const double xj = g16_first(xw);
                xw -= lcv * xj;
                *(valid && gl == 0 ? x + j : dsink) = xj;
                xw = g16_next(xw);
                if (gl == kl) xw = nxv;
            };
            int j0 = 0;
            for (; j0 + D <= n - 1; j0 += D) {
                static_for<0, D>([&](auto S_) CFX_INLINE {
                    constexpr int s = decltype(S_)::value;
                    step(j0 + s, lc[s], nx[s], pj[s], j0 + s + D);
                });
            }
            static_for<0, D>([&](auto S_) CFX_INLINE {
                constexpr int s = decltype(S_)::value;
                if (j0 + s < n - 1) step(j0 + s, lc[s], nx[s], pj[s], n);
            });
            if (valid && gl == 0) x[n - 1] = xw;
            __threadfence();  // the backward pass re-reads what this one stored
        }
        auto ucol_ok = [&](int j) { return j >= 0 && gl <= min(kv, j); };
        auto ucol = [&](int j) { return ab[ucol_ok(j) ? j * ldab + kv - gl : 0]; };
        auto enter_ok = [&](int j) { return gl == kv && j - 1 - kv >= 0; };
        auto enter = [&](int j) { return x[enter_ok(j) ? j - 1 - kv : 0]; };
        double xw = (gl <= kv && n - 1 - gl >= 0) ? x[n - 1 - gl] : 0.0;
        double uc[D], nx[D];
        static_for<0, D>([&](auto S_) CFX_INLINE {
            constexpr int s = decltype(S_)::value;
            uc[s] = ucol(n - 1 - s);
            nx[s] = enter(n - 1 - s);
        });
        auto step = [&](int j, double& ucs, double& nxs, int jpre) CFX_INLINE {
            double ucv = ucol_ok(j) ? ucs : 0.0, nxv = enter_ok(j) ? nxs : 0.0;
            asm volatile("" : "+v"(ucv), "+v"(nxv)::"memory");
            ucs = ucol(jpre);
            nxs = enter(jpre);
            const double xj = g16_first(xw) / g16_first(ucv);
            *(valid && gl == 0 ? x + j : dsink) = xj;
            xw -= gl == 0 ? 0.0 : ucv * xj;
            xw = g16_next(xw);
            if (gl == kv) xw = nxv;
        };
        int j0 = n - 1;
        for (; j0 - D + 1 >= 0; j0 -= D) {
            static_for<0, D>([&](auto S_) CFX_INLINE {
                constexpr int s = decltype(S_)::value;
                step(j0 - s, uc[s], nx[s], j0 - s - D);
            });
        }
        static_for<0, D>([&](auto S_) CFX_INLINE {
            constexpr int s = decltype(S_)::value;
            if (j0 - s >= 0) step(j0 - s, uc[s], nx[s], -1);
        });
    }
}

template <int D>
__global__ void __launch_bounds__(64) k_band_lu_reg16(int64_t batch, int n, int kl, int ku, int nrhs,
                                                      double* __restrict__ AB, int32_t* __restrict__ IPIV,
                                                      double* __restrict__ RHS, int32_t* __restrict__ INFO) {
    constexpr int KLM = kG16Klm;
    const int gl = threadIdx.x & 15;
    const int64_t b0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 4);
    const bool valid = b0 < batch;
    const int64_t b = valid ? b0 : batch - 1;  // the spare groups of the last wave read a valid instance
    const int ldab = 2 * kl + ku + 1, kv = kl + ku;
    double* ab = AB + b * (int64_t)n * ldab;
    int32_t* piv = IPIV + b * n;
    const int cofs = gl * (ldab - 1) + kv;  // U(j, j + gl) at ab[j ldab + cofs]
    const bool uok = gl <= kv;
    const bool eok = gl >= KLM - kl && gl <= KLM + ku;
    auto entering_ok = [&](int j) { return eok && j + 1 + KLM < n && j + 1 + gl < n; };
    auto fetch = [&](int j) { return ab[entering_ok(j) ? (j + 1) * ldab + cofs + KLM : 0]; };
    double* const sinkb = block_sink();
    double* dsink = sinkb + threadIdx.x;
    int32_t* isink = reinterpret_cast<int32_t*>(sinkb + 64 * 2) + threadIdx.x;

    double r[KLM + 1];  // r[i]: row j + i of the window, column j + gl
    static_for<0, KLM + 1>([&](auto I) CFX_INLINE {
        constexpr int i = decltype(I)::value;
        r[i] = (i < n && gl < n && i - gl <= kl && gl - i <= ku) ? ab[gl * ldab + kv + i - gl] : 0.0;
    });
    if (valid && gl < min(kv, n))
        for (int q = 0; q < min(kl, kv - gl); ++q) ab[gl * ldab + q] = 0.0;
    double nxt[D];
    static_for<0, D>([&](auto S_) CFX_INLINE { nxt[decltype(S_)::value] = fetch(decltype(S_)::value); });
    int info = 0;

    auto step = [&](int j, double& pre, int jpre) CFX_INLINE {
        double ent = entering_ok(j) ? pre : 0.0;
        asm volatile("" : "+v"(ent)::"memory");
        pre = fetch(jpre);
        // pivot: first largest |A(j + i, j)| on the group's lane 0 (column j)
        double best = fabs(r[0]);
        int p = 0;
        static_for<1, KLM + 1>([&](auto I) CFX_INLINE {
            constexpr int i = decltype(I)::value;
            const double a = fabs(r[i]);
            p = a > best ? i : p;
            best = fmax(best, a);
        });
        p = g16_first_i(p);
        *(valid && gl == 0 ? piv + j : isink) = j + p;
        static_for<1, KLM + 1>([&](auto I) CFX_INLINE {  // rows 0 and p (group-uniform p) by selects
            constexpr int i = decltype(I)::value;
            const bool sw = p == i;
            const double t = r[0];
            r[0] = sw ? r[i] : r[0];
            r[i] = sw ? t : r[i];
        });
        const double u = r[0];
        *(valid && uok && j + gl < n ? ab + j * ldab + cofs : dsink) = u;
        const double pv = g16_first(u);
        const double inv = pv != 0.0 ? 1.0 / pv : 0.0;
        if (pv == 0.0 && info == 0) info = j + 1;
        double lg = 0.0;  // group lane i gathers L(j + i, j)
        static_for<1, KLM + 1>([&](auto I) CFX_INLINE {
            constexpr int i = decltype(I)::value;
            const double l = g16_first(r[i] * inv);
            lg = gl == i ? l : lg;
            r[i] -= l * u;
        });
        *(valid && gl >= 1 && gl <= min(kl, n - 1 - j) ? ab + j * ldab + kv + gl : dsink + 64) = lg;
        static_for<0, KLM>([&](auto I) CFX_INLINE {
            constexpr int i = decltype(I)::value;
            r[i] = g16_next(r[i + 1]);
        });
        r[KLM] = ent;
    };
    int j0 = 0;
    for (; j0 + D <= n; j0 += D) {
        static_for<0, D>([&](auto S_) CFX_INLINE {
            constexpr int s = decltype(S_)::value;
            step(j0 + s, nxt[s], j0 + s + D);
        });
    }
    static_for<0, D>([&](auto S_) CFX_INLINE {
        constexpr int s = decltype(S_)::value;
        if (j0 + s < n) step(j0 + s, nxt[s], n);
    });
    if (valid && gl == 0) INFO[b] = info;
    if (nrhs > 0) {
        __threadfence();  // the solve reads the factors stored above
        reg16_solve<D>(n, kl, ku, nrhs, ab, piv, RHS + b * (int64_t)n * nrhs, valid);
    }
}

template <int D>
__global__ void __launch_bounds__(64) k_band_solve_reg16(int64_t batch, int n, int kl, int ku, int nrhs,
                                                         const double* __restrict__ AB,
                                                         const int32_t* __restrict__ IPIV, double* __restrict__ RHS) {
    const int64_t b0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 4);
    const bool valid = b0 < batch;
    const int64_t b = valid ? b0 : batch - 1;
    reg16_solve<D>(n, kl, ku, nrhs, AB + b * (int64_t)n * (2 * kl + ku + 1), IPIV + b * n,
                   RHS + b * (int64_t)n * nrhs, valid);
}

// ---------------------------------------------------------------------------------------------------
// lane placement: one lane per instance (large batches of narrow bands)
// ---------------------------------------------------------------------------------------------------
// Once the batch alone fills the chip, a wavefront per instance spends every column step on cross-lane
// operations for one instance while thousands of such waves queue for the CUs.  Here a lane owns an instance
// and runs dgbtf2's column loop on its own register window — rows j .. j + K, columns j .. j + 2K, K = max(kl,
// ku) <= 8 a compile-time bound — so a step is plain FP64 arithmetic: the pivot row (lane-varying) is exchanged
// by selects, the window slides by register moves, and the next row of the band enters from a D-step-deep
// prefetch.  Same storage, pivots and zero-pivot convention as the other placements (the factors are
// interchangeable).  Every lane stores every step (to its sink slot when it has nothing to store), so no store
// sits under a branch and the waits for the prefetches count exactly.
constexpr int kLaneD = 2;  // prefetch depth (steps)

// Element strides: band entry e (LAPACK column-major index within the instance) at ab[e ae], pivot j at
// piv[j pe], right-hand-side entry i at x[i xe] — 1 for the caller's instance-major arrays, the batch for the
// instance-minor copies of the coalesced path.
template <int K>
__device__ __forceinline__ void lane_solve(int n, int kl, int ku, const double* ab, int64_t ae, const int32_t* piv,
                                           int64_t pe, double* x, int64_t xe) {
    constexpr int KV = 2 * K, D = kLaneD;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku;
    if (kl > 0) {  // x <- L^-1 P x: the window holds x[j .. j + K]
        auto lok = [&](int j, int i) { return i <= kl && j + i < n; };
        auto lget = [&](int j, int i) { return ab[(lok(j, i) ? (int64_t)j * ldab + kv + i : 0) * ae]; };
        auto eok = [&](int j) { return j + 1 + K < n; };
        auto eget = [&](int j) { return x[(eok(j) ? j + 1 + K : 0) * xe]; };
        double xw[K + 1];
        static_for<0, K + 1>([&](auto I) CFX_INLINE {
            constexpr int i = decltype(I)::value;
            xw[i] = i < n ? x[i * xe] : 0.0;
        });
        double lp[D][K + 1], ep[D];
        int pp[D];
        static_for<0, D>([&](auto S_) CFX_INLINE {
            constexpr int s = decltype(S_)::value;
            static_for<1, K + 1>([&](auto I) CFX_INLINE { lp[s][decltype(I)::value] = lget(s, decltype(I)::value); });
            ep[s] = eget(s);
            pp[s] = piv[min(s, n - 1) * pe];
        });
        auto step = [&](int j, double (&lps)[K + 1], double& eps, int& pps, int jpre) CFX_INLINE {
            double lv[K + 1], ev = eok(j) ? eps : 0.0;
            int p = pps - j;
            static_for<1, K + 1>([&](auto I) CFX_INLINE {
                constexpr int i = decltype(I)::value;
                lv[i] = lok(j, i) ? lps[i] : 0.0;
                asm volatile("" : "+v"(lv[i])::"memory");
                lps[i] = lget(jpre, i);
            });
            asm volatile("" : "+v"(ev), "+v"(p)::"memory");
            eps = eget(jpre);
            pps = piv[min(jpre, n - 1) * pe];
            double x0 = xw[0];
            static_for<1, K + 1>([&](auto I) CFX_INLINE {
                constexpr int i = decltype(I)::value;
                const double t = xw[i];
                xw[i] = p == i ? xw[0] : t;
                x0 = p == i ? t : x0;
            });
            x[j * xe] = x0;
            static_for<1, K + 1>([&](auto I) CFX_INLINE {
                constexpr int i = decltype(I)::value;
                xw[i - 1] = xw[i] - lv[i] * x0;
            });
            xw[K] = ev;
        };
        int j0 = 0;
        for (; j0 + D <= n - 1; j0 += D)
            static_for<0, D>([&](auto S_) CFX_INLINE {
                constexpr int s = decltype(S_)::value;
                step(j0 + s, lp[s], ep[s], pp[s], j0 + s + D);
            });
        static_for<0, D>([&](auto S_) CFX_INLINE {
            constexpr int s = decltype(S_)::value;
            if (j0 + s < n - 1) step(j0 + s, lp[s], ep[s], pp[s], n);
        });
        x[(n - 1) * xe] = xw[0];
        __threadfence();  // the backward pass re-reads what this one stored
    }
    // x <- U^-1 x: the window holds x[j - KV .. j] reversed (xw[t] = x[j - t])
    auto uok = [&](int j, int t) { return j >= 0 && t <= kv && j - t >= 0; };
    auto uget = [&](int j, int t) { return ab[(uok(j, t) ? (int64_t)j * ldab + kv - t : 0) * ae]; };
    auto eok = [&](int j) { return j - 1 - KV >= 0; };
    auto eget = [&](int j) { return x[(eok(j) ? j - 1 - KV : 0) * xe]; };
    double xw[KV + 1];
    static_for<0, KV + 1>([&](auto T) CFX_INLINE {
        constexpr int t = decltype(T)::value;
        xw[t] = n - 1 - t >= 0 ? x[(n - 1 - t) * xe] : 0.0;
    });
    double up[D][KV + 1], ep[D];
    static_for<0, D>([&](auto S_) CFX_INLINE {
        constexpr int s = decltype(S_)::value;
        static_for<0, KV + 1>([&](auto T) CFX_INLINE { up[s][decltype(T)::value] = uget(n - 1 - s, decltype(T)::value); });
        ep[s] = eget(n - 1 - s);
    });
    auto step = [&](int j, double (&ups)[KV + 1], double& eps, int jpre) CFX_INLINE {
        double uv[KV + 1], ev = eok(j) ? eps : 0.0;
        static_for<0, KV + 1>([&](auto T) CFX_INLINE {
            constexpr int t = decltype(T)::value;
            uv[t] = uok(j, t) ? ups[t] : 0.0;
            asm volatile("" : "+v"(uv[t])::"memory");
            ups[t] = uget(jpre, t);
        });
        asm volatile("" : "+v"(ev)::"memory");
        eps = eget(jpre);
        const double xj = xw[0] / uv[0];
        x[j * xe] = xj;
        static_for<1, KV + 1>([&](auto T) CFX_INLINE {
            constexpr int t = decltype(T)::value;
            xw[t - 1] = xw[t] - uv[t] * xj;
        });
        xw[KV] = ev;
    };
    int j0 = n - 1;
    for (; j0 - D + 1 >= 0; j0 -= D)
        static_for<0, D>([&](auto S_) CFX_INLINE {
            constexpr int s = decltype(S_)::value;
            step(j0 - s, up[s], ep[s], j0 - s - D);
        });
    static_for<0, D>([&](auto S_) CFX_INLINE {
        constexpr int s = decltype(S_)::value;
        if (j0 - s >= 0) step(j0 - s, up[s], ep[s], -1);
    });
}

// instance b's arrays start at b * *_inst; element strides as lane_solve (x_rhs: between right-hand sides)
struct LaneLayout {
    int64_t ab_inst, ab_el, pv_inst, pv_el, x_inst, x_el, x_rhs;
};

template <int K>
__global__ void __launch_bounds__(64) k_band_lu_lane(int64_t batch, int n, int kl, int ku, int nrhs,
                                                     double* __restrict__ AB, int32_t* __restrict__ IPIV,
                                                     double* __restrict__ RHS, int32_t* __restrict__ INFO,
                                                     LaneLayout L) {
    constexpr int KW = 2 * K + 1, D = kLaneD;
    const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (b >= batch) return;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku;  // n * ldab < 2^31 (checked at dispatch)
    const int64_t ae = L.ab_el, pe = L.pv_el;
    double* ab = AB + b * L.ab_inst;
    int32_t* piv = IPIV + b * L.pv_inst;
    double* const sink = block_sink() + threadIdx.x;  // stores with nothing to store land here
    int32_t* const isink = reinterpret_cast<int32_t*>(block_sink() + 64 * 4) + threadIdx.x;
    // A(i, c) of the original band: i - c <= kl, c - i <= ku, inside the matrix
    auto bok = [&](int i, int c) { return i < n && c < n && i - c <= kl && c - i <= ku; };
    auto bget = [&](int i, int c) { return ab[(bok(i, c) ? (int64_t)c * ldab + kv + i - c : 0) * ae]; };
    double W[K + 1][KW];  // W[i][c] = A(j + i, j + c) of the current step
    static_for<0, K + 1>([&](auto I) CFX_INLINE {
        constexpr int i = decltype(I)::value;
        static_for<0, KW>([&](auto C_) CFX_INLINE {
            constexpr int c = decltype(C_)::value;
            W[i][c] = bok(i, c) ? bget(i, c) : 0.0;
        });
    });
    for (int c = 0; c < min(kv, n); ++c)  // fill-in positions above the matrix, which no U row reaches
        for (int q = 0; q < min(kl, kv - c); ++q) ab[((int64_t)c * ldab + q) * ae] = 0.0;
    double nxt[D][KW];  // row j + 1 + K (columns j + 1 ..) enters after step j; fetched D steps ahead
    static_for<0, D>([&](auto S_) CFX_INLINE {
        constexpr int s = decltype(S_)::value;
        static_for<0, KW>([&](auto C_) CFX_INLINE {
            constexpr int c = decltype(C_)::value;
            nxt[s][c] = bget(s + 1 + K, s + 1 + c);
        });
    });
    int info = 0;
    auto step = [&](int j, double (&pre)[KW], int jpre) CFX_INLINE {
        double ent[KW];
        static_for<0, KW>([&](auto C_) CFX_INLINE {
            constexpr int c = decltype(C_)::value;
            ent[c] = bok(j + 1 + K, j + 1 + c) ? pre[c] : 0.0;
            asm volatile("" : "+v"(ent[c])::"memory");  // taken before this step's stores
            pre[c] = bget(jpre + 1 + K, jpre + 1 + c);
        });
        // pivot: first largest |A(j + i, j)|
        double best = fabs(W[0][0]);
        int p = 0;
        static_for<1, K + 1>([&](auto I) CFX_INLINE {
            constexpr int i = decltype(I)::value;
            const double a = fabs(W[i][0]);
            p = a > best ? i : p;
            best = fmax(best, a);
        });
        *(j < n ? piv + j * pe : isink) = j + p;
        // U: row p; row p takes row 0
        double U[KW];
        static_for<0, KW>([&](auto C_) CFX_INLINE { U[decltype(C_)::value] = W[0][decltype(C_)::value]; });
        static_for<1, K + 1>([&](auto I) CFX_INLINE {
            constexpr int i = decltype(I)::value;
            static_for<0, KW>([&](auto C_) CFX_INLINE {
                constexpr int c = decltype(C_)::value;
                const double t = W[i][c];
                W[i][c] = p == i ? W[0][c] : t;
                U[c] = p == i ? t : U[c];
            });
        });
        static_for<0, KW>([&](auto C_) CFX_INLINE {  // U(j, j + c) at band row kv - c of column j + c
            constexpr int c = decltype(C_)::value;
            *(c <= kv && j + c < n ? ab + ((int64_t)(j + c) * ldab + kv - c) * ae : sink) = U[c];
        });
        const double inv = U[0] != 0.0 ? 1.0 / U[0] : 0.0;  // zero pivot: zero column, zero multipliers
        if (U[0] == 0.0 && info == 0) info = j + 1;
        static_for<1, K + 1>([&](auto I) CFX_INLINE {
            constexpr int i = decltype(I)::value;
            const double l = W[i][0] * inv;
            *(i <= kl && j + i < n ? ab + ((int64_t)j * ldab + kv + i) * ae : sink) = l;
            static_for<1, KW>([&](auto C_) CFX_INLINE {
                constexpr int c = decltype(C_)::value;
                W[i - 1][c - 1] = W[i][c] - l * U[c];  // update and slide up-left in one move
            });
            W[i - 1][KW - 1] = 0.0;
        });
        static_for<0, KW>([&](auto C_) CFX_INLINE { W[K][decltype(C_)::value] = ent[decltype(C_)::value]; });
    };
    int j0 = 0;
    for (; j0 + D <= n; j0 += D)
        static_for<0, D>([&](auto S_) CFX_INLINE {
            constexpr int s = decltype(S_)::value;
            step(j0 + s, nxt[s], j0 + s + D);
        });
    static_for<0, D>([&](auto S_) CFX_INLINE {  // the last steps prefetch nothing (their rows are past n)
        constexpr int s = decltype(S_)::value;
        if (j0 + s < n) step(j0 + s, nxt[s], n);
    });
    INFO[b] = info;
    if (nrhs > 0) __threadfence();  // the solve reads the factors stored above
    for (int c = 0; c < nrhs; ++c) lane_solve<K>(n, kl, ku, ab, ae, piv, pe, RHS + b * L.x_inst + c * L.x_rhs, L.x_el);
}

template <int K>
__global__ void __launch_bounds__(64) k_band_solve_lane(int64_t batch, int n, int kl, int ku, int nrhs,
                                                        const double* __restrict__ AB, const int32_t* __restrict__ IPIV,
                                                        double* __restrict__ RHS) {
    const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (b >= batch) return;
    const int64_t ldab = 2 * kl + ku + 1;
    for (int c = 0; c < nrhs; ++c)
        lane_solve<K>(n, kl, ku, AB + b * n * ldab, 1, IPIV + b * n, 1, RHS + (b * nrhs + c) * (int64_t)n, 1);
}

// [rows][cols] -> [cols][rows] through 64 x 64 LDS tiles (the coalesced lane path's instance-minor copies)
template <class T>
__global__ void __launch_bounds__(256) k_band_transpose(const T* __restrict__ src, T* __restrict__ dst, int64_t rows,
                                                        int64_t cols) {
    __shared__ T tile[64][65];
    const int64_t r0 = (int64_t)blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int64_t c0 = (int64_t)blockIdx.y * 64; c0 < cols; c0 += (int64_t)gridDim.y * 64) {
        for (int r = ty; r < 64; r += 4)
            if (r0 + r < rows && c0 + tx < cols) tile[r][tx] = src[(r0 + r) * cols + c0 + tx];
        __syncthreads();
        for (int r = ty; r < 64; r += 4)
            if (c0 + r < cols && r0 + tx < rows) dst[(c0 + r) * rows + r0 + tx] = tile[tx][r];
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------------
// panel placement: single wide bands, factored NB columns at a time
// ---------------------------------------------------------------------------------------------------
// The global placement's column step is five barrier-separated phases over L2 (pivot search, swap, scale,
// update): ≈ 13 µs per column for the 1,500-interval MSK KKT (n = 119,640, kl = ku = 108), 1.5 s per
// factorisation.  Here, per panel of NB columns j0 .. j0 + NB - 1:
//  1. the panel (its rows j0 .. j0 + NB - 1 + kl) is factored in one wavefront's registers, no LDS round trip
//     and no barrier per column (an LDS version with one barrier per column spent ≈ 1 µs per column), and with
//     look-ahead: wavefront 0 takes the next panel's columns of step 2 first and factors that panel while the
//     other waves finish step 2 for the current one;
//  2. the trailing columns j0 + NB .. ju (ju <= j0 + NB - 1 + kv) take the panel's interchanges and
//     elimination at once, one wave per column with the lanes over the panel's rows (band-storage columns are
//     contiguous): row r starts from original row q[r] (the interchanges composed), and for k = 0 .. NB - 1 the
//     final U12 element of row k is broadcast (readlane) and subtracted times Lt(r, k) — U12 = L11^-1 P A12 in
//     the lanes above NB, A22 -= L21 U12 below, no LDS image and no barrier; the column loads run one group
//     ahead.  Lt(r, k) = L(sigma_k(r), k) are the panel's multipliers with its later interchanges applied,
//     sigma_k(r) the row that held at step k what ends in row r; the stored multipliers stay position-based
//     (dgbtf2's, what every solve kernel reads).
// Every element receives the same operations in the same order as in the column step (the interchanges
// commute with the eliminations they are moved past), so factors, pivots and zero-pivot reports equal the
// global placement's (tested bit for bit).  Fill rows (storage rows < kl) are zeroed lazily, as columns
// enter the trailing reach.  RH: 64-row chunks per lane (NB + kl <= 64 RH).
#ifdef CFX_BAND_PROF
// phase clocks of instance 0 (micro build only): [0, 8) thread 0 (wavefront 0), [8, 16) thread 64 (wavefront 1)
__device__ unsigned long long g_panel_prof[16];
#define PANEL_STAMP(i)                                                  \
    do {                                                                \
        if (blockIdx.x == 0 && (t == 0 || t == 64)) {                   \
            const unsigned long long now_ = wall_clock64();             \
            prof[i] += now_ - last_;                                    \
            last_ = now_;                                               \
        }                                                               \
    } while (0)
#else
#define PANEL_STAMP(i) \
    do {               \
    } while (0)
#endif
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    return from32(__builtin_amdgcn_mov_dpp(lo32(v), CTRL, 0xf, 0xf, false),
                  __builtin_amdgcn_mov_dpp(hi32(v), CTRL, 0xf, 0xf, false));
}
// max over the wave (every lane gets it): quad swaps, half-row and row mirrors (each lane then holds its
// 16-lane row's max), then the four rows through readlane
__device__ __forceinline__ double wave_max(double v) {
    v = fmax(v, dpp_d<0xB1>(v));   // quad_perm [1, 0, 3, 2]
    v = fmax(v, dpp_d<0x4E>(v));   // quad_perm [2, 3, 0, 1]
    v = fmax(v, dpp_d<0x141>(v));  // row_half_mirror
    v = fmax(v, dpp_d<0x140>(v));  // row_mirror
    return fmax(fmax(lane_read(v, 0), lane_read(v, 16)), fmax(lane_read(v, 32), lane_read(v, 48)));
}
__device__ __forceinline__ int wave_min_i(int v) {
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xf, 0xf, false));
    return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
               min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

template <int NB, int RH, int NT>
__global__ void __launch_bounds__(NT) k_band_lu_panel(int n, int kl, int ku, double* __restrict__ AB,
                                                      int32_t* __restrict__ IPIV, int32_t* __restrict__ INFO) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
#ifdef CFX_PANEL_CG  // (micro builds: columns per load group)
    constexpr int NW = NT / 64, US = NB + 1, CG = CFX_PANEL_CG;
#else
    constexpr int NW = NT / 64, US = NB + 1, CG = RH >= 3 ? 2 : 4;  // US: row stride of Lt (conflict-free); CG: columns per load group
#endif
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku, PR = NB + kl;
    double* const ab = AB + (int64_t)blockIdx.x * n * ldab;
    int32_t* const piv = IPIV + (int64_t)blockIdx.x * n;
    double* const P0 = smem;               // the factored panel, column-major [c][r], stride PR
    double* const Lt = P0 + NB * PR;       // blocked multipliers, row-major [r][k], stride US
    int* const q = reinterpret_cast<int*>(Lt + PR * US);  // panel row r ends up holding original row q[r]
    int* const sp = q + PR;                                // pivot row of each panel step (panel-relative)
    int* const snz = sp + NB;                              // its pivot was non-zero
    auto at = [&](int i, int j) CFX_INLINE -> double& { return ab[(int64_t)j * ldab + kv + i - j]; };
#ifdef CFX_BAND_PROF
    unsigned long long prof[8] = {}, last_ = wall_clock64();
#endif
    // fill rows (storage rows < kl) of columns zhi + 1 .. zend, as columns enter the reach of a panel's rows
    auto zero_fill = [&](int zhi, int zend, int tid, int nthr) CFX_INLINE {
        for (int64_t e = tid; e < (int64_t)(zend - zhi) * kl; e += nthr)
            ab[(int64_t)(zhi + 1 + e / kl) * ldab + e % kl] = 0.0;
    };
    // 1. panel j0p (width wp, rows prp) in wavefront 0's registers (lane: rows lane + 64 h; no LDS and no barrier per
    //    column): per step the pivot (DPP reductions), the pivot row and row jj broadcast by readlane, and every row
    //    of the active block rewritten in place with the interchange folded into its source row — the column step's
    //    expressions, operand for operand.  Leaves the factored panel in P0 and the pivots in sp / snz.
    auto factor_panel = [&](int j0p, int wp, int prp) CFX_INLINE {
        double pa[RH][NB];
#pragma unroll
        for (int h = 0; h < RH; ++h)
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                const int r = lane + 64 * h;
                pa[h][c] = (r < prp && c < wp && r - c <= kl && c - r <= kv) ? at(j0p + r, j0p + c) : 0.0;
            }
        PANEL_STAMP(0);
#pragma unroll
        for (int jj = 0; jj < NB; ++jj) {
            if (jj < wp) {
                const int rmax = min(prp - 1, jj + kl);  // rows of the column step (km)
                double av = -1.0;
                int ai = jj;
#pragma unroll
                for (int h = 0; h < RH; ++h) {  // first row of the largest |A(r, jj)| (NaN never wins)
                    const int r = lane + 64 * h;
                    const double v = fabs(pa[h][jj]);
                    if (r >= jj && r <= rmax && v > av) {
                        av = v;
                        ai = r;
                    }
                }
                const double amax = wave_max(av);
                const int pj = wave_min_i(av == amax ? ai : 0x7fffffff), ph = pj >> 6, pl = pj & 63;
                double u[NB];  // the pivot row, columns jj .. NB - 1 (uniform: readlane)
#pragma unroll
                for (int h = 0; h < RH; ++h)
                    if (ph == h) {  // (uniform branch: one register's readlanes)
#pragma unroll
                        for (int c = 0; c < NB; ++c)  // (full-range loops: unrolled before jj is, registers throughout)
                            if (c >= jj) u[c] = lane_read(pa[h][c], pl);
                    }
                const double pv = u[jj];
                const bool nz = pv != 0.0;
                const double inv = nz ? 1.0 / pv : 0.0;
                // the ordinary rows jj < r <= rmax (not pj): l = A(r, jj) / pv, A(r, c) -= l u(c); the others keep
                // their values (l = 0: an exact no-op for finite pivot rows)
#pragma unroll
                for (int h = 0; h < RH; ++h) {
                    const int r = lane + 64 * h;
                    const bool elim = nz && r > jj && r <= rmax && r != pj;
                    const double l = elim ? pa[h][jj] * inv : 0.0;
#pragma unroll
                    for (int c = 0; c < NB; ++c)
                        if (c > jj) pa[h][c] -= l * u[c];
                    pa[h][jj] = elim ? l : pa[h][jj];
                }
                if (nz && pj != jj) {  // row pj takes row jj's elements, eliminated (uniform values, one lane)
                    double rj[NB];
#pragma unroll
                    for (int c = 0; c < NB; ++c)
                        if (c >= jj) rj[c] = lane_read(pa[0][c], jj);
                    const double lp = rj[jj] * inv;
#pragma unroll
                    for (int h = 0; h < RH; ++h)
                        if (ph == h) {
#pragma unroll
                            for (int c = 0; c < NB; ++c)
                                if (c >= jj) pa[h][c] = lane == pl ? (c == jj ? lp : rj[c] - lp * u[c]) : pa[h][c];
                        }
                }
                if (nz) {  // row jj takes the pivot row
#pragma unroll
                    for (int c = 0; c < NB; ++c)
                        if (c >= jj) pa[0][c] = lane == jj ? u[c] : pa[0][c];
                }
                if (lane == 0) {
                    sp[jj] = pj;
                    snz[jj] = nz;
                }
            }
        }
        PANEL_STAMP(1);
#pragma unroll
        for (int h = 0; h < RH; ++h)
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                const int r = lane + 64 * h;
                if (r < prp && c < wp) P0[c * PR + r] = pa[h][c];
            }
        PANEL_STAMP(7);
    };
    // 2. trailing columns c0 + cc (cc = cb, cb + stride, ... < ce) of panel j0 (width w, rows pr), one wave each: lane
    //    holds rows lane + 64 h; row r starts from original row q[r], and for k = 0 .. w - 1 the final U12 element of
    //    row k is broadcast (readlane) and subtracted times Lt(r, k) (zero for r <= k); the loads run one group ahead
    auto trail = [&](int j0, int w, int pr, int c0, int cb0, int ce, int stride) CFX_INLINE {
        double lr[RH][NB];
        int qr[RH];
#pragma unroll
        for (int h = 0; h < RH; ++h) {
            const int r = lane + 64 * h;
            qr[h] = r < pr ? q[r] : -1;
#pragma unroll
            for (int k = 0; k < NB; ++k) lr[h][k] = r < pr ? Lt[r * US + k] : 0.0;
        }
        auto load = [&](int cc, double (&x)[RH]) CFX_INLINE {
            const int c = c0 + cc;
#pragma unroll
            for (int h = 0; h < RH; ++h)
                x[h] = (cc < ce && qr[h] >= 0 && c - (j0 + qr[h]) <= kv) ? at(j0 + qr[h], c) : 0.0;
        };
        double cur[CG][RH], nxt[CG][RH];
#pragma unroll
        for (int g = 0; g < CG; ++g) load(cb0 + g * stride, cur[g]);
        for (int cb = cb0; cb < ce; cb += stride * CG) {
#pragma unroll
            for (int g = 0; g < CG; ++g) load(cb + (g + CG) * stride, nxt[g]);
            // the CG columns' chains interleaved step by step (row k of each: final U12 once steps 0 .. k - 1 are in);
            // full panels without the k < w test, so that the whole update is one block for the scheduler
            auto step = [&](int k) CFX_INLINE {
#pragma unroll
                for (int g = 0; g < CG; ++g) {
                    const double xk = lane_read(cur[g][0], k);
#pragma unroll
                    for (int h = 0; h < RH; ++h) cur[g][h] -= lr[h][k] * xk;
                }
            };
            if (w == NB) {
#pragma unroll
                for (int k = 0; k < NB; ++k) step(k);
            } else {
#pragma unroll
                for (int k = 0; k < NB; ++k)
                    if (k < w) step(k);  // (uniform; no break: the loop stays fully unrolled, lr in registers)
            }
#pragma unroll
            for (int g = 0; g < CG; ++g) {
                const int cc = cb + g * stride, c = c0 + cc;
                double (&x)[RH] = cur[g];
                if (cc < ce) {
#pragma unroll
                    for (int h = 0; h < RH; ++h) {
                        const int r = lane + 64 * h;
                        if (r < pr && (r >= w || c - (j0 + r) <= kv)) at(j0 + r, c) = x[h];
                    }
                }
            }
#pragma unroll
            for (int g = 0; g < CG; ++g)
#pragma unroll
                for (int h = 0; h < RH; ++h) cur[g][h] = nxt[g][h];
        }
    };
    int info = 0, ju = 0, zhi = -1;
    {  // prologue: the first panel
        const int w0 = min(NB, n), zend = min(w0 - 1 + kv, n - 1);
        zero_fill(zhi, zend, t, NT);
        zhi = zend;
        __syncthreads();
        if (wave == 0) factor_panel(0, w0, min(w0 + kl, n));
        __syncthreads();
    }
    for (int j0 = 0; j0 < n; j0 += NB) {
        const int w = min(NB, n - j0), pr = min(w + kl, n - j0);
        // the factored panel (P0, sp, snz): LAPACK's column reach and first zero pivot in every thread; the panel back
        // to the band, the pivots, the blocked multipliers and the composed interchanges
        for (int jj = 0; jj < w; ++jj) {
            if (snz[jj])
                ju = max(ju, min(j0 + ku + sp[jj], n - 1));
            else if (info == 0)
                info = j0 + jj + 1;
        }
        PANEL_STAMP(2);
        int spr[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) spr[i] = i < w ? sp[i] : i;
        auto sigma = [&](int r, int k) CFX_INLINE {  // interchanges w - 1 .. k + 1 undone
            int s = r;
#pragma unroll
            for (int i = NB - 1; i >= 0; --i)
                if (i > k && i < w) s = s == i ? spr[i] : (s == spr[i] ? i : s);
            return s;
        };
        for (int e = t; e < w * pr; e += NT) {
            const int c = e / pr, r = e - c * pr;
            if (r - c <= kl && c - r <= kv) at(j0 + r, j0 + c) = P0[c * PR + r];
        }
        for (int e = t; e < NB * pr; e += NT) {
            const int k = e % NB, rr = e / NB;
            Lt[rr * US + k] = (rr > k && k < w) ? P0[k * PR + sigma(rr, k)] : 0.0;
        }
        for (int r = t; r < pr; r += NT) q[r] = sigma(r, -1);
        if (t < w) piv[j0 + t] = j0 + sp[t];
        // LDS only (Lt, q; P0 and sp free after it): the panel's global stores are read again only after the next
        // full barrier
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        PANEL_STAMP(3);
        // 2. the trailing columns c0 .. ju, with look-ahead: wavefront 0 updates the next panel's columns, zeroes the
        //    fill rows entering that panel's reach, re-reads the panel and factors it (step 1) while the other waves
        //    update the rest
        const int c0 = j0 + w, wt = ju - c0 + 1, jn = c0, wn = min(NB, n - jn);
        const int zend = wn > 0 ? min(jn + wn - 1 + kv, n - 1) : zhi;
        if (wave == 0) {
            if (wn > 0) {
                if (wt > 0) trail(j0, w, pr, c0, 0, min(wn, wt), 1);
                PANEL_STAMP(4);
                zero_fill(zhi, zend, lane, 64);
                __threadfence_block();  // this wave's stores before its loads of the next panel
                factor_panel(jn, wn, min(wn + kl, n - jn));
                PANEL_STAMP(5);
            }
        } else if (wt > wn) {
            trail(j0, w, pr, c0, wn + wave - 1, wt, NW - 1);
            PANEL_STAMP(4);
        }
        zhi = max(zhi, zend);
        __syncthreads();
        PANEL_STAMP(6);
    }
#ifdef CFX_BAND_PROF
    if (blockIdx.x == 0 && t == 0)
        for (int i = 0; i < 8; ++i) g_panel_prof[i] = prof[i];
    if (blockIdx.x == 0 && t == 64)
        for (int i = 0; i < 8; ++i) g_panel_prof[8 + i] = prof[i];
#endif
    if (t == 0) INFO[blockIdx.x] = info;
}

// Solves with the factors of any placement for single wide bands: one wavefront runs the substitution's
// dependent chain with its window in registers (as the register placement's solve), the other waves stream
// the band columns it needs into LDS ahead of it, CH columns per buffer, one barrier per CH columns — the
// global placement's substitutions pay two barriers and an L2 round trip per column instead.
// Forward pass: x <- L^-1 P x, lane i + 64 f holding x[j + i + 64 f] (i + 64 f <= kl < 64 KF); per column the
// buffer holds the multipliers L(j + i, j) at slot i (zero outside 1 .. min(kl, n - 1 - j)), the pivot row
// and x[j + 1 + kl], the element entering the window.
template <int KF, int NT>
__global__ void __launch_bounds__(NT) k_band_fwd_stream(int n, int kl, int ku, int nrhs,
                                                        const double* __restrict__ AB,
                                                        const int32_t* __restrict__ IPIV, double* RHS) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int CW = 64 * KF, CH = 128 / KF, NP = NT - 64, SD = 4;
    const int t = threadIdx.x, lane = t & 63;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku, fk = kl >> 6, lk = kl & 63;
    const double* const ab = AB + (int64_t)blockIdx.x * n * ldab;
    const int32_t* const piv = IPIV + (int64_t)blockIdx.x * n;
    double* const M = smem;                // [buffer][column][slot]
    double* const X = M + 2 * CH * CW;     // [buffer][column]
    int* const Pv = reinterpret_cast<int*>(X + 2 * CH);
    double* dsink = block_sink() + lane;
    const int steps = n - 1, nch = (steps + CH - 1) / CH;
    if (kl == 0 || steps <= 0) return;
    for (int c = 0; c < nrhs; ++c) {
        double* x = RHS + ((int64_t)blockIdx.x * nrhs + c) * n;
        auto produce = [&](int ci) {
            const int b = ci & 1, jb = ci * CH, tp = t - 64;
#pragma unroll 8
            for (int e = tp; e < CH * CW; e += NP) {
                const int jj = e / CW, i = e - jj * CW, j = jb + jj;
                M[(b * CH + jj) * CW + i] =
                    (j < steps && i >= 1 && i <= min(kl, n - 1 - j)) ? ab[(int64_t)j * ldab + kv + i] : 0.0;
            }
            for (int jj = tp; jj < CH; jj += NP) {
                const int j = jb + jj;
                Pv[b * CH + jj] = j < steps ? piv[j] - j : 0;
                X[b * CH + jj] = j + 1 + kl < n ? x[j + 1 + kl] : 0.0;
            }
        };
        double xw[KF];
        if (t < 64) {
#pragma unroll
            for (int f = 0; f < KF; ++f) {
                const int i = lane + 64 * f;
                xw[f] = (i <= kl && i < n) ? x[i] : 0.0;
            }
        } else {
            produce(0);
        }
        __syncthreads();
        for (int ci = 0; ci < nch; ++ci) {
            if (t < 64) {
                const int b = ci & 1, jb = ci * CH, cnt = min(CH, steps - jb);
                const double* Mb = M + b * CH * CW;
                // the buffer's reads run SD steps ahead of their use (a register ring, unrolled)
                auto fetch = [&](int jj, double (&lc)[KF], int& p, double& nx) CFX_INLINE {
                    const int jc = min(jj, CH - 1);
#pragma unroll
                    for (int f = 0; f < KF; ++f) lc[f] = Mb[jc * CW + lane + 64 * f];
                    p = Pv[b * CH + jc];
                    nx = X[b * CH + jc];
                };
                double lr[SD][KF], nr[SD];
                int pr[SD];
#pragma unroll
                for (int s = 0; s < SD; ++s) fetch(s, lr[s], pr[s], nr[s]);
                for (int jj0 = 0; jj0 < cnt; jj0 += SD) {
#pragma unroll
                    for (int s = 0; s < SD; ++s) {
                        const int jj = jj0 + s, j = jb + jj;
                        if (jj < cnt) {
                            double lc[KF];
#pragma unroll
                            for (int f = 0; f < KF; ++f) lc[f] = lr[s][f];
                            const int p = __builtin_amdgcn_readfirstlane(pr[s]);
                            const double nxv = nr[s];
                            fetch(jj + SD, lr[s], pr[s], nr[s]);
                            if (p != 0) {
                                const int fp = p >> 6, lp = p & 63;
                                double src = xw[0];
#pragma unroll
                                for (int f = 1; f < KF; ++f)
                                    if (f == fp) src = xw[f];
                                const double a = lane_read(xw[0], 0), bv = lane_read(src, lp);
                                xw[0] = lane == 0 ? bv : xw[0];
#pragma unroll
                                for (int f = 0; f < KF; ++f)
                                    if (f == fp) xw[f] = lane == lp ? a : xw[f];
                            }
                            const double xj = lane_read(xw[0], 0);
#pragma unroll
                            for (int f = 0; f < KF; ++f) xw[f] -= lc[f] * xj;
                            *(lane == 0 ? x + j : dsink) = xj;
                            slide<KF>(xw);
#pragma unroll
                            for (int f = 0; f < KF; ++f)
                                if (f == fk && lane == lk) xw[f] = nxv;
                        }
                    }
                }
            } else if (ci + 1 < nch) {
                produce(ci + 1);
            }
            __syncthreads();
        }
        if (t == 0) x[n - 1] = xw[0];
        __syncthreads();
    }
}

// Backward pass: x <- U^-1 x, lane i + 64 k holding x[j - i - 64 k] (i + 64 k <= kv < 64 KB); per column the
// buffer holds U(j - i, j) at slot i (zero past min(kv, j)) and x[j - 1 - kv].
template <int KB, int NT>
__global__ void __launch_bounds__(NT) k_band_bwd_stream(int n, int kl, int ku, int nrhs,
                                                        const double* __restrict__ AB, double* RHS) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int CW = 64 * KB, CH = 128 / KB, NP = NT - 64, SD = 4;
    const int t = threadIdx.x, lane = t & 63;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku, fk = kv >> 6, lk = kv & 63;
    const double* const ab = AB + (int64_t)blockIdx.x * n * ldab;
    double* const U = smem;
    double* const X = U + 2 * CH * CW;
    double* dsink = block_sink() + lane;
    const int nch = (n + CH - 1) / CH;
    for (int c = 0; c < nrhs; ++c) {
        double* x = RHS + ((int64_t)blockIdx.x * nrhs + c) * n;
        auto produce = [&](int ci) {  // chunk ci: columns n - 1 - ci CH downwards
            const int b = ci & 1, jb = n - 1 - ci * CH, tp = t - 64;
#pragma unroll 8
            for (int e = tp; e < CH * CW; e += NP) {
                const int jj = e / CW, i = e - jj * CW, j = jb - jj;
                U[(b * CH + jj) * CW + i] = (j >= 0 && i <= min(kv, j)) ? ab[(int64_t)j * ldab + kv - i] : 0.0;
            }
            for (int jj = tp; jj < CH; jj += NP) {
                const int j = jb - jj;
                X[b * CH + jj] = j - 1 - kv >= 0 ? x[j - 1 - kv] : 0.0;
            }
        };
        double xw[KB];
        if (t < 64) {
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                const int i = lane + 64 * k;
                xw[k] = (i <= kv && n - 1 - i >= 0) ? x[n - 1 - i] : 0.0;
            }
        } else {
            produce(0);
        }
        __syncthreads();
        for (int ci = 0; ci < nch; ++ci) {
            if (t < 64) {
                const int b = ci & 1, jb = n - 1 - ci * CH, cnt = min(CH, jb + 1);
                const double* Ub = U + b * CH * CW;
                auto fetch = [&](int jj, double (&uc)[KB], double& nx) CFX_INLINE {
                    const int jc = min(jj, CH - 1);
#pragma unroll
                    for (int k = 0; k < KB; ++k) uc[k] = Ub[jc * CW + lane + 64 * k];
                    nx = X[b * CH + jc];
                };
                double ur[SD][KB], nr[SD];
#pragma unroll
                for (int s = 0; s < SD; ++s) fetch(s, ur[s], nr[s]);
                for (int jj0 = 0; jj0 < cnt; jj0 += SD) {
#pragma unroll
                    for (int s = 0; s < SD; ++s) {
                        const int jj = jj0 + s, j = jb - jj;
                        if (jj < cnt) {
                            double uc[KB];
#pragma unroll
                            for (int k = 0; k < KB; ++k) uc[k] = ur[s][k];
                            const double nxv = nr[s];
                            fetch(jj + SD, ur[s], nr[s]);
                            const double xj = lane_read(xw[0], 0) / lane_read(uc[0], 0);
                            *(lane == 0 ? x + j : dsink) = xj;
#pragma unroll
                            for (int k = 0; k < KB; ++k) {  // one fused multiply-subtract per element, as the column kernels
                                const double u = (k == 0 && lane == 0) ? 0.0 : uc[k];
                                xw[k] -= u * xj;
                            }
                            slide<KB>(xw);
#pragma unroll
                            for (int k = 0; k < KB; ++k)
                                if (k == fk && lane == lk) xw[k] = nxv;
                        }
                    }
                }
            } else if (ci + 1 < nch) {
                produce(ci + 1);
            }
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------------------------------
// Raise a kernel's dynamic-LDS limit above 64 KiB only when a launch needs more than it was last raised to (one
// attribute call per kernel and size, not one per launch).
// The limit raised so far is kept per kernel ADDRESS: several instantiations share one function-pointer type
// (k_band_fwd_stream<1/2/4>, k_band_bwd_stream<KB>, k_band_lu_panel<RH>), so a per-type static would skip the attribute
// call for an instantiation that was never raised.
static std::mutex g_lds_mutex;
static std::map<const void*, size_t> g_lds_raised;
template <class K>
static hipError_t allow_lds(K kernel, size_t bytes) {
    const void* fn = reinterpret_cast<const void*>(kernel);
    std::lock_guard<std::mutex> lock(g_lds_mutex);
    auto it = g_lds_raised.find(fn);
    const size_t raised = it == g_lds_raised.end() ? 65536 : it->second;
    if (bytes <= raised) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) g_lds_raised[fn] = bytes;
    return e;
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

template <int NCH, int KC, int D = (NCH <= 2 && KC == 1) ? 8 : 2>
static hipError_t launch_reg(int64_t n, int32_t kl, int32_t ku, int64_t batch, double* ab, int32_t* ipiv,
                             int32_t* info, int32_t nrhs, double* rhs, hipStream_t s, int factor) {
    if (factor)
        hipLaunchKernelGGL((k_band_lu_reg<NCH, KC, D>), dim3((unsigned)batch), dim3(64), 0, s, (int)n, kl, ku, nrhs,
                           ab, ipiv, rhs, info);
    else
        hipLaunchKernelGGL((k_band_solve_reg<KC, D>), dim3((unsigned)batch), dim3(64), 0, s, (int)n, kl, ku, nrhs,
                           (const double*)ab, (const int32_t*)ipiv, rhs);
    return hipGetLastError();
}

// Register placement when the window fits: the padded rows (8 NCH - 1 >= kl) plus the ku + 1 columns of
// the pivot row within 64 KC lanes, and 32-bit offsets within an instance.
static int reg_chunks(int64_t n, int32_t kl, int32_t ku) {
    const int64_t ldab = 2 * (int64_t)kl + ku + 1;
    if (n * ldab >= (int64_t)1 << 31) return -1;
    const int nch = kl / 8 + 1;  // 8 nch - 1 >= kl
    if (nch > 6 || 8 * nch + ku > 128) return -1;
    return nch;
}

// Grouped register placement (four instances per wave): windows of at most 16 lanes, batches of at least
// kGroupBatch instances (CFX_BAND_GROUP=0 / 1 forces it off / on where it fits).
constexpr int64_t kGroupBatch = 256;
static bool group_ok(int64_t n, int32_t kl, int32_t ku, int64_t batch) {
    if (kl > kG16Klm || 8 + ku > 16 || n * (2 * (int64_t)kl + ku + 1) >= ((int64_t)1 << 31)) return false;
    if (const char* e = std::getenv("CFX_BAND_GROUP")) return *e == '1';
    return batch >= kGroupBatch;
}

static hipError_t reg_dispatch(int64_t n, int32_t kl, int32_t ku, int64_t batch, double* ab, int32_t* ipiv,
                               int32_t* info, int32_t nrhs, double* rhs, hipStream_t s, int factor) {
#define CFX_REG(M, C) launch_reg<M, C>(n, kl, ku, batch, ab, ipiv, info, nrhs, rhs, s, factor)
    if (group_ok(n, kl, ku, batch)) {
        const dim3 grid((unsigned)((batch + 3) / 4));
        if (factor)
            hipLaunchKernelGGL(k_band_lu_reg16<8>, grid, dim3(64), 0, s, batch, (int)n, kl, ku, nrhs, ab, ipiv, rhs,
                               info);
        else
            hipLaunchKernelGGL(k_band_solve_reg16<8>, grid, dim3(64), 0, s, batch, (int)n, kl, ku, nrhs,
                               (const double*)ab, (const int32_t*)ipiv, rhs);
        return hipGetLastError();
    }
    const int nch = reg_chunks(n, kl, ku);
    if (8 * nch + ku <= 64) {
        switch (nch) {
            case 1: return CFX_REG(1, 1);
            case 2: return CFX_REG(2, 1);
            case 3: return CFX_REG(3, 1);
            case 4: return CFX_REG(4, 1);
            case 5: return CFX_REG(5, 1);
            default: return CFX_REG(6, 1);
        }
    }
    switch (nch) {
        case 1: return CFX_REG(1, 2);
        case 2: return CFX_REG(2, 2);
        case 3: return CFX_REG(3, 2);
        case 4: return CFX_REG(4, 2);
        case 5: return CFX_REG(5, 2);
        default: return CFX_REG(6, 2);
    }
#undef CFX_REG
}

// Lane placement: batches of at least kLaneBatch instances with max(kl, ku) <= kLaneMaxK.  Each lane runs its
// instance's ~30-instruction-deep dependent chain per column alone (one wave per SIMD, nothing to hide the
// latency: ~4.4 us per column against the register kernel's ~0.3 us), so it only wins once the register kernel's
// waves queue for the CUs — cfg-3 KKT (n = 502, kl = ku = 6), factor + solve: 0.51 / 2.29 ms (register / lane) at
// 1,024 instances, 1.74 / 2.56 at 4,096, 7.75 / 3.66 at 16,384; solve alone 2.54 / 0.79 ms at 16,384
// (scripts/band_lane_probe.py, profiles/round2/band_lane_probe.jsonl).
constexpr int64_t kLaneBatch = 8192;
constexpr int kLaneMaxK = 8;
static bool lane_ok(int64_t n, int32_t kl, int32_t ku) {
    return std::max(kl, ku) <= kLaneMaxK && n * (2 * (int64_t)kl + ku + 1) < ((int64_t)1 << 31);
}
// Device workspace of the coalesced lane path (instance-minor copies of the band, pivots and right-hand sides):
// grown on demand, one per device, kept for the process.
static std::mutex g_lane_ws_mutex;
static void* g_lane_ws[64];
static size_t g_lane_ws_bytes[64];
static void* lane_workspace(size_t bytes) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lock(g_lane_ws_mutex);
    if (g_lane_ws_bytes[dev] < bytes) {
        if (g_lane_ws[dev]) (void)hipFree(g_lane_ws[dev]);
        g_lane_ws[dev] = nullptr;
        g_lane_ws_bytes[dev] = 0;
        if (hipMalloc(&g_lane_ws[dev], bytes) != hipSuccess) return nullptr;
        g_lane_ws_bytes[dev] = bytes;
    }
    return g_lane_ws[dev];
}
template <class T>
static void transpose(const T* src, T* dst, int64_t rows, int64_t cols, hipStream_t s) {
    const dim3 grid((unsigned)((rows + 63) / 64), (unsigned)std::min<int64_t>((cols + 63) / 64, 65535));
    hipLaunchKernelGGL(k_band_transpose<T>, grid, dim3(256), 0, s, src, dst, rows, cols);
}

template <int K>
static hipError_t launch_lane_k(int64_t n, int32_t kl, int32_t ku, int64_t batch, double* ab, int32_t* ipiv,
                                int32_t* info, int32_t nrhs, double* rhs, hipStream_t s, int factor) {
    const dim3 grid((unsigned)((batch + 63) / 64));
    const int64_t ldab = 2 * (int64_t)kl + ku + 1, len = n * ldab, xl = (int64_t)nrhs * n;
    if (factor && !std::getenv("CFX_BAND_LANE_DIRECT")) {
        // coalesced: every lane access of a wave is one contiguous 512-byte run in the instance-minor copies
        const size_t bytes = (size_t)batch * ((len + xl) * sizeof(double) + n * sizeof(int32_t));
        double* wab = static_cast<double*>(lane_workspace(bytes));
        if (!wab) return hipErrorOutOfMemory;
        double* wx = wab + batch * len;
        int32_t* wp = reinterpret_cast<int32_t*>(wx + batch * xl);
        transpose<double>(ab, wab, batch, len, s);
        if (nrhs) transpose<double>(rhs, wx, batch, xl, s);
        const LaneLayout L{1, batch, 1, batch, 1, batch, n * batch};
        hipLaunchKernelGGL(k_band_lu_lane<K>, grid, dim3(64), 0, s, batch, (int)n, kl, ku, nrhs, wab, wp, wx, info, L);
        transpose<double>(wab, ab, len, batch, s);
        transpose<int32_t>(wp, ipiv, n, batch, s);
        if (nrhs) transpose<double>(wx, rhs, xl, batch, s);
    } else if (factor) {
        const LaneLayout L{len, 1, n, 1, xl, 1, n};
        hipLaunchKernelGGL(k_band_lu_lane<K>, grid, dim3(64), 0, s, batch, (int)n, kl, ku, nrhs, ab, ipiv, rhs, info, L);
    } else
        hipLaunchKernelGGL(k_band_solve_lane<K>, grid, dim3(64), 0, s, batch, (int)n, kl, ku, nrhs,
                           (const double*)ab, (const int32_t*)ipiv, rhs);
    return hipGetLastError();
}
static hipError_t lane_dispatch(int64_t n, int32_t kl, int32_t ku, int64_t batch, double* ab, int32_t* ipiv,
                                int32_t* info, int32_t nrhs, double* rhs, hipStream_t s, int factor) {
#define CFX_LANE(K) launch_lane_k<K>(n, kl, ku, batch, ab, ipiv, info, nrhs, rhs, s, factor)
    switch (std::max(std::max(kl, ku), 1)) {
        case 1: return CFX_LANE(1);
        case 2: return CFX_LANE(2);
        case 3: return CFX_LANE(3);
        case 4: return CFX_LANE(4);
        case 5: return CFX_LANE(5);
        case 6: return CFX_LANE(6);
        case 7: return CFX_LANE(7);
        default: return CFX_LANE(8);
    }
#undef CFX_LANE
}

// Panel placement (single bands too wide for LDS and registers: what the global placement would take): 16-column
// panels with the panel's rows (16 + kl <= 256) in at most four 64-row chunks per lane; LDS bytes of k_band_lu_panel.
constexpr int kPanelNB = 16;
static size_t panel_lds(int32_t kl) {
    const int64_t pr = kPanelNB + (int64_t)kl;
    return (size_t)(8 * (kPanelNB * pr + pr * (kPanelNB + 1)) + 4 * (pr + 2 * kPanelNB));
}
static int panel_rh(int32_t kl) {  // 64-row chunks per lane, 0: not applicable
    const int64_t pr = kPanelNB + (int64_t)kl;
    return (pr <= 256 && panel_lds(kl) <= (size_t)kBandLds) ? (int)((pr + 63) / 64) : 0;
}
// streamed solves: window registers per lane (forward kl < 64 KF, backward kl + ku < 64 KB)
static bool stream_ok(int32_t kl, int32_t ku) { return kl <= 255 && kl + ku <= 511; }
constexpr int kStreamNT = 512;

template <int KF>
static hipError_t launch_fwd(int64_t n, int32_t kl, int32_t ku, int64_t batch, const double* ab, const int32_t* ipiv,
                             int32_t nrhs, double* rhs, hipStream_t s) {
    constexpr int CH = 128 / KF;
    const size_t lds = (size_t)2 * CH * 64 * KF * 8 + (size_t)2 * CH * 8 + (size_t)2 * CH * 4;
    hipError_t e = allow_lds(&k_band_fwd_stream<KF, kStreamNT>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_band_fwd_stream<KF, kStreamNT>), dim3((unsigned)batch), dim3(kStreamNT), lds, s, (int)n, kl,
                       ku, nrhs, ab, ipiv, rhs);
    return hipGetLastError();
}
template <int KB>
static hipError_t launch_bwd(int64_t n, int32_t kl, int32_t ku, int64_t batch, const double* ab, int32_t nrhs,
                             double* rhs, hipStream_t s) {
    constexpr int CH = 128 / KB;
    const size_t lds = (size_t)2 * CH * 64 * KB * 8 + (size_t)2 * CH * 8;
    hipError_t e = allow_lds(&k_band_bwd_stream<KB, kStreamNT>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_band_bwd_stream<KB, kStreamNT>), dim3((unsigned)batch), dim3(kStreamNT), lds, s, (int)n, kl,
                       ku, nrhs, ab, rhs);
    return hipGetLastError();
}

template <int RH>
static hipError_t launch_panel_rh(int64_t n, int32_t kl, int32_t ku, int64_t batch, double* ab, int32_t* ipiv,
                                  int32_t* info, hipStream_t s) {
    const size_t lds = panel_lds(kl);
    hipError_t e = allow_lds(&k_band_lu_panel<kPanelNB, RH, 512>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_band_lu_panel<kPanelNB, RH, 512>), dim3((unsigned)batch), dim3(512), lds, s, (int)n, kl, ku,
                       ab, ipiv, info);
    return hipGetLastError();
}

static hipError_t launch_panel(int64_t n, int32_t kl, int32_t ku, int64_t batch, double* ab, int32_t* ipiv,
                               int32_t* info, int32_t nrhs, double* rhs, hipStream_t s, int factor) {
    hipError_t e = hipSuccess;
    if (factor) {
        switch (panel_rh(kl)) {
            case 1: e = launch_panel_rh<1>(n, kl, ku, batch, ab, ipiv, info, s); break;
            case 2: e = launch_panel_rh<2>(n, kl, ku, batch, ab, ipiv, info, s); break;
            case 3: e = launch_panel_rh<3>(n, kl, ku, batch, ab, ipiv, info, s); break;
            default: e = launch_panel_rh<4>(n, kl, ku, batch, ab, ipiv, info, s); break;
        }
        if (e != hipSuccess) return e;
    }
    if (nrhs < 1) return hipSuccess;
    if (!stream_ok(kl, ku)) {  // the global placement's substitutions
        hipLaunchKernelGGL((k_band_lu<false, 1024>), dim3((unsigned)batch), dim3(1024), 0, s, (int)n, kl, ku, nrhs, ab,
                           ipiv, rhs, info, 0);
        return hipGetLastError();
    }
    if (kl > 0) {
        e = kl < 64 ? launch_fwd<1>(n, kl, ku, batch, ab, ipiv, nrhs, rhs, s)
                    : (kl < 128 ? launch_fwd<2>(n, kl, ku, batch, ab, ipiv, nrhs, rhs, s)
                                : launch_fwd<4>(n, kl, ku, batch, ab, ipiv, nrhs, rhs, s));
        if (e != hipSuccess) return e;
    }
    const int kv = kl + ku;
    return kv < 64    ? launch_bwd<1>(n, kl, ku, batch, ab, nrhs, rhs, s)
           : kv < 128 ? launch_bwd<2>(n, kl, ku, batch, ab, nrhs, rhs, s)
           : kv < 256 ? launch_bwd<4>(n, kl, ku, batch, ab, nrhs, rhs, s)
                      : launch_bwd<8>(n, kl, ku, batch, ab, nrhs, rhs, s);
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
    // placement: the register kernels whenever the window fits a wavefront's registers; otherwise small
    // batches keep the whole band resident when it fits LDS (latency-bound), larger ones use the window,
    // and bands too wide for both take the panel kernels (the global copy where even those do not fit).
    // CFX_BAND_PLACEMENT=0..5 forces one (where it fits; 1: resident, else global; 2: global; 4: lane; 5:
    // panel); CFX_BAND_FULL forces resident / global.  Batches of >= kLaneBatch narrow bands take the lane
    // placement.
    int placement;
    const bool force_full = std::getenv("CFX_BAND_FULL") != nullptr;
    const char* forced = std::getenv("CFX_BAND_PLACEMENT");
    const bool win_ok = lds_win <= (size_t)kBandLds && chunk >= 4;
    // the register solve (one wave per instance) loses to the windowed one once the batch fills the chip
    const bool reg_ok = reg_chunks(n, kl, ku) > 0 && (factor || batch < 2048 || !win_ok || group_ok(n, kl, ku, batch));
    if (forced && *forced == '4' && lane_ok(n, kl, ku))
        placement = 4;
    else if (forced && *forced == '3' && reg_chunks(n, kl, ku) > 0)
        placement = 3;
    else if (!force_full && !forced && batch >= kLaneBatch && lane_ok(n, kl, ku))
        placement = 4;
    else if (forced && *forced == '0' && win_ok)
        placement = 0;
    else if (forced && *forced == '1')
        placement = lds_full <= (size_t)kBandLds ? 1 : 2;
    else if (forced && *forced == '2')
        placement = 2;
    else if (forced && *forced == '5' && panel_rh(kl) > 0)
        placement = 5;
    else if (!force_full && !forced && reg_ok)
        placement = 3;
    else if (!force_full && !(batch < 128 && lds_full <= (size_t)kBandLds) && win_ok)
        placement = 0;
    else
        placement = lds_full <= (size_t)kBandLds ? 1 : 2;
    if (placement == 2 && !force_full && !forced && panel_rh(kl) > 0) placement = 5;
    const size_t lds = placement == 0 ? lds_win : (placement == 1 ? lds_full : 0);
    // threads per instance: enough lanes for the rank-1 update of the trailing km x (kl + ku) block
    const int64_t work = (int64_t)kl * (kl + ku);
    const hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    if (placement == 5)
        e = launch_panel(n, kl, ku, batch, ab, ipiv, info, nrhs, rhs, s, factor);
    else if (placement == 4)
        e = lane_dispatch(n, kl, ku, batch, ab, ipiv, info, nrhs, rhs, s, factor);
    else if (placement == 3)
        e = reg_dispatch(n, kl, ku, batch, ab, ipiv, info, nrhs, rhs, s, factor);
    else if (work <= 192)
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

// internal (cfx_internal.h): does the register placement apply to (n, kl, ku)
int cfx_band_reg_ok(int64_t n, int32_t kl, int32_t ku) { return cfx::reg_chunks(n, kl, ku) > 0; }

// internal (cfx_internal.h): parallel right-hand sides with the factors of cfx_band_lu (register placement only)
int cfx_band_solve_multi(int64_t n, int32_t kl, int32_t ku, int64_t batch, int32_t parts, const double* ab,
                         const int32_t* ipiv, double* X, int64_t x_inst, int64_t x_part, int64_t x_rhs, int32_t nx,
                         double* Y, int64_t y_inst, int64_t y_part, void* stream) {
    const int nch = cfx::reg_chunks(n, kl, ku);
    const int ny = Y ? 1 : 0;
    if (nch <= 0 || batch < 1 || batch > 0x7fffffff || parts < 1 || batch % parts || nx < 0 || nx + ny < 1 ||
        nx + ny > 65535 || (nx && !X)) {
        g_create_error = "cfx_band_solve_multi: invalid argument";
        return CFX_EINVAL;
    }
    const dim3 grid((unsigned)batch, (unsigned)(nx + ny));
    const hipStream_t s = (hipStream_t)stream;
    if (8 * nch + ku <= 64)
        hipLaunchKernelGGL((cfx::k_band_solve_reg_multi<1, 8>), grid, dim3(64), 0, s, (int)n, kl, ku, ab, ipiv,
                           parts, X, x_inst, x_part, x_rhs, nx, Y, y_inst, y_part);
    else
        hipLaunchKernelGGL((cfx::k_band_solve_reg_multi<2, 2>), grid, dim3(64), 0, s, (int)n, kl, ku, ab, ipiv,
                           parts, X, x_inst, x_part, x_rhs, nx, Y, y_inst, y_part);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_create_error = std::string("cfx_band_solve_multi: ") + hipGetErrorString(e);
        return CFX_EHIP;
    }
    return CFX_OK;
}

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
