// cfx_chain.hip — batched block-tridiagonal factorisation and solves by block cyclic reduction (gfx950).
//
// Replaces, for single large OCPs, the sequential band factorisation of the interior point's KKT matrix
// (round 4: k_band_lu_panel, one 512-thread workgroup walking 119,640 pivot columns of the reaching task's band,
// 248 ms per factorisation with 255 of 256 CUs idle).  In Ipopt this is MUMPS' job (Solver.IPOPT as built at
// cocofest/optimization/fes_ocp.py:171-190; reaching_task_pulse_duration_optimization.py:117).
//
// Structure.  Group the KKT unknowns by stage: node k holds the free variables of shooting node k and the constraint
// rows that "arrive" at it (the continuity rows Phi(x_{k-1}, u_{k-1}) - x_k, whose -I falls on x_k; the per-pulse tie
// rows u_k - u_{k-1}; path rows of node k).  Every KKT entry then couples a node with itself or a neighbour: the
// matrix is block tridiagonal with M diagonal blocks D_k (padded to SP x SP), L_k = block (k, k-1) and
// U_k = block (k, k+1).  cfx_ipm builds this grouping from the callbacks' triplets (rows matched one-to-one to a
// variable of their node; rows that cannot be matched — marker rows, end conditions on fixed states — go to a small
// dense border, solved by its Schur complement as for the Hmed parameters).  With that matching every principal
// submatrix over a contiguous range of nodes is a KKT matrix whose constraint block has full row rank, so the pivot
// blocks below are nonsingular for any Hessian: no pivoting across blocks is needed.
//
// Block cyclic reduction (log2 M levels).  Level l (h = 2^l) eliminates the nodes i = h mod 2h, every one
// independently:  D_i^-1 (Gauss-Jordan with partial pivoting in LDS), X_i = D_i^-1 L_i, Y_i = D_i^-1 U_i (FP64 MFMA,
// v_mfma_f64_16x16x4f64), and each survivor p = 0 mod 2h takes the Schur complement of its two eliminated neighbours
// i = p + h, j = p - h:
//     D_p -= U_p X_i + L_p Y_j,   U_p <- -U_p Y_i  (now coupling to p + 2h),   L_p <- -L_p X_j  (to p - 2h)
// four SP x SP x SP products on the matrix cores.  The pre-update U_p, L_p are kept (Cl_i, Cr_j) for the solves.
// After the last level node 0 alone remains and is inverted.  Level 0 of the reaching task (M = 1,501, SP = 80) runs
// 750 eliminations side by side: the chip is full where the band factorisation ran one workgroup.
// Solve: forward over the levels (t_i = D_i^-1 r_i, r_p -= Cl_i t_i + Cr_j t_j), x_0 = D_0^-1 r_0, backward
// (x_i = t_i - X_i x_{i-h} - Y_i x_{i+h}).
//
// Storage (per instance, instance stride `stride` doubles): D [M][SP][SP], L [M][SP][SP], U [M][SP][SP], row-major.
// After the factorisation D_k holds D_k^-1 of the level where node k was eliminated, L_k / U_k of an eliminated node
// hold X_k / Y_k; work (per instance `wstride`): Cl [M][SP][SP], Cr [M][SP][SP].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/cfx.h"
#include "cfx_internal.h"

namespace cfx_chain {

typedef double d4 __attribute__((ext_vector_type(4)));

struct Chain {
    double *D, *L, *U;  // instance b at + b * stride
    double *Cl, *Cr;    // instance b at + b * wstride
    int64_t stride, wstride;
    int M;
};

// One 16 x 16 tile of C = A B over K = SP (A row-major lda, B row-major ldb), B's column block in registers:
// breg[kk] = B[4 kk + (lane >> 4)][16 J + (lane & 15)].  v_mfma_f64_16x16x4f64: lane l holds A[l & 15][l >> 4] and
// B[l >> 4][l & 15] of each 16 x 4 / 4 x 16 step; result element r of lane l is C[(l >> 4) + 4 r][l & 15].
template <int SP, class AF>
__device__ __forceinline__ d4 tile_mm(const AF& a_at, const double (&breg)[SP / 4], int I, d4 acc) {
    const int lane = threadIdx.x & 63;
    const int r = 16 * I + (lane & 15), kq = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < SP / 4; ++kk) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a_at(r, 4 * kk + kq), breg[kk], acc, 0, 0, 0);
    return acc;
}

template <int SP>
__device__ __forceinline__ void load_bcol(const double* __restrict__ B, int J, double (&breg)[SP / 4]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int kk = 0; kk < SP / 4; ++kk) breg[kk] = B[(4 * kk + (lane >> 4)) * SP + 16 * J + (lane & 15)];
}

template <int SP>
__device__ __forceinline__ void store_tile(double* __restrict__ C, int I, int J, d4 v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < 4; ++r) C[(16 * I + (lane >> 4) + 4 * r) * SP + 16 * J + (lane & 15)] = v[r];
}

constexpr int kNT = 256;  // threads per workgroup (4 waves)

// Eliminate nodes i = first + step * blockIdx.x (instance blockIdx.y): D_i <- D_i^-1, L_i <- D_i^-1 L_i (when node
// i - h exists), U_i <- D_i^-1 U_i (when node i + h exists).  A zero pivot sets info[b] (0-based slot + 1) if unset.
template <int SP>
__global__ void __launch_bounds__(kNT) k_chain_elim(Chain C, int first, int step, int h, int32_t* __restrict__ info) {
    // In-place Gauss-Jordan with partial pivoting (first largest |A(r, k)|, r >= k; columns unscrambled at the end),
    // the matrix in registers: thread t owns row t % SP and the columns cg + G c (cg = t / SP, G = kNT / SP groups).
    // Per pivot column three barriers: the column (double-buffered, written by its owners at the end of the previous
    // step) -> wave 0's argmax -> the pivot row and row k through LDS -> every thread updates its own entries.
    constexpr int G = kNT / SP, CW = (SP + G - 1) / G, SPP = G * CW;  // SPP: columns padded to the groups
    __shared__ double A[SP][SP + 1];
    __shared__ double colv[2][SP];
    __shared__ double rowp[SPP], rowk[SPP];
    __shared__ int piv[SP], perm[SP];
    __shared__ int s_p;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int i = first + step * blockIdx.x;
    const int64_t b = blockIdx.y;
    if (i >= C.M) return;
    constexpr int64_t NB = (int64_t)SP * SP;
    double* D = C.D + b * C.stride + i * NB;
    const int row = t % SP, cg = min(t / SP, G - 1);
    const bool own = t < G * SP;  // threads past G SP groups own nothing (they shadow the last group, never store)
    double a[CW];
#pragma unroll
    for (int c = 0; c < CW; ++c) {
        const int j = cg + G * c;
        a[c] = j < SP ? D[(int64_t)row * SP + j] : 0.0;
    }
    if (own && cg == 0) colv[0][row] = a[0];                           // column 0
    for (int j = SP + t; j < SPP; j += kNT) rowp[j] = rowk[j] = 0.0;  // padding columns stay zero
    __syncthreads();
    int sing = 0;
    {
#pragma unroll 1
        for (int k = 0; k < SP; ++k) {
            const int par = k & 1;
            if (wave == 0) {
                double av = -1.0;
                int ai = SP;
                for (int r = k + lane; r < SP; r += 64) {
                    const double v = fabs(colv[par][r]);
                    if (v > av) av = v, ai = r;
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const double ov = __shfl_xor(av, o);
                    const int oi = __shfl_xor(ai, o);
                    if (ov > av || (ov == av && oi < ai)) av = ov, ai = oi;
                }
                if (lane == 0) s_p = piv[k] = ai;
            }
            __syncthreads();
            const int p = s_p;
            if (own && (row == p || row == k)) {
                double* dst = row == p ? rowp : rowk;
#pragma unroll
                for (int c = 0; c < CW; ++c) dst[cg + G * c] = a[c];
            }
            __syncthreads();
            const double pv = colv[par][p];
            if (pv == 0.0 && !sing) sing = k + 1;
            const double inv = pv != 0.0 ? 1.0 / pv : 0.0;
            // row p now holds the old row k (its column-k value colv[k]); row k the scaled pivot row.  Branch-free:
            // all LDS reads first, then selects
            const bool isk = row == k, isp = row == p && p != k;
            const double f = colv[par][isp ? k : row];
            double pr[CW], rk[CW];
#pragma unroll
            for (int c = 0; c < CW; ++c) pr[c] = rowp[cg + G * c];
#pragma unroll
            for (int c = 0; c < CW; ++c) rk[c] = rowk[cg + G * c];
            const int kn = k + 1;
            double nxt = 0.0;
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                const int j = cg + G * c;
                const double prc = (j == k ? 1.0 : pr[c]) * inv;
                const double src = isp ? rk[c] : a[c];
                const double upd = (j == k ? 0.0 : src) - f * prc;
                a[c] = isk ? prc : upd;
                nxt = (j == kn) ? a[c] : nxt;
            }
            // the next pivot column, by its owners, into the other buffer
            if (own && kn < SP && cg == kn % G) colv[par ^ 1][row] = nxt;
            __syncthreads();
        }
    }
    // columns: final column j is the eliminated matrix's column perm[j] (the interchanges undone in reverse order)
    if (t == 0) {
        for (int j = 0; j < SP; ++j) perm[j] = j;
        for (int k = SP - 1; k >= 0; --k) {
            const int q = piv[k], tmp = perm[k];
            perm[k] = perm[q];
            perm[q] = tmp;
        }
    }
    if (own) {
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            const int j = cg + G * c;
            if (j < SP) A[row][j] = a[c];
        }
    }
    __syncthreads();
    if (own) {
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            const int j = cg + G * c;
            if (j < SP) a[c] = A[row][perm[j]];
        }
    }
    __syncthreads();
    if (own) {
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            const int j = cg + G * c;
            if (j < SP) A[row][j] = a[c];
        }
    }
    __syncthreads();
    if (t == 0 && sing && info && info[b] == 0) info[b] = (int32_t)(i * SP + sing);
    for (int e = t; e < SP * SP; e += kNT) D[e] = A[e / SP][e % SP];
    // X_i = D_i^-1 L_i, Y_i = D_i^-1 U_i in place: a wave owns whole column blocks J (read into registers first)
    auto a_at = [&](int r, int c) { return A[r][c]; };
    for (int side = 0; side < 2; ++side) {
        if (side == 0 ? i - h < 0 : i + h >= C.M) continue;
        double* Bm = (side == 0 ? C.L : C.U) + b * C.stride + i * NB;
        for (int J = wave; J < SP / 16; J += kNT / 64) {
            double breg[SP / 4];
            load_bcol<SP>(Bm, J, breg);
#pragma unroll 1
            for (int I = 0; I < SP / 16; ++I) {
                d4 acc = {0.0, 0.0, 0.0, 0.0};
                acc = tile_mm<SP>(a_at, breg, I, acc);
                store_tile<SP>(Bm, I, J, acc);
            }
        }
    }
}

// Survivors p = 2 h blockIdx.x of level h (instance blockIdx.y) take the Schur complement of their eliminated
// neighbours i = p + h and j = p - h.  The pre-update U_p / L_p are copied to Cl_i / Cr_j first; every product reads
// its left operand from those copies, so the in-place updates of U_p / L_p never race with their reads.
template <int SP>
__global__ void __launch_bounds__(kNT) k_chain_upd(Chain C, int h) {
    const int t = threadIdx.x, wave = t >> 6;
    const int p = 2 * h * blockIdx.x;
    const int64_t b = blockIdx.y;
    if (p >= C.M) return;
    constexpr int64_t NB = (int64_t)SP * SP;
    const int i = p + h, j = p - h;
    const bool hi = i < C.M, hj = j >= 0;
    const bool hyi = hi && i + h < C.M;  // Y_i exists (node i + h = p + 2h)
    double* Dp = C.D + b * C.stride + p * NB;
    double* Up = C.U + b * C.stride + p * NB;
    double* Lp = C.L + b * C.stride + p * NB;
    double* Cli = hi ? C.Cl + b * C.wstride + i * NB : nullptr;
    double* Crj = hj ? C.Cr + b * C.wstride + j * NB : nullptr;
    for (int e = t; e < SP * SP; e += kNT) {
        if (hi) Cli[e] = Up[e];
        if (hj) Crj[e] = Lp[e];
    }
    __threadfence_block();
    __syncthreads();
    const double* Xi = hi ? C.L + b * C.stride + i * NB : nullptr;
    const double* Yi = hyi ? C.U + b * C.stride + i * NB : nullptr;
    const double* Xj = hj ? C.L + b * C.stride + j * NB : nullptr;
    const double* Yj = hj ? C.U + b * C.stride + j * NB : nullptr;
    auto cl_at = [&](int r, int c) { return Cli[r * SP + c]; };
    auto cr_at = [&](int r, int c) { return Crj[r * SP + c]; };
    for (int J = wave; J < SP / 16; J += kNT / 64) {
        double breg[SP / 4];
        d4 accD[SP / 16];
#pragma unroll
        for (int I = 0; I < SP / 16; ++I) accD[I] = d4{0.0, 0.0, 0.0, 0.0};
        if (hi) {  // D_p -= U_p X_i
            load_bcol<SP>(Xi, J, breg);
#pragma unroll
            for (int I = 0; I < SP / 16; ++I) accD[I] = tile_mm<SP>(cl_at, breg, I, accD[I]);
        }
        if (hj) {  // D_p -= L_p Y_j
            load_bcol<SP>(Yj, J, breg);
#pragma unroll
            for (int I = 0; I < SP / 16; ++I) accD[I] = tile_mm<SP>(cr_at, breg, I, accD[I]);
        }
        if (hi || hj) {
            const int lane = t & 63;
#pragma unroll
            for (int I = 0; I < SP / 16; ++I)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t e = (16 * I + (lane >> 4) + 4 * r) * SP + 16 * J + (lane & 15);
                    Dp[e] -= accD[I][r];
                }
        }
        if (hi) {  // U_p <- -U_p Y_i (zero when node p + 2h does not exist)
            if (hyi) load_bcol<SP>(Yi, J, breg);
#pragma unroll 1
            for (int I = 0; I < SP / 16; ++I) {
                d4 acc = {0.0, 0.0, 0.0, 0.0};
                if (hyi) acc = tile_mm<SP>(cl_at, breg, I, acc);
                store_tile<SP>(Up, I, J, -acc);
            }
        }
        if (hj) {  // L_p <- -L_p X_j
            load_bcol<SP>(Xj, J, breg);
#pragma unroll 1
            for (int I = 0; I < SP / 16; ++I) {
                d4 acc = {0.0, 0.0, 0.0, 0.0};
                acc = tile_mm<SP>(cr_at, breg, I, acc);
                store_tile<SP>(Lp, I, J, -acc);
            }
        }
    }
}

// y = M x for an SP x SP row-major matrix and an LDS vector, rows over threads [t0, t0 + SP)
template <int SP>
__device__ __forceinline__ double row_dot(const double* __restrict__ Mx, int r, const double* x) {
    double acc = 0.0;
    const double* row = Mx + (int64_t)r * SP;
#pragma unroll 8
    for (int k = 0; k < SP; ++k) acc = fma(row[k], x[k], acc);
    return acc;
}

struct Rhs {
    double* R;  // right-hand side c of instance b, node k at R + b r_inst + c r_rhs + k SP
    int64_t r_inst, r_rhs;
    double* T;  // t_i of the eliminated nodes, same shape as R (t_inst, t_rhs)
    int64_t t_inst, t_rhs;
};

// forward step of level h: survivor p (blockIdx.x), right-hand side blockIdx.y, instance blockIdx.z
template <int SP>
__global__ void __launch_bounds__(kNT) k_chain_fwd(Chain C, Rhs X, int h) {
    static_assert(SP <= 128, "rows over two thread halves");
    __shared__ double vi[SP], vj[SP], ti[SP], tj[SP];
    const int t = threadIdx.x;
    const int p = 2 * h * blockIdx.x;
    const int64_t b = blockIdx.z, c = blockIdx.y;
    if (p >= C.M) return;
    constexpr int64_t NB = (int64_t)SP * SP;
    const int i = p + h, j = p - h;
    const bool hi = i < C.M, hj = j >= 0;
    double* R = X.R + b * X.r_inst + c * X.r_rhs;
    double* T = X.T + b * X.t_inst + c * X.t_rhs;
    for (int r = t; r < SP; r += kNT) {
        vi[r] = hi ? R[(int64_t)i * SP + r] : 0.0;
        vj[r] = hj ? R[(int64_t)j * SP + r] : 0.0;
    }
    __syncthreads();
    if (t < SP) {
        if (hi) {
            const double v = row_dot<SP>(C.D + b * C.stride + i * NB, t, vi);
            ti[t] = v;
            T[(int64_t)i * SP + t] = v;
        }
    } else if (t >= 128 && t < 128 + SP) {
        if (hj) tj[t - 128] = row_dot<SP>(C.D + b * C.stride + j * NB, t - 128, vj);
    }
    __syncthreads();
    if (t < SP && (hi || hj)) {
        double acc = R[(int64_t)p * SP + t];
        if (hi) acc -= row_dot<SP>(C.Cl + b * C.wstride + i * NB, t, ti);
        if (hj) acc -= row_dot<SP>(C.Cr + b * C.wstride + j * NB, t, tj);
        R[(int64_t)p * SP + t] = acc;
    }
}

// node 0 after the last level: x_0 = D_0^-1 r_0
template <int SP>
__global__ void __launch_bounds__(kNT) k_chain_top(Chain C, Rhs X) {
    __shared__ double v[SP];
    const int t = threadIdx.x;
    const int64_t b = blockIdx.z, c = blockIdx.y;
    double* R = X.R + b * X.r_inst + c * X.r_rhs;
    for (int r = t; r < SP; r += kNT) v[r] = R[r];
    __syncthreads();
    if (t < SP) R[t] = row_dot<SP>(C.D + b * C.stride, t, v);
}

// backward step of level h: eliminated i = h + 2h blockIdx.x: x_i = t_i - X_i x_{i-h} - Y_i x_{i+h}
template <int SP>
__global__ void __launch_bounds__(kNT) k_chain_bwd(Chain C, Rhs X, int h) {
    __shared__ double xl[SP], xr[SP];
    const int t = threadIdx.x;
    const int i = h + 2 * h * blockIdx.x;
    const int64_t b = blockIdx.z, c = blockIdx.y;
    if (i >= C.M) return;
    constexpr int64_t NB = (int64_t)SP * SP;
    const bool hr = i + h < C.M;
    double* R = X.R + b * X.r_inst + c * X.r_rhs;
    const double* T = X.T + b * X.t_inst + c * X.t_rhs;
    for (int r = t; r < SP; r += kNT) {
        xl[r] = R[(int64_t)(i - h) * SP + r];
        xr[r] = hr ? R[(int64_t)(i + h) * SP + r] : 0.0;
    }
    __syncthreads();
    if (t < SP) {
        double acc = T[(int64_t)i * SP + t] - row_dot<SP>(C.L + b * C.stride + i * NB, t, xl);
        if (hr) acc -= row_dot<SP>(C.U + b * C.stride + i * NB, t, xr);
        R[(int64_t)i * SP + t] = acc;
    }
}

static int levels(int M) {
    int L = 0;
    while ((1 << L) < M) ++L;
    return L;
}

template <int SP>
static hipError_t factor_sp(const Chain& C, int64_t B, int32_t* info, hipStream_t s) {
    const int L = levels(C.M);
    for (int l = 0; l < L; ++l) {
        const int h = 1 << l;
        const int ne = (C.M - h + 2 * h - 1) / (2 * h), ns = (C.M + 2 * h - 1) / (2 * h);
        hipLaunchKernelGGL(k_chain_elim<SP>, dim3((unsigned)ne, (unsigned)B), dim3(kNT), 0, s, C, h, 2 * h, h, info);
        hipLaunchKernelGGL(k_chain_upd<SP>, dim3((unsigned)ns, (unsigned)B), dim3(kNT), 0, s, C, h);
    }
    hipLaunchKernelGGL(k_chain_elim<SP>, dim3(1, (unsigned)B), dim3(kNT), 0, s, C, 0, 1, 1 << L, info);
    return hipGetLastError();
}

template <int SP>
static hipError_t solve_sp(const Chain& C, int64_t B, const Rhs& X, int nrhs, hipStream_t s) {
    const int L = levels(C.M);
    for (int l = 0; l < L; ++l) {
        const int h = 1 << l;
        const int ns = (C.M + 2 * h - 1) / (2 * h);
        hipLaunchKernelGGL(k_chain_fwd<SP>, dim3((unsigned)ns, (unsigned)nrhs, (unsigned)B), dim3(kNT), 0, s, C, X, h);
    }
    hipLaunchKernelGGL(k_chain_top<SP>, dim3(1, (unsigned)nrhs, (unsigned)B), dim3(kNT), 0, s, C, X);
    for (int l = L - 1; l >= 0; --l) {
        const int h = 1 << l;
        const int ne = (C.M - h + 2 * h - 1) / (2 * h);
        hipLaunchKernelGGL(k_chain_bwd<SP>, dim3((unsigned)ne, (unsigned)nrhs, (unsigned)B), dim3(kNT), 0, s, C, X, h);
    }
    return hipGetLastError();
}

#define CFX_CHAIN_SP(F, ...)                                     \
    switch (sp) {                                                \
        case 16: e = F<16>(__VA_ARGS__); break;                  \
        case 32: e = F<32>(__VA_ARGS__); break;                  \
        case 48: e = F<48>(__VA_ARGS__); break;                  \
        case 64: e = F<64>(__VA_ARGS__); break;                  \
        case 80: e = F<80>(__VA_ARGS__); break;                  \
        case 96: e = F<96>(__VA_ARGS__); break;                  \
        case 112: e = F<112>(__VA_ARGS__); break;                \
        case 128: e = F<128>(__VA_ARGS__); break;                \
        default: e = hipErrorInvalidValue; break;                \
    }

}  // namespace cfx_chain

int cfx_chain_sp_ok(int32_t sp) { return sp >= 16 && sp <= 128 && sp % 16 == 0; }

int cfx_chain_factor_s(int64_t batch, int32_t M, int32_t sp, double* D, double* L, double* U, int64_t stride,
                       double* Cl, double* Cr, int64_t wstride, int32_t* info, void* stream) {
    if (batch < 1 || batch > 65535 || M < 1 || !cfx_chain_sp_ok(sp) || !D || !L || !U || !Cl || !Cr) {
        g_create_error = "cfx_chain_factor: invalid argument";
        return CFX_EINVAL;
    }
    const hipStream_t s = (hipStream_t)stream;
    if (info && hipMemsetAsync(info, 0, batch * sizeof(int32_t), s) != hipSuccess) {
        g_create_error = "cfx_chain_factor: hipMemsetAsync failed";
        return CFX_EHIP;
    }
    const cfx_chain::Chain C{D, L, U, Cl, Cr, stride, wstride, M};
    hipError_t e;
    CFX_CHAIN_SP(cfx_chain::factor_sp, C, batch, info, s)
    if (e != hipSuccess) {
        g_create_error = std::string("cfx_chain_factor: ") + hipGetErrorString(e);
        return CFX_EHIP;
    }
    return CFX_OK;
}

int cfx_chain_solve_s(int64_t batch, int32_t M, int32_t sp, const double* D, const double* L, const double* U,
                      int64_t stride, const double* Cl, const double* Cr, int64_t wstride, int32_t nrhs, double* R,
                      int64_t r_inst, int64_t r_rhs, double* T, int64_t t_inst, int64_t t_rhs, void* stream) {
    if (batch < 1 || batch > 65535 || M < 1 || !cfx_chain_sp_ok(sp) || nrhs < 1 || nrhs > 65535 || !R || !T) {
        g_create_error = "cfx_chain_solve: invalid argument";
        return CFX_EINVAL;
    }
    const cfx_chain::Chain C{const_cast<double*>(D), const_cast<double*>(L), const_cast<double*>(U),
                             const_cast<double*>(Cl), const_cast<double*>(Cr), stride, wstride, M};
    const cfx_chain::Rhs X{R, r_inst, r_rhs, T, t_inst, t_rhs};
    hipError_t e;
    CFX_CHAIN_SP(cfx_chain::solve_sp, C, batch, X, nrhs, (hipStream_t)stream)
    if (e != hipSuccess) {
        g_create_error = std::string("cfx_chain_solve: ") + hipGetErrorString(e);
        return CFX_EHIP;
    }
    return CFX_OK;
}

// ---- C ABI (include/cfx.h): contiguous layout [batch][M][sp][sp] per array ------------------------------------
extern "C" int cfx_btri_factor(int64_t batch, int32_t M, int32_t sp, double* D, double* L, double* U, double* work,
                               int32_t* info, void* stream) {
    if (!work) {
        g_create_error = "cfx_btri_factor: work is NULL";
        return CFX_EINVAL;
    }
    const int64_t st = (int64_t)M * sp * sp;
    return cfx_chain_factor_s(batch, M, sp, D, L, U, st, work, work + batch * st, st, info, stream);
}

extern "C" int cfx_btri_solve(int64_t batch, int32_t M, int32_t sp, const double* D, const double* L, const double* U,
                              const double* work, int32_t nrhs, double* rhs, double* scratch, void* stream) {
    if (!work) {
        g_create_error = "cfx_btri_solve: work is NULL";
        return CFX_EINVAL;
    }
    const int64_t st = (int64_t)M * sp * sp, nv = (int64_t)M * sp;
    return cfx_chain_solve_s(batch, M, sp, D, L, U, st, work, work + batch * st, st, nrhs, rhs, nrhs * nv, nv, scratch,
                             nrhs * nv, nv, stream);
}
