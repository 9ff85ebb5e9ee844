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
// submatrix over a contiguous range of nodes is a KKT matrix whose constraint block has full structural row rank, so
// the pivot blocks below are structurally nonsingular and the factorisation pivots within each block only.  That is
// not numerical nonsingularity: a block [W_k J_k^T; J_k -dc] whose W_k is singular on null(J_k) is (nearly) singular,
// and no pivoting across blocks rescues it.  An exactly zero pivot, or a column with no finite pivot candidate, is
// reported in info (the interior point then raises its regularisation dw); the inertia test (cfx_btri_inertia) counts
// such blocks' eigenvalues, the default curvature test sees them only through the step they produce.
//
// Block cyclic reduction (log2 M levels).  Level l (h = 2^l) eliminates the nodes i = h mod 2h, every one
// independently:  D_i^-1 (Gauss-Jordan with partial pivoting in LDS), X_i = D_i^-1 L_i, Y_i = D_i^-1 U_i (FP64 MFMA,
// v_mfma_f64_16x16x4f64), and each survivor p = 0 mod 2h takes the Schur complement of its two eliminated neighbours
// i = p + h, j = p - h:
//     D_p -= U_p X_i + L_p Y_j,   U_p <- -U_p Y_i  (now coupling to p + 2h),   L_p <- -L_p X_j  (to p - 2h)
// four SP x SP x SP products on the matrix cores.  The updated couplings go to work slots (cur_u / cur_l below), so
// the pre-update U_p, L_p stay in place for the solves.
// After the last level node 0 alone remains and is inverted.  Level 0 of the reaching task (M = 1,501, SP = 80) runs
// 750 eliminations side by side: the chip is full where the band factorisation ran one workgroup.
// Solve: forward over the levels (t_i = D_i^-1 r_i, r_p -= U_p t_i + L_p t_j), x_0 = D_0^-1 r_0, backward
// (x_i = t_i - X_i x_{i-h} - Y_i x_{i+h}).
//
// Storage (per instance, instance stride `stride` doubles): D [M][SP][SP], L [M][SP][SP], U [M][SP][SP], row-major.
// Work (per instance `wstride`): Cl [M][SP][SP], Cr [M][SP][SP].  After the factorisation D_k holds D_k^-1 of the
// level where node k was eliminated, and node k's couplings at that level (cur_u / cur_l: in U / L for level 0, in
// Cl / Cr above) hold X_k / Y_k.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/cfx.h"
#include "cfx_inertia.h"
#include "cfx_internal.h"

namespace cfx_chain {

typedef double d4 __attribute__((ext_vector_type(4)));

struct Chain {
    double *D, *L, *U;  // instance b at + b * stride
    double *Cl, *Cr;    // instance b at + b * wstride
    int64_t stride, wstride;
    int M;
};

// Where node k's couplings live at the start of level h (h = 1: the input blocks; after level h / 2 the Schur update
// wrote them to the work slot of the node it eliminated: U_k to Cl[k + h/2], L_k to Cr[k - h/2]).  A node eliminated
// at level h keeps X_k = D_k^-1 L_k, Y_k = D_k^-1 U_k in those same places, and the pre-update couplings a survivor's
// solve step needs stay where they are — no block is copied.  Work slot Cl[x] (Cr[x]) is written at one level only,
// the one at which x is eliminated.
template <int SP>
__device__ __forceinline__ double* cur_u(const Chain& C, int64_t b, int k, int h) {
    constexpr int64_t NB = (int64_t)SP * SP;
    return h == 1 ? C.U + b * C.stride + k * NB : C.Cl + b * C.wstride + (k + h / 2) * NB;
}
template <int SP>
__device__ __forceinline__ double* cur_l(const Chain& C, int64_t b, int k, int h) {
    constexpr int64_t NB = (int64_t)SP * SP;
    return h == 1 ? C.L + b * C.stride + k * NB : C.Cr + b * C.wstride + (k - h / 2) * NB;
}

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

// Pivot key of a candidate row r with value v: |v| with its 7 low mantissa bits replaced by 127 - r (non-negative
// doubles order like their bits), -1 for a non-finite value.  The wave maximum picks the largest |v| (to 2^-45), ties
// to the lowest row.  (A 32-bit key of the high word, 2^-13, took one instruction less per DPP step but moved the
// reaching task's iteration path measurably; not kept.)
__device__ __forceinline__ double pivot_key(double v, int r) {
    const uint64_t bits = (uint64_t)__double_as_longlong(fabs(v));
    if (bits >= 0x7ff0000000000000ull) return -1.0;
    return __longlong_as_double((long long)((bits & ~0x7Full) | (uint64_t)(127 - r)));
}

// Maximum of v over the 64 lanes (every lane gets it): DPP max-scan within rows of 16 lanes, row broadcasts to lane 63,
// readlane.  Lanes a shift leaves without a source keep their own value.
#define CFX_DPP_MAX(v, CTRL, RM, BM)                                                                              \
    do {                                                                                                          \
        const int lo_ = __double2loint(v), hi_ = __double2hiint(v);                                               \
        const int slo_ = __builtin_amdgcn_update_dpp(lo_, lo_, CTRL, RM, BM, false);                              \
        const int shi_ = __builtin_amdgcn_update_dpp(hi_, hi_, CTRL, RM, BM, false);                              \
        v = fmax(v, __hiloint2double(shi_, slo_));                                                                \
    } while (0)
__device__ __forceinline__ double wave_max(double v) {
    CFX_DPP_MAX(v, 0x111, 0xf, 0xf);  // row_shr:1
    CFX_DPP_MAX(v, 0x112, 0xf, 0xf);  // row_shr:2
    CFX_DPP_MAX(v, 0x114, 0xf, 0xf);  // row_shr:4
    CFX_DPP_MAX(v, 0x118, 0xf, 0xf);  // row_shr:8  (lane 15 of each row: the row's maximum)
    CFX_DPP_MAX(v, 0x142, 0xa, 0xf);  // row_bcast:15 into rows 1 and 3
    CFX_DPP_MAX(v, 0x143, 0xc, 0xf);  // row_bcast:31 into rows 2 and 3 (lane 63: the wave's maximum)
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), 63), hi = __builtin_amdgcn_readlane(__double2hiint(v), 63);
    return __hiloint2double(hi, lo);
}

constexpr int kNT = 256;  // threads per workgroup (4 waves)

__device__ __forceinline__ double readlane_d(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}

// Eliminate nodes i = first + step * blockIdx.x (instance blockIdx.y): D_i <- D_i^-1, L_i <- D_i^-1 L_i (when node
// i - h exists), U_i <- D_i^-1 U_i (when node i + h exists).  A zero pivot sets info[b] (0-based slot + 1) if unset.
template <int SP>
__global__ void __launch_bounds__(kNT) k_chain_elim(Chain C, int first, int step, int h, int32_t* __restrict__ info) {
    // Blocked in-place Gauss-Jordan with partial pivoting (largest |A(r, k)| over the rows not yet pivots, to within
    // pivot_key's 2^-45, ties to the lowest row) without moving rows: step k pivots on physical row P_k, so the array
    // ends as (Q D)^-1 = D^-1 Q^T, D^-1[k][j] = array[P_k][s_j] with s_j the step at which row j was pivot (undone at the
    // end).  The matrix sits in LDS; the SP columns go in panels of 16.  Panel j: wavefront 0 runs its 16 pivot steps
    // on the panel's columns alone, in registers (lane l holds rows l and l + 64; DPP pivot search, the pivot row by
    // readlane, no LDS and no barrier per step).  The composite of the 16 steps acts on every other column as
    // M <- Z + W V, W the processed panel columns (SP x 16), V the 16 pivot rows before the panel, Z the column with
    // those rows zeroed — a rank-16 update on v_mfma_f64_16x16x4f64, each wave owning whole 16-column blocks (it reads
    // V of its blocks before writing them: no barrier between).  Two barriers per panel instead of two per column
    // (round 5's column-by-column version, register tiles: 83 us per 80 x 80 block, issue- and barrier-bound).
    constexpr int T = SP / 16;
    static_assert(SP % 16 == 0 && SP <= 128 && kNT == 256, "16-column panels; 7-bit row index in the pivot key");
    constexpr int LDA = SP + 1;
    __shared__ double A[SP * LDA];
    // P_k (row pivoted at step k), s_j (step at which row j was pivot); bytes
    __shared__ uint8_t prow[SP], pstep[SP];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int i = first + step * blockIdx.x;
    const int64_t b = blockIdx.y;
    if (i >= C.M) return;
    constexpr int64_t NB = (int64_t)SP * SP;
    double* D = C.D + b * C.stride + i * NB;
    for (int e = t; e < SP * SP; e += kNT) A[(e / SP) * LDA + e % SP] = D[e];
    for (int r = t; r < SP; r += kNT) pstep[r] = 255;
    __syncthreads();
    int sing = 0;                       // (wave 0)
    bool used0 = false, used1 = false;  // (wave 0) rows lane and lane + 64 already pivots
    const bool has0 = lane < SP, has1 = lane + 64 < SP;
#pragma unroll 1
    for (int j = 0; j < T; ++j) {
        if (wave == 0) {
            double a0[16], a1[16];
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                a0[c] = has0 ? A[lane * LDA + 16 * j + c] : 0.0;
                a1[c] = has1 ? A[(lane + 64) * LDA + 16 * j + c] : 0.0;
            }
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) {
                const int k = 16 * j + kk;
                double key = -1.0;
                if (has0 && !used0) key = pivot_key(a0[kk], lane);
                if (has1 && !used1) key = fmax(key, pivot_key(a1[kk], lane + 64));
                key = wave_max(key);
                int p;
                if (key >= 0.0) {
                    p = 127 - (int)((uint64_t)__double_as_longlong(key) & 0x7Full);
                } else {  // no finite candidate: singular; the lowest unused row keeps the indices in range
                    const unsigned long long m0 = __ballot(has0 && !used0), m1 = __ballot(has1 && !used1);
                    p = m0 ? __ffsll((long long)m0) - 1 : 64 + __ffsll((long long)m1) - 1;
                    if (!sing) sing = k + 1;
                }
                used0 = used0 || p == lane;
                used1 = used1 || p == lane + 64;
                if (lane == 0) prow[k] = (uint8_t)p, pstep[p] = (uint8_t)k;
                double prv[16];  // the pivot row's panel values (wave-uniform)
                if (p < 64) {
#pragma unroll
                    for (int c = 0; c < 16; ++c) prv[c] = readlane_d(a0[c], p);
                } else {
#pragma unroll
                    for (int c = 0; c < 16; ++c) prv[c] = readlane_d(a1[c], p - 64);
                }
                const double pv = prv[kk];
                if (pv == 0.0 && !sing) sing = k + 1;
                const double inv = pv != 0.0 ? 1.0 / pv : 0.0;
                double sc[16];  // the scaled pivot row, column k replaced by 1 / pv
#pragma unroll
                for (int c = 0; c < 16; ++c) sc[c] = c == kk ? inv : prv[c] * inv;
                // every row r -= A(r, k) x the scaled pivot row; column k -> -A(r, k) / pv; row p -> the scaled row
                const bool ip0 = lane == p, ip1 = lane + 64 == p;
                const double m0 = a0[kk], m1 = a1[kk];
#pragma unroll
                for (int c = 0; c < 16; ++c) {
                    if (c == kk) continue;
                    a0[c] = ip0 ? sc[c] : fma(-m0, sc[c], a0[c]);
                    a1[c] = ip1 ? sc[c] : fma(-m1, sc[c], a1[c]);
                }
                a0[kk] = ip0 ? inv : -m0 * inv;
                a1[kk] = ip1 ? inv : -m1 * inv;
            }
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                if (has0) A[lane * LDA + 16 * j + c] = a0[c];
                if (has1) A[(lane + 64) * LDA + 16 * j + c] = a1[c];
            }
        }
        __syncthreads();
        // the other column blocks: M <- Z + W V (wave w: blocks w, w + 4, ... other than j)
        for (int q = wave; q < T - 1; q += kNT / 64) {
            const int Jc = q < j ? q : q + 1;
            double breg[4];  // V[4 kk + lane / 16][16 Jc + lane % 16]: pivot row of step 16 j + 4 kk + lane / 16
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) breg[kk] = A[prow[16 * j + 4 * kk + (lane >> 4)] * LDA + 16 * Jc + (lane & 15)];
#pragma unroll 1
            for (int I = 0; I < T; ++I) {
                d4 acc;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 16 * I + (lane >> 4) + 4 * r;
                    const int ps = pstep[row];
                    const bool piv = ps >= 16 * j && ps < 16 * j + 16;  // a pivot row of this panel: zeroed (Z)
                    acc[r] = piv ? 0.0 : A[row * LDA + 16 * Jc + (lane & 15)];
                }
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(16 * I + (lane & 15)) * LDA + 16 * j + 4 * kk + (lane >> 4)],
                                                               breg[kk], acc, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; ++r) A[(16 * I + (lane >> 4) + 4 * r) * LDA + 16 * Jc + (lane & 15)] = acc[r];
            }
        }
        __syncthreads();
    }
    // D^-1[r][c] = array[P_r][s_c]
    const int tr = t >> 4, tc = t & 15;
    double a[T][T];
#pragma unroll
    for (int ii = 0; ii < T; ++ii)
#pragma unroll
        for (int jj = 0; jj < T; ++jj) a[ii][jj] = A[prow[tr + 16 * ii] * LDA + pstep[tc + 16 * jj]];
    __syncthreads();
#pragma unroll
    for (int ii = 0; ii < T; ++ii)
#pragma unroll
        for (int jj = 0; jj < T; ++jj) A[(tr + 16 * ii) * LDA + tc + 16 * jj] = a[ii][jj];
    __syncthreads();
    if (t == 0 && sing && info && info[b] == 0) info[b] = (int32_t)(i * SP + sing);
    for (int e = t; e < SP * SP; e += kNT) D[e] = A[(e / SP) * LDA + e % SP];
    // X_i = D_i^-1 L_i, Y_i = D_i^-1 U_i in place: items (side, column block J) over the waves, each read into
    // registers before its tiles are stored
    auto a_at = [&](int r, int c) { return A[r * LDA + c]; };
    const bool xl = i - h >= 0, yu = i + h < C.M;
    for (int it = wave; it < 2 * (SP / 16); it += kNT / 64) {
        const int side = it / (SP / 16), J = it % (SP / 16);
        if (side == 0 ? !xl : !yu) continue;
        double* Bm = side == 0 ? cur_l<SP>(C, b, i, h) : cur_u<SP>(C, b, i, h);
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

// Survivors p = 2 h blockIdx.x of level h (instance blockIdx.y) take the Schur complement of their eliminated
// neighbours i = p + h and j = p - h, in three workgroups per survivor (blockIdx.z):
//   0: D_p -= U_p X_i + L_p Y_j      1: U_p' = -U_p Y_i (zero without node p + 2h)      2: L_p' = -L_p X_j
// with U_p' / L_p' written to the work slots Cl[i] / Cr[j] (cur_u / cur_l), so no workgroup reads what another
// writes and U_p / L_p stay for the solves.  Each product stages its two operands in LDS (the left operand read by every tile, the
// right one too when both fit: SP <= 96) and spreads its 16 x 16 output tiles over the four waves; the sums run in
// the order of one K loop per product, products in the order above.  (Round 5 first version: one workgroup per
// survivor, left operands read from global memory per MFMA, output column blocks per wave — 115 us per tail level
// for SP = 80, where the FP64 matrix cores need ~7.)
// BLDS: the right operand staged in LDS too (when both fit: SP <= 96).  The launcher stages it only for levels with
// fewer than kUpdGlobalB survivors: at the wide levels the doubled LDS halves the workgroups per CU, and reading the
// right operand from L2 is faster (reaching task, micro: level 0 249 -> 155 us, level 1 108 -> 86 us; the tail
// levels the other way, 35 vs 48 us)
constexpr int kUpdGlobalB = 256;
template <int SP>
constexpr bool chain_b_fits() {
    return 2 * SP * (SP + 1) * 8 <= 150 * 1024;
}
template <int SP, bool BLDS>
constexpr size_t chain_upd_lds() {
    return (size_t)(BLDS ? 2 : 1) * SP * (SP + 1) * sizeof(double);
}
template <int SP, bool BLDS>
__global__ void __launch_bounds__(kNT) k_chain_upd(Chain C, int h) {
    constexpr int T16 = SP / 16, NT = T16 * T16, TPW = (NT + 3) / 4;  // output tiles, per wave
    constexpr int LD = SP + 1;
    constexpr bool BL = BLDS && chain_b_fits<SP>();
    extern __shared__ double sm[];
    double* sA = sm;
    double* sB = sm + SP * LD;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const int p = 2 * h * blockIdx.x, part = blockIdx.z;
    const int64_t b = blockIdx.y;
    if (p >= C.M) return;
    constexpr int64_t NB = (int64_t)SP * SP;
    const int i = p + h, j = p - h;
    const bool hi = i < C.M, hj = j >= 0;
    const bool hyi = hi && i + h < C.M;  // Y_i exists (node i + h = p + 2h)
    if ((part == 0 && !hi && !hj) || (part == 1 && !hi) || (part == 2 && !hj)) return;
    const double* Up = hi ? cur_u<SP>(C, b, p, h) : nullptr;  // the pre-update couplings (stay in place)
    const double* Lp = hj ? cur_l<SP>(C, b, p, h) : nullptr;
    d4 acc[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
    // acc[q] += A Bm over the wave's tiles q (tile wave + 4 q: I = tile / T16, J = tile % T16)
    auto product = [&](const double* __restrict__ Ag, const double* __restrict__ Bg) {
        __syncthreads();  // the previous product's readers are done with the buffers
        for (int e = t; e < SP * SP; e += kNT) {
            const int r = e / SP, c = e - r * SP;
            sA[r * LD + c] = Ag[e];
            if constexpr (BL) sB[r * LD + c] = Bg[e];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < TPW; ++q) {
            const int tile = wave + 4 * q;
            if (tile < NT) {
                const int I = tile / T16, J = tile % T16;
                const int ra = 16 * I + (lane & 15), kq = lane >> 4, cb = 16 * J + (lane & 15);
                d4 a = acc[q];
#pragma unroll
                for (int kk = 0; kk < SP / 4; ++kk) {
                    const double bv = BL ? sB[(4 * kk + kq) * LD + cb] : Bg[(4 * kk + kq) * SP + cb];
                    a = __builtin_amdgcn_mfma_f64_16x16x4f64(sA[ra * LD + 4 * kk + kq], bv, a, 0, 0, 0);
                }
                acc[q] = a;
            }
        }
    };
    double* out;
    if (part == 0) {
        if (hi) product(Up, cur_l<SP>(C, b, i, h));  // U_p X_i
        if (hj) product(Lp, cur_u<SP>(C, b, j, h));  // L_p Y_j
        out = C.D + b * C.stride + p * NB;
    } else if (part == 1) {
        if (hyi) product(Up, cur_u<SP>(C, b, i, h));  // U_p Y_i
        out = C.Cl + b * C.wstride + i * NB;            // = cur_u(p, 2h)
    } else {
        product(Lp, cur_l<SP>(C, b, j, h));  // L_p X_j
        out = C.Cr + b * C.wstride + j * NB;  // = cur_l(p, 2h)
    }
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int tile = wave + 4 * q;
        if (tile < NT) {
            const int I = tile / T16, J = tile % T16;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t e = (16 * I + (lane >> 4) + 4 * r) * SP + 16 * J + (lane & 15);
                if (part == 0) out[e] -= acc[q][r];
                else out[e] = -acc[q][r];
            }
        }
    }
}

// y = M x for an SP x SP row-major matrix and an LDS vector, rows over threads [t0, t0 + SP)
template <int SP>
// (four interleaved partial sums: the single chain of sp dependent FMAs was the solve kernels' latency)
__device__ __forceinline__ double row_dot(const double* __restrict__ Mx, int r, const double* x) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    const double* row = Mx + (int64_t)r * SP;
#pragma unroll 4
    for (int k = 0; k < SP; k += 4) {
        a0 = fma(row[k], x[k], a0);
        a1 = fma(row[k + 1], x[k + 1], a1);
        a2 = fma(row[k + 2], x[k + 2], a2);
        a3 = fma(row[k + 3], x[k + 3], a3);
    }
    return (a0 + a1) + (a2 + a3);
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
    // the two coupling products in the two thread halves, summed through LDS (vi / vj are free again)
    if (t < SP) {
        if (hi) vi[t] = row_dot<SP>(cur_u<SP>(C, b, p, h), t, ti);
    } else if (t >= 128 && t < 128 + SP) {
        if (hj) vj[t - 128] = row_dot<SP>(cur_l<SP>(C, b, p, h), t - 128, tj);
    }
    __syncthreads();
    if (t < SP && (hi || hj)) {
        double acc = R[(int64_t)p * SP + t];
        if (hi) acc -= vi[t];
        if (hj) acc -= vj[t];
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
    const bool hr = i + h < C.M;
    double* R = X.R + b * X.r_inst + c * X.r_rhs;
    const double* T = X.T + b * X.t_inst + c * X.t_rhs;
    for (int r = t; r < SP; r += kNT) {
        xl[r] = R[(int64_t)(i - h) * SP + r];
        xr[r] = hr ? R[(int64_t)(i + h) * SP + r] : 0.0;
    }
    __syncthreads();
    __shared__ double yl[SP], yr[SP];
    if (t < SP) yl[t] = row_dot<SP>(cur_l<SP>(C, b, i, h), t, xl);
    else if (t >= 128 && t < 128 + SP && hr) yr[t - 128] = row_dot<SP>(cur_u<SP>(C, b, i, h), t - 128, xr);
    __syncthreads();
    if (t < SP) {
        double acc = T[(int64_t)i * SP + t] - yl[t];
        if (hr) acc -= yr[t];
        R[(int64_t)i * SP + t] = acc;
    }
}

static int levels(int M) {
    int L = 0;
    while ((1 << L) < M) ++L;
    return L;
}

// the dynamic LDS limit of one k_chain_upd instantiation raised (once) when it needs more than the default 64 KiB
template <int SP, bool BL>
static hipError_t allow_upd_lds() {
    if (chain_upd_lds<SP, BL>() <= 65536) return hipSuccess;
    static const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_chain_upd<SP, BL>),
                                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                                    (int)chain_upd_lds<SP, BL>());
    return e;
}

template <int SP>
static hipError_t factor_sp(const Chain& C, int64_t B, int32_t* info, hipStream_t s) {
    const int L = levels(C.M);
    constexpr bool FITS = chain_b_fits<SP>();
    // both instantiations the levels below can launch (SP = 96 without BLDS needs 74,496 B)
    hipError_t e = allow_upd_lds<SP, FITS>();
    if (e == hipSuccess) e = allow_upd_lds<SP, false>();
    if (e != hipSuccess) return e;
    for (int l = 0; l < L; ++l) {
        const int h = 1 << l;
        const int ne = (C.M - h + 2 * h - 1) / (2 * h), ns = (C.M + 2 * h - 1) / (2 * h);
        hipLaunchKernelGGL(k_chain_elim<SP>, dim3((unsigned)ne, (unsigned)B), dim3(kNT), 0, s, C, h, 2 * h, h, info);
        if (FITS && ns < kUpdGlobalB)
            k_chain_upd<SP, FITS><<<dim3((unsigned)ns, (unsigned)B, 3), dim3(kNT), chain_upd_lds<SP, FITS>(), s>>>(C, h);
        else
            k_chain_upd<SP, false><<<dim3((unsigned)ns, (unsigned)B, 3), dim3(kNT), chain_upd_lds<SP, false>(), s>>>(C, h);
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

// Negative eigenvalues of the factored symmetric block-tridiagonal matrix (the interior point's inertia correction,
// cfx_inertia.h), added to neg[b]: block cyclic reduction is a sequence of congruences, so the matrix's inertia is the
// sum of its pivot blocks' (node k at its elimination level), and node k's D slot holds that block's inverse, whose
// inertia is the block's.  One workgroup per node (grid M x batch); the inverse is symmetrised on its way to LDS.
template <int SP>
constexpr size_t chain_inertia_lds() {
    return (size_t)SP * (SP + 1) * sizeof(double);
}
template <int SP>
__global__ void __launch_bounds__(kNT) k_chain_inertia(Chain C, int32_t* __restrict__ neg) {
    extern __shared__ double A[];
    constexpr int64_t NB = (int64_t)SP * SP;
    const int64_t b = blockIdx.y;
    const double* D = C.D + b * C.stride + blockIdx.x * NB;
    for (int e = threadIdx.x; e < SP * SP; e += kNT) {
        const int r = e / SP, c = e % SP;
        A[r * (SP + 1) + c] = 0.5 * (D[r * SP + c] + D[c * SP + r]);
    }
    __syncthreads();
    const int cnt = cfx_inertia::sym_neg_count(A, SP + 1, SP);
    if (threadIdx.x == 0 && cnt) atomicAdd(neg + b, cnt);
}

template <int SP>
static hipError_t inertia_sp(const Chain& C, int64_t B, int32_t* neg, hipStream_t s) {
    if (chain_inertia_lds<SP>() > 65536) {
        static const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_chain_inertia<SP>),
                                                        hipFuncAttributeMaxDynamicSharedMemorySize,
                                                        (int)chain_inertia_lds<SP>());
        if (e != hipSuccess) return e;
    }
    k_chain_inertia<SP><<<dim3((unsigned)C.M, (unsigned)B), dim3(kNT), chain_inertia_lds<SP>(), s>>>(C, neg);
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

int cfx_chain_inertia_s(int64_t batch, int32_t M, int32_t sp, const double* D, int64_t stride, int32_t* neg,
                        void* stream) {
    if (batch < 1 || batch > 65535 || M < 1 || !cfx_chain_sp_ok(sp) || !D || !neg) {
        g_create_error = "cfx_chain_inertia: invalid argument";
        return CFX_EINVAL;
    }
    const cfx_chain::Chain C{const_cast<double*>(D), nullptr, nullptr, nullptr, nullptr, stride, 0, M};
    hipError_t e;
    CFX_CHAIN_SP(cfx_chain::inertia_sp, C, batch, neg, (hipStream_t)stream)
    if (e != hipSuccess) {
        g_create_error = std::string("cfx_chain_inertia: ") + hipGetErrorString(e);
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

extern "C" int cfx_btri_inertia(int64_t batch, int32_t M, int32_t sp, const double* D, int32_t* neg, void* stream) {
    if (!neg || batch < 1 || batch > 65535) {
        g_create_error = "cfx_btri_inertia: invalid argument";
        return CFX_EINVAL;
    }
    if (hipMemsetAsync(neg, 0, batch * sizeof(int32_t), (hipStream_t)stream) != hipSuccess) {
        g_create_error = "cfx_btri_inertia: hipMemsetAsync failed";
        return CFX_EHIP;
    }
    return cfx_chain_inertia_s(batch, M, sp, D, (int64_t)M * sp * sp, neg, stream);
}
