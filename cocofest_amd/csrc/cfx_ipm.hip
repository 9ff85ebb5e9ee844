// cfx_ipm.hip — the batched interior-point driver of libcfx (include/cfx.h, cfx_ipm_*).
//
// Plays the part of `ocp.solve(Solver.IPOPT(...))` in the reference (bioptim's Ipopt interface, e.g.
// examples/getting_started/frequency_optimization.py:22): Ipopt's primal-dual barrier algorithm, for the B
// instances of one libcfx handle in lockstep, with every iteration resident on the handle's GPU.
//
// The algorithm is the one of cocofest_amd/solver.py (BatchedIpm), which is its executable specification and is
// cross-checked there against scipy's trust-constr on the CPU; this file restates it as a handful of fused HIP
// kernels around the libcfx callbacks and the batched band LU, so that one iteration is ~10 launches and two host
// reads of a 16-byte counter instead of ~1,500 small tensor operations:
//   eval_all_h(x) (g, J_g, f, grad f and the Hessian in one call: cfx_eval_all_h; eval_all then eval_h at the
//   start and after least-squares multipliers) -> k_ipm_begin (scaling, KKT error, convergence, barrier update, Sigma,
//   Newton rhs) -> k_ipm_kkt (band assembly + rhs permutation) -> band LU + solve -> k_ipm_curv (inertia)   [read]
//   k_ipm_dir (dz, fraction to the boundary, filter quantities, first trial point)
//   eval g, f (trial) -> k_ipm_accept (filter acceptance, second-order correction set-up)               [read]
//   k_ipm_update (filter augmentation, primal / dual steps, z safeguard)
// Rare paths (wrong inertia, backtracking, second-order corrections, restoration, least-squares multipliers) add
// launches only for the iterations that need them.
//
// Data: every per-instance vector is instance-major ([B][len], the callbacks' AoS layout); one 256-thread block
// owns one instance in the vector kernels (coalesced rows, block reductions in a fixed order, so a solve is
// reproducible run to run).  The sparse products (J^T y, the band assembly) gather through CSR tables built once
// on the host from the callbacks' fixed triplet structure — no atomics.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/cfx.h"
#include "cfx_inertia.h"
#include "cfx_internal.h"

namespace {

constexpr int kIB = 256;    // threads per instance block
constexpr int kFilt = 64;   // filter entries per instance (a ring, as solver.py)
constexpr int kSlots = 64;  // counter ring: one 4-int slot per host read
constexpr int kMaxY = 65535;
constexpr int kMaxBorder = 32;  // free parameters handled as a dense border
constexpr int kWideParts = 128;  // blocks per instance of the wide-instance reductions (IpmK::wide)
constexpr int kWP = 20;          // partial values per block (IpmK::wpart)
constexpr int kWF = 12;          // decisions per instance (IpmK::wflag)

// per-instance scalars of the iteration
struct Scal {
    double mu, tau, sf, fS, theta, phi, dphi, alpha, a_p, a_z, theta_max, theta_min, dw, dwl, err0, theta_soc, a_c,
        theta_r, a_r;
    double wd_theta, wd_phi, wd_dphi, wd_ap, wd_mu;  // watchdog reference: the iterate where it started
    int32_t done, acc, iters, fpos, accepted, armijo, soc, reinit, todo;
    int32_t wd_short, wd_on, wd_trial, skip_first, forced;
    int32_t rejf, nsucc, nreset;  // filter reset heuristic: last rejection by the filter, successive such iterations,
                                  // resets done
    int32_t acc_ok;  // the iterate meets Ipopt's acceptable-level tests (k_ipm_begin)
    // limited-memory Hessian (L-BFGS): sigma, pairs held, next ring slot, previous iterate saved
    double lsig;
    int32_t lcount, lhead, lprev, lpad;
    // restoration phase (CFX_RESTORATION_PHASE): its barrier, the original infeasibility where it started, its own
    // regularisation, line-search and filter quantities
    double rs_mu, rs_tau, rs_th0, rs_dw, rs_dwl, rs_theta, rs_phi, rs_dphi, rs_alpha, rs_ap, rs_az, rs_tmax, rs_tmin;
    // rs_on: the instance is in the phase (its iterations run in the same launches as the main iterations of the
    // others); rs_exit: how its phase ended this iteration (RS_*; 0: still running), acted on by k_ipm_update
    int32_t rs_on, rs_exit, rs_acc, rs_arm, rs_it;
    int32_t stop;    // done, not converged (status says why)
    int32_t status;  // CFX_IPM_STATUS_* once done
    int32_t spad;
    // soft restoration: its step and the primal-dual error at x; taking soft steps, how many, tried this iteration,
    // the try was accepted by the original filter
    double soft_a, soft_pd;
    int32_t soft_on, soft_cnt, soft_try, soft_ok;
    int32_t rs_rr;  // consecutive phase iterations that reset p, n (Ipopt's RestoRestorationPhase) instead of stepping
    int32_t rpad;
    // Ipopt's structural-degeneracy test of the Hessian (PDPerturbationHandler, degen_iters_max = 3): hdeg 0 not yet
    // determined, 1 not degenerate (an iteration's first trial with dw = 0 passed), 2 degenerate (the first
    // kDegenIters iterations all needed dw > 0): from then on each iteration's first trial is dw = max(1e-20, dw_last / 3)
    // instead of 0; degit counts those iterations
    int32_t hdeg, degit;
    // adaptive barrier parameter (o.mu_strategy == CFX_MU_ADAPTIVE; IpAdaptiveMuUpdate): free-mu mode, insertions into
    // the globalisation filter (its ring position), mu_max (set at the first iteration), this iteration's average
    // complementarity and the squared 2-norms of the scaled dual / primal infeasibility (the quality function's terms)
    int32_t mfree, mfpos;
    double mu_max, avgc, qd, qp;
};
constexpr int kDegenIters = 3;  // Ipopt degen_iters_max

// how a restoration phase ended (Scal::rs_exit)
enum { RS_RUNNING = 0, RS_OK = 1, RS_FAILED = 2, RS_INFEASIBLE = 3, RS_BUDGET = 4 };

struct IpmK {
    int64_t B;
    int n, m, nf, nj, nh, nK, kl, ku, ldab, nfix, nnzj, nnzh;
    cfx_ipm_options o;
    // problem data shared by the batch
    const int32_t *free, *fixed;
    const double *lb_full, *d, *lbF, *ubF, *lbF0, *ubF0;
    const uint8_t *hasL, *hasU;
    const int32_t *jsel, *jr, *jc;  // J_g triplets over the free columns
    const int32_t *hsel, *hr, *hc;  // Hessian triplets (lower triangle) over the free variables
    const uint8_t* hoff;
    const int32_t *jt_ptr, *jt_idx;    // triplets of each free column (J^T y)
    const int32_t *jrw_ptr, *jrw_idx;  // triplets of each constraint row (row scaling)
    const int32_t *kkt_ptr, *kkt_src;  // sources of each band-storage entry
    const int32_t* pos;                // KKT unknown (free variables, then rows) -> band order
    // Stage-chain layout (chain = 1): the unknowns grouped by stage into cM nodes of csp (padded) unknowns, the KKT
    // matrix block tridiagonal and factored by block cyclic reduction (cfx_chain.hip); P = 1 and nA = cM csp, the
    // band storage `ab` holds [D | L | U] ([3][cM][csp][csp] per instance, NE_A entries), cw the reduction's work
    // ([B][2][cM][csp][csp]), ct its solve scratch ([B][max(na, 1)][nA]); a border (np > 0) as below.
    int chain, cM, csp;
    double *cw, *ct;
    // chain: the band-storage positions with a source (the rest of [D | L | U] is zero and is cleared by a memset, not
    // by one thread per entry: 28.8 M entries of which ~1 in 6 has a source for the reaching task)
    const int32_t* nzpos;
    int64_t nnzA;
    // Wide instances (wide = 1: small batches of large NLPs, e.g. the reaching task's 2.4 M J_g values in one instance):
    // the gather loops of k_ipm_begin (J_g scaling, J^T y), k_ipm_curv (unpacking, x^T W x) and the border's back
    // substitution run as grids of many blocks per instance (k_wide_*) instead of one block's serial loop; gj [B][nf]
    // holds grad f + J^T y, part [B][kWideParts][4] the per-block partial sums (x^T W x, non-finite, x^T (Sigma +
    // dw) x, |x|^2), reduced in a fixed order
    int wide;
    double *gj, *part;
    // wpart [B][kWideParts][kWP]: per-block partials of the split barrier-algebra kernels (k_w*_a), reduced by the
    // one-block kernel in breduce_n's fixed order; wflag [B][kWF]: that kernel's decisions for the k_w*_c loops
    double *wpart, *wflag;
    // KKT layout.  P = 1, np = 0: one band of nA = nK unknowns (factor + solve in one launch).  Otherwise the
    // unknowns split into P diagonal band blocks of nA rows each (padded with unit rows) and a dense border of np
    // unknowns — Hmed intensity parameters, whose sliding windows couple most stages, and the separators between
    // the blocks (nested dissection of the stage chain, so that the P blocks factor side by side) — solved by a
    // Schur complement on the border (np <= kMaxBorder).  rb (right-hand side / solution, per instance nKp =
    // P nA + np): block q at q nA, the border at P nA.
    int P, nA, np, nKp;
    int64_t NE_A, NE_tot;  // band-storage entries of the P blocks; all assembled entries (bands, Cr, Cc, D)
    // the border is sparse in the blocks: block q couples to na_q <= na border unknowns act[q][.] (its "active"
    // columns: Cr_q and A_q^-1 Cr_q are stored for those only, slot sl[q][k] of border unknown k, -1: none), and
    // Cc is a list of non-zeros grouped by border row (ccr_ptr; block ccr_q, block row ccr_a)
    int na, ncc;
    const int32_t *act, *sl, *ccr_ptr, *ccr_q, *ccr_a;
    // per instance
    double *x, *zl, *zu, *dx, *dzl, *dzu, *xt, *xacc, *xr, *dxr, *sig, *gF;  // [B][nf]
    double *lbI, *ubI;                                                      // [B][nf] bounds (moved per instance)
    double *wx, *wzl, *wzu, *wy;                                            // watchdog iterate [B][nf] / [B][m]
    double *rhs, *rb;                                                       // [B][nK]
    double *y, *dy, *gS, *csoc, *sg, *ysc, *graw, *gt;                      // [B][m]
    double *vx, *vt, *grad;                                                 // [B][n]
    double *jac, *jv, *hv;                                                  // [B][nnzj], [B][nj], [B][nnzh]
    double *fraw, *ft, *of;                                                 // [B]
    double* ab;                                                             // [B][P][nA][ldab]
    // [B][P][na][nA] Cr -> A^-1 Cr (active columns), [B][ncc] Cc non-zeros, [B][np][np] D, LU of the Schur complement
    double *Xb, *Ccb, *Db, *Sf;
    int32_t* Sp;  // [B][np] its pivots
    // inertia test (o.inertia_test, stage chain): [B] negative eigenvalues of the last factorisation (the chain's pivot
    // blocks by cfx_chain_inertia_s, the border's Schur complement by k_ipm_schur); null: the curvature test
    int32_t* inert;
    int32_t *ipiv, *info;                                                   // [B][P][nA], [B][P]
    double* filt;                                                           // [B][kFilt][2]
    Scal* sc;                                                               // [B]
    int32_t* cnt;                                                           // [kSlots][4]
    // limited-memory Hessian (o.hessian_approximation == CFX_HESSIAN_LIMITED_MEMORY): hmax pairs (s, y) per instance
    // in a ring, the previous iterate, the compact form's middle matrix M, the Woodbury columns P = K0^-1 Z in band
    // order ([2 hmax][B][nKp], one rb-shaped array per column) and the LU of C = M - Z^T P
    int lbfgs, hmax;
    double *Sh, *Yh;           // [B][hmax][nf]
    double *xprev, *gprev;     // [B][nf]
    double* jvprev;            // [B][nj]
    double *Mm, *Cl;           // [B][2 hmax][2 hmax]
    int32_t* Cp;               // [B][2 hmax]
    double* Zb;                // [2 hmax][B][nKp]
    // restoration phase: p, n (the constraint relaxation c(x) - p + n = 0), their multipliers, steps and trial values,
    // the phase's constraint multipliers, the eliminated (2,2) block -(p / zp + n / zn) of its KKT matrix ([B][m]);
    // the phase's multipliers of the x bounds ([B][nf]); its filter; a zero objective factor for its Hessian ([B])
    int rsphase;
    double *rp, *rn, *rzp, *rzn, *rdp, *rdn, *rdzp, *rdzn, *rpt, *rnt, *ry, *rdc;
    double *rzl, *rzu;
    double* rfilt;
    unsigned long long* rstat;  // [4] phases entered, phase iterations, soft steps, switches of the adaptive mu update
                                // to its monotone mode (summed over the instances)
    // soft restoration (o.soft_resto_pderror_reduction_factor > 0): the trial point's J_g values and gradient; npd =
    // nf + m + bounded sides, the number of terms of the primal-dual system error
    double *jact, *gradt;  // [B][nnzj], [B][n]
    int npd;
    // adaptive barrier parameter (adapt = o.mu_strategy == CFX_MU_ADAPTIVE): the (f, ||c||_1) filter of its
    // globalisation [B][kFilt][2], the unit-centering part of the Newton right-hand side 1 / s_L - 1 / s_U [B][nf] (the
    // affine part stays in rhs) and its solution in band order [B][nKp]; ncomp = the bounded sides
    int adapt, ncomp;
    double *mfilt, *rhsmu, *rbc;
    double* mgs;  // wide instances: k_wmu_ctl's golden-section state [B][kGS]
    int mu_block;  // 1: the small-instance oracle in the whole block (CFX_IPM_MU_ORACLE=block, tests / A-B)
};

enum { KKT_NEWTON = 0, KKT_LSMULT = 1, KKT_RESTO = 2, KKT_RSNLP = 3 };
enum { SRC_W = 0, SRC_JV = 1, SRC_DIAG = 2, SRC_DC = 3 };
constexpr int kSrcShift = 29;
constexpr int32_t kSrcMask = (1 << kSrcShift) - 1;

// NaN-propagating min / max and torch.clamp semantics (a NaN input stays NaN)
__host__ __device__ inline double max_n(double a, double b) { return (a != a) ? a : ((b != b) ? b : (a > b ? a : b)); }
__host__ __device__ inline double min_n(double a, double b) { return (a != a) ? a : ((b != b) ? b : (a < b ? a : b)); }
__host__ __device__ inline double clamp_lo(double a, double lo) { return a < lo ? lo : a; }
__host__ __device__ inline double clamp_hi(double a, double hi) { return a > hi ? hi : a; }

struct OpSum {
    __device__ double operator()(double a, double b) const { return a + b; }
};
struct OpMax {
    __device__ double operator()(double a, double b) const { return max_n(a, b); }
};
struct OpMin {
    __device__ double operator()(double a, double b) const { return min_n(a, b); }
};

// Block-wide reduction, same result in every thread; the order is fixed (lane butterfly, then the waves in
// order), so the value is reproducible.
template <class Op>
__device__ double breduce(double v, Op op, double* sh) {
    for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = sh[0];
#pragma unroll
    for (int i = 1; i < kIB / 64; ++i) r = op(r, sh[i]);
    return r;
}

// Several block-wide reductions with one pair of barriers: v[i] reduced with op[i] (0 sum, 1 max, 2 min), each in
// breduce's order, so every value is bit-identical to its own breduce.
template <int N>
__device__ void breduce_n(double (&v)[N], const int (&op)[N]) {
    __shared__ double shn[kIB / 64][N];
    auto apply = [&](int i, double a, double c) { return op[i] == 0 ? a + c : (op[i] == 1 ? max_n(a, c) : min_n(a, c)); };
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = apply(i, v[i], __shfl_xor(v[i], o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int i = 0; i < N; ++i) shn[threadIdx.x >> 6][i] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double r = shn[0][i];
#pragma unroll
        for (int w = 1; w < kIB / 64; ++w) r = apply(i, r, shn[w][i]);
        v[i] = r;
    }
}

// Wide instances: a block of a k_w*_a grid (B, kWideParts) stores its partials of N reductions; the one-block
// kernel that follows reduces the kWideParts partials of each (thread q holding partial q) in breduce_n's order, so
// the values are reproducible (their order differs from the one-block loops': the wide path is its own
// deterministic sum).
__device__ inline double red_identity(int op) { return op == 0 ? 0.0 : (op == 1 ? -INFINITY : INFINITY); }
template <int N>
__device__ void wide_put(const IpmK& K, int64_t b, double (&v)[N], const int (&op)[N]) {
    static_assert(N <= kWP, "partials per block");
    breduce_n(v, op);
    if (threadIdx.x == 0)
#pragma unroll
        for (int k = 0; k < N; ++k) K.wpart[(b * kWideParts + blockIdx.y) * kWP + k] = v[k];
}
template <int N>
__device__ void wide_get(const IpmK& K, int64_t b, double (&v)[N], const int (&op)[N]) {
    static_assert(kWideParts <= kIB, "a partial per thread");
#pragma unroll
    for (int k = 0; k < N; ++k)
        v[k] = threadIdx.x < kWideParts ? K.wpart[(b * kWideParts + threadIdx.x) * kWP + k] : red_identity(op[k]);
    breduce_n(v, op);
}

// counter slot: thread 0 of block 0 clears the next slot (the next counting kernel runs after this one)
__device__ inline void count_add(const IpmK& K, int slot, int which, int v) {
    if (threadIdx.x == 0) {
        if (blockIdx.x == 0 && blockIdx.y == 0) {
            int32_t* nx = K.cnt + 4 * ((slot + 1) % kSlots);
            nx[0] = nx[1] = nx[2] = nx[3] = 0;
        }
        if (v) atomicAdd(K.cnt + 4 * slot + which, v);
    }
}

__device__ inline void load_scal(const IpmK& K, int64_t b, Scal& S) {
    if (threadIdx.x == 0) S = K.sc[b];
    __syncthreads();
}
__device__ inline void store_scal(const IpmK& K, int64_t b, const Scal& S) {
    __syncthreads();
    if (threadIdx.x == 0) K.sc[b] = S;
}

// solver.py _max_step: min(1, min_i (has_i & ds_i < 0 ? -tau s_i / ds_i : inf)) over the block
__device__ inline double step_term(bool has, double s, double ds, double tau) {
    return (has && ds < 0) ? (-tau * s) / ds : INFINITY;
}

// Ipopt's safe slacks (solver.py _safe_slacks): a slack in [0, eps min(1, mu)) — a point that landed on its bound in
// floating point — is measured to the bound moved outwards by slack_move max(1, |bound|); k_ipm_update makes the move
// of an accepted point permanent
constexpr double kEps = 2.220446049250313e-16;
constexpr double kSlackMove = 1.8189894035458565e-12;  // eps^(3/4), Ipopt slack_move
__device__ inline double slack_min(double mu) { return kEps * clamp_hi(mu, 1.0); }
__device__ inline double moved_lb(double lb, double s, double smin) {
    return (s < smin && s >= 0) ? lb - kSlackMove * clamp_lo(fabs(lb), 1.0) : lb;
}
__device__ inline double moved_ub(double ub, double s, double smin) {
    return (s < smin && s >= 0) ? ub + kSlackMove * clamp_lo(fabs(ub), 1.0) : ub;
}

// solver.py _barrier_obj: f - mu (sum ln sl + sum ln su), +inf outside the bounds
__device__ double barrier_obj(const IpmK& K, int64_t b, const double* x, double f, double mu, double* sh) {
    double sL = 0.0, sU = 0.0, bad = 0.0;
    const double* lbI = K.lbI + b * K.nf;
    const double* ubI = K.ubI + b * K.nf;
    const double smin = slack_min(mu);
    for (int i = threadIdx.x; i < K.nf; i += kIB) {
        if (K.hasL[i]) {
            double sl = x[i] - lbI[i];
            sl = x[i] - moved_lb(lbI[i], sl, smin);
            if (sl <= 0) bad = 1.0;
            sL += log(clamp_lo(sl, 1e-300));
        }
        if (K.hasU[i]) {
            double su = ubI[i] - x[i];
            su = moved_ub(ubI[i], su, smin) - x[i];
            if (su <= 0) bad = 1.0;
            sU += log(clamp_lo(su, 1e-300));
        }
    }
    {
        double rv[3] = {sL, sU, bad};
        const int ro[3] = {0, 0, 1};
        breduce_n(rv, ro);
        sL = rv[0];
        sU = rv[1];
        bad = rv[2];
    }
    return bad > 0 ? INFINITY : f - mu * (sL + sU);
}

// (tt, pt) dominated by an entry of the filter (block-wide, same in every thread)
__device__ bool filter_dominated(const double* filt, double tt, double pt, double* sh) {
    double inf_ = 0.0;
    for (int k = threadIdx.x; k < kFilt; k += kIB)
        if (tt >= filt[2 * k] && pt >= filt[2 * k + 1]) inf_ = 1.0;
    return breduce(inf_, OpMax(), sh) > 0;
}

// Ipopt's filter test of a trial (tt = ||c||_1, pt = barrier objective) against the current point (theta, phi,
// directional derivative dphi, step alpha): (accepted, by the Armijo / f-type rule)
__device__ void filter_core(const IpmK& K, const double* filt, double theta, double phi, double dphi, double theta_max,
                            double theta_min, double tt, double pt, double alpha, double* sh, bool& ok, bool& arm,
                            bool* rejf = nullptr) {
    const bool dominated = filter_dominated(filt, tt, pt, sh);
    const bool finite = isfinite(pt) && isfinite(tt);
    const bool switching = (dphi < 0) && (alpha * pow(clamp_lo(-dphi, 0.0), 2.3) > 1.0 * pow(theta, 1.1)) &&
                           (theta <= theta_min);
    // Ipopt's Compare_le(lhs, rhs, base): lhs - rhs <= 10 eps |base| (round-off in phi near an optimum)
    const double tol_phi = 10 * kEps * fabs(phi);
    const bool armijo_ok = (pt - phi) - K.o.armijo * alpha * dphi <= tol_phi;
    const bool suff = (tt - (1 - 1e-5) * theta <= 10 * kEps * theta) || ((pt - phi) + 1e-5 * theta <= tol_phi);
    ok = finite && (tt <= theta_max) && !dominated && (switching ? armijo_ok : suff);
    arm = switching && armijo_ok;
    // rejected by the filter alone: it passed Ipopt's theta_max and Armijo / sufficient-decrease tests
    if (rejf) *rejf = finite && (tt <= theta_max) && dominated && (switching ? armijo_ok : suff);
}

// solver.py _filter_accept: (accepted, by the Armijo / f-type rule) for a trial with tt = ||g||_1, pt = barrier
__device__ void filter_accept(const IpmK& K, const Scal& S, const double* filt, double tt, double pt, double alpha,
                              double* sh, bool& ok, bool& arm, bool* rejf = nullptr) {
    // in the watchdog, trial points are judged against the iterate where it started (with its full step length)
    const double theta = S.wd_on ? S.wd_theta : S.theta, phi = S.wd_on ? S.wd_phi : S.phi;
    const double dphi = S.wd_on ? S.wd_dphi : S.dphi;
    if (S.wd_on) alpha = S.wd_ap;
    filter_core(K, filt, theta, phi, dphi, S.theta_max, S.theta_min, tt, pt, alpha, sh, ok, arm, rejf);
}

// x -> full decision vector (fixed entries are already in place)
__device__ inline void write_full(const IpmK& K, int64_t b, const double* xs, double* v) {
    for (int i = threadIdx.x; i < K.nf; i += kIB) v[b * K.n + K.free[i]] = xs[i] * K.d[i];
}

// restoration phase: weight zeta D_R,i^2 of the proximity term zeta/2 |D_R (x - x_r)|^2, zeta = sqrt(mu_R),
// D_R,i = min(1, 1 / |x_r,i|) (Ipopt resto_proximity_weight 1); x_r is the iterate where the phase started (K.x)
__device__ inline double rs_weight(double mu, double xref) {
    const double r = clamp_lo(fabs(xref), 1.0);
    return sqrt(mu) / (r * r);
}
__device__ inline double rs_prox(const IpmK& K, int64_t b, int i) {
    return rs_weight(K.sc[b].rs_mu, K.x[b * K.nf + i]);
}

// ---------------------------------------------------------------------------------------------------------------
// kernels (grid = B blocks of kIB threads unless noted)
// ---------------------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kIB) k_ipm_fix(const IpmK K, const double* __restrict__ fv) {
    const int64_t b = blockIdx.x;
    for (int j = threadIdx.x; j < K.nfix; j += kIB) {
        const int e = K.fixed[j];
        K.vx[b * K.n + e] = fv ? fv[b * K.nfix + j] : K.lb_full[e];
    }
}

// after eval_all at the starting point: gradient-based scaling (solver.py _set_function_scaling), bound push,
// z = mu / s, y = 0, empty filter
// Warm start (Ipopt warm_start_init_point; ws = the unscaled multipliers of cfx_ipm_set_warm_start, else NULL): y and
// the bound multipliers from them (scaled problem: y_s = sf y / s_g, z_s = sf d z, z raised to
// warm_start_mult_bound_push), x pushed by warm_start_bound_push / warm_start_bound_frac, no least-squares step.
__global__ void __launch_bounds__(kIB) k_ipm_init(const IpmK K, const double* __restrict__ wy,
                                                  const double* __restrict__ wzl, const double* __restrict__ wzu) {
    __shared__ double sh[kIB / 64];
    const int64_t b = blockIdx.x;
    const bool warm = wy != nullptr;
    const double* grad = K.grad + b * K.n;
    const double* jac = K.jac + b * K.nnzj;
    double gmax = 0.0;
    for (int i = threadIdx.x; i < K.nf; i += kIB) gmax = max_n(gmax, fabs(grad[K.free[i]] * K.d[i]));
    gmax = breduce(gmax, OpMax(), sh);
    // Ipopt's gradient-based scaling: min(1, max_gradient / max |gradient|), at least nlp_scaling_min_value; none: 1
    const bool scl = K.o.nlp_scaling_method != 0;
    const double gm = K.o.nlp_scaling_max_gradient, smin = K.o.nlp_scaling_min_value;
    const double sf = scl ? clamp_lo(clamp_hi(gm / clamp_lo(gmax, 1e-300), 1.0), smin) : 1.0;
    for (int r = threadIdx.x; r < K.m; r += kIB) {
        double rmax = 0.0;
        for (int k = K.jrw_ptr[r]; k < K.jrw_ptr[r + 1]; ++k) {
            const int s = K.jrw_idx[k];
            rmax = max_n(rmax, fabs(jac[K.jsel[s]] * K.d[K.jc[s]]));
        }
        const double sgr = scl ? clamp_lo(clamp_hi(gm / clamp_lo(rmax, 1e-300), 1.0), smin) : 1.0;
        K.sg[b * K.m + r] = sgr;
        K.y[b * K.m + r] = warm ? sf * wy[b * K.m + r] / sgr : 0.0;
    }
    const double mu = K.o.mu_init;
    const double push = warm ? K.o.warm_start_bound_push : K.o.bound_push;
    const double frac = warm ? K.o.warm_start_bound_frac : K.o.bound_frac;
    for (int i = threadIdx.x; i < K.nf; i += kIB) {
        double xi = K.vx[b * K.n + K.free[i]] / K.d[i];
        const bool hL = K.hasL[i], hU = K.hasU[i];
        const double lb = K.lbF[i], ub = K.ubF[i];
        K.lbI[b * K.nf + i] = lb;
        K.ubI[b * K.nf + i] = ub;
        double pl = push * clamp_lo(hL ? fabs(lb) : 1.0, 1.0);
        double pu = push * clamp_lo(hU ? fabs(ub) : 1.0, 1.0);
        const double width = (hL && hU) ? ub - lb : INFINITY;
        pl = min_n(pl, frac * width);
        pu = min_n(pu, frac * width);
        if (hL) xi = max_n(xi, lb + pl);
        if (hU) xi = min_n(xi, ub - pu);
        const double sl = hL ? xi - lb : 1.0, su = hU ? ub - xi : 1.0;
        K.x[b * K.nf + i] = xi;
        if (warm) {
            const int64_t e = b * K.n + K.free[i];
            const double zs = sf * K.d[i];
            K.zl[b * K.nf + i] = hL ? max_n(zs * wzl[e], K.o.warm_start_mult_bound_push) : 0.0;
            K.zu[b * K.nf + i] = hU ? max_n(zs * wzu[e], K.o.warm_start_mult_bound_push) : 0.0;
        } else if (K.o.bound_mult_init_method == 0) {  // Ipopt's "constant"
            K.zl[b * K.nf + i] = hL ? K.o.bound_mult_init_val : 0.0;
            K.zu[b * K.nf + i] = hU ? K.o.bound_mult_init_val : 0.0;
        } else {
            K.zl[b * K.nf + i] = hL ? mu / sl : 0.0;
            K.zu[b * K.nf + i] = hU ? mu / su : 0.0;
        }
        K.vx[b * K.n + K.free[i]] = xi * K.d[i];
    }
    for (int k = threadIdx.x; k < kFilt; k += kIB) {
        K.filt[(b * kFilt + k) * 2] = INFINITY;
        K.filt[(b * kFilt + k) * 2 + 1] = -INFINITY;
        if (K.adapt) K.mfilt[(b * kFilt + k) * 2] = K.mfilt[(b * kFilt + k) * 2 + 1] = INFINITY;
    }
    if (threadIdx.x == 0) {
        Scal S{};
        S.mu = mu;
        S.sf = sf;
        S.mfree = K.adapt;  // Ipopt's adaptive update starts in the free mode
        S.mu_max = -1.0;
        S.lsig = 1.0;  // Ipopt limited_memory_init_val
        S.err0 = INFINITY;
        S.reinit = K.m > 0 && !warm;
        K.sc[b] = S;
    }
}

// Iteration start (solver.py solve loop, up to the Newton right-hand side).  mode bit 0: scale the callback
// outputs of x (g, J_g, f, grad f); bit 1: stop after the scaling (least-squares multipliers come next).
// Instances in the restoration phase are k_rs_begin's.
__global__ void __launch_bounds__(kIB) k_ipm_begin(const IpmK K, int mode, int slot) {
    __shared__ double sh[kIB / 64];
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    if (S.rs_on) {  // block-uniform
        count_add(K, slot, 0, 0);
        return;
    }
    double* gS = K.gS + b * m;
    double* jv = K.jv + b * K.nj;
    double* gF = K.gF + b * nf;
    if (mode & 1) {
        const double* sg = K.sg + b * m;
        const double* jac = K.jac + b * K.nnzj;
        if (!K.wide) {  // (wide: k_wide_scale did these)
            for (int j = threadIdx.x; j < m; j += kIB) gS[j] = K.graw[b * m + j] * sg[j];
            // (unrolled: several gathers in flight per thread — one instance of ~10^6 J_g entries is one block's loop)
#pragma unroll 8
            for (int s = threadIdx.x; s < K.nj; s += kIB) jv[s] = jac[K.jsel[s]] * K.d[K.jc[s]] * sg[K.jr[s]];
            for (int i = threadIdx.x; i < nf; i += kIB) gF[i] = K.grad[b * K.n + K.free[i]] * K.d[i] * S.sf;
        }
        if (threadIdx.x == 0) S.fS = K.fraw[b] * S.sf;
        __syncthreads();
        if (mode & 2) {
            store_scal(K, b, S);
            return;
        }
    }
    const double* x = K.x + b * nf;
    const double* zl = K.zl + b * nf;
    const double* zu = K.zu + b * nf;
    const double* y = K.y + b * m;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    double* rhs = K.rhs + b * K.nK;
    double szl = 0, szu = 0, sy = 0, ed = 0, ep = 0, ecl = 0, ecu = 0, edu = 0, epu = 0;
    double pLmax = -INFINITY, pLmin = INFINITY, pUmax = -INFINITY, pUmin = INFINITY;  // (wide: k_wbegin_a's)
    // the adaptive update's sums: complementarity (its average), ||c||_1, |grad L|^2, |c|^2
    double scl = 0, scu = 0, th = 0, rd2 = 0, g2 = 0;
    const double* sg = K.sg + b * m;
    if (K.wide) {
        double rv[18];
        const int ro[18] = {0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 2, 1, 2, 0, 0, 0, 0, 0};
        wide_get(K, b, rv, ro);
        szl = rv[0], szu = rv[1], sy = rv[2], ed = rv[3], ep = rv[4], ecl = rv[5], ecu = rv[6], edu = rv[7],
        epu = rv[8], pLmax = rv[9], pLmin = rv[10], pUmax = rv[11], pUmin = rv[12];
        scl = rv[13], scu = rv[14], th = rv[15], rd2 = rv[16], g2 = rv[17];
    } else {
    for (int i = threadIdx.x; i < nf; i += kIB) {
        double gj;
        if (K.wide) {  // k_wide_jty, the same sum in the same order
            gj = K.gj[b * nf + i];
        } else {
            double jty = 0.0;
#pragma unroll 4
            for (int k = K.jt_ptr[i]; k < K.jt_ptr[i + 1]; ++k) {
                const int s = K.jt_idx[k];
                jty += jv[s] * y[K.jr[s]];
            }
            gj = gF[i] + jty;
        }
        rhs[i] = gj;  // completed below, once mu is final
        const double rd = gj - zl[i] + zu[i];
        szl += fabs(zl[i]);
        szu += fabs(zu[i]);
        const double cl = K.hasL[i] ? (x[i] - lbI[i]) * zl[i] : 0.0;
        const double cu = K.hasU[i] ? (ubI[i] - x[i]) * zu[i] : 0.0;
        ed = max_n(ed, fabs(rd));
        edu = max_n(edu, fabs(rd) / K.d[i]);
        ecl = max_n(ecl, fabs(cl));
        ecu = max_n(ecu, fabs(cu));
        scl += cl;
        scu += cu;
        rd2 += rd * rd;
    }
    for (int j = threadIdx.x; j < m; j += kIB) {
        sy += fabs(y[j]);
        ep = max_n(ep, fabs(gS[j]));
        epu = max_n(epu, fabs(gS[j]) / sg[j]);
        th += fabs(gS[j]);
        g2 += gS[j] * gS[j];
    }
    {
        double rv[14] = {szl, szu, sy, ed, ep, ecl, ecu, edu, epu, scl, scu, th, rd2, g2};
        const int ro[14] = {0, 0, 0, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
        breduce_n(rv, ro);
        szl = rv[0];
        szu = rv[1];
        sy = rv[2];
        ed = rv[3];
        ep = rv[4];
        ecl = rv[5];
        ecu = rv[6];
        edu = rv[7];
        epu = rv[8];
        scl = rv[9];
        scu = rv[10];
        th = rv[11];
        rd2 = rv[12];
        g2 = rv[13];
    }
    }
    const double smax = K.o.s_max;
    const double sd = clamp_lo((szl + szu + sy) / (2.0 * nf + m), smax) / smax;
    const double sc = clamp_lo((szl + szu) / (2.0 * nf), smax) / smax;
    const double e_d = ed / sd, e_p = m ? ep : 0.0, e_c0 = max_n(ecl, ecu) / sc;
    if (threadIdx.x == 0) {
        S.err0 = max_n(max_n(e_d, e_p), e_c0);
        // Ipopt's unscaled tests (IpOptErrorConv): constraint violation, dual infeasibility (x = d x_s, the multipliers
        // of the scaled problem over sf), complementarity with mu = 0
        const double e_pu = m ? epu : 0.0, e_du = edu / S.sf, e_cu = max_n(ecl, ecu) / S.sf;
        const bool conv = S.err0 <= K.o.tol && e_pu <= K.o.constr_viol_tol && e_du <= K.o.dual_inf_tol &&
                          e_cu <= K.o.compl_inf_tol;
        S.acc_ok = S.err0 <= K.o.acceptable_tol && e_pu <= K.o.acceptable_constr_viol_tol &&
                   e_du <= K.o.acceptable_dual_inf_tol && e_cu <= K.o.acceptable_compl_inf_tol;
        S.acc = S.acc_ok ? S.acc + 1 : 0;
        const bool newly = !S.done && (conv || S.acc >= K.o.acceptable_iter);
        if (newly) S.status = conv ? CFX_IPM_SOLVE_SUCCEEDED : CFX_IPM_SOLVED_TO_ACCEPTABLE_LEVEL;
        S.done = S.done || newly;
        if (!S.done && S.iters >= K.o.max_iter) {  // per-instance budget
            S.done = S.stop = 1;
            S.status = CFX_IPM_MAXIMUM_ITERATIONS_EXCEEDED;
        }
    }
    __syncthreads();
    // Adaptive strategy (IpAdaptiveMuUpdate; solver.py BatchedIpm.solve): the globalisation decides the mode — a
    // free-mode iterate not acceptable to the (f, ||c||_1) filter switches to the monotone mode at mu =
    // adaptive_mu_monotone_init_factor * average complementarity; a monotone-mode one acceptable to it returns to the
    // free mode; acceptable iterates enter the filter.  Free-mode mu comes from k_mu_oracle after the factorisation.
    __shared__ int s_mono;
    const double mu_prev = S.mu;
    int passes = 5;  // the monotone strategy's fast decrease (mu_allow_fast_monotone_decrease)
    if (threadIdx.x == 0) s_mono = !S.done;
    if (K.adapt) {
        passes = 1;
        static_assert(kFilt == 64, "the globalisation filter: one entry per lane of wavefront 0");
        if (threadIdx.x < 64 && !S.done) {  // (S.done is block-uniform)
            const int k = threadIdx.x;
            const double avg = K.ncomp ? (scl + scu) / K.ncomp : 0.0;
            const double thc = m ? th : 0.0;
            double* mf = K.mfilt + b * kFilt * 2;
            const double fk = mf[2 * k], tk = mf[2 * k + 1];
            // IpFilter::Acceptable: f <= f_i or theta < theta_i for every entry
            const bool okk = K.o.adaptive_mu_globalization != CFX_MU_GLOBAL_OBJ_CONSTR_FILTER || S.fS <= fk || thc < tk;
            const bool ok = __ballot(!okk) == 0ull;
            if (ok) {  // RememberCurrentPointAsAccepted: the entries it dominates leave, then the first free slot
                const double margin = K.o.filter_margin_fact * clamp_hi(thc, K.o.filter_max_margin);
                const double fe = S.fS - margin, te = thc - margin;
                const bool dom = fe <= fk && te <= tk;
                const unsigned long long fr = __ballot(dom || (isinf(fk) && isinf(tk)));
                const int slot = fr ? __ffsll((long long)fr) - 1 : S.mfpos % kFilt;
                if (k == slot) {
                    mf[2 * k] = fe;
                    mf[2 * k + 1] = te;
                } else if (dom) {
                    mf[2 * k] = mf[2 * k + 1] = INFINITY;
                }
            }
            __builtin_amdgcn_wave_barrier();  // every lane has read S.fS / S.mfpos before lane 0 updates S
            if (k == 0) {
            if (ok) S.mfpos += 1;
            S.avgc = avg;
            S.qd = rd2;
            S.qp = m ? g2 : 0.0;
            if (S.mu_max < 0) S.mu_max = K.o.mu_max > 0 ? K.o.mu_max : K.o.mu_max_fact * avg;
            s_mono = 0;
            if (S.mfree && !ok) {  // to the monotone mode
                S.mfree = 0;
                S.mu = min_n(clamp_lo(K.o.adaptive_mu_monotone_init_factor * avg, K.o.mu_min), S.mu_max);
                atomicAdd(K.rstat + 3, 1ull);
            } else if (!S.mfree && ok) {  // back to the free mode
                S.mfree = 1;
            } else {
                s_mono = !S.mfree;
            }
            }
        }
    }
    __syncthreads();
    // floor of the monotone mu: tol / 10, or Ipopt's min(tol, compl_inf_tol) / (barrier_tol_factor + 1)
    const double mufl = K.o.monotone_mu_floor ? min_n(K.o.tol, K.o.compl_inf_tol) / (K.o.kappa_eps + 1.0) : K.o.tol / 10;
    // monotone barrier update: while the barrier sub-problem is solved, decrease mu (at most `passes` times)
    for (int pass = 0; pass < passes && s_mono; ++pass) {
        const double mu = S.mu;
        double ecm = 0.0;
        if (K.wide) {  // max_i |p_i - mu| = max(p_max - mu, mu - p_min), exactly (fl(p - mu) is monotone in p)
            ecm = max_n(max_n(max_n(ecm, pLmax - mu), max_n(mu - pLmin, pUmax - mu)), mu - pUmin) / sc;
        } else {
        for (int i = threadIdx.x; i < nf; i += kIB) {
            const double cl = K.hasL[i] ? (x[i] - lbI[i]) * zl[i] - mu : 0.0;
            const double cu = K.hasU[i] ? (ubI[i] - x[i]) * zu[i] - mu : 0.0;
            ecm = max_n(ecm, max_n(fabs(cl), fabs(cu)));
        }
        ecm = breduce(ecm, OpMax(), sh) / sc;
        }
        const double e_mu = max_n(max_n(e_d, e_p), ecm);
        const bool dec = !S.done && (e_mu <= K.o.kappa_eps * mu) && (mu > mufl);
        if (!dec) break;
        __syncthreads();
        if (threadIdx.x == 0) S.mu = clamp_lo(min_n(K.o.kappa_mu * mu, pow(mu, K.o.theta_mu)), mufl);
        __syncthreads();
    }
    const double mu = S.mu;
    // Ipopt restarts the line search's filter whenever mu changes (linesearch_->Reset()): every free-mode iteration of
    // the adaptive strategy, a changed mu of either strategy (the monotone one only with mu_change_resets_filter)
    const bool ls_reset = !S.done && (K.adapt ? (S.mfree || mu != mu_prev) : (K.o.mu_change_resets_filter && mu != mu_prev));
    if (ls_reset)
        for (int k = threadIdx.x; k < kFilt; k += kIB) {
            K.filt[(b * kFilt + k) * 2] = INFINITY;
            K.filt[(b * kFilt + k) * 2 + 1] = -INFINITY;
        }
    double* sig = K.sig + b * nf;
    if (!K.wide) {  // (wide: k_wbegin_c)
    for (int i = threadIdx.x; i < nf; i += kIB) {
        const bool hL = K.hasL[i], hU = K.hasU[i];
        const double sl = hL ? x[i] - lbI[i] : 1.0, su = hU ? ubI[i] - x[i] : 1.0;
        sig[i] = (hL ? zl[i] / sl : 0.0) + (hU ? zu[i] / su : 0.0);
        if (K.adapt) {  // rhs = -(grad f + J^T y) + mu (1 / s_L - 1 / s_U): the affine part and the unit centering
            rhs[i] = -rhs[i];
            K.rhsmu[b * nf + i] = (hL ? 1.0 / sl : 0.0) - (hU ? 1.0 / su : 0.0);
        } else {
            const double bar = (hL ? mu / sl : 0.0) - (hU ? mu / su : 0.0);
            rhs[i] = -(rhs[i] - bar);
        }
    }
    for (int j = threadIdx.x; j < m; j += kIB) {
        rhs[nf + j] = -gS[j];
        K.ysc[b * m + j] = y[j] * K.sg[b * m + j];
    }
    }
    if (threadIdx.x == 0) {
        S.tau = clamp_lo(1.0 - mu, K.o.tau_min);
        // Ipopt's first trial: dw = 0, or straight from the last one when the Hessian is known to be degenerate
        S.dw = S.hdeg == 2 ? (S.dwl > 0 ? clamp_lo(S.dwl / 3, 1e-20) : 1e-4) : 0.0;
        K.of[b] = S.sf;
    }
    store_scal(K, b, S);
    count_add(K, slot, 0, !S.done);
}

// KKT matrix in band storage and the permuted right-hand side.  grid (B, ceil(nK ldab / kIB)).
//   NEWTON: [[W + Sigma + dw, J^T], [J, -delta_c]], rhs as k_ipm_begin left it
//   LSMULT: [[I, J^T], [J, -delta_c]], rhs [-(grad f - zl + zu); 0]   (least-squares multipliers)
//   RESTO : [[Sigma + I, J^T], [J, -delta_c]], rhs [0; -g]            (restoration step)
// one band-storage entry of the KKT matrix (p < NE_tot) from its sources
__device__ inline void kkt_entry(const IpmK& K, int64_t b, int64_t p, int mode) {
    double v = 0.0;
    const double* hv = K.hv + b * K.nnzh;
    const double* jv = K.jv + b * K.nj;
    const double* sig = K.sig + b * K.nf;
    // L-BFGS: W = sigma I - low rank (Woodbury); restoration phase (the Newton matrix of an instance in it): its
    // own regularisation and proximity term
    const bool rs = mode == KKT_RSNLP || (mode == KKT_NEWTON && K.sc[b].rs_on);
    const double dw = rs ? K.sc[b].rs_dw : K.sc[b].dw + (K.lbfgs ? K.sc[b].lsig : 0.0);
    for (int k = K.kkt_ptr[p]; k < K.kkt_ptr[p + 1]; ++k) {
        const int32_t code = K.kkt_src[k];
        const int idx = code & kSrcMask;
        switch (code >> kSrcShift) {
            case SRC_W:
                if (mode == KKT_NEWTON || rs) v += hv[K.hsel[idx]] * K.d[K.hr[idx]] * K.d[K.hc[idx]];
                break;
            case SRC_JV: v += jv[idx]; break;
            case SRC_DIAG:
                if (rs)
                    v += sig[idx] + dw + rs_prox(K, b, idx);
                else
                    v += mode == KKT_NEWTON ? sig[idx] + dw : (mode == KKT_LSMULT ? 1.0 : sig[idx] + 1.0);
                break;
            default:  // unit diagonal of a padding row / -delta_c (restoration: - p / zp - n / zn of row idx)
                v += idx == kSrcMask ? 1.0 : -K.o.delta_c + (rs ? K.rdc[b * K.m + idx] : 0.0);
                break;
        }
    }
    if (p < K.NE_A) {
        K.ab[b * K.NE_A + p] = v;
    } else {  // the border: Cr (active columns per block, as right-hand sides), Cc non-zeros, D
        const int64_t nb = (int64_t)K.P * K.na * K.nA;
        int64_t q = p - K.NE_A;
        if (q < nb)
            K.Xb[b * nb + q] = v;
        else if ((q -= nb) < K.ncc)
            K.Ccb[b * K.ncc + q] = v;
        else
            K.Db[b * K.np * K.np + (q - K.ncc)] = v;
    }
}

// the permuted right-hand side entry p < nK
__device__ inline void kkt_rhs(const IpmK& K, int64_t b, int64_t p, int mode) {
    const int nf = K.nf;
    double r;
    if (mode == KKT_NEWTON || mode == KKT_RSNLP) {
        r = K.rhs[b * K.nK + p];
        // adaptive strategy: the monotone-mode instances' mu term (free-mode ones solve mu = 0 here, k_mu_oracle adds
        // mu times the centering solution)
        if (K.adapt && mode == KKT_NEWTON && p < nf && !K.sc[b].rs_on && !K.sc[b].mfree)
            r += K.sc[b].mu * K.rhsmu[b * nf + p];
    }
    else if (mode == KKT_LSMULT)
        r = p < nf ? -(K.gF[b * nf + p] - K.zl[b * nf + p] + K.zu[b * nf + p]) : 0.0;
    else
        r = p < nf ? 0.0 : -K.gS[b * K.m + (p - nf)];
    K.rb[b * K.nKp + K.pos[p]] = r;
}

__global__ void __launch_bounds__(kIB) k_ipm_kkt(const IpmK K, int mode) {
    const int64_t b = blockIdx.x;
    // chain with a source list (nzpos): entries t < nnzA are the positions with sources in [D | L | U] (the rest was
    // cleared), then the border's; otherwise every entry.  grid-stride: grid.y is capped at kMaxY
    const int64_t NE = K.nzpos ? K.nnzA + (K.NE_tot - K.NE_A) : K.NE_tot;
    for (int64_t t = (int64_t)blockIdx.y * kIB + threadIdx.x; t < NE || t < K.nK; t += (int64_t)gridDim.y * kIB) {
        if (t < NE) {
            const int64_t p = K.nzpos ? (t < K.nnzA ? (int64_t)K.nzpos[t] : K.NE_A + (t - K.nnzA)) : t;
            kkt_entry(K, b, p, mode);
        }
        if (t < K.nK) kkt_rhs(K, b, t, mode);
    }
}

// Bordered / dissected KKT: after the band factorisations of the P blocks A_q and the solves A_q^-1 [Cr_q | r_q]
// (X and the block parts of rb), the Schur complement S = D - sum_q Cc_q A_q^-1 Cr_q (np x np, LU with partial
// pivoting in LDS, kept for the second-order corrections: factor = 0 re-uses it), the border x_p =
// S^-1 (r_p - sum_q Cc_q y_q) and the blocks x_q = y_q - (A_q^-1 Cr_q) x_p, written back into rb.  A zero pivot
// of S is reported in info like one of a block (P nA + k + 1).
// ordering point for the single-wavefront phases below: LDS traffic of the wave completed, no compiler motion
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

constexpr int kSchurStage = 2048;  // Cc non-zeros / active-slot entries staged in LDS (else read from global)
// Operands (A^-1 Cr)(., j) of every Cc non-zero z and border column j, gathered by all threads at once before the S
// entries sum their products: the per-entry loops otherwise walk their row's non-zeros with one dependent L2 load each
// (cfg 3 at batch 1: 29.6 us per call, of a ~180 us iteration).  The sums keep the fused multiply-subtract of the
// ungathered loop, so the results are bit-identical to it (the interior point's trajectories are sensitive to rounding)
constexpr int kSchurProd = 1536;

__global__ void __launch_bounds__(kIB) k_ipm_schur(const IpmK K, int factor, int back = 1) {
    __shared__ double S[kMaxBorder][kMaxBorder + 1];
    __shared__ double sv[kMaxBorder];
    __shared__ int piv[kMaxBorder];
    __shared__ double ccv[kSchurStage];
    __shared__ int ccq[kSchurStage], cca[kSchurStage], slt[kSchurStage];
    __shared__ double prod[kSchurProd];
    const int64_t b = blockIdx.x;
    const int nA = K.nA, np = K.np, P = K.P, na = K.na, t = threadIdx.x;
    const int64_t nb = (int64_t)na * nA;  // per block
    const double* X = K.Xb + b * P * nb;
    const double* Cc = K.Ccb + b * K.ncc;
    double* rb = K.rb + b * K.nKp;
    double* Sf = K.Sf + b * np * np;
    int32_t* Sp = K.Sp + b * np;
    const int PA = P * nA;
    // the sparse coupling of the border rows, staged once (every S entry and s_i walks its row)
    const bool staged = K.ncc <= kSchurStage && P * np <= kSchurStage;
    if (staged) {
        for (int z = t; z < K.ncc; z += kIB) ccv[z] = Cc[z], ccq[z] = K.ccr_q[z], cca[z] = K.ccr_a[z];
        for (int e = t; e < P * np; e += kIB) slt[e] = K.sl[e];
        __syncthreads();
    }
    auto cval = [&](int z) { return staged ? ccv[z] : Cc[z]; };
    auto cq = [&](int z) { return staged ? ccq[z] : K.ccr_q[z]; };
    auto ca = [&](int z) { return staged ? cca[z] : K.ccr_a[z]; };
    auto slot = [&](int q, int j) { return staged ? slt[q * np + j] : K.sl[q * np + j]; };
    const bool pstage = staged && K.ncc * np <= kSchurProd && K.ncc <= kSchurProd;
    if (factor) {
        if (pstage) {  // every operand at once (independent loads), then the sums from LDS
            for (int e = t; e < K.ncc * np; e += kIB) {
                const int z = e / np, j = e - z * np;
                const int q = ccq[z], c = slt[q * np + j];
                prod[e] = c >= 0 ? X[q * nb + (int64_t)c * nA + cca[z]] : 0.0;
            }
            __syncthreads();
        }
        for (int e = t; e < np * np; e += kIB) {  // S(i, j) = D(i, j) - sum over row i's Cc non-zeros
            const int i = e / np, j = e - (e / np) * np;
            double acc = K.Db[b * np * np + e];
            for (int z = K.ccr_ptr[i]; z < K.ccr_ptr[i + 1]; ++z) {
                if (pstage) {
                    acc = fma(-ccv[z], prod[z * np + j], acc);
                } else {
                    const int q = cq(z), c = slot(q, j);
                    if (c >= 0) acc = fma(-cval(z), X[q * nb + (int64_t)c * nA + ca(z)], acc);
                }
            }
            S[i][j] = acc;
        }
        __syncthreads();
        if (K.inert) {  // inertia test: the border's share of the KKT matrix's negative eigenvalues (Haynsworth)
            __shared__ double S2[kMaxBorder * (kMaxBorder + 1)];
            for (int e = t; e < np * np; e += kIB) {
                const int i = e / np, j = e - (e / np) * np;
                S2[i * (kMaxBorder + 1) + j] = 0.5 * (S[i][j] + S[j][i]);
            }
            __syncthreads();
            const int cnt = cfx_inertia::sym_neg_count(S2, kMaxBorder + 1, np);
            if (t == 0 && cnt) atomicAdd(K.inert + b, cnt);
        }
        if (t < 64) {  // LU with partial pivoting (first largest |S(i, k)|, i >= k) in one wavefront
            int sing = 0;
            for (int k = 0; k < np; ++k) {
                double a = (t >= k && t < np) ? fabs(S[t][k]) : -1.0;
                int idx = t;
                for (int o = 32; o > 0; o >>= 1) {
                    const double a2 = __shfl_xor(a, o, 64);
                    const int i2 = __shfl_xor(idx, o, 64);
                    if (a2 > a || (a2 == a && i2 < idx)) {
                        a = a2;
                        idx = i2;
                    }
                }
                const int p = idx;  // the same in every lane
                if (t == 0) piv[k] = p;
                if (p != k && t < np) {  // lanes over columns
                    const double tmp = S[k][t];
                    S[k][t] = S[p][t];
                    S[p][t] = tmp;
                }
                wave_sync();
                const double pv = S[k][k];
                const double inv = pv != 0.0 ? 1.0 / pv : 0.0;
                if (pv == 0.0 && !sing) sing = PA + k + 1;
                if (t > k && t < np) S[t][k] *= inv;
                wave_sync();
                if (t > k && t < np) {  // lane t updates column t of the trailing rows
                    const double ukt = S[k][t];
                    for (int i = k + 1; i < np; ++i) S[i][t] -= S[i][k] * ukt;
                }
                wave_sync();
            }
            if (t == 0 && sing && K.info[b * P] == 0) K.info[b * P] = sing;
        }
        __syncthreads();
        for (int e = t; e < np * np; e += kIB) Sf[e] = S[e / np][e - (e / np) * np];
        if (t < np) Sp[t] = piv[t];
    } else {
        for (int e = t; e < np * np; e += kIB) S[e / np][e - (e / np) * np] = Sf[e];
        if (t < np) piv[t] = Sp[t];
        __syncthreads();
    }
    if (pstage) {  // the y operands of Cc y at once (the factor phase's reads of prod are behind the barriers above)
        for (int z = t; z < K.ncc; z += kIB) prod[z] = rb[ccq[z] * nA + cca[z]];
        __syncthreads();
    }
    if (t < 64) {  // x_p = S^-1 (r_p - sum_q Cc_q y_q), lane i holding component i (getrs)
        double x = 0.0;
        if (t < np) {
            x = rb[PA + t];
            for (int z = K.ccr_ptr[t]; z < K.ccr_ptr[t + 1]; ++z)
                x = fma(-cval(z), pstage ? prod[z] : rb[cq(z) * nA + ca(z)], x);
        }
        for (int k = 0; k < np; ++k) {  // row interchanges in order
            const int p = piv[k];
            if (p != k) {
                const double xk = __shfl(x, k, 64), xp = __shfl(x, p, 64);
                if (t == k) x = xp;
                if (t == p) x = xk;
            }
        }
        for (int k = 0; k < np; ++k) {  // unit lower
            const double xk = __shfl(x, k, 64);
            if (t > k && t < np) x -= S[t][k] * xk;
        }
        for (int k = np - 1; k >= 0; --k) {  // upper
            if (t == k) x = x / S[k][k];
            const double xk = __shfl(x, k, 64);
            if (t < k) x -= S[t][k] * xk;
        }
        if (t < np) sv[t] = x;
    }
    __syncthreads();
    if (!back) {  // k_wide_border_back does the blocks
        for (int c = t; c < np; c += kIB) rb[PA + c] = sv[c];
        return;
    }
    for (int e = t; e < PA; e += kIB) {
        const int q = e / nA, a = e - (e / nA) * nA;
        double acc = rb[e];
        // four columns' loads issued together (independent), then their updates
        for (int c0 = 0; c0 < na; c0 += 4) {
            double xv[4], sk[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int c = c0 + u, k = c < na ? K.act[q * na + c] : -1;
                xv[u] = k >= 0 ? X[q * nb + (int64_t)c * nA + a] : 0.0;
                sk[u] = k >= 0 ? sv[k] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) acc -= xv[u] * sk[u];
        }
        rb[e] = acc;
    }
    for (int c = t; c < np; c += kIB) rb[PA + c] = sv[c];
}


// ---- wide instances (IpmK::wide): the long gather loops of one instance over a grid of blocks ----------------
// grid (B, ceil(max(nj, m, nf) / kIB)): the scaled callback outputs of k_ipm_begin's mode bit 0 (gS, jv, gF)
__global__ void __launch_bounds__(kIB) k_wide_scale(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;
    const int64_t p = (int64_t)blockIdx.y * kIB + threadIdx.x;
    const int m = K.m, nf = K.nf;
    const double* sg = K.sg + b * m;
    if (p < K.nj) K.jv[b * K.nj + p] = K.jac[b * K.nnzj + K.jsel[p]] * K.d[K.jc[p]] * sg[K.jr[p]];
    if (p < m) K.gS[b * m + p] = K.graw[b * m + p] * sg[p];
    if (p < nf) K.gF[b * nf + p] = K.grad[b * K.n + K.free[p]] * K.d[p] * K.sc[b].sf;
}

// grid (B, ceil(nf / kIB)): gj = grad f + J^T y per free variable, k_ipm_begin's sum in its order
__global__ void __launch_bounds__(kIB) k_wide_jty(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;
    const int i = blockIdx.y * kIB + threadIdx.x;
    if (i >= K.nf) return;
    const double* jv = K.jv + b * K.nj;
    const double* y = K.y + b * K.m;
    double jty = 0.0;
#pragma unroll 4
    for (int k = K.jt_ptr[i]; k < K.jt_ptr[i + 1]; ++k) {
        const int s = K.jt_idx[k];
        jty += jv[s] * y[K.jr[s]];
    }
    K.gj[b * K.nf + i] = K.gF[b * K.nf + i] + jty;
}

// grid (B, kWideParts): the Newton step in natural order (dx / dxr, dy) from rb, and a non-finite flag per block
__global__ void __launch_bounds__(kIB) k_wide_unpack(const IpmK K) {
    const int64_t b = blockIdx.x;
    const Scal& S = K.sc[b];
    const bool rs = S.rs_on;
    const bool active = rs ? S.rs_exit == RS_RUNNING : !S.done;
    const int nf = K.nf;
    const double* rb = K.rb + b * K.nKp;
    double* dx = (rs ? K.dxr : K.dx) + b * nf;
    double* dy = K.dy + b * K.m;
    const int64_t per = (K.nK + kWideParts - 1) / kWideParts;
    const int64_t lo = blockIdx.y * per, hi = std::min<int64_t>(K.nK, lo + per);
    double nonfin = 0.0, dd = 0.0, nrm = 0.0;
    const double dwc = rs ? S.rs_dw : S.dw;
    const double* sig = K.sig + b * nf;
    if (active || !rs)
        for (int64_t i = lo + threadIdx.x; i < hi; i += kIB) {
            const double r = rb[K.pos[i]];
            if (!isfinite(r)) nonfin = 1.0;
            if (i < nf) {
                dx[i] = r;
                dd += (sig[i] + dwc + (rs ? rs_prox(K, b, (int)i) : 0.0)) * r * r;  // k_ipm_curv's terms
                nrm += r * r;
            } else {
                dy[i - nf] = r;
            }
        }
    double rv[3] = {nonfin, dd, nrm};
    const int ro[3] = {1, 0, 0};
    breduce_n(rv, ro);
    if (threadIdx.x == 0) {
        double* pp = K.part + (b * kWideParts + blockIdx.y) * 4;
        pp[1] = rv[0];
        pp[2] = rv[1];
        pp[3] = rv[2];
    }
}

// grid (B, kWideParts): partial sums of dx^T W dx over contiguous ranges of the Hessian entries
__global__ void __launch_bounds__(kIB) k_wide_quad(const IpmK K) {
    __shared__ double sh[kIB / 64];
    const int64_t b = blockIdx.x;
    const bool rs = K.sc[b].rs_on;
    const double* dx = (rs ? K.dxr : K.dx) + b * K.nf;
    const double* hv = K.hv + b * K.nnzh;
    const int64_t per = (K.nh + kWideParts - 1) / kWideParts;
    const int64_t lo = blockIdx.y * per, hi = std::min<int64_t>(K.nh, lo + per);
    double quad = 0.0;
#pragma unroll 8
    for (int64_t s = lo + threadIdx.x; s < hi; s += kIB) {
        const int r = K.hr[s], c = K.hc[s];
        const double w = hv[K.hsel[s]] * K.d[r] * K.d[c];
        quad += w * dx[r] * dx[c] * (K.hoff[s] ? 2.0 : 1.0);
    }
    quad = breduce(quad, OpSum(), sh);
    if (threadIdx.x == 0) K.part[(b * kWideParts + blockIdx.y) * 4] = quad;
}

// grid (B, ceil(P nA / kIB)): the chain's back substitution of the border, x_A = y_A - (A^-1 Cr) x_p (k_ipm_schur's
// last loop, same order per entry), after k_ipm_schur with back = 0 left x_p in rb's border slots
__global__ void __launch_bounds__(kIB) k_wide_border_back(const IpmK K) {
    const int64_t b = blockIdx.x;
    const int64_t PA = (int64_t)K.P * K.nA;
    const int64_t e = (int64_t)blockIdx.y * kIB + threadIdx.x;
    if (e >= PA) return;
    const int nA = K.nA, na = K.na, np = K.np;
    const int64_t nb = (int64_t)na * nA;
    const double* X = K.Xb + b * K.P * nb;
    double* rb = K.rb + b * K.nKp;
    const int q = (int)(e / nA), a = (int)(e - (int64_t)q * nA);
    double acc = rb[e];
    for (int c0 = 0; c0 < na; c0 += 4) {
        double xv[4], sk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int c = c0 + u, k = c < na ? K.act[q * na + c] : -1;
            xv[u] = k >= 0 ? X[q * nb + (int64_t)c * nA + a] : 0.0;
            sk[u] = k >= 0 ? rb[PA + k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc -= xv[u] * sk[u];
    }
    rb[e] = acc;
    (void)np;
}

// ---- wide instances: k_ipm_begin / k_ipm_dir / k_ipm_accept / k_ipm_update split into a grid pass that forms the
// per-block partials (k_w*_a, grid (B, kWideParts), strided loops), the one-block kernel (its scalar logic on the reduced
// values, unchanged) and a grid pass over the elementwise updates that depend on them (k_w*_c, grid (B, ceil(max(nf,
// m) / kIB)), reading the decisions the one-block kernel left in K.sc / K.wflag).  The one-block kernels' own loops
// over ~10^5 variables were 0.5-1.4 ms each on the reaching task.
#define WIDE_LOOP(i, n) for (int i = blockIdx.y * kIB + threadIdx.x; i < (n); i += kWideParts * kIB)

// k_ipm_begin's sums and maxima (9) and the extremes of the complementarity products (4), from which the monotone
// mu update's max_i |(x - l) z - mu| follows exactly for any mu (fl(p - mu) is monotone in p)
__global__ void __launch_bounds__(kIB) k_wbegin_a(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;
    const int nf = K.nf, m = K.m;
    const double* x = K.x + b * nf;
    const double* zl = K.zl + b * nf;
    const double* zu = K.zu + b * nf;
    const double* y = K.y + b * m;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    const double* gS = K.gS + b * m;
    const double* sg = K.sg + b * m;
    double* rhs = K.rhs + b * K.nK;
    double szl = 0, szu = 0, sy = 0, ed = 0, ep = 0, ecl = 0, ecu = 0, edu = 0, epu = 0;
    double pLmax = -INFINITY, pLmin = INFINITY, pUmax = -INFINITY, pUmin = INFINITY;
    double scl = 0, scu = 0, th = 0, rd2 = 0, g2 = 0;
    WIDE_LOOP(i, nf) {
        const double gj = K.gj[b * nf + i];
        rhs[i] = gj;
        const double rd = gj - zl[i] + zu[i];
        szl += fabs(zl[i]);
        szu += fabs(zu[i]);
        const double cl = K.hasL[i] ? (x[i] - lbI[i]) * zl[i] : 0.0;
        const double cu = K.hasU[i] ? (ubI[i] - x[i]) * zu[i] : 0.0;
        ed = max_n(ed, fabs(rd));
        edu = max_n(edu, fabs(rd) / K.d[i]);
        ecl = max_n(ecl, fabs(cl));
        ecu = max_n(ecu, fabs(cu));
        if (K.hasL[i]) pLmax = max_n(pLmax, cl), pLmin = min_n(pLmin, cl);
        if (K.hasU[i]) pUmax = max_n(pUmax, cu), pUmin = min_n(pUmin, cu);
        scl += cl;
        scu += cu;
        rd2 += rd * rd;
    }
    WIDE_LOOP(j, m) {
        sy += fabs(y[j]);
        ep = max_n(ep, fabs(gS[j]));
        epu = max_n(epu, fabs(gS[j]) / sg[j]);
        th += fabs(gS[j]);
        g2 += gS[j] * gS[j];
    }
    double rv[18] = {szl, szu, sy, ed, ep, ecl, ecu, edu, epu, pLmax, pLmin, pUmax, pUmin, scl, scu, th, rd2, g2};
    const int ro[18] = {0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 2, 1, 2, 0, 0, 0, 0, 0};
    wide_put(K, b, rv, ro);
}

// k_ipm_begin's Newton right-hand side and Sigma at the final mu (k_ipm_begin stored it)
__global__ void __launch_bounds__(kIB) k_wbegin_c(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;
    const int nf = K.nf, m = K.m;
    const int i = blockIdx.y * kIB + threadIdx.x;
    const double mu = K.sc[b].mu;
    double* rhs = K.rhs + b * K.nK;
    if (i < nf) {
        const double xi = K.x[b * nf + i];
        const bool hL = K.hasL[i], hU = K.hasU[i];
        const double sl = hL ? xi - K.lbI[b * nf + i] : 1.0, su = hU ? K.ubI[b * nf + i] - xi : 1.0;
        K.sig[b * nf + i] = (hL ? K.zl[b * nf + i] / sl : 0.0) + (hU ? K.zu[b * nf + i] / su : 0.0);
        if (K.adapt) {  // the affine part and the unit centering (k_ipm_begin)
            rhs[i] = -rhs[i];
            K.rhsmu[b * nf + i] = (hL ? 1.0 / sl : 0.0) - (hU ? 1.0 / su : 0.0);
        } else {
            const double bar = (hL ? mu / sl : 0.0) - (hU ? mu / su : 0.0);
            rhs[i] = -(rhs[i] - bar);
        }
    }
    if (i < m) {
        rhs[nf + i] = -K.gS[b * m + i];
        K.ysc[b * m + i] = K.y[b * m + i] * K.sg[b * m + i];
    }
}

// k_ipm_dir's loops: dz, the fraction-to-the-boundary minima, grad phi . dx, ||c||_1 and the barrier terms at x
__global__ void __launch_bounds__(kIB) k_wdir_a(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;
    const int nf = K.nf, m = K.m;
    const double mu = K.sc[b].mu, tau = K.sc[b].tau, smin = slack_min(mu);
    const double* x = K.x + b * nf;
    const double* zl = K.zl + b * nf;
    const double* zu = K.zu + b * nf;
    const double* dx = K.dx + b * nf;
    const double* gF = K.gF + b * nf;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    double apl = INFINITY, apu = INFINITY, azl = INFINITY, azu = INFINITY, dphi = 0.0, theta = 0.0;
    double sL = 0.0, sU = 0.0, bad = 0.0;
    WIDE_LOOP(i, nf) {
        const bool hL = K.hasL[i], hU = K.hasU[i];
        const double sl = hL ? x[i] - lbI[i] : 1.0, su = hU ? ubI[i] - x[i] : 1.0;
        const double vzl = hL ? mu / sl - zl[i] - zl[i] / sl * dx[i] : 0.0;
        const double vzu = hU ? mu / su - zu[i] + zu[i] / su * dx[i] : 0.0;
        K.dzl[b * nf + i] = vzl;
        K.dzu[b * nf + i] = vzu;
        apl = min_n(apl, step_term(hL, sl, dx[i], tau));
        apu = min_n(apu, step_term(hU, su, -dx[i], tau));
        azl = min_n(azl, step_term(hL, zl[i], vzl, tau));
        azu = min_n(azu, step_term(hU, zu[i], vzu, tau));
        const double bar = (hL ? mu / sl : 0.0) - (hU ? mu / su : 0.0);
        dphi += (gF[i] - bar) * dx[i];
        if (hL) {  // barrier_obj's terms
            const double s2 = x[i] - moved_lb(lbI[i], sl, smin);
            if (s2 <= 0) bad = 1.0;
            sL += log(clamp_lo(s2, 1e-300));
        }
        if (hU) {
            const double s2 = moved_ub(ubI[i], su, smin) - x[i];
            if (s2 <= 0) bad = 1.0;
            sU += log(clamp_lo(s2, 1e-300));
        }
    }
    WIDE_LOOP(j, m) theta += fabs(K.gS[b * m + j]);
    double rv[9] = {apl, apu, azl, azu, dphi, theta, sL, sU, bad};
    const int ro[9] = {2, 2, 2, 2, 0, 0, 0, 0, 1};
    wide_put(K, b, rv, ro);
}

// k_ipm_dir's first trial point x + alpha0 dx (alpha0: S.alpha as k_ipm_dir left it)
__global__ void __launch_bounds__(kIB) k_wdir_c(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;
    const int nf = K.nf;
    const int i = blockIdx.y * kIB + threadIdx.x;
    if (i >= nf) return;
    const double a0 = K.sc[b].alpha, xi = K.x[b * nf + i];
    const double xt = xi + a0 * K.dx[b * nf + i];
    K.xacc[b * nf + i] = xi;
    K.xt[b * nf + i] = xt;
    K.vt[b * K.n + K.free[i]] = xt * K.d[i];
}

// k_ipm_accept's ||c(x_t)||_1 and the barrier terms at the trial point
// (soc: the second-order-corrected trial in xr, for k_ipm_soc_accept)
__global__ void __launch_bounds__(kIB) k_wacc_a(const IpmK K, int soc) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;
    const int nf = K.nf, m = K.m;
    const double mu = K.sc[b].mu, smin = slack_min(mu);
    const double* xt = (soc ? K.xr : K.xt) + b * nf;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    double tt = 0.0, sL = 0.0, sU = 0.0, bad = 0.0;
    WIDE_LOOP(j, m) tt += fabs(K.gt[b * m + j] * K.sg[b * m + j]);
    WIDE_LOOP(i, nf) {
        if (K.hasL[i]) {
            double sl = xt[i] - lbI[i];
            sl = xt[i] - moved_lb(lbI[i], sl, smin);
            if (sl <= 0) bad = 1.0;
            sL += log(clamp_lo(sl, 1e-300));
        }
        if (K.hasU[i]) {
            double su = ubI[i] - xt[i];
            su = moved_ub(ubI[i], su, smin) - xt[i];
            if (su <= 0) bad = 1.0;
            sU += log(clamp_lo(su, 1e-300));
        }
    }
    double rv[4] = {tt, sL, sU, bad};
    const int ro[4] = {0, 0, 0, 1};
    wide_put(K, b, rv, ro);
}

// k_ipm_accept's second-order-correction right-hand side (wflag[1]) and the accepted point (wflag[2])
__global__ void __launch_bounds__(kIB) k_wacc_c(const IpmK K) {
    const int64_t b = blockIdx.x;
    const double* wf = K.wflag + b * kWF;
    if (wf[0] == 0.0) return;
    const int nf = K.nf, m = K.m;
    const int i = blockIdx.y * kIB + threadIdx.x;
    if (wf[1] != 0.0 && i < m) K.csoc[b * m + i] = wf[3] * K.gS[b * m + i] + K.gt[b * m + i] * K.sg[b * m + i];
    if (wf[2] != 0.0 && i < nf) K.xacc[b * nf + i] = K.xt[b * nf + i];
}

// the line search's backtracking and second-order corrections on wide instances (their one-block kernels loop over the
// instance: k_ipm_next_trial 86 us, k_ipm_soc_trial 0.66 ms, k_ipm_soc_accept 0.51 ms, k_ipm_soc_rhs 0.30 ms per call
// on the reaching task, ~1.3 ms of an iteration under the Ipopt profile)
// grid (B, ceil(nf / kIB)): k_ipm_next_trial's trial x + (alpha / 2) dx; k_wnext_b halves alpha after it
__global__ void __launch_bounds__(kIB) k_wnext_a(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].accepted || K.sc[b].rs_on) return;
    const int nf = K.nf, i = blockIdx.y * kIB + threadIdx.x;
    if (i >= nf) return;
    const double a = K.sc[b].alpha * 0.5;
    const double xt = K.x[b * nf + i] + a * K.dx[b * nf + i];
    K.xt[b * nf + i] = xt;
    K.vt[b * K.n + K.free[i]] = xt * K.d[i];
}
__global__ void __launch_bounds__(kIB) k_wnext_b(const IpmK K) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= K.B || K.sc[b].accepted || K.sc[b].rs_on) return;
    K.sc[b].alpha = K.sc[b].alpha * 0.5;
}
// grid (B, ceil(nK / kIB)): k_ipm_soc_rhs elementwise
__global__ void __launch_bounds__(kIB) k_wsoc_rhs(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;
    const int nf = K.nf, i = blockIdx.y * kIB + threadIdx.x;
    if (i >= K.nK) return;
    const double a = K.sc[b].alpha, mu = K.sc[b].mu;
    const double rx = i < nf ? (K.adapt ? K.rhs[b * K.nK + i] + mu * K.rhsmu[b * nf + i] : K.rhs[b * K.nK + i]) : 0.0;
    K.rb[b * K.nKp + K.pos[i]] = i < nf ? rx * a : -K.csoc[b * K.m + (i - nf)];
}
// k_ipm_soc_trial: partial fractions to the boundary of the corrected step (grid (B, kWideParts)), then every block of
// a grid over the variables reduces them (the same a_c in each) and forms its part of the trial
__global__ void __launch_bounds__(kIB) k_wsoct_a(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;
    const int nf = K.nf;
    const double* x = K.x + b * nf;
    const double* rb = K.rb + b * K.nKp;
    const double tau = K.sc[b].tau;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    double apl = INFINITY, apu = INFINITY;
    WIDE_LOOP(i, nf) {
        const double d = rb[K.pos[i]];
        if (K.hasL[i]) apl = min_n(apl, step_term(true, x[i] - lbI[i], d, tau));
        if (K.hasU[i]) apu = min_n(apu, step_term(true, ubI[i] - x[i], -d, tau));
    }
    double rv[2] = {apl, apu};
    const int ro[2] = {2, 2};
    wide_put(K, b, rv, ro);
}
__global__ void __launch_bounds__(kIB) k_wsoct_c(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;  // (block-uniform)
    double rv[2];
    const int ro[2] = {2, 2};
    wide_get(K, b, rv, ro);
    const double a_c = min_n(clamp_hi(rv[0], 1.0), clamp_hi(rv[1], 1.0));
    const int nf = K.nf, i = blockIdx.y * kIB + threadIdx.x;
    if (i < nf) {
        const double xr = K.x[b * nf + i] + a_c * K.rb[b * K.nKp + K.pos[i]];
        K.xr[b * nf + i] = xr;
        K.vt[b * K.n + K.free[i]] = xr * K.d[i];
    }
    if (blockIdx.y == 0 && threadIdx.x == 0) K.sc[b].a_c = a_c;
}
// k_ipm_soc_accept's elementwise part: the correction's constraint values (wflag[1]) and the accepted point (wflag[2])
__global__ void __launch_bounds__(kIB) k_wsoca_c(const IpmK K) {
    const int64_t b = blockIdx.x;
    const double* wf = K.wflag + b * kWF;
    if (wf[0] == 0.0) return;
    const int nf = K.nf, m = K.m;
    const int i = blockIdx.y * kIB + threadIdx.x;
    if (wf[1] != 0.0 && i < m) K.csoc[b * m + i] = wf[3] * K.csoc[b * m + i] + K.gt[b * m + i] * K.sg[b * m + i];
    if (wf[2] != 0.0 && i < nf) K.xacc[b * nf + i] = K.xr[b * nf + i];
}

// k_ipm_update's non-finite checks of the step
__global__ void __launch_bounds__(kIB) k_wupd_a(const IpmK K) {
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    double nfy = 0.0, nfz = 0.0;
    WIDE_LOOP(j, m)
    if (!isfinite(K.dy[b * m + j])) nfy = 1.0;
    WIDE_LOOP(i, nf)
    if (!isfinite(K.dzl[b * nf + i]) || !isfinite(K.dzu[b * nf + i])) nfz = 1.0;
    double rv[2] = {nfy, nfz};
    const int ro[2] = {1, 1};
    wide_put(K, b, rv, ro);
}

// k_ipm_update's step of x, the bound multipliers (with Ipopt's kappa_sigma safeguard) and the moved bounds, the
// constraint multipliers, and the decision vector; wflag: [0] go, [1] step, [2] reset, [3] mz, [4] az, [5] mu,
// [6] back to the watchdog iterate, [7] y update (0 none, 1 watchdog, 2 zero, 3 alpha dy), [8] alpha
__global__ void __launch_bounds__(kIB) k_wupd_c(const IpmK K) {
    const int64_t b = blockIdx.x;
    const double* wf = K.wflag + b * kWF;
    if (wf[0] == 0.0) return;
    const int nf = K.nf, m = K.m;
    const int i = blockIdx.y * kIB + threadIdx.x;
    const bool step = wf[1] != 0.0, reset = wf[2] != 0.0, mz = wf[3] != 0.0, wd_back = wf[6] != 0.0;
    const double az = wf[4], mu = wf[5], smin = slack_min(mu);
    if (i < nf) {
        const int64_t e = b * nf + i;
        const double* xnew = reset ? K.xr : K.xacc;
        double xi = step ? xnew[e] : K.x[e];
        double l = K.zl[e], u = K.zu[e];
        if (mz) {
            l = l + az * K.dzl[e];
            u = u + az * K.dzu[e];
        }
        if (K.hasL[i]) {
            const double lbv = moved_lb(K.lbI[e], xi - K.lbI[e], smin);
            K.lbI[e] = lbv;
            const double sl = xi - lbv;
            l = clamp_hi(clamp_lo(l, mu / (1e10 * sl)), 1e10 * mu / sl);
        }
        if (K.hasU[i]) {
            const double ubv = moved_ub(K.ubI[e], K.ubI[e] - xi, smin);
            K.ubI[e] = ubv;
            const double su = ubv - xi;
            u = clamp_hi(clamp_lo(u, mu / (1e10 * su)), 1e10 * mu / su);
        }
        if (wd_back) {
            xi = K.wx[e];
            l = K.wzl[e];
            u = K.wzu[e];
        }
        K.x[e] = xi;
        K.zl[e] = l;
        K.zu[e] = u;
        K.vx[b * K.n + K.free[i]] = xi * K.d[i];
    }
    if (i < m) {
        const int64_t e = b * m + i;
        const int ym = (int)wf[7];
        double yv = K.y[e];
        if (ym == 1) yv = K.wy[e];
        else if (ym == 2) yv = 0.0;
        else if (ym == 3) yv = yv + wf[8] * K.dy[e];
        K.y[e] = yv;
        K.ysc[e] = yv * K.sg[e];
    }
}
// ---- wide instances in the restoration phase: k_rs_begin's loops over the instance as grids (one block's loops over the
// reaching task's 2.4 M J_g values and 10^5 variables were ~7 ms per call)
// grid (B, ceil(max(nj, m) / kIB)): the scaled constraint values and J_g values of the phase's instances
__global__ void __launch_bounds__(kIB) k_wrs_scale(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (!K.sc[b].rs_on || K.sc[b].rs_exit != RS_RUNNING) return;
    const int64_t p = (int64_t)blockIdx.y * kIB + threadIdx.x;
    const int m = K.m;
    const double* sg = K.sg + b * m;
    if (p < K.nj) K.jv[b * K.nj + p] = K.jac[b * K.nnzj + K.jsel[p]] * K.d[K.jc[p]] * sg[K.jr[p]];
    if (p < m) K.gS[b * m + p] = K.graw[b * m + p] * sg[p];
}
// grid (B, kWideParts): J^T y into rhs (k_rs_begin's sum in its order), the phase's dual and primal errors, and the
// extremes of its complementarity products, from which max_i |p_i - mu| follows exactly for any mu
__global__ void __launch_bounds__(kIB) k_wrs_a(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (!K.sc[b].rs_on || K.sc[b].rs_exit != RS_RUNNING) return;
    const int nf = K.nf, m = K.m;
    const double rho = K.o.resto_penalty, mu = K.sc[b].rs_mu;
    const double* jv = K.jv + b * K.nj;
    const double* x = K.xr + b * nf;
    const double* xref = K.x + b * nf;
    const double* zl = K.rzl + b * nf;
    const double* zu = K.rzu + b * nf;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    const double* p = K.rp + b * m;
    const double* nn = K.rn + b * m;
    const double* zp = K.rzp + b * m;
    const double* zn = K.rzn + b * m;
    const double* y = K.ry + b * m;
    const double* gS = K.gS + b * m;
    double* rhs = K.rhs + b * K.nK;
    double ed = 0.0, ep = 0.0, pmax = -INFINITY, pmin = INFINITY;
    WIDE_LOOP(i, nf) {
        double jty = 0.0;
#pragma unroll 4
        for (int k = K.jt_ptr[i]; k < K.jt_ptr[i + 1]; ++k) {
            const int q = K.jt_idx[k];
            jty += jv[q] * y[K.jr[q]];
        }
        rhs[i] = jty;
        ed = max_n(ed, fabs(rs_weight(mu, xref[i]) * (x[i] - xref[i]) + jty - zl[i] + zu[i]));
        if (K.hasL[i]) {
            const double pr = (x[i] - lbI[i]) * zl[i];
            pmax = max_n(pmax, pr), pmin = min_n(pmin, pr);
        }
        if (K.hasU[i]) {
            const double pr = (ubI[i] - x[i]) * zu[i];
            pmax = max_n(pmax, pr), pmin = min_n(pmin, pr);
        }
    }
    WIDE_LOOP(j, m) {
        ep = max_n(ep, fabs(gS[j] - p[j] + nn[j]));
        ed = max_n(ed, max_n(fabs(rho - y[j] - zp[j]), fabs(rho + y[j] - zn[j])));
        const double pp = p[j] * zp[j], pn = nn[j] * zn[j];
        pmax = max_n(pmax, max_n(pp, pn)), pmin = min_n(pmin, min_n(pp, pn));
    }
    double rv[4] = {ed, ep, pmax, pmin};
    const int ro[4] = {1, 1, 1, 2};
    wide_put(K, b, rv, ro);
}
// grid (B, ceil(max(nf, m) / kIB)): k_rs_begin's Newton system of the phase at its final mu (instances it kept going)
__global__ void __launch_bounds__(kIB) k_wrs_c(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (!K.sc[b].rs_on || K.sc[b].rs_exit != RS_RUNNING) return;
    const int nf = K.nf, m = K.m, i = blockIdx.y * kIB + threadIdx.x;
    const double rho = K.o.resto_penalty, mu = K.sc[b].rs_mu;
    double* rhs = K.rhs + b * K.nK;
    if (i < nf) {
        const int64_t e = b * nf + i;
        const double xi = K.xr[e], xref = K.x[e];
        const bool hL = K.hasL[i], hU = K.hasU[i];
        const double sl = hL ? xi - K.lbI[e] : 1.0, su = hU ? K.ubI[e] - xi : 1.0;
        K.sig[e] = (hL ? K.rzl[e] / sl : 0.0) + (hU ? K.rzu[e] / su : 0.0);
        const double bar = (hL ? mu / sl : 0.0) - (hU ? mu / su : 0.0);
        rhs[i] = -(rs_weight(mu, xref) * (xi - xref) + rhs[i] - bar);
    }
    if (i < m) {
        const int64_t e = b * m + i;
        const double p = K.rp[e], nn = K.rn[e], y = K.ry[e];
        const double Sp = K.rzp[e] / p, Sn = K.rzn[e] / nn;
        const double ap = mu / p - rho + y, an = mu / nn - rho - y;
        rhs[nf + i] = -(K.gS[e] - p + nn) + ap / Sp - an / Sn;
        K.rdc[e] = -(1.0 / Sp + 1.0 / Sn);
        K.ysc[e] = y * K.sg[e];
    }
}

#undef WIDE_LOOP

// Newton step in natural order and the curvature test (solver.py inertia loop); bumps dw where it fails.  An instance
// in the restoration phase takes the phase's step (its dx in dxr, its own dw, the proximity weights).  Counters: [0]
// instances iterating, [1] of them with the wrong inertia, [2] of them in the restoration phase
__global__ void __launch_bounds__(kIB) k_ipm_curv(const IpmK K, int slot) {
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf;
    load_scal(K, b, S);
    const bool rs = S.rs_on;
    const bool active = rs ? S.rs_exit == RS_RUNNING : !S.done;
    const double dwc = rs ? S.rs_dw : S.dw;
    const double* rb = K.rb + b * K.nKp;
    double* dx = (rs ? K.dxr : K.dx) + b * nf;
    double* dy = K.dy + b * K.m;
    double nonfin = 0.0, quad = 0.0, dd = 0.0, nrm = 0.0;
    if (K.wide) {  // k_wide_unpack / k_wide_quad: partial sums of the blocks (thread q holds block q's)
        if (threadIdx.x < kWideParts) {
            const double* pt = K.part + (b * kWideParts + threadIdx.x) * 4;
            quad = pt[0];
            nonfin = pt[1];
            dd = pt[2];
            nrm = pt[3];
        }
    } else {
        if (active || !rs)
            for (int i = threadIdx.x; i < K.nK; i += kIB) {
                const double r = rb[K.pos[i]];
                if (!isfinite(r)) nonfin = 1.0;
                if (i < nf)
                    dx[i] = r;
                else
                    dy[i - nf] = r;
            }
        __syncthreads();
        const double* hv = K.hv + b * K.nnzh;
#pragma unroll 8
        for (int s = threadIdx.x; s < K.nh; s += kIB) {  // (sums in the same order; gathers in flight)
            const int r = K.hr[s], c = K.hc[s];
            const double w = hv[K.hsel[s]] * K.d[r] * K.d[c];
            quad += w * dx[r] * dx[c] * (K.hoff[s] ? 2.0 : 1.0);
        }
    }
    const double* sig = K.sig + b * nf;
    if (!K.wide)
        for (int i = threadIdx.x; i < nf; i += kIB) {
            dd += (sig[i] + dwc + (rs ? rs_prox(K, b, i) : 0.0)) * dx[i] * dx[i];
            nrm += dx[i] * dx[i];
        }
    {
        double rv[4] = {quad, dd, nrm, nonfin};
        const int ro[4] = {0, 0, 0, 1};
        breduce_n(rv, ro);
        quad = rv[0];
        dd = rv[1];
        nrm = rv[2];
        nonfin = rv[3];
    }
    const double curv = quad + dd;
    bool sing = false;
    for (int q = 0; q < K.P; ++q) sing = sing || K.info[b * K.P + q] != 0;
    // L-BFGS: the approximation is positive definite by construction (pairs with s^T y <= 0 are skipped), so only a
    // singular or non-finite factorisation asks for more regularisation
    // (inertia test: the factorisation's negative eigenvalues must number the constraints, Ipopt's inertia correction)
    const bool weak = (K.lbfgs && !rs) ? false
                      : K.inert        ? (K.inert[b] != K.m || !isfinite(curv))
                                       : ((curv <= K.o.curv_min * nrm) || !isfinite(curv));
    const bool bad = active && (weak || sing || nonfin > 0);
    if (threadIdx.x == 0 && bad) {
        double& dw = rs ? S.rs_dw : S.dw;
        const double dwl = rs ? S.rs_dwl : S.dwl;
        if (dw == 0.0)
            dw = dwl > 0 ? clamp_lo(dwl / 3, 1e-20) : 1e-4;
        else
            dw = dw * 8;
    }
    if (threadIdx.x == 0 && active && !bad && !rs && S.hdeg == 0) {  // the iteration's trial passed: degeneracy test
        if (S.dw == 0.0) {
            S.hdeg = 1;
        } else if (++S.degit >= kDegenIters) {
            S.hdeg = 2;
        }
    }
    store_scal(K, b, S);
    if (threadIdx.x == 0) {
        count_add(K, slot, 0, active);
        if (bad) atomicAdd(K.cnt + 4 * slot + 1, 1);
        if (rs && active) atomicAdd(K.cnt + 4 * slot + 2, 1);
    }
}

// ---- adaptive barrier parameter: Ipopt's quality-function mu oracle (IpQualityFunctionMuOracle::CalculateMu,
// 2-norm-squared, no centrality or balancing term; recalled, see solver.py BatchedIpm._mu_oracle, its specification)
// For the free-mode instances the Newton step is affine in mu: rb holds the solution of the affine right-hand side
// (mu = 0, kkt_rhs), rbc that of the unit centering [1 / s_L - 1 / s_U; 0] with the same factors, and the step for
// mu = sigma * avgc is rb + mu rbc.

// the unit-centering right-hand side in band order (zero for the other instances, so rbc stays bounded)
__global__ void __launch_bounds__(kIB) k_mu_cen_rhs(const IpmK K) {
    const int64_t b = blockIdx.x;
    const bool on = !K.sc[b].done && !K.sc[b].rs_on && K.sc[b].mfree;
    for (int i = threadIdx.x; i < K.nK; i += kIB)
        K.rbc[b * K.nKp + K.pos[i]] = (on && i < K.nf) ? K.rhsmu[b * K.nf + i] : 0.0;
}

// the quality function at mu: predicted (1 - a_d)^2 |grad L|^2 / n_x + (1 - a_p)^2 |c|^2 / m + |(s + a_p ds)(z + a_d
// dz)|^2 / n_bounds after the step of mu, a_p / a_d its fractions to the boundary (tau = max(tau_min, 1 - mu))
__device__ double mu_quality(const IpmK& K, int64_t b, const Scal& S, double mu) {
    const int nf = K.nf;
    const double tau = clamp_lo(1.0 - mu, K.o.tau_min);
    const double* x = K.x + b * nf;
    const double* zl = K.zl + b * nf;
    const double* zu = K.zu + b * nf;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    const double* ra = K.rb + b * K.nKp;
    const double* rc = K.rbc + b * K.nKp;
    double apl = INFINITY, apu = INFINITY, azl = INFINITY, azu = INFINITY;
    for (int i = threadIdx.x; i < nf; i += kIB) {
        const int q = K.pos[i];
        const double dx = ra[q] + mu * rc[q];
        const bool hL = K.hasL[i], hU = K.hasU[i];
        const double sl = hL ? x[i] - lbI[i] : 1.0, su = hU ? ubI[i] - x[i] : 1.0;
        const double vzl = hL ? mu / sl - zl[i] - zl[i] / sl * dx : 0.0;
        const double vzu = hU ? mu / su - zu[i] + zu[i] / su * dx : 0.0;
        apl = min_n(apl, step_term(hL, sl, dx, tau));
        apu = min_n(apu, step_term(hU, su, -dx, tau));
        azl = min_n(azl, step_term(hL, zl[i], vzl, tau));
        azu = min_n(azu, step_term(hU, zu[i], vzu, tau));
    }
    {
        double rv[4] = {apl, apu, azl, azu};
        const int ro[4] = {2, 2, 2, 2};
        breduce_n(rv, ro);
        apl = rv[0], apu = rv[1], azl = rv[2], azu = rv[3];
    }
    const double ap = min_n(clamp_hi(apl, 1.0), clamp_hi(apu, 1.0));
    const double ad = min_n(clamp_hi(azl, 1.0), clamp_hi(azu, 1.0));
    double cs = 0.0;
    for (int i = threadIdx.x; i < nf; i += kIB) {
        const int q = K.pos[i];
        const double dx = ra[q] + mu * rc[q];
        const bool hL = K.hasL[i], hU = K.hasU[i];
        if (hL) {
            const double sl = x[i] - lbI[i];
            const double t = (sl + ap * dx) * (zl[i] + ad * (mu / sl - zl[i] - zl[i] / sl * dx));
            cs += t * t;
        }
        if (hU) {
            const double su = ubI[i] - x[i];
            const double t = (su - ap * dx) * (zu[i] + ad * (mu / su - zu[i] + zu[i] / su * dx));
            cs += t * t;
        }
    }
    {
        double rv[1] = {cs};
        const int ro[1] = {0};
        breduce_n(rv, ro);
        cs = rv[0];
    }
    double val = (1.0 - ad) * (1.0 - ad) * S.qd / (nf > 0 ? nf : 1);
    if (K.m) val += (1.0 - ap) * (1.0 - ap) * S.qp / K.m;
    if (K.ncomp) val += cs / K.ncomp;
    return val;
}

// Small instances (nf <= 64 kMuWave): the oracle in wavefront 0 alone, each lane's elements (i = lane + 64 e) and
// their reciprocals held in registers across the section's evaluations, the reductions lane butterflies — no block
// barriers — and no division per evaluation: min_i (-tau s_i / ds_i) over ds_i < 0 is formed as tau / max_i (-ds_i
// (1 / s_i)) (cfg 3 at batch 1: 77 us per call with the block's loops, of which ~13 quality evaluations of four
// divisions per element).  Its own rounding (and another reduction order), so its decisions may differ from the
// block path's in the last bits of a quality value.
constexpr int kMuWave = 6;
struct MuLane {
    double a[kMuWave], c[kMuWave], sl[kMuWave], su[kMuWave], zl[kMuWave], zu[kMuWave];
    double isl[kMuWave], isu[kMuWave], izl[kMuWave], izu[kMuWave];  // 1 / s, 1 / z
    bool hL[kMuWave], hU[kMuWave];
};
__device__ __forceinline__ void mu_lane_load(const IpmK& K, int64_t b, MuLane& E) {
    const int nf = K.nf, lane = threadIdx.x;
#pragma unroll
    for (int e = 0; e < kMuWave; ++e) {
        const int i = lane + 64 * e;
        const bool in = i < nf;
        const int q = in ? K.pos[i] : 0;
        E.hL[e] = in && K.hasL[i];
        E.hU[e] = in && K.hasU[i];
        E.a[e] = in ? K.rb[b * K.nKp + q] : 0.0;
        E.c[e] = in ? K.rbc[b * K.nKp + q] : 0.0;
        const double x = in ? K.x[b * nf + i] : 0.0;
        E.sl[e] = E.hL[e] ? x - K.lbI[b * nf + i] : 1.0;
        E.su[e] = E.hU[e] ? K.ubI[b * nf + i] - x : 1.0;
        E.zl[e] = E.hL[e] ? K.zl[b * nf + i] : 1.0;
        E.zu[e] = E.hU[e] ? K.zu[b * nf + i] : 1.0;
        E.isl[e] = 1.0 / E.sl[e];
        E.isu[e] = 1.0 / E.su[e];
        E.izl[e] = 1.0 / E.zl[e];
        E.izu[e] = 1.0 / E.zu[e];
    }
}
// wave reduction by DPP (row_shr scans within rows of 16 lanes, row broadcasts, readlane 63): lanes a shift leaves
// without a source combine with the identity.  (__shfl_xor lowers to ds_bpermute, an LDS round trip per step.)
#define CFX_DPP_OP(v, op, id, CTRL, RM, BM)                                                                      \
    do {                                                                                                        \
        const int slo_ = __builtin_amdgcn_update_dpp(__double2loint(id), __double2loint(v), CTRL, RM, BM, false); \
        const int shi_ = __builtin_amdgcn_update_dpp(__double2hiint(id), __double2hiint(v), CTRL, RM, BM, false); \
        v = op(v, __hiloint2double(shi_, slo_));                                                                \
    } while (0)
template <class Op>
__device__ __forceinline__ double wreduce(double v, Op op, double id) {
    CFX_DPP_OP(v, op, id, 0x111, 0xf, 0xf);  // row_shr:1
    CFX_DPP_OP(v, op, id, 0x112, 0xf, 0xf);  // row_shr:2
    CFX_DPP_OP(v, op, id, 0x114, 0xf, 0xf);  // row_shr:4
    CFX_DPP_OP(v, op, id, 0x118, 0xf, 0xf);  // row_shr:8 (lane 15 of each row: the row's value)
    CFX_DPP_OP(v, op, id, 0x142, 0xa, 0xf);  // row_bcast:15 into rows 1 and 3
    CFX_DPP_OP(v, op, id, 0x143, 0xc, 0xf);  // row_bcast:31 into rows 2 and 3 (lane 63: the wave's)
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63), __builtin_amdgcn_readlane(__double2loint(v), 63));
}
// -ds / s where the step shrinks a positive quantity (has, ds < 0), else 0
__device__ __forceinline__ double shrink_rate(bool has, double ds, double inv_s) { return (has && ds < 0) ? -ds * inv_s : 0.0; }
__device__ __forceinline__ double step_from_rate(double r, double tau) { return r > 0 ? tau / r : (r != r ? r : INFINITY); }
// the wave's maximum of non-negative rates by v_max_f64 steps, NaN if any lane holds one (fmax would drop it)
__device__ __forceinline__ double wmax_rate(double r) {
    const bool nan = __ballot(r != r) != 0ull;
    const double v = wreduce(r, [](double a, double c) { return fmax(a, c); }, 0.0);
    return nan ? __longlong_as_double(0x7ff8000000000000ll) : v;
}
__device__ __forceinline__ double mu_quality_w(const IpmK& K, const MuLane& E, const Scal& S, double mu) {
    const int nf = K.nf;
    const double tau = clamp_lo(1.0 - mu, K.o.tau_min);
    // the primal and the dual fraction to the boundary: min over both sides = tau / the larger shrink rate
    double rp = 0.0, rz = 0.0;
#pragma unroll
    for (int e = 0; e < kMuWave; ++e) {
        if (threadIdx.x + 64 * e >= nf) break;
        const double dx = E.a[e] + mu * E.c[e];
        const bool hL = E.hL[e], hU = E.hU[e];
        const double vzl = mu * E.isl[e] - E.zl[e] - E.zl[e] * E.isl[e] * dx;
        const double vzu = mu * E.isu[e] - E.zu[e] + E.zu[e] * E.isu[e] * dx;
        rp = max_n(rp, max_n(shrink_rate(hL, dx, E.isl[e]), shrink_rate(hU, -dx, E.isu[e])));
        rz = max_n(rz, max_n(shrink_rate(hL, vzl, E.izl[e]), shrink_rate(hU, vzu, E.izu[e])));
    }
    const double ap = clamp_hi(step_from_rate(wmax_rate(rp), tau), 1.0);
    const double ad = clamp_hi(step_from_rate(wmax_rate(rz), tau), 1.0);
    double cs = 0.0;
#pragma unroll
    for (int e = 0; e < kMuWave; ++e) {
        if (threadIdx.x + 64 * e >= nf) break;
        const double dx = E.a[e] + mu * E.c[e];
        if (E.hL[e]) {
            const double t = (E.sl[e] + ap * dx) * (E.zl[e] + ad * (mu * E.isl[e] - E.zl[e] - E.zl[e] * E.isl[e] * dx));
            cs += t * t;
        }
        if (E.hU[e]) {
            const double t = (E.su[e] - ap * dx) * (E.zu[e] + ad * (mu * E.isu[e] - E.zu[e] + E.zu[e] * E.isu[e] * dx));
            cs += t * t;
        }
    }
    cs = wreduce(cs, OpSum(), 0.0);
    double val = (1.0 - ad) * (1.0 - ad) * S.qd / (nf > 0 ? nf : 1);
    if (K.m) val += (1.0 - ap) * (1.0 - ap) * S.qp / K.m;
    if (K.ncomp) val += cs / K.ncomp;
    return val;
}

// sigma from the quality function Q(sigma) by the golden section over log sigma (CalculateMu / PerformGoldenSection),
// as a state machine that asks for one or two quality values at a time (so each caller evaluates Q at one call site:
// the inlined evaluation appears once in the code, and the wide path can run each request as grid passes).  phase 1:
// Q(1 - sigma_tol), Q(1) pending; 2: Q(e^m1), Q(e^m2); 3: one section point (which 1: m1, 2: m2); 4: the end point;
// 5: done, mu = sigma avgc within [mu_min, mu_max].
struct MuSec {
    int phase, nc, which, k;
    double c0, c1, a, bb, a0, b0, m1, m2, qm1, qm2, q_lo, q_hi, qbest, best, ep, mu;
};
__device__ __forceinline__ void musec_start(MuSec& M, const IpmK& K) {
    M.phase = 1;
    M.nc = 2;
    M.c0 = 1.0 - max_n(1e-4, K.o.quality_function_section_sigma_tol);
    M.c1 = 1.0;
}
__device__ __forceinline__ void musec_step(MuSec& M, const IpmK& K, const Scal& S, const double (&Qv)[2]) {
    const double avg = S.avgc;
    const bool safe = avg > 0;
    const double avgs = safe ? avg : 1.0;
    const double g = (3.0 - sqrt(5.0)) / 2.0;
    bool fin = false;
    double sig = 0.0;
    // the next request: one point e^m (which: the section point it becomes, 1 m1, 2 m2, 0 the end point)
    int req = -1;
    double rm = 0.0;
    if (M.phase == 1) {  // which way the quality decreases from sigma = 1
        const double s1m = M.c0, q1m = Qv[0], q1 = Qv[1];
        const bool up = q1m > q1;
        const double s_hi = up ? clamp_hi(S.mu_max / avgs, K.o.sigma_max) : clamp_lo(K.o.mu_min / avgs, K.o.sigma_min);
        const double lo = up ? 1.0 : s_hi;
        const double hi = up ? s_hi : max_n(s_hi, s1m);
        M.q_lo = up ? q1 : -1.0;  // -1: not evaluated
        M.q_hi = up ? -1.0 : q1m;
        if (lo >= hi) {
            sig = up ? hi : lo;
            fin = true;
        } else {
            M.a = M.a0 = log(lo);
            M.bb = M.b0 = log(hi);
            M.m1 = M.a + g * (M.bb - M.a);
            M.m2 = M.a + (1.0 - g) * (M.bb - M.a);
            M.nc = 2;
            M.c0 = exp(M.m1);
            M.c1 = exp(M.m2);
            M.k = 0;
            M.phase = 2;
        }
    } else if (M.phase == 2 || M.phase == 3) {
        // (value selects throughout, no field chosen by a branch: that form keeps M out of registers)
        const bool two = M.phase == 2, w1 = M.which == 1;
        M.qm1 = two || w1 ? Qv[0] : M.qm1;
        M.qm2 = two ? Qv[1] : (w1 ? M.qm2 : Qv[0]);
        bool stop = M.k >= K.o.quality_function_max_section_steps;
        if (!stop) {
            double qmin = INFINITY, qmax = -INFINITY;
            const double qs[4] = {M.q_lo, M.q_hi, M.qm1, M.qm2};
            for (int t = 0; t < 4; ++t)
                if (qs[t] >= 0) qmin = fmin(qmin, qs[t]), qmax = fmax(qmax, qs[t]);
            stop = !(exp(M.bb) - exp(M.a) >= K.o.quality_function_section_sigma_tol * exp(M.bb)) ||
                   !(1.0 - qmin / qmax >= K.o.quality_function_section_qf_tol);
        }
        if (!stop) {
            // the minimum is in [m1, b] (right): a = m1, q_lo = qm1, m1 = m2, qm1 = qm2, m2 = a + (1 - g)(b - a) asked
            // for; else b = m2, q_hi = qm2, m2 = m1, qm2 = qm1, m1 = a + g (b - a) asked for
            const bool right = M.qm1 > M.qm2;
            const double a = right ? M.m1 : M.a, bb = right ? M.bb : M.m2;
            const double m1 = right ? M.m2 : a + g * (bb - a);
            const double m2 = right ? a + (1.0 - g) * (bb - a) : M.m1;
            M.q_lo = right ? M.qm1 : M.q_lo;
            M.q_hi = right ? M.q_hi : M.qm2;
            const double qm1 = right ? M.qm2 : M.qm1, qm2 = right ? M.qm2 : M.qm1;
            M.a = a, M.bb = bb, M.m1 = m1, M.m2 = m2, M.qm1 = qm1, M.qm2 = qm2;
            rm = right ? m2 : m1;
            req = right ? 2 : 1;
            M.k += 1;
            M.phase = 3;
        } else {
            double best = M.qm1 < M.qm2 ? M.m1 : M.m2;
            const double qbest = M.qm1 < M.qm2 ? M.qm1 : M.qm2;
            const bool hi_end = M.bb == M.b0, lo_end = M.a == M.a0 && !hi_end;  // an end point never moved competes
            if (hi_end || lo_end) {
                const double qe = hi_end ? M.q_hi : M.q_lo, ep = hi_end ? M.bb : M.a;
                if (qe < 0) {
                    M.best = best;
                    M.qbest = qbest;
                    M.ep = ep;
                    rm = ep, req = 0;
                    M.phase = 4;
                } else {
                    if (qe < qbest) best = ep;
                    sig = exp(best);
                    fin = true;
                }
            } else {
                sig = exp(best);
                fin = true;
            }
        }
    } else if (M.phase == 4) {
        sig = exp(Qv[0] < M.qbest ? M.ep : M.best);
        fin = true;
    }
    if (req >= 0) {
        M.nc = 1;
        M.c0 = exp(rm);
        M.which = req;
    }
    if (fin) {
        M.mu = safe ? clamp_lo(min_n(sig * avg, S.mu_max), K.o.mu_min) : K.o.mu_min;
        M.phase = 5;
    }
}
// the section driven to its end by one evaluation site (every thread of the caller runs the same decisions)
template <class QF>
__device__ __forceinline__ double mu_section(const IpmK& K, const Scal& S, QF Q) {
    MuSec M;
    musec_start(M, K);
#pragma unroll 1
    while (M.phase != 5) {
        double q0 = 0.0, q1 = 0.0;
#pragma unroll 1
        for (int c = 0; c < M.nc; ++c) {
            const double q = Q((c == 0 ? M.c0 : M.c1) * S.avgc);
            q0 = c == 0 ? q : q0;
            q1 = c == 0 ? q1 : q;
        }
        const double Qv[2] = {q0, q1};
        musec_step(M, K, S, Qv);
    }
    return M.mu;
}

// mu = sigma avgc within [mu_min, mu_max] from mu_section; then the Newton step rb += mu rbc, mu and tau stored
__global__ void __launch_bounds__(kIB) k_mu_oracle(const IpmK K) {
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    load_scal(K, b, S);
    if (S.done || S.rs_on || !S.mfree) return;  // block-uniform
    double* rb = K.rb + b * K.nKp;
    const double* rc = K.rbc + b * K.nKp;
    if (K.nf <= 64 * kMuWave && !K.mu_block) {  // wavefront 0 alone (block-uniform branch; the other waves leave)
        if (threadIdx.x >= 64) return;
        MuLane E;
        mu_lane_load(K, b, E);
        const double mu = mu_section(K, S, [&](double m) { return mu_quality_w(K, E, S, m); });
        for (int i = threadIdx.x; i < K.nK; i += 64) {
            const int q = K.pos[i];
            rb[q] += mu * rc[q];
        }
        if (threadIdx.x == 0) {
            K.sc[b].mu = mu;
            K.sc[b].tau = clamp_lo(1.0 - mu, K.o.tau_min);
        }
        return;
    }
    const double mu = mu_section(K, S, [&](double m) { return mu_quality(K, b, S, m); });
    __syncthreads();
    for (int i = threadIdx.x; i < K.nK; i += kIB) {
        const int q = K.pos[i];
        rb[q] += mu * rc[q];
    }
    if (threadIdx.x == 0) {
        S.mu = mu;
        S.tau = clamp_lo(1.0 - mu, K.o.tau_min);
    }
    store_scal(K, b, S);
}

// ---- adaptive mu on wide instances (IpmK::wide): the section's requests (MuSec) as rounds of three launches — the
// candidates' partial step-fraction minima over a grid (k_wmu_min), the partial complementarity sums with every block
// reducing those minima in wide_get's order (k_wmu_sum), the one-block step of the machine on the quality values
// (k_wmu_ctl) — so that a quality evaluation is a grid pass instead of one block's loop over the instance (9.6 ms per
// call on the reaching task, 65 % of an iteration's kernels).  State [B][kGS] (musec_load / musec_store); rounds after
// the machine's phase 5 return at once, and k_wmu_apply adds mu rbc to rb.
constexpr int kGS = 24;
enum { MG_PHASE = 0, MG_NC, MG_C0, MG_C1, MG_MU };  // MuSec's fields in st[]: these first, the rest after
__device__ inline MuSec musec_load(const double* st) {
    MuSec M;
    M.phase = (int)st[MG_PHASE], M.nc = (int)st[MG_NC], M.c0 = st[MG_C0], M.c1 = st[MG_C1], M.mu = st[MG_MU];
    M.which = (int)st[5], M.k = (int)st[6], M.a = st[7], M.bb = st[8], M.a0 = st[9], M.b0 = st[10], M.m1 = st[11];
    M.m2 = st[12], M.qm1 = st[13], M.qm2 = st[14], M.q_lo = st[15], M.q_hi = st[16], M.qbest = st[17], M.best = st[18];
    M.ep = st[19];
    return M;
}
__device__ inline void musec_store(const MuSec& M, double* st) {
    st[MG_PHASE] = M.phase, st[MG_NC] = M.nc, st[MG_C0] = M.c0, st[MG_C1] = M.c1, st[MG_MU] = M.mu;
    st[5] = M.which, st[6] = M.k, st[7] = M.a, st[8] = M.bb, st[9] = M.a0, st[10] = M.b0, st[11] = M.m1;
    st[12] = M.m2, st[13] = M.qm1, st[14] = M.qm2, st[15] = M.q_lo, st[16] = M.q_hi, st[17] = M.qbest, st[18] = M.best;
    st[19] = M.ep;
}

// grid (B, ceil(nK / kIB)): k_mu_cen_rhs elementwise
__global__ void __launch_bounds__(kIB) k_wmu_cen_rhs(const IpmK K) {
    const int64_t b = blockIdx.x;
    const int i = blockIdx.y * kIB + threadIdx.x;
    if (i >= K.nK) return;
    const bool on = !K.sc[b].done && !K.sc[b].rs_on && K.sc[b].mfree;
    K.rbc[b * K.nKp + K.pos[i]] = (on && i < K.nf) ? K.rhsmu[b * K.nf + i] : 0.0;
}

__global__ void __launch_bounds__(kIB) k_wmu_init(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (threadIdx.x != 0) return;
    const Scal& S = K.sc[b];
    double* st = K.mgs + b * kGS;
    if (S.done || S.rs_on || !S.mfree) {
        st[MG_PHASE] = 0.0;
        return;
    }
    MuSec M{};
    musec_start(M, K);
    musec_store(M, st);
}

// the candidates' mu = sigma avgc (at most two)
__device__ inline int wmu_cands(const IpmK& K, int64_t b, double (&mu)[2]) {
    const double* st = K.mgs + b * kGS;
    const int ph = (int)st[MG_PHASE];
    if (ph < 1 || ph > 4) return 0;
    const double avg = K.sc[b].avgc;
    const int nc = (int)st[MG_NC];
    mu[0] = st[MG_C0] * avg;
    mu[1] = nc > 1 ? st[MG_C1] * avg : mu[0];
    return nc;
}

// grid (B, kWideParts): partial minima of the candidates' primal / dual fractions to the boundary (mu_quality's first
// loop), wpart slots 0..7
__global__ void __launch_bounds__(kIB) k_wmu_min(const IpmK K) {
    const int64_t b = blockIdx.x;
    double mu[2];
    const int nc = wmu_cands(K, b, mu);
    if (nc == 0) return;
    const int nf = K.nf;
    const double tau[2] = {clamp_lo(1.0 - mu[0], K.o.tau_min), clamp_lo(1.0 - mu[1], K.o.tau_min)};
    const double* x = K.x + b * nf;
    const double* zl = K.zl + b * nf;
    const double* zu = K.zu + b * nf;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    const double* ra = K.rb + b * K.nKp;
    const double* rc = K.rbc + b * K.nKp;
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = INFINITY;
    for (int i = blockIdx.y * kIB + threadIdx.x; i < nf; i += kWideParts * kIB) {
        const int q = K.pos[i];
        const double a = ra[q], c = rc[q];
        const bool hL = K.hasL[i], hU = K.hasU[i];
        const double sl = hL ? x[i] - lbI[i] : 1.0, su = hU ? ubI[i] - x[i] : 1.0;
        const double zli = zl[i], zui = zu[i];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const double dx = a + mu[t] * c;
            const double vzl = hL ? mu[t] / sl - zli - zli / sl * dx : 0.0;
            const double vzu = hU ? mu[t] / su - zui + zui / su * dx : 0.0;
            v[4 * t] = min_n(v[4 * t], step_term(hL, sl, dx, tau[t]));
            v[4 * t + 1] = min_n(v[4 * t + 1], step_term(hU, su, -dx, tau[t]));
            v[4 * t + 2] = min_n(v[4 * t + 2], step_term(hL, zli, vzl, tau[t]));
            v[4 * t + 3] = min_n(v[4 * t + 3], step_term(hU, zui, vzu, tau[t]));
        }
    }
    const int ro[8] = {2, 2, 2, 2, 2, 2, 2, 2};
    wide_put(K, b, v, ro);
}

// the candidates' (a_p, a_d) from k_wmu_min's partials (every block and the control kernel the same values)
__device__ inline void wmu_fractions(const IpmK& K, int64_t b, double (&ap)[2], double (&ad)[2]) {
    double v[8];
    const int ro[8] = {2, 2, 2, 2, 2, 2, 2, 2};
    wide_get(K, b, v, ro);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        ap[t] = min_n(clamp_hi(v[4 * t], 1.0), clamp_hi(v[4 * t + 1], 1.0));
        ad[t] = min_n(clamp_hi(v[4 * t + 2], 1.0), clamp_hi(v[4 * t + 3], 1.0));
    }
}

// grid (B, kWideParts): partial sums of the predicted complementarity (mu_quality's second loop), wpart slots 8, 9
__global__ void __launch_bounds__(kIB) k_wmu_sum(const IpmK K) {
    const int64_t b = blockIdx.x;
    double mu[2];
    if (wmu_cands(K, b, mu) == 0) return;  // (block-uniform)
    double ap[2], ad[2];
    wmu_fractions(K, b, ap, ad);
    const int nf = K.nf;
    const double* x = K.x + b * nf;
    const double* zl = K.zl + b * nf;
    const double* zu = K.zu + b * nf;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    const double* ra = K.rb + b * K.nKp;
    const double* rc = K.rbc + b * K.nKp;
    double cs[2] = {0.0, 0.0};
    for (int i = blockIdx.y * kIB + threadIdx.x; i < nf; i += kWideParts * kIB) {
        const int q = K.pos[i];
        const bool hL = K.hasL[i], hU = K.hasU[i];
        if (!hL && !hU) continue;
        const double a = ra[q], c = rc[q];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const double dx = a + mu[t] * c;
            if (hL) {
                const double sl = x[i] - lbI[i];
                const double u = (sl + ap[t] * dx) * (zl[i] + ad[t] * (mu[t] / sl - zl[i] - zl[i] / sl * dx));
                cs[t] += u * u;
            }
            if (hU) {
                const double su = ubI[i] - x[i];
                const double u = (su - ap[t] * dx) * (zu[i] + ad[t] * (mu[t] / su - zu[i] + zu[i] / su * dx));
                cs[t] += u * u;
            }
        }
    }
    const int ro[2] = {0, 0};
    breduce_n(cs, ro);
    if (threadIdx.x == 0) {
        double* pp = K.wpart + (b * kWideParts + blockIdx.y) * kWP;
        pp[8] = cs[0];
        pp[9] = cs[1];
    }
}

// one block per instance: the candidates' quality values and one step of k_mu_oracle's section
__global__ void __launch_bounds__(kIB) k_wmu_ctl(const IpmK K) {
    const int64_t b = blockIdx.x;
    double mu[2];
    const int nc = wmu_cands(K, b, mu);
    if (nc == 0) return;  // (block-uniform)
    double ap[2], ad[2];
    wmu_fractions(K, b, ap, ad);
    double cs[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
        cs[t] = threadIdx.x < kWideParts ? K.wpart[(b * kWideParts + threadIdx.x) * kWP + 8 + t] : 0.0;
    const int ro[2] = {0, 0};
    breduce_n(cs, ro);
    if (threadIdx.x != 0) return;
    const Scal& S = K.sc[b];
    const int nf = K.nf;
    double Qv[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        double val = (1.0 - ad[t]) * (1.0 - ad[t]) * S.qd / (nf > 0 ? nf : 1);
        if (K.m) val += (1.0 - ap[t]) * (1.0 - ap[t]) * S.qp / K.m;
        if (K.ncomp) val += cs[t] / K.ncomp;
        Qv[t] = val;
    }
    double* st = K.mgs + b * kGS;
    MuSec M = musec_load(st);
    musec_step(M, K, S, Qv);
    musec_store(M, st);
    if (M.phase == 5) {
        K.sc[b].mu = M.mu;
        K.sc[b].tau = clamp_lo(1.0 - M.mu, K.o.tau_min);
    }
}

// grid (B, ceil(nK / kIB)): the Newton step rb += mu rbc of the instances whose section finished
__global__ void __launch_bounds__(kIB) k_wmu_apply(const IpmK K) {
    const int64_t b = blockIdx.x;
    const double* st = K.mgs + b * kGS;
    if ((int)st[MG_PHASE] != 5) return;
    const int i = blockIdx.y * kIB + threadIdx.x;
    if (i >= K.nK) return;
    const int q = K.pos[i];
    K.rb[b * K.nKp + q] += st[MG_MU] * K.rbc[b * K.nKp + q];
}

// dz, fraction to the boundary, filter quantities at x, first trial point (solver.py, after the inertia loop)
__global__ void __launch_bounds__(kIB) k_ipm_dir(const IpmK K, int it) {
    __shared__ double sh[kIB / 64];
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    if (S.rs_on) return;  // block-uniform: k_rs_dir's
    const double* x = K.x + b * nf;
    const double* zl = K.zl + b * nf;
    const double* zu = K.zu + b * nf;
    const double* dx = K.dx + b * nf;
    const double* gF = K.gF + b * nf;
    double* dzl = K.dzl + b * nf;
    double* dzu = K.dzu + b * nf;
    const double mu = S.mu, tau = S.tau;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    double apl = INFINITY, apu = INFINITY, azl = INFINITY, azu = INFINITY, dphi = 0.0, theta = 0.0;
    double phi;
    if (K.wide) {  // k_wdir_a's partials
        double rv[9];
        const int ro[9] = {2, 2, 2, 2, 0, 0, 0, 0, 1};
        wide_get(K, b, rv, ro);
        apl = rv[0], apu = rv[1], azl = rv[2], azu = rv[3], dphi = rv[4], theta = rv[5];
        phi = rv[8] > 0 ? INFINITY : S.fS - mu * (rv[6] + rv[7]);
    } else {
    for (int i = threadIdx.x; i < nf; i += kIB) {
        const bool hL = K.hasL[i], hU = K.hasU[i];
        const double sl = hL ? x[i] - lbI[i] : 1.0, su = hU ? ubI[i] - x[i] : 1.0;
        const double vzl = hL ? mu / sl - zl[i] - zl[i] / sl * dx[i] : 0.0;
        const double vzu = hU ? mu / su - zu[i] + zu[i] / su * dx[i] : 0.0;
        dzl[i] = vzl;
        dzu[i] = vzu;
        apl = min_n(apl, step_term(hL, sl, dx[i], tau));
        apu = min_n(apu, step_term(hU, su, -dx[i], tau));
        azl = min_n(azl, step_term(hL, zl[i], vzl, tau));
        azu = min_n(azu, step_term(hU, zu[i], vzu, tau));
        const double bar = (hL ? mu / sl : 0.0) - (hU ? mu / su : 0.0);
        dphi += (gF[i] - bar) * dx[i];
    }
    for (int j = threadIdx.x; j < m; j += kIB) theta += fabs(K.gS[b * m + j]);
    {
        double rv[6] = {apl, apu, azl, azu, dphi, theta};
        const int ro[6] = {2, 2, 2, 2, 0, 0};
        breduce_n(rv, ro);
        apl = rv[0];
        apu = rv[1];
        azl = rv[2];
        azu = rv[3];
        dphi = rv[4];
        theta = rv[5];
    }
    phi = barrier_obj(K, b, x, S.fS, mu, sh);
    }
    const double a_p = min_n(clamp_hi(apl, 1.0), clamp_hi(apu, 1.0));
    // watchdog start (Ipopt StartWatchDog): remember this iterate and its line-search reference values
    const int trig = K.o.watchdog_shortened_iter_trigger;
    const bool wd_start = !S.done && !S.wd_on && trig > 0 && S.wd_short >= trig;
    if (wd_start) {
        for (int i = threadIdx.x; i < nf; i += kIB) {
            K.wx[b * nf + i] = x[i];
            K.wzl[b * nf + i] = zl[i];
            K.wzu[b * nf + i] = zu[i];
        }
        for (int j = threadIdx.x; j < m; j += kIB) K.wy[b * m + j] = K.y[b * m + j];
    }
    const double alpha0 = S.skip_first ? 0.5 * a_p : a_p;
    __syncthreads();
    if (threadIdx.x == 0) {
        S.dwl = S.dw;
        S.a_p = a_p;
        S.a_z = min_n(clamp_hi(azl, 1.0), clamp_hi(azu, 1.0));
        S.theta = theta;
        S.phi = phi;
        S.dphi = dphi;
        if (it == 0) {
            S.theta_max = 1e4 * clamp_lo(theta, 1.0);
            S.theta_min = 1e-4 * clamp_lo(theta, 1.0);
        }
        if (wd_start) {
            S.wd_on = 1;
            S.wd_trial = 0;
            S.wd_theta = theta;
            S.wd_phi = phi;
            S.wd_dphi = dphi;
            S.wd_ap = a_p;
            S.wd_mu = mu;
        }
        S.alpha = alpha0;
        S.accepted = S.done || S.soft_on;  // soft-restoration steps replace the line search (k_soft_trial)
        S.armijo = 0;
        S.soc = 0;
        S.forced = 0;
        S.rejf = 0;  // Ipopt's InitThisLineSearch
    }
    if (!K.wide) {  // (wide: k_wdir_c)
        double* xacc = K.xacc + b * nf;
        double* xt = K.xt + b * nf;
        for (int i = threadIdx.x; i < nf; i += kIB) {
            xacc[i] = x[i];
            xt[i] = x[i] + alpha0 * dx[i];
        }
        __syncthreads();
        write_full(K, b, xt, K.vt);
    }
    store_scal(K, b, S);
}

// after g, f at the trial point: filter acceptance (solver.py line search); at ls == 0 the second-order
// correction set-up.  counters: [0] not accepted (instances in the restoration phase counted after k_rs_accept),
// [1] second-order corrections wanted
__global__ void __launch_bounds__(kIB) k_ipm_accept(const IpmK K, int ls, int slot) {
    __shared__ double sh[kIB / 64];
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    if (S.rs_on) {  // block-uniform
        count_add(K, slot, 0, S.rs_exit == RS_RUNNING && !S.rs_acc);
        if (K.wide && threadIdx.x == 0) K.wflag[b * kWF] = 0.0;  // k_wacc_c: nothing to do
        return;
    }
    const double* sg = K.sg + b * m;
    const double* gt = K.gt + b * m;
    double tt = 0.0, pt;
    const double* xt = K.xt + b * nf;
    if (K.wide) {  // k_wacc_a's partials
        double rv[4];
        const int ro[4] = {0, 0, 0, 1};
        wide_get(K, b, rv, ro);
        tt = rv[0];
        pt = rv[3] > 0 ? INFINITY : K.ft[b] * S.sf - S.mu * (rv[1] + rv[2]);
    } else {
        for (int j = threadIdx.x; j < m; j += kIB) tt += fabs(gt[j] * sg[j]);
        tt = breduce(tt, OpSum(), sh);
        pt = barrier_obj(K, b, xt, K.ft[b] * S.sf, S.mu, sh);
    }
    bool ok, arm, rejf;
    filter_accept(K, S, K.filt + b * kFilt * 2, tt, pt, S.alpha, sh, ok, arm, &rejf);
    const bool rej_here = rejf && !S.accepted;
    ok = ok && !S.accepted;
    // a watchdog iteration takes its full step whether or not it is acceptable (no corrections, no backtracking)
    const bool forced = ls == 0 && S.wd_on && !ok && !S.accepted;
    bool soc = false;
    if (ls == 0) soc = !S.accepted && !ok && !forced && (tt >= S.theta) && !S.skip_first;
    if (K.wide) {  // (k_wacc_c)
        if (threadIdx.x == 0) {
            double* wf = K.wflag + b * kWF;
            wf[0] = 1.0;
            wf[1] = ls == 0;
            wf[2] = ok || forced;
            wf[3] = S.alpha;
        }
    } else {
        if (ls == 0) {
            double* cs = K.csoc + b * m;
            for (int j = threadIdx.x; j < m; j += kIB) cs[j] = S.alpha * K.gS[b * m + j] + gt[j] * sg[j];
        }
        if (ok || forced) {
            double* xacc = K.xacc + b * nf;
            for (int i = threadIdx.x; i < nf; i += kIB) xacc[i] = xt[i];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (ls == 0) {
            S.soc = soc;
            S.theta_soc = tt;
        }
        if (rej_here) S.rejf = 1;
        if (ok) {
            S.armijo = arm;
            S.accepted = 1;
        }
        if (forced) {
            S.forced = 1;
            S.accepted = 1;
        }
    }
    store_scal(K, b, S);
    if (threadIdx.x == 0) {
        count_add(K, slot, 0, !S.accepted);
        if (S.soc) atomicAdd(K.cnt + 4 * slot + 1, 1);
        if (S.soft_on && !S.done) atomicAdd(K.cnt + 4 * slot + 2, 1);  // taking soft steps (no line search)
    }
}

// backtracking: halve alpha where no trial was accepted, next trial point
__global__ void __launch_bounds__(kIB) k_ipm_next_trial(const IpmK K) {
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    load_scal(K, b, S);
    if (S.accepted || S.rs_on) return;  // block-uniform
    const double a = S.alpha * 0.5;
    const int nf = K.nf;
    const double* x = K.x + b * nf;
    const double* dx = K.dx + b * nf;
    double* xt = K.xt + b * nf;
    for (int i = threadIdx.x; i < nf; i += kIB) xt[i] = x[i] + a * dx[i];
    __syncthreads();
    write_full(K, b, xt, K.vt);
    if (threadIdx.x == 0) K.sc[b].alpha = a;
}

// second-order correction: rhs [alpha rhs_x; -c_soc] in band order (the factors of the iteration are reused)
__global__ void __launch_bounds__(kIB) k_ipm_soc_rhs(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;  // block-uniform
    const double a = K.sc[b].alpha, mu = K.sc[b].mu;
    const int nf = K.nf;
    for (int i = threadIdx.x; i < K.nK; i += kIB) {
        // (adaptive: rhs holds the affine part, the final mu's term added)
        const double rx = i < nf ? (K.adapt ? K.rhs[b * K.nK + i] + mu * K.rhsmu[b * nf + i] : K.rhs[b * K.nK + i]) : 0.0;
        K.rb[b * K.nKp + K.pos[i]] = i < nf ? rx * a : -K.csoc[b * K.m + (i - nf)];
    }
}

// corrected trial x + a_c dx_c (into xr)
__global__ void __launch_bounds__(kIB) k_ipm_soc_trial(const IpmK K) {
    const int64_t b = blockIdx.x;
    if (K.sc[b].rs_on) return;  // block-uniform: xr, vt hold the phase's iterate and trial
    const int nf = K.nf;
    const double* x = K.x + b * nf;
    const double* rb = K.rb + b * K.nKp;
    const double tau = K.sc[b].tau;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    double apl = INFINITY, apu = INFINITY;
    for (int i = threadIdx.x; i < nf; i += kIB) {
        const double d = rb[K.pos[i]];
        if (K.hasL[i]) apl = min_n(apl, step_term(true, x[i] - lbI[i], d, tau));
        if (K.hasU[i]) apu = min_n(apu, step_term(true, ubI[i] - x[i], -d, tau));
    }
    {
        double rv[2] = {apl, apu};
        const int ro[2] = {2, 2};
        breduce_n(rv, ro);
        apl = rv[0];
        apu = rv[1];
    }
    const double a_c = min_n(clamp_hi(apl, 1.0), clamp_hi(apu, 1.0));
    double* xr = K.xr + b * nf;
    for (int i = threadIdx.x; i < nf; i += kIB) xr[i] = x[i] + a_c * rb[K.pos[i]];
    __syncthreads();
    write_full(K, b, xr, K.vt);
    if (threadIdx.x == 0) K.sc[b].a_c = a_c;
}

__global__ void __launch_bounds__(kIB) k_ipm_soc_accept(const IpmK K, int slot) {
    __shared__ double sh[kIB / 64];
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    if (S.rs_on) {  // block-uniform
        count_add(K, slot, 0, S.rs_exit == RS_RUNNING && !S.rs_acc);
        if (K.wide && threadIdx.x == 0) K.wflag[b * kWF] = 0.0;  // k_wacc_c: nothing to do
        return;
    }
    const double* sg = K.sg + b * m;
    const double* gt = K.gt + b * m;
    double tt = 0.0, pt;
    const double* xr = K.xr + b * nf;
    if (K.wide) {  // k_wacc_a's partials (soc = 1)
        double rv[4];
        const int ro[4] = {0, 0, 0, 1};
        wide_get(K, b, rv, ro);
        tt = rv[0];
        pt = rv[3] > 0 ? INFINITY : K.ft[b] * S.sf - S.mu * (rv[1] + rv[2]);
    } else {
        for (int j = threadIdx.x; j < m; j += kIB) tt += fabs(gt[j] * sg[j]);
        tt = breduce(tt, OpSum(), sh);
        pt = barrier_obj(K, b, xr, K.ft[b] * S.sf, S.mu, sh);
    }
    bool okc, armc, rejfc;
    filter_accept(K, S, K.filt + b * kFilt * 2, tt, pt, S.alpha, sh, okc, armc, &rejfc);
    const bool rej_here = rejfc && S.soc && !S.accepted;
    okc = okc && S.soc && (S.a_c >= 0.99);
    if (K.wide) {  // (k_wsoca_c)
        if (threadIdx.x == 0) {
            double* wf = K.wflag + b * kWF;
            wf[0] = 1.0;
            wf[1] = 1.0;
            wf[2] = okc;
            wf[3] = S.a_c;
        }
    } else {
        if (okc) {
            double* xacc = K.xacc + b * nf;
            for (int i = threadIdx.x; i < nf; i += kIB) xacc[i] = xr[i];
        }
        double* cs = K.csoc + b * m;
        for (int j = threadIdx.x; j < m; j += kIB) cs[j] = S.a_c * cs[j] + gt[j] * sg[j];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (okc) {
            S.armijo = armc;
            S.accepted = 1;
        }
        if (rej_here) S.rejf = 1;
        S.soc = S.soc && !okc && (S.a_c >= 0.99) && (tt <= K.o.kappa_soc * S.theta_soc);
        S.theta_soc = tt;
    }
    store_scal(K, b, S);
    if (threadIdx.x == 0) {
        count_add(K, slot, 0, !S.accepted);
        if (S.soc) atomicAdd(K.cnt + 4 * slot + 1, 1);
    }
}

// restoration (solver.py _restoration_step), for the instances whose line search failed: step from the band
// solve of [[Sigma + I, J^T], [J, 0]] [dx; .] = [0; -g], fraction to the boundary, first trial
__global__ void __launch_bounds__(kIB) k_ipm_resto_init(const IpmK K, int slot) {
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    const double* x = K.x + b * nf;
    const double* rb = K.rb + b * K.nKp;
    double* dxr = K.dxr + b * nf;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    double apl = INFINITY, apu = INFINITY, th = 0.0;
    for (int i = threadIdx.x; i < nf; i += kIB) {
        const double d = rb[K.pos[i]];
        dxr[i] = d;
        if (K.hasL[i]) apl = min_n(apl, step_term(true, x[i] - lbI[i], d, S.tau));
        if (K.hasU[i]) apu = min_n(apu, step_term(true, ubI[i] - x[i], -d, S.tau));
    }
    for (int j = threadIdx.x; j < m; j += kIB) th += fabs(K.gS[b * m + j]);
    {
        double rv[3] = {apl, apu, th};
        const int ro[3] = {2, 2, 0};
        breduce_n(rv, ro);
        apl = rv[0];
        apu = rv[1];
        th = rv[2];
    }
    const double a = min_n(clamp_hi(apl, 1.0), clamp_hi(apu, 1.0));
    const bool failed = !S.accepted && !S.done;
    double* xr = K.xr + b * nf;
    double* xt = K.xt + b * nf;
    for (int i = threadIdx.x; i < nf; i += kIB) {
        xr[i] = x[i];
        xt[i] = x[i] + a * dxr[i];
    }
    __syncthreads();
    if (failed) write_full(K, b, xt, K.vt);
    if (threadIdx.x == 0) {
        S.a_r = a;
        S.theta_r = th;
        S.todo = failed;
    }
    store_scal(K, b, S);
    count_add(K, slot, 0, failed);
}

__global__ void __launch_bounds__(kIB) k_ipm_resto_accept(const IpmK K, int slot) {
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    const double* sg = K.sg + b * m;
    const double* gt = K.gt + b * m;
    double tt = 0.0, nonfin = 0.0;
    for (int j = threadIdx.x; j < m; j += kIB) {
        const double v = gt[j] * sg[j];
        if (!isfinite(v)) nonfin = 1.0;
        tt += fabs(v);
    }
    {
        double rv[2] = {tt, nonfin};
        const int ro[2] = {0, 1};
        breduce_n(rv, ro);
        tt = rv[0];
        nonfin = rv[1];
    }
    const bool ok = S.todo && !(nonfin > 0) && (tt < S.theta_r);
    const double* x = K.x + b * nf;
    const double* dxr = K.dxr + b * nf;
    double* xt = K.xt + b * nf;
    double* xr = K.xr + b * nf;
    if (ok)
        for (int i = threadIdx.x; i < nf; i += kIB) xr[i] = xt[i];
    const bool todo = S.todo && !ok;
    const double a = S.a_r * 0.5;
    if (todo)
        for (int i = threadIdx.x; i < nf; i += kIB) xt[i] = x[i] + a * dxr[i];
    __syncthreads();
    if (todo) write_full(K, b, xt, K.vt);
    if (threadIdx.x == 0) {
        S.todo = todo;
        S.a_r = a;
    }
    store_scal(K, b, S);
    count_add(K, slot, 0, todo);
}

// ---- Ipopt's soft restoration (IpBacktrackingLineSearch::TrySoftRestoStep; solver.py, soft_resto_...) ----------
// Ipopt's primal-dual system error of the scaled problem at (x, y, zl, zu): (|grad L|_1 + |c|_1 + sum |s z - mu|) / npd.
// gF / gS: the scaled objective gradient and constraints at x; the scaled J_g values are jac[jsel] d sg (jac_raw) or jv
__device__ double pd_error(const IpmK& K, int64_t b, const double* x, const double* y, double ay, const double* dy,
                           const double* zl, const double* zu, double az, const double* dzl, const double* dzu,
                           const double* gF, const double* jac_raw, const double* jv, const double* gS, double mu) {
    const int nf = K.nf, m = K.m;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    const double* sg = K.sg + b * m;
    double sd = 0.0, sp = 0.0, scl = 0.0, scu = 0.0;
    for (int i = threadIdx.x; i < nf; i += kIB) {
        double jty = 0.0;
#pragma unroll 4
        for (int k = K.jt_ptr[i]; k < K.jt_ptr[i + 1]; ++k) {
            const int s = K.jt_idx[k], r = K.jr[s];
            const double jvs = jac_raw ? jac_raw[K.jsel[s]] * K.d[K.jc[s]] * sg[r] : jv[s];
            jty += jvs * (y[r] + ay * dy[r]);
        }
        const double l = zl[i] + az * dzl[i], u = zu[i] + az * dzu[i];
        sd += fabs(gF[i] + jty - l + u);
        if (K.hasL[i]) scl += fabs((x[i] - lbI[i]) * l - mu);
        if (K.hasU[i]) scu += fabs((ubI[i] - x[i]) * u - mu);
    }
    for (int j = threadIdx.x; j < m; j += kIB) sp += fabs(gS ? gS[j] : 0.0);
    double rv[4] = {sd, sp, scl, scu};
    const int ro[4] = {0, 0, 0, 0};
    breduce_n(rv, ro);
    return (((rv[0] + rv[1]) + rv[2]) + rv[3]) / K.npd;
}

// after the line search: the instances taking soft steps count one more (past max_soft_resto_iters their search counts
// as failed); the candidates — failed searches outside the watchdog, instances taking soft steps — get the trial
// x + a dx, a = min(a_p, a_z), in xt / vt and the primal-dual error at x.  counters: [0] candidates, [1] instances
// whose soft steps ran out
__global__ void __launch_bounds__(kIB) k_soft_trial(const IpmK K, int slot) {
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf;
    load_scal(K, b, S);
    if (S.rs_on || S.done) {  // block-uniform
        count_add(K, slot, 0, 0);
        return;
    }
    const bool was = S.soft_on;
    const int cnt = S.soft_cnt + (was ? 1 : 0);
    const bool over = was && cnt > K.o.max_soft_resto_iters;
    const bool cand = (!S.accepted && !S.wd_on) || (was && !over);
    const double a = min_n(S.a_p, S.a_z);
    double pd = 0.0;
    if (cand) {
        const double* x = K.x + b * nf;
        const double* dx = K.dx + b * nf;
        double* xt = K.xt + b * nf;
        for (int i = threadIdx.x; i < nf; i += kIB) xt[i] = x[i] + a * dx[i];
        __syncthreads();
        write_full(K, b, xt, K.vt);
        pd = pd_error(K, b, x, K.y + b * K.m, 0.0, K.dy + b * K.m, K.zl + b * nf, K.zu + b * nf, 0.0, K.dzl + b * nf,
                      K.dzu + b * nf, K.gF + b * nf, nullptr, K.jv + b * K.nj, K.gS + b * K.m, S.mu);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (over) {
            S.soft_on = 0;
            S.accepted = 0;  // to the restoration phase
        }
        S.soft_cnt = over ? 0 : cnt;
        S.soft_try = cand;
        S.soft_a = a;
        S.soft_pd = pd;
    }
    store_scal(K, b, S);
    if (threadIdx.x == 0) {
        count_add(K, slot, 0, cand);
        if (over) atomicAdd(K.cnt + 4 * slot + 1, 1);
    }
}

// after eval_all at the soft trial points (gt, jact, ft, gradt): take the step when the original filter accepts it
// (alpha 0: the sufficient-decrease test) or it cuts the primal-dual error by soft_resto_pderror_reduction_factor;
// instances whose step the filter did not accept keep taking soft steps, rejected ones go to the restoration phase.
// counters: [0] not accepted (as k_ipm_accept's: instances in the phase counted by their own line search)
__global__ void __launch_bounds__(kIB) k_soft_accept(const IpmK K, int slot) {
    __shared__ double sh[kIB / 64];
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    if (S.rs_on) {  // block-uniform
        count_add(K, slot, 0, S.rs_exit == RS_RUNNING && !S.rs_acc);
        return;
    }
    if (S.done || !S.soft_try) {  // block-uniform
        count_add(K, slot, 0, !S.accepted);
        return;
    }
    const double* sg = K.sg + b * m;
    const double* gt = K.gt + b * m;
    const double* xt = K.xt + b * nf;
    double* gFt = K.sig + b * nf;  // scratch: Sigma is rebuilt by the next k_ipm_begin
    for (int i = threadIdx.x; i < nf; i += kIB) gFt[i] = K.gradt[b * K.n + K.free[i]] * K.d[i] * S.sf;
    double* gSt = K.csoc + b * m;  // scratch: set up again by the next line search
    double tt = 0.0;
    for (int j = threadIdx.x; j < m; j += kIB) {
        gSt[j] = gt[j] * sg[j];
        tt += fabs(gSt[j]);
    }
    tt = breduce(tt, OpSum(), sh);
    const double a = S.soft_a;
    const double pd = pd_error(K, b, xt, K.y + b * m, a, K.dy + b * m, K.zl + b * nf, K.zu + b * nf, a, K.dzl + b * nf,
                               K.dzu + b * nf, gFt, K.jact + b * K.nnzj, nullptr, gSt, S.mu);
    const double pt = barrier_obj(K, b, xt, K.ft[b] * S.sf, S.mu, sh);
    bool ok, arm;
    filter_accept(K, S, K.filt + b * kFilt * 2, tt, pt, 0.0, sh, ok, arm);
    const bool acc = isfinite(pd) && (ok || pd <= K.o.soft_resto_pderror_reduction_factor * S.soft_pd);
    if (acc) {
        double* xacc = K.xacc + b * nf;
        for (int i = threadIdx.x; i < nf; i += kIB) xacc[i] = xt[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        S.accepted = acc;
        S.armijo = 0;
        S.forced = 0;
        S.soft_ok = acc && ok;
        S.soft_on = acc && !ok;
        if (!S.soft_on) S.soft_cnt = 0;
        if (acc) {
            S.alpha = a;  // primal and dual steps of the same length (k_ipm_update)
            S.a_z = a;
            atomicAdd(K.rstat + 2, 1ull);
        }
    }
    store_scal(K, b, S);
    count_add(K, slot, 0, !S.accepted);
}

// least-squares multipliers (Ipopt's constr_mult_init), for the instances flagged reinit
__global__ void __launch_bounds__(kIB) k_ipm_lsmult(const IpmK K) {
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    load_scal(K, b, S);
    if (!S.reinit) return;  // block-uniform
    const int nf = K.nf, m = K.m;
    const double* rb = K.rb + b * K.nKp;
    double big = 0.0, nonfin = 0.0;
    for (int j = threadIdx.x; j < m; j += kIB) {
        const double v = rb[K.pos[nf + j]];
        if (!isfinite(v)) nonfin = 1.0;
        big = max_n(big, fabs(v));
    }
    {
        double rv[2] = {big, nonfin};
        const int ro[2] = {1, 1};
        breduce_n(rv, ro);
        big = rv[0];
        nonfin = rv[1];
    }
    const bool ok = !(nonfin > 0) && big <= 1e3;
    for (int j = threadIdx.x; j < m; j += kIB) K.y[b * m + j] = ok ? rb[K.pos[nf + j]] : 0.0;
    if (threadIdx.x == 0) K.sc[b].reinit = 0;
}

// end of an iteration: filter augmentation, restoration outcome, primal-dual steps, z safeguard.  resto 1: the
// instances whose line search failed took a restoration step (xr); resto 2 (restoration phase): an instance whose phase
// ended this iteration (k_rs_update / k_rs_begin set rs_exit) returns to the main iteration at the phase's point, or —
// when the phase failed or found a point of local infeasibility — stops there, as Ipopt's solve does
// (Restoration_Failed / Infeasible_Problem_Detected); an instance still in the phase (or entering it, k_rs_init) is
// left alone; an instance whose search failed with its iteration budget spent does not move.
__global__ void __launch_bounds__(kIB) k_ipm_update(const IpmK K, int resto) {
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    if (K.wide && threadIdx.x == 0) K.wflag[b * kWF] = 0.0;  // k_wupd_c: nothing to do unless set below
    if (S.rs_on && S.rs_exit == RS_RUNNING) return;  // block-uniform
    const bool phase_end = S.rs_on;
    // a failed phase stops the instance (Ipopt: Restoration_Failed) unless resto_failure_restart (an extension) sends
    // it back to the main iteration from the phase's last point, as a successful phase would
    const bool rs_stop = phase_end && (S.rs_exit == RS_INFEASIBLE ||
                                       (S.rs_exit == RS_FAILED && !K.o.resto_failure_restart));
    if (rs_stop) {
        __syncthreads();
        if (threadIdx.x == 0) {
            S.done = S.stop = 1;
            S.status = S.rs_exit == RS_FAILED ? CFX_IPM_RESTORATION_FAILED : CFX_IPM_INFEASIBLE_PROBLEM_DETECTED;
            S.iters += 1;  // the main iteration whose line search failed
            S.rs_on = 0;
            S.rs_exit = RS_RUNNING;
        }
        store_scal(K, b, S);
        return;
    }
    const bool failed = !S.accepted && !S.done;
    const bool forced = S.forced;
    // a soft-restoration step augments the filter only when the original filter accepted it (as an h-type step)
    const bool grow = !S.done && S.accepted && !S.armijo && !forced && (!S.soft_try || S.soft_ok);
    const bool reset = resto == 2 ? phase_end : (failed && resto && m > 0);
    // watchdog bookkeeping (solver.py): an acceptable point ends it; after watchdog_trial_iter_max unacceptable full
    // steps the iterate returns to where it started, and the next line search starts at half its step
    const bool wd_ok = S.wd_on && S.accepted && !forced;
    const int wd_trial = S.wd_trial + (forced ? 1 : 0);
    const bool wd_back = forced && wd_trial > K.o.watchdog_trial_iter_max;
    const bool shortened = S.accepted && !forced && S.alpha < S.a_p;
    double* filt = K.filt + b * kFilt * 2;
    // Ipopt's filter reset heuristic (FilterLSAcceptor::UpdateForNextIteration), before the augmentation
    int nsucc = S.nsucc;
    bool freset = false;
    if (!S.done && S.accepted && !forced && !S.soft_try && S.nreset < K.o.max_filter_resets) {
        if (S.rejf) {
            if (++nsucc >= K.o.filter_reset_trigger) {
                freset = true;
                nsucc = 0;
            }
        } else {
            nsucc = 0;
        }
    }
    if (freset)
        for (int k = threadIdx.x; k < kFilt; k += kIB) {
            filt[2 * k] = INFINITY;
            filt[2 * k + 1] = -INFINITY;
        }
    __syncthreads();
    if (threadIdx.x == 0 && grow) {
        const int k = S.fpos % kFilt;
        filt[2 * k] = (1 - 1e-5) * S.theta;
        filt[2 * k + 1] = S.phi - 1e-5 * S.theta;
    }
    __syncthreads();
    if (reset)  // a fresh filter after a restoration (step or phase, see k_rs_init)
        for (int k = threadIdx.x; k < kFilt; k += kIB) {
            filt[2 * k] = INFINITY;
            filt[2 * k + 1] = -INFINITY;
        }
    const bool step = !S.done;
    double alpha = S.alpha;
    if (reset || failed || !step) alpha = 0.0;
    double* x = K.x + b * nf;
    double* zl = K.zl + b * nf;
    double* zu = K.zu + b * nf;
    const double* dzl = K.dzl + b * nf;
    const double* dzu = K.dzu + b * nf;
    const double* dy = K.dy + b * m;
    double nfy = 0.0, nfz = 0.0;
    if (K.wide) {  // k_wupd_a's partials
        double rv[2];
        const int ro[2] = {1, 1};
        wide_get(K, b, rv, ro);
        nfy = rv[0];
        nfz = rv[1];
    } else {
        for (int j = threadIdx.x; j < m; j += kIB)
            if (!isfinite(dy[j])) nfy = 1.0;
        for (int i = threadIdx.x; i < nf; i += kIB)
            if (!isfinite(dzl[i]) || !isfinite(dzu[i])) nfz = 1.0;
        double rv[2] = {nfy, nfz};
        const int ro[2] = {1, 1};
        breduce_n(rv, ro);
        nfy = rv[0];
        nfz = rv[1];
    }
    const bool mv = alpha > 0 && !(nfy > 0);
    const double az = (step && !failed) ? S.a_z : 0.0;
    const bool mz = az > 0 && !(nfz > 0);
    const double* xnew = reset ? K.xr + b * nf : K.xacc + b * nf;
    const double mu = S.mu, smin = slack_min(mu);
    double* lbI = K.lbI + b * nf;
    double* ubI = K.ubI + b * nf;
    if (K.wide) {  // (k_wupd_c)
        if (threadIdx.x == 0) {
            double* wf = K.wflag + b * kWF;
            wf[1] = step;
            wf[2] = reset;
            wf[3] = mz;
            wf[4] = az;
            wf[5] = mu;
            wf[6] = wd_back;
            wf[7] = wd_back ? 1 : ((reset && resto == 2) ? 2 : (mv ? 3 : 0));
            wf[8] = alpha;
            wf[0] = 1.0;
        }
    } else {
    for (int i = threadIdx.x; i < nf; i += kIB) {
        double xi = step ? xnew[i] : x[i];
        x[i] = xi;
        double l = zl[i], u = zu[i];
        if (mz) {
            l = l + az * dzl[i];
            u = u + az * dzu[i];
        }
        if (K.hasL[i]) {
            const double lbv = moved_lb(lbI[i], xi - lbI[i], smin);
            lbI[i] = lbv;
            const double sl = xi - lbv;
            l = clamp_hi(clamp_lo(l, mu / (1e10 * sl)), 1e10 * mu / sl);
        }
        if (K.hasU[i]) {
            const double ubv = moved_ub(ubI[i], ubI[i] - xi, smin);
            ubI[i] = ubv;
            const double su = ubv - xi;
            u = clamp_hi(clamp_lo(u, mu / (1e10 * su)), 1e10 * mu / su);
        }
        zl[i] = l;
        zu[i] = u;
        if (wd_back) {  // back to the watchdog iterate
            x[i] = K.wx[b * nf + i];
            zl[i] = K.wzl[b * nf + i];
            zu[i] = K.wzu[b * nf + i];
        }
    }
    if (wd_back)
        for (int j = threadIdx.x; j < m; j += kIB) K.y[b * m + j] = K.wy[b * m + j];
    else if (reset && resto == 2)  // after the phase: zero multipliers (Ipopt constr_mult_reset_threshold = 0)
        for (int j = threadIdx.x; j < m; j += kIB) K.y[b * m + j] = 0.0;
    else if (mv)
        for (int j = threadIdx.x; j < m; j += kIB) K.y[b * m + j] = K.y[b * m + j] + alpha * dy[j];
    // the Hessian's multipliers at the new iterate, as k_ipm_begin will form them: the next iteration evaluates
    // g, J_g and the Hessian in one call (cfx_eval_all_h) before k_ipm_begin runs
    for (int j = threadIdx.x; j < m; j += kIB) K.ysc[b * m + j] = K.y[b * m + j] * K.sg[b * m + j];
    __syncthreads();
    write_full(K, b, x, K.vx);
    }
    if (threadIdx.x == 0) {
        K.of[b] = S.sf;  // the phase evaluated its Hessian with objective factor 0
        if (grow) S.fpos += 1;
        if (reset) {
            S.reinit = resto == 1;  // the step re-estimates the multipliers by least squares
            S.lcount = S.lhead = S.lprev = 0;  // the quasi-Newton pairs describe the abandoned region
            S.lsig = 1.0;
        }
        S.rs_on = 0;
        S.rs_exit = RS_RUNNING;
        S.alpha = alpha;
        S.iters += step;
        S.nsucc = nsucc;
        S.nreset += freset;
        S.wd_trial = wd_trial;
        S.wd_on = S.wd_on && !wd_ok && !wd_back;
        S.wd_short = (wd_ok || wd_back || failed || !shortened || S.soft_try) ? 0 : S.wd_short + 1;
        S.soft_try = 0;
        S.skip_first = wd_back;
        if (wd_back) S.mu = S.wd_mu;
    }
    store_scal(K, b, S);
}

// ---- Ipopt's feasibility-restoration phase (CFX_RESTORATION_PHASE) -------------------------------------------------
// For the instances whose line search failed:  min rho sum(p + n) + 1/2 sum_i zeta D_R,i^2 (x_i - x_r,i)^2  s.t.
// c(x) - p + n = 0, p, n >= 0 and the bounds — c the scaled constraints, x_r the iterate where the phase started
// (K.x) — solved by the interior point itself with its own barrier mu_R, filter and line search.  With dp, dn and
// the bound multipliers' steps eliminated its Newton system
//   [[W_c + zeta D_R^2 + Sigma_x + dw, J^T], [J, -(p / zp + n / zn) - delta_c]] [dx; dy] = [r_x; r_c],
//   dp = (dy + mu_R / p - rho + y) p / zp,   dn = (-dy + mu_R / n - rho - y) n / zn
// has the original band structure (W_c: the Hessian of y^T c, eval_h with objective factor 0), so band assembly,
// factorisation, curvature test and callbacks are the main loop's.  The phase iterate is xr (direction dxr), its bound
// multipliers rzl / rzu; the main iteration's x, zl, zu, y stay untouched until it ends.  It ends when its point is
// acceptable to the original filter (augmented with the starting point) with ||c||_1 <= required_infeasibility_
// reduction times the value where it started (Ipopt RestoConvergenceCheck); the original bound multipliers then take
// a Newton step for complementarity over the phase's whole dx (cut by the fraction to the boundary; all reset to 1
// above Ipopt's bound_mult_reset_threshold 1000), the constraint multipliers restart from zero (Ipopt's
// constr_mult_reset_threshold = 0 discards the least-squares estimate) and the filter from empty (k_ipm_update;
// measured: cfg 5 from 16 perturbed starts converges 13 / 16 with a fresh filter, 9 / 16 keeping the augmented one).
// A failed line search of the phase, a point of local infeasibility (its own problem converged) or max_resto_iter of
// its iterations end the solve of that instance, as in Ipopt.
//
// Scheduling: an instance's phase iterations run inside the host's main iterations — one host iteration advances every
// instance by one iteration of its own mode (main or phase), through the same callback launches, factorisations and
// line-search loop (the k_ipm_* kernels skip the instances in the phase, the k_rs_* kernels the others).  A batch
// whose instances enter the phase at staggered times therefore costs max over the instances of their iterations, not
// their sum (round 3 ran each phase as a nested loop over the whole batch with the other instances idle: 512 starts of
// cfg 5 serialised into an unbounded number of batch-wide iterations).

// p, n minimising rho (p + n) - mu (ln p + ln n) on c - p + n = 0 (Ipopt's closed form, evaluated without
// cancellation)
__device__ inline void rs_pn(double c, double mu, double rho, double& p, double& n) {
    const double s = hypot(mu, rho * c);
    n = c > 0 ? (mu + mu * mu / (s + rho * c)) / (2 * rho) : (mu - rho * c + s) / (2 * rho);
    p = c < 0 ? (mu + mu * mu / (s - rho * c)) / (2 * rho) : (mu + rho * c + s) / (2 * rho);
}

// the phase's barrier objective at (x, p, n) with barrier mu: +inf outside the bounds or at p, n <= 0
__device__ double rs_merit(const IpmK& K, int64_t b, const double* x, const double* p, const double* nn, double mu,
                           double* sh) {
    const int nf = K.nf, m = K.m;
    double prox = 0.0, lin = 0.0, lg = 0.0, bad = 0.0;
    for (int i = threadIdx.x; i < nf; i += kIB) {
        const double xref = K.x[b * nf + i], e = x[i] - xref;
        prox += rs_weight(mu, xref) * e * e;
    }
    for (int j = threadIdx.x; j < m; j += kIB) {
        if (!(p[j] > 0) || !(nn[j] > 0)) bad = 1.0;
        lin += p[j] + nn[j];
        lg += log(clamp_lo(p[j], 1e-300)) + log(clamp_lo(nn[j], 1e-300));
    }
    {
        double rv[4] = {prox, lin, lg, bad};
        const int ro[4] = {0, 0, 0, 1};
        breduce_n(rv, ro);
        prox = rv[0];
        lin = rv[1];
        lg = rv[2];
        bad = rv[3];
    }
    const double fx = barrier_obj(K, b, x, K.o.resto_penalty * lin + 0.5 * prox, mu, sh);
    return bad > 0 ? INFINITY : fx - mu * lg;
}

// enter the phase: the instances in the main iteration whose line search failed (with iterations left: the phase's
// iterations count among the instance's); their first phase iteration is the next host iteration, at vx = x
__global__ void __launch_bounds__(kIB) k_rs_init(const IpmK K) {
    __shared__ double sh[kIB / 64];
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    const bool failed = !S.rs_on && !S.accepted && !S.done;
    // Ipopt (BacktrackingLineSearch): "Restoration phase called at acceptable point" — the solve ends there, solved to
    // the acceptable level (err0 is the current point's scaled KKT error)
    const bool acceptable = failed && S.acc_ok;
    const bool go = failed && !acceptable && S.iters < K.o.max_iter;
    if (acceptable && threadIdx.x == 0) {
        S.done = 1;
        S.status = CFX_IPM_SOLVED_TO_ACCEPTABLE_LEVEL;
    }
    if (go) {  // block-uniform
        const double rho = K.o.resto_penalty;
        const double* c = K.gS + b * m;
        double cinf = 0.0;
        for (int j = threadIdx.x; j < m; j += kIB) cinf = max_n(cinf, fabs(c[j]));
        cinf = breduce(cinf, OpMax(), sh);
        const double mu = max_n(S.mu, cinf);  // Ipopt: mu_R = max(mu, ||c||_inf)
        for (int j = threadIdx.x; j < m; j += kIB) {
            double p, n;
            rs_pn(c[j], mu, rho, p, n);
            K.rp[b * m + j] = p;
            K.rn[b * m + j] = n;
            K.rzp[b * m + j] = mu / p;
            K.rzn[b * m + j] = mu / n;
            K.ry[b * m + j] = 0.0;
            K.ysc[b * m + j] = 0.0;  // the multipliers of its first Hessian (objective factor 0)
        }
        for (int i = threadIdx.x; i < nf; i += kIB) {
            K.xr[b * nf + i] = K.x[b * nf + i];
            K.rzl[b * nf + i] = K.hasL[i] ? min_n(rho, K.zl[b * nf + i]) : 0.0;
            K.rzu[b * nf + i] = K.hasU[i] ? min_n(rho, K.zu[b * nf + i]) : 0.0;
        }
        double* rf = K.rfilt + b * kFilt * 2;
        for (int k = threadIdx.x; k < kFilt; k += kIB) {
            rf[2 * k] = INFINITY;
            rf[2 * k + 1] = -INFINITY;
        }
        if (threadIdx.x == 0) {  // the original filter takes the point where the phase starts
            double* filt = K.filt + b * kFilt * 2;
            const int k = S.fpos % kFilt;
            filt[2 * k] = (1 - 1e-5) * S.theta;
            filt[2 * k + 1] = S.phi - 1e-5 * S.theta;
            S.fpos += 1;
            S.rs_mu = mu;
            S.rs_th0 = S.theta;
            S.rs_dw = S.rs_dwl = 0.0;
            S.rs_it = 0;
            S.rs_rr = 0;
            S.rs_on = 1;
            S.rs_exit = RS_RUNNING;
            S.soc = 0;
            S.lcount = S.lhead = S.lprev = 0;  // L-BFGS: no pairs (no Woodbury correction) during the phase
            S.lsig = 1.0;
            K.of[b] = 0.0;
            atomicAdd(K.rstat, 1ull);
        }
        __syncthreads();
        write_full(K, b, K.xr + b * nf, K.vx);
    }
    store_scal(K, b, S);
}

// after g, J_g at the phase iterate (vx = xr): scaling, the phase's optimality error and barrier update, Sigma, the
// Newton right-hand side, the eliminated (2,2) block and the multipliers of its constraint Hessian
__global__ void __launch_bounds__(kIB) k_rs_begin(const IpmK K) {
    __shared__ double sh[kIB / 64];
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    if (!S.rs_on || S.rs_exit != RS_RUNNING) return;  // block-uniform
    const double rho = K.o.resto_penalty;
    const double* sg = K.sg + b * m;
    double* gS = K.gS + b * m;
    double* jv = K.jv + b * K.nj;
    const double* jac = K.jac + b * K.nnzj;
    if (!K.wide) {  // (wide: k_wrs_scale)
        for (int j = threadIdx.x; j < m; j += kIB) gS[j] = K.graw[b * m + j] * sg[j];
#pragma unroll 8
        for (int q = threadIdx.x; q < K.nj; q += kIB) jv[q] = jac[K.jsel[q]] * K.d[K.jc[q]] * sg[K.jr[q]];
    }
    __syncthreads();
    const double* x = K.xr + b * nf;
    const double* xref = K.x + b * nf;
    const double* zl = K.rzl + b * nf;
    const double* zu = K.rzu + b * nf;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    const double* p = K.rp + b * m;
    const double* nn = K.rn + b * m;
    const double* zp = K.rzp + b * m;
    const double* zn = K.rzn + b * m;
    const double* y = K.ry + b * m;
    double* rhs = K.rhs + b * K.nK;
    double ed = 0.0, ep = 0.0, pmax = -INFINITY, pmin = INFINITY;
    if (K.wide) {  // k_wrs_a's partials
        double rv[4];
        const int ro[4] = {1, 1, 1, 2};
        wide_get(K, b, rv, ro);
        ed = rv[0], ep = rv[1], pmax = rv[2], pmin = rv[3];
    } else {
    for (int i = threadIdx.x; i < nf; i += kIB) {
        double jty = 0.0;
#pragma unroll 4
        for (int k = K.jt_ptr[i]; k < K.jt_ptr[i + 1]; ++k) {
            const int q = K.jt_idx[k];
            jty += jv[q] * y[K.jr[q]];
        }
        rhs[i] = jty;  // completed below, once mu_R is final
        ed = max_n(ed, fabs(rs_weight(S.rs_mu, xref[i]) * (x[i] - xref[i]) + jty - zl[i] + zu[i]));
    }
    for (int j = threadIdx.x; j < m; j += kIB) {
        ep = max_n(ep, fabs(gS[j] - p[j] + nn[j]));
        ed = max_n(ed, max_n(fabs(rho - y[j] - zp[j]), fabs(rho + y[j] - zn[j])));
    }
    {
        double rv[2] = {ed, ep};
        const int ro[2] = {1, 1};
        breduce_n(rv, ro);
        ed = rv[0];
        ep = rv[1];
    }
    }
    // the phase's monotone barrier update (the main loop's rule, on its unscaled errors)
    double e_mu = INFINITY;
    for (int pass = 0; pass < 5; ++pass) {
        const double mu = S.rs_mu;
        double ecm = 0.0;
        if (K.wide) {  // max_i |p_i - mu| = max(p_max - mu, mu - p_min), exactly (fl(p - mu) is monotone in p)
            ecm = max_n(max_n(ecm, pmax - mu), mu - pmin);
        } else {
        for (int i = threadIdx.x; i < nf; i += kIB) {
            if (K.hasL[i]) ecm = max_n(ecm, fabs((x[i] - lbI[i]) * zl[i] - mu));
            if (K.hasU[i]) ecm = max_n(ecm, fabs((ubI[i] - x[i]) * zu[i] - mu));
        }
        for (int j = threadIdx.x; j < m; j += kIB)
            ecm = max_n(ecm, max_n(fabs(p[j] * zp[j] - mu), fabs(nn[j] * zn[j] - mu)));
        ecm = breduce(ecm, OpMax(), sh);
        }
        e_mu = max_n(max_n(ed, ep), ecm);
        if (!((e_mu <= K.o.kappa_eps * mu) && (mu > K.o.tol / 10))) break;
        __syncthreads();
        if (threadIdx.x == 0) S.rs_mu = clamp_lo(min_n(K.o.kappa_mu * mu, pow(mu, K.o.theta_mu)), K.o.tol / 10);
        __syncthreads();
    }
    const double mu = S.rs_mu;
    // the phase has converged (barrier at its floor, its sub-problem solved) without reaching a point the original
    // problem accepts: a local minimiser of the infeasibility (Ipopt: "converged to a point of local infeasibility")
    if (mu <= K.o.tol / 10 && e_mu <= K.o.kappa_eps * mu) {
        __syncthreads();
        if (threadIdx.x == 0) S.rs_exit = RS_INFEASIBLE;
        store_scal(K, b, S);
        return;
    }
    double* sig = K.sig + b * nf;
    if (!K.wide)  // (wide: k_wrs_c)
    for (int i = threadIdx.x; i < nf; i += kIB) {
        const bool hL = K.hasL[i], hU = K.hasU[i];
        const double sl = hL ? x[i] - lbI[i] : 1.0, su = hU ? ubI[i] - x[i] : 1.0;
        sig[i] = (hL ? zl[i] / sl : 0.0) + (hU ? zu[i] / su : 0.0);
        const double bar = (hL ? mu / sl : 0.0) - (hU ? mu / su : 0.0);
        rhs[i] = -(rs_weight(mu, xref[i]) * (x[i] - xref[i]) + rhs[i] - bar);
    }
    if (!K.wide)
    for (int j = threadIdx.x; j < m; j += kIB) {
        const double Sp = zp[j] / p[j], Sn = zn[j] / nn[j];
        const double ap = mu / p[j] - rho + y[j], an = mu / nn[j] - rho - y[j];
        rhs[nf + j] = -(gS[j] - p[j] + nn[j]) + ap / Sp - an / Sn;
        K.rdc[b * m + j] = -(1.0 / Sp + 1.0 / Sn);
        K.ysc[b * m + j] = y[j] * sg[j];
    }
    if (threadIdx.x == 0) {
        S.rs_tau = clamp_lo(1.0 - mu, K.o.tau_min);
        S.rs_dw = 0.0;
    }
    store_scal(K, b, S);
}

// the phase's step: dp, dn and the multiplier steps from (dx, dy), fraction to the boundary, filter quantities at
// the phase iterate, first trial point
__global__ void __launch_bounds__(kIB) k_rs_dir(const IpmK K) {
    __shared__ double sh[kIB / 64];
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    if (!S.rs_on || S.rs_exit != RS_RUNNING) return;  // block-uniform
    const double rho = K.o.resto_penalty, mu = S.rs_mu, tau = S.rs_tau;
    const double* x = K.xr + b * nf;
    const double* xref = K.x + b * nf;
    const double* dx = K.dxr + b * nf;
    const double* zl = K.rzl + b * nf;
    const double* zu = K.rzu + b * nf;
    const double* lbI = K.lbI + b * nf;
    const double* ubI = K.ubI + b * nf;
    double* dzl = K.dzl + b * nf;
    double* dzu = K.dzu + b * nf;
    const double* p = K.rp + b * m;
    const double* nn = K.rn + b * m;
    const double* zp = K.rzp + b * m;
    const double* zn = K.rzn + b * m;
    const double* y = K.ry + b * m;
    const double* dy = K.dy + b * m;
    double apl = INFINITY, apu = INFINITY, azl = INFINITY, azu = INFINITY, dphi = 0.0, theta = 0.0;
    for (int i = threadIdx.x; i < nf; i += kIB) {
        const bool hL = K.hasL[i], hU = K.hasU[i];
        const double sl = hL ? x[i] - lbI[i] : 1.0, su = hU ? ubI[i] - x[i] : 1.0;
        const double vzl = hL ? mu / sl - zl[i] - zl[i] / sl * dx[i] : 0.0;
        const double vzu = hU ? mu / su - zu[i] + zu[i] / su * dx[i] : 0.0;
        dzl[i] = vzl;
        dzu[i] = vzu;
        apl = min_n(apl, step_term(hL, sl, dx[i], tau));
        apu = min_n(apu, step_term(hU, su, -dx[i], tau));
        azl = min_n(azl, step_term(hL, zl[i], vzl, tau));
        azu = min_n(azu, step_term(hU, zu[i], vzu, tau));
        const double bar = (hL ? mu / sl : 0.0) - (hU ? mu / su : 0.0);
        dphi += (rs_weight(mu, xref[i]) * (x[i] - xref[i]) - bar) * dx[i];
    }
    for (int j = threadIdx.x; j < m; j += kIB) {
        const double Sp = zp[j] / p[j], Sn = zn[j] / nn[j];
        const double dpj = (dy[j] + mu / p[j] - rho + y[j]) / Sp;
        const double dnj = (-dy[j] + mu / nn[j] - rho - y[j]) / Sn;
        const double dzpj = mu / p[j] - zp[j] - Sp * dpj, dznj = mu / nn[j] - zn[j] - Sn * dnj;
        K.rdp[b * m + j] = dpj;
        K.rdn[b * m + j] = dnj;
        K.rdzp[b * m + j] = dzpj;
        K.rdzn[b * m + j] = dznj;
        apl = min_n(apl, min_n(step_term(true, p[j], dpj, tau), step_term(true, nn[j], dnj, tau)));
        azl = min_n(azl, min_n(step_term(true, zp[j], dzpj, tau), step_term(true, zn[j], dznj, tau)));
        dphi += (rho - mu / p[j]) * dpj + (rho - mu / nn[j]) * dnj;
        theta += fabs(K.gS[b * m + j] - p[j] + nn[j]);
    }
    {
        double rv[6] = {apl, apu, azl, azu, dphi, theta};
        const int ro[6] = {2, 2, 2, 2, 0, 0};
        breduce_n(rv, ro);
        apl = rv[0];
        apu = rv[1];
        azl = rv[2];
        azu = rv[3];
        dphi = rv[4];
        theta = rv[5];
    }
    const double phi = rs_merit(K, b, x, p, nn, mu, sh);
    const double a_p = min_n(clamp_hi(apl, 1.0), clamp_hi(apu, 1.0));
    __syncthreads();
    if (threadIdx.x == 0) {
        S.rs_dwl = S.rs_dw;
        S.rs_theta = theta;
        S.rs_phi = phi;
        S.rs_dphi = dphi;
        S.rs_ap = a_p;
        S.rs_az = min_n(clamp_hi(azl, 1.0), clamp_hi(azu, 1.0));
        S.rs_alpha = a_p;
        S.rs_acc = 0;
        S.rs_arm = 0;
        if (S.rs_it == 0) {
            S.rs_tmax = 1e4 * clamp_lo(theta, 1.0);
            S.rs_tmin = 1e-4 * clamp_lo(theta, 1.0);
        }
    }
    double* xt = K.xt + b * nf;
    for (int i = threadIdx.x; i < nf; i += kIB) xt[i] = x[i] + a_p * dx[i];
    for (int j = threadIdx.x; j < m; j += kIB) {
        K.rpt[b * m + j] = p[j] + a_p * K.rdp[b * m + j];
        K.rnt[b * m + j] = nn[j] + a_p * K.rdn[b * m + j];
    }
    __syncthreads();
    write_full(K, b, xt, K.vt);
    store_scal(K, b, S);
}

// after g (and f) at the phase's trial point: its own filter test (k_ipm_accept, launched next, counts the phase
// instances not accepted)
__global__ void __launch_bounds__(kIB) k_rs_accept(const IpmK K) {
    __shared__ double sh[kIB / 64];
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    if (S.rs_on && S.rs_exit == RS_RUNNING && !S.rs_acc) {  // block-uniform
        const double* sg = K.sg + b * m;
        const double* gt = K.gt + b * m;
        const double* pt = K.rpt + b * m;
        const double* nt = K.rnt + b * m;
        double tt = 0.0;
        for (int j = threadIdx.x; j < m; j += kIB) tt += fabs(gt[j] * sg[j] - pt[j] + nt[j]);
        tt = breduce(tt, OpSum(), sh);
        const double ph = rs_merit(K, b, K.xt + b * nf, pt, nt, S.rs_mu, sh);
        bool ok, arm;
        filter_core(K, K.rfilt + b * kFilt * 2, S.rs_theta, S.rs_phi, S.rs_dphi, S.rs_tmax, S.rs_tmin, tt, ph,
                    S.rs_alpha, sh, ok, arm);
        __syncthreads();
        if (threadIdx.x == 0 && ok) {
            S.rs_acc = 1;
            S.rs_arm = arm;
        }
    }
    store_scal(K, b, S);
}

// the phase's backtracking: halve its step where no trial was accepted
__global__ void __launch_bounds__(kIB) k_rs_next_trial(const IpmK K) {
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    if (!S.rs_on || S.rs_exit != RS_RUNNING || S.rs_acc) return;  // block-uniform
    const double a = S.rs_alpha * 0.5;
    const double* x = K.xr + b * nf;
    const double* dx = K.dxr + b * nf;
    double* xt = K.xt + b * nf;
    for (int i = threadIdx.x; i < nf; i += kIB) xt[i] = x[i] + a * dx[i];
    for (int j = threadIdx.x; j < m; j += kIB) {
        K.rpt[b * m + j] = K.rp[b * m + j] + a * K.rdp[b * m + j];
        K.rnt[b * m + j] = K.rn[b * m + j] + a * K.rdn[b * m + j];
    }
    __syncthreads();
    write_full(K, b, xt, K.vt);
    if (threadIdx.x == 0) K.sc[b].rs_alpha = a;
}

// consecutive p, n resets after which a phase whose line search keeps failing gives up (Ipopt has no such bound: its
// RestoRestorationPhase always succeeds and the phase runs on to max_resto_iter); CFX_RS_RR_MAX for experiments
__device__ __constant__ int g_rs_rr_max = 1;
__device__ inline int rs_rr_max() { return g_rs_rr_max; }

// end of a phase iteration: the step (primal-dual, z safeguard), the phase's filter, the exit test on the original
// problem and, on exit, the original bound multipliers; rs_exit records how the phase ended (k_ipm_update acts on it).
// A failed line search of the phase is answered as Ipopt's RestoRestorationPhase does: x stays, p and n take their
// closed form at x (the phase's own constraints c - p + n = 0 then hold), the phase's filter takes the point; a second
// failed search in a row, or max_resto_iter iterations, fail the phase (Ipopt: Restoration_Failed).  The instances
// that go on get their next evaluation point (vx = xr) and Hessian multipliers ready.
__global__ void __launch_bounds__(kIB) k_rs_update(const IpmK K) {
    __shared__ double sh[kIB / 64];
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, m = K.m;
    load_scal(K, b, S);
    if (!S.rs_on || S.rs_exit != RS_RUNNING) return;  // block-uniform
    if (!S.rs_acc && S.rs_rr >= rs_rr_max()) {
        __syncthreads();
        if (threadIdx.x == 0) {
            S.rs_exit = RS_FAILED;
            S.iters += 1;  // Ipopt counts the phase's iterations among the solve's
            atomicAdd(K.rstat + 1, 1ull);
        }
    } else if (!S.rs_acc) {  // Ipopt's restoration of the restoration phase
        const double rho = K.o.resto_penalty, mu = S.rs_mu;
        for (int j = threadIdx.x; j < m; j += kIB) {
            double p, n;
            rs_pn(K.gS[b * m + j], mu, rho, p, n);
            K.rp[b * m + j] = p;
            K.rn[b * m + j] = n;
            K.rzp[b * m + j] = mu / p;
            K.rzn[b * m + j] = mu / n;
        }
        const bool budget = S.iters + 1 >= K.o.max_iter, limit = S.rs_it + 1 >= K.o.max_resto_iter;
        if (!budget && !limit) {
            write_full(K, b, K.xr + b * nf, K.vx);
            for (int j = threadIdx.x; j < m; j += kIB) K.ysc[b * m + j] = K.ry[b * m + j] * K.sg[b * m + j];
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double* rf = K.rfilt + b * kFilt * 2;
            const int k = S.rs_it % kFilt;
            rf[2 * k] = (1 - 1e-5) * S.rs_theta;
            rf[2 * k + 1] = S.rs_phi - 1e-5 * S.rs_theta;
            S.rs_rr += 1;
            S.rs_it += 1;
            S.iters += 1;
            atomicAdd(K.rstat + 1, 1ull);
            if (budget)
                S.rs_exit = RS_BUDGET;
            else if (limit)
                S.rs_exit = RS_FAILED;
        }
    } else {
        const double a = S.rs_alpha, az = S.rs_az, mu = S.rs_mu;
        if (threadIdx.x == 0 && !S.rs_arm) {
            double* rf = K.rfilt + b * kFilt * 2;
            const int k = S.rs_it % kFilt;
            rf[2 * k] = (1 - 1e-5) * S.rs_theta;
            rf[2 * k + 1] = S.rs_phi - 1e-5 * S.rs_theta;
        }
        double* x = K.xr + b * nf;
        double* zl = K.rzl + b * nf;
        double* zu = K.rzu + b * nf;
        const double* lbI = K.lbI + b * nf;
        const double* ubI = K.ubI + b * nf;
        for (int i = threadIdx.x; i < nf; i += kIB) {
            const double xi = K.xt[b * nf + i];
            x[i] = xi;
            if (K.hasL[i]) {
                const double sl = xi - lbI[i];
                zl[i] = clamp_hi(clamp_lo(zl[i] + az * K.dzl[b * nf + i], mu / (1e10 * sl)), 1e10 * mu / sl);
            }
            if (K.hasU[i]) {
                const double su = ubI[i] - xi;
                zu[i] = clamp_hi(clamp_lo(zu[i] + az * K.dzu[b * nf + i], mu / (1e10 * su)), 1e10 * mu / su);
            }
        }
        for (int j = threadIdx.x; j < m; j += kIB) {
            const int64_t e = b * m + j;
            const double p = K.rpt[e], n = K.rnt[e];
            K.rp[e] = p;
            K.rn[e] = n;
            K.ry[e] += a * K.dy[e];
            K.rzp[e] = clamp_hi(clamp_lo(K.rzp[e] + az * K.rdzp[e], mu / (1e10 * p)), 1e10 * mu / p);
            K.rzn[e] = clamp_hi(clamp_lo(K.rzn[e] + az * K.rdzn[e], mu / (1e10 * n)), 1e10 * mu / n);
        }
        __syncthreads();
        // exit test on the original problem, from g, f of the accepted trial
        const double* sg = K.sg + b * m;
        double th = 0.0;
        for (int j = threadIdx.x; j < m; j += kIB) th += fabs(K.gt[b * m + j] * sg[j]);
        th = breduce(th, OpSum(), sh);
        const double ph = barrier_obj(K, b, x, K.ft[b] * S.sf, S.mu, sh);
        const bool ok = isfinite(th) && isfinite(ph) && th <= K.o.required_infeasibility_reduction * S.rs_th0 &&
                        !filter_dominated(K.filt + b * kFilt * 2, th, ph, sh);
        if (ok) {  // the original bound multipliers: Newton step for complementarity over the phase's dx
            const double* x0 = K.x + b * nf;
            double* zl0 = K.zl + b * nf;
            double* zu0 = K.zu + b * nf;
            const double mu0 = S.mu, tau0 = S.tau;
            double al = INFINITY;
            for (int i = threadIdx.x; i < nf; i += kIB) {
                const bool hL = K.hasL[i], hU = K.hasU[i];
                const double sl = hL ? x0[i] - lbI[i] : 1.0, su = hU ? ubI[i] - x0[i] : 1.0, d = x[i] - x0[i];
                const double vzl = hL ? mu0 / sl - zl0[i] - zl0[i] / sl * d : 0.0;
                const double vzu = hU ? mu0 / su - zu0[i] + zu0[i] / su * d : 0.0;
                al = min_n(al, min_n(step_term(hL, zl0[i], vzl, tau0), step_term(hU, zu0[i], vzu, tau0)));
            }
            al = clamp_hi(breduce(al, OpMin(), sh), 1.0);
            double zmax = 0.0;
            for (int i = threadIdx.x; i < nf; i += kIB) {
                const bool hL = K.hasL[i], hU = K.hasU[i];
                const double sl = hL ? x0[i] - lbI[i] : 1.0, su = hU ? ubI[i] - x0[i] : 1.0, d = x[i] - x0[i];
                if (hL) zl0[i] += al * (mu0 / sl - zl0[i] - zl0[i] / sl * d);
                if (hU) zu0[i] += al * (mu0 / su - zu0[i] + zu0[i] / su * d);
                zmax = max_n(zmax, max_n(zl0[i], zu0[i]));
            }
            zmax = breduce(zmax, OpMax(), sh);
            if (zmax > 1e3)
                for (int i = threadIdx.x; i < nf; i += kIB) {
                    zl0[i] = K.hasL[i] ? 1.0 : 0.0;
                    zu0[i] = K.hasU[i] ? 1.0 : 0.0;
                }
        }
        const bool budget = S.iters + 1 >= K.o.max_iter, limit = S.rs_it + 1 >= K.o.max_resto_iter;
        if (!ok && !budget && !limit) {  // the phase goes on from xr
            write_full(K, b, x, K.vx);
            for (int j = threadIdx.x; j < m; j += kIB) K.ysc[b * m + j] = K.ry[b * m + j] * sg[j];
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            S.rs_rr = 0;
            S.rs_it += 1;
            S.iters += 1;
            atomicAdd(K.rstat + 1, 1ull);
            if (ok)
                S.rs_exit = RS_OK;
            else if (budget)
                S.rs_exit = RS_BUDGET;
            else if (limit)
                S.rs_exit = RS_FAILED;
        }
    }
    store_scal(K, b, S);
}

// after the last host iteration: the instances still in the phase leave it, not converged (a failed phase k_ipm_update
// has not seen yet stops the instance as it would have)
__global__ void __launch_bounds__(kIB) k_rs_finish(const IpmK K) {
    if (threadIdx.x == 0) {
        Scal& S = K.sc[blockIdx.x];
        if (S.rs_on && (S.rs_exit == RS_FAILED || S.rs_exit == RS_INFEASIBLE)) {
            S.status = S.rs_exit == RS_FAILED ? CFX_IPM_RESTORATION_FAILED : CFX_IPM_INFEASIBLE_PROBLEM_DETECTED;
            S.done = S.stop = 1;
            S.iters += 1;  // the iteration k_ipm_update's stop path counts (solver.py: rstop.long()), ADVICE round 4
        }
        S.rs_on = 0;
        S.rs_exit = RS_RUNNING;
    }
}

// project onto the original bounds (Ipopt honor_original_bounds) and write the final point into vx
// (honor_original_bounds only), and the bound multipliers of the unscaled problem (z_l, z_u [B][n]; 0 at fixed ones)
__global__ void __launch_bounds__(kIB) k_ipm_final(const IpmK K, double* __restrict__ zlo, double* __restrict__ zuo) {
    const int64_t b = blockIdx.x;
    double* x = K.x + b * K.nf;
    if (K.o.honor_original_bounds)
        for (int i = threadIdx.x; i < K.nf; i += kIB) x[i] = min_n(max_n(x[i], K.lbF0[i]), K.ubF0[i]);
    const double sf = K.sc[b].sf;
    for (int j = threadIdx.x; j < K.nfix; j += kIB) zlo[b * K.n + K.fixed[j]] = zuo[b * K.n + K.fixed[j]] = 0.0;
    for (int i = threadIdx.x; i < K.nf; i += kIB) {
        zlo[b * K.n + K.free[i]] = K.zl[b * K.nf + i] / (sf * K.d[i]);
        zuo[b * K.n + K.free[i]] = K.zu[b * K.nf + i] / (sf * K.d[i]);
    }
    __syncthreads();
    write_full(K, b, x, K.vx);
}

// results: y of the unscaled problem, converged / iterations / KKT error
__global__ void __launch_bounds__(kIB) k_ipm_out(const IpmK K, double* __restrict__ yo, int32_t* __restrict__ conv,
                                                 int32_t* __restrict__ its, double* __restrict__ kkt,
                                                 int32_t* __restrict__ status, int wall) {
    const int64_t b = blockIdx.x;
    const Scal& S = K.sc[b];
    if (yo)
        for (int j = threadIdx.x; j < K.m; j += kIB) yo[b * K.m + j] = K.y[b * K.m + j] * K.sg[b * K.m + j] / S.sf;
    if (threadIdx.x == 0) {
        if (conv) conv[b] = S.done && !S.stop;
        if (its) its[b] = S.iters;
        if (kkt) kkt[b] = S.err0;
        // still iterating when the host loop ended: its bound (max_iter host iterations) or max_wall_time
        if (status)
            status[b] = S.done ? S.status
                               : (wall ? CFX_IPM_MAXIMUM_WALLTIME_EXCEEDED : CFX_IPM_MAXIMUM_ITERATIONS_EXCEEDED);
    }
}

// Publish one counter slot to host-mapped memory: the four counts, then (release, system scope) the sequence
// number the host spins on.  Replaces a device-to-host copy + stream synchronisation (~25 us of host wake-up
// and relaunch latency per read on the batch-1 path) by a poll of pinned memory.
__global__ void k_ipm_publish(const int32_t* __restrict__ cnt, int32_t* pub, int32_t seq) {
    if (threadIdx.x == 0) {
        for (int i = 0; i < 4; ++i) __hip_atomic_store(pub + 1 + i, cnt[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(pub, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---- limited-memory Hessian (Ipopt hessian_approximation = limited-memory, BFGS update, scalar1 initialisation) --
// W ~ B = sigma I - Z M^-1 Z^T with Z = [sigma S, Y] (the last c <= hmax steps s = x+ - x and gradient-of-the-
// Lagrangian changes y = grad L(x+, y+) - grad L(x, y+), oldest first) and M = [[sigma S^T S, L], [L^T, -D]]
// (S^T Y = L + D + U).  The band factors are those of K0 = K with W replaced by sigma I; the Newton / correction
// solves use  K^-1 r = K0^-1 r + P C^-1 Z^T K0^-1 r,  P = K0^-1 Z,  C = M - Z^T P  (Sherman-Morrison-Woodbury; Z is
// zero on the constraint rows).  Unused slots of the 2 hmax columns are zero with an identity block in M and C.

// pair slot of the r-th stored pair (oldest first)
__device__ inline int lb_slot(const Scal& S, int H, int r) { return (S.lhead - S.lcount + r + 2 * H) % H; }

// column q of Z at free variable i (q < H: sigma s_q, else y_{q-H}; zero past the stored pairs)
__device__ inline double lb_z(const IpmK& K, const Scal& S, int64_t b, int q, int i) {
    const int H = K.hmax;
    const int r = q < H ? q : q - H;
    if (r >= S.lcount) return 0.0;
    const int64_t o = ((int64_t)b * H + lb_slot(S, H, r)) * K.nf + i;
    return q < H ? S.lsig * K.Sh[o] : K.Yh[o];
}

// after k_ipm_begin: the pair of the last step (skipped unless s^T y > 1e-8 |s| |y|), sigma = s^T y / s^T s, the
// current iterate saved, and M
__global__ void __launch_bounds__(kIB) k_lbfgs_update(const IpmK K) {
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    const int nf = K.nf, H = K.hmax, H2 = 2 * H;
    load_scal(K, b, S);
    const double* x = K.x + b * nf;
    const double* gF = K.gF + b * nf;
    const double* jv = K.jv + b * K.nj;
    const double* y = K.y + b * K.m;
    double* xp = K.xprev + b * nf;
    double* gp = K.gprev + b * nf;
    double* jp = K.jvprev + b * K.nj;
    if (!S.done && S.lprev) {
        double sy = 0.0, ss = 0.0, yy = 0.0;
        for (int i = threadIdx.x; i < nf; i += kIB) {
            double jty = 0.0, jtyp = 0.0;
#pragma unroll 4
            for (int k = K.jt_ptr[i]; k < K.jt_ptr[i + 1]; ++k) {
                const int t = K.jt_idx[k];
                const double yk = y[K.jr[t]];
                jty += jv[t] * yk;
                jtyp += jp[t] * yk;
            }
            const double si = x[i] - xp[i], yi = (gF[i] - gp[i]) + (jty - jtyp);
            xp[i] = si;  // the previous iterate is no longer needed: its arrays hold the candidate pair
            gp[i] = yi;
            sy += si * yi;
            ss += si * si;
            yy += yi * yi;
        }
        {
            double rv[3] = {sy, ss, yy};
            const int ro[3] = {0, 0, 0};
            breduce_n(rv, ro);
            sy = rv[0];
            ss = rv[1];
            yy = rv[2];
        }
        const bool take = isfinite(sy) && isfinite(yy) && ss > 0.0 && sy > 1e-8 * sqrt(ss * yy);
        if (take) {
            double* sn = K.Sh + ((int64_t)b * H + S.lhead) * nf;
            double* yn = K.Yh + ((int64_t)b * H + S.lhead) * nf;
            for (int i = threadIdx.x; i < nf; i += kIB) {
                sn[i] = xp[i];
                yn[i] = gp[i];
            }
        }
        __syncthreads();
        if (threadIdx.x == 0 && take) {
            S.lhead = (S.lhead + 1) % H;
            S.lcount = S.lcount < H ? S.lcount + 1 : H;
            S.lsig = clamp_hi(clamp_lo(sy / ss, 1e-8), 1e8);
        }
        __syncthreads();
    }
    for (int i = threadIdx.x; i < nf; i += kIB) {
        xp[i] = x[i];
        gp[i] = gF[i];
    }
    for (int t = threadIdx.x; t < K.nj; t += kIB) jp[t] = jv[t];
    if (threadIdx.x == 0) S.lprev = 1;
    __syncthreads();
    // M over the stored pairs (S rows / columns at 0.., Y at H..), identity elsewhere
    double* Mb = K.Mm + b * H2 * H2;
    for (int e = threadIdx.x; e < H2 * H2; e += kIB) {
        const int r = e / H2, c = e - (e / H2) * H2;
        const bool used = (r % H) < S.lcount && (c % H) < S.lcount;
        Mb[e] = used ? 0.0 : (r == c ? 1.0 : 0.0);
    }
    __syncthreads();
    const int c = S.lcount;
    for (int i = 0; i < c; ++i)
        for (int j = 0; j < c; ++j) {
            const double* si = K.Sh + ((int64_t)b * H + lb_slot(S, H, i)) * nf;
            const double* sj = K.Sh + ((int64_t)b * H + lb_slot(S, H, j)) * nf;
            const double* yj = K.Yh + ((int64_t)b * H + lb_slot(S, H, j)) * nf;
            double dss = 0.0, dsy = 0.0;
            for (int t = threadIdx.x; t < nf; t += kIB) {
                dss += si[t] * sj[t];
                dsy += si[t] * yj[t];
            }
            double rv[2] = {dss, dsy};
            const int ro[2] = {0, 0};
            breduce_n(rv, ro);
            if (threadIdx.x == 0) {
                Mb[i * H2 + j] = S.lsig * rv[0];              // sigma S^T S
                if (i > j) Mb[i * H2 + H + j] = rv[1];        // L
                if (i > j) Mb[(H + j) * H2 + i] = rv[1];      // L^T
                if (i == j) Mb[(H + i) * H2 + H + i] = -rv[1];  // -D
            }
        }
    store_scal(K, b, S);
}

// the 2 H columns of Z in band order, one rb-shaped array per column (then solved in place: P = K0^-1 Z)
__global__ void __launch_bounds__(kIB) k_lbfgs_zcols(const IpmK K) {
    __shared__ Scal S;
    const int64_t b = blockIdx.x;
    load_scal(K, b, S);
    const int H2 = 2 * K.hmax;
    for (int q = 0; q < H2; ++q) {
        double* z = K.Zb + ((int64_t)q * K.B + b) * K.nKp;
        for (int i = threadIdx.x; i < K.nKp; i += kIB) z[i] = 0.0;
        __syncthreads();
        for (int i = threadIdx.x; i < K.nf; i += kIB) z[K.pos[i]] = lb_z(K, S, b, q, i);
        __syncthreads();
    }
}

// C = M - Z^T P and its LU with partial pivoting, in place in Cl (2 hmax <= 128: the whole block, a barrier per
// pivot step; the pivot search by wavefront 0, two rows per lane)
__global__ void __launch_bounds__(kIB) k_lbfgs_factor(const IpmK K) {
    __shared__ Scal S;
    __shared__ int piv_s;
    const int64_t b = blockIdx.x;
    load_scal(K, b, S);
    const int H2 = 2 * K.hmax, t = threadIdx.x;
    const double* Mb = K.Mm + b * H2 * H2;
    double* C = K.Cl + b * H2 * H2;
    int32_t* piv = K.Cp + b * H2;
    for (int e = t; e < H2 * H2; e += kIB) {
        const int r = e / H2, c = e - (e / H2) * H2;
        const double* P = K.Zb + ((int64_t)c * K.B + b) * K.nKp;
        double acc = 0.0;
        if ((r % K.hmax) < S.lcount && (c % K.hmax) < S.lcount)
            for (int i = 0; i < K.nf; ++i) acc += lb_z(K, S, b, r, i) * P[K.pos[i]];
        C[e] = Mb[e] - acc;
    }
    __syncthreads();
    for (int k = 0; k < H2; ++k) {
        if (t < 64) {  // argmax |C[r][k]| over r >= k (first index on ties), rows t and t + 64
            double a = -1.0;
            int idx = H2;
            for (int r = t; r < H2; r += 64)
                if (r >= k && fabs(C[r * H2 + k]) > a) a = fabs(C[r * H2 + k]), idx = r;
            for (int o = 32; o > 0; o >>= 1) {
                const double a2 = __shfl_xor(a, o, 64);
                const int i2 = __shfl_xor(idx, o, 64);
                if (a2 > a || (a2 == a && i2 < idx)) {
                    a = a2;
                    idx = i2;
                }
            }
            if (t == 0) {
                piv_s = idx;
                piv[k] = idx;
            }
        }
        __syncthreads();
        const int p = piv_s;
        if (p != k)
            for (int c = t; c < H2; c += kIB) {
                const double tmp = C[k * H2 + c];
                C[k * H2 + c] = C[p * H2 + c];
                C[p * H2 + c] = tmp;
            }
        __syncthreads();
        const double pv = C[k * H2 + k];
        const double inv = pv != 0.0 ? 1.0 / pv : 0.0;
        for (int r = k + 1 + t; r < H2; r += kIB) C[r * H2 + k] *= inv;
        __syncthreads();
        const int n1 = H2 - k - 1;
        for (int e = t; e < n1 * n1; e += kIB) {
            const int r = k + 1 + e / n1, c = k + 1 + e % n1;
            C[r * H2 + c] -= C[r * H2 + k] * C[k * H2 + c];
        }
        __syncthreads();
    }
}

// rb (= K0^-1 r, band order) += P C^-1 Z^T rb   (2 hmax <= 128 values in LDS)
__global__ void __launch_bounds__(kIB) k_lbfgs_apply(const IpmK K) {
    constexpr int HM2 = 128;
    __shared__ Scal S;
    __shared__ double w[HM2];
    const int64_t b = blockIdx.x;
    load_scal(K, b, S);
    const int H2 = 2 * K.hmax, t = threadIdx.x;
    double* rb = K.rb + b * K.nKp;
    if (t < H2) {  // (Z^T u)_t
        double v = 0.0;
        if ((t % K.hmax) < S.lcount)
            for (int i = 0; i < K.nf; ++i) v += lb_z(K, S, b, t, i) * rb[K.pos[i]];
        w[t] = v;
    }
    __syncthreads();
    const double* L = K.Cl + b * H2 * H2;
    const int32_t* pv = K.Cp + b * H2;
    if (t == 0)  // row interchanges (getrs), in order
        for (int k = 0; k < H2; ++k) {
            const int p = pv[k];
            if (p != k) {
                const double tmp = w[k];
                w[k] = w[p];
                w[p] = tmp;
            }
        }
    __syncthreads();
    for (int k = 0; k < H2; ++k) {  // unit lower
        const double wk = w[k];
        __syncthreads();
        if (t > k && t < H2) w[t] -= L[t * H2 + k] * wk;
        __syncthreads();
    }
    for (int k = H2 - 1; k >= 0; --k) {  // upper
        if (t == 0) w[k] = w[k] / L[k * H2 + k];
        __syncthreads();
        const double wk = w[k];
        if (t < k) w[t] -= L[t * H2 + k] * wk;
        __syncthreads();
    }
    for (int e = t; e < K.nKp; e += kIB) {
        double acc = 0.0;
        for (int q = 0; q < H2; ++q)
            if ((q % K.hmax) < S.lcount) acc += K.Zb[((int64_t)q * K.B + b) * K.nKp + e] * w[q];
        rb[e] += acc;
    }
}

}  // namespace

// ---------------------------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------------------------
struct cfx_ipm {
    cfx_handle* h = nullptr;
    int64_t B = 1;
    int device = 0;
    IpmK K{};
    std::vector<void*> allocs;
    int32_t* h_cnt = nullptr;
    int32_t *h_pub = nullptr, *d_pub = nullptr;  // host-mapped counter mailbox [seq, 4 counts]
    int32_t seq = 0;
    bool poll = true;  // CFX_IPM_SYNC=stream: copy + hipStreamSynchronize instead
    int slot = 0;
    cfx_ipm_stats st{};
    std::string err;
    hipStream_t stream = nullptr;
    // staging for host inputs / outputs
    double *d_fv = nullptr, *d_yo = nullptr, *d_kkt = nullptr;
    // warm start inputs (cfx_ipm_set_warm_start; allocated on first use) and the last solve's bound multipliers
    double *d_wy = nullptr, *d_wzl = nullptr, *d_wzu = nullptr, *d_zlo = nullptr, *d_zuo = nullptr;
    bool warm_set = false;
    bool trace = false;  // CFX_IPM_TRACE=1: one stderr line per iteration (instance 0)
    int32_t *d_conv = nullptr, *d_its = nullptr, *d_status = nullptr;
    std::vector<int32_t> h_status;  // CFX_IPM_* status per instance of the last solve (cfx_ipm_get_status)
    // J_g's constant values (cfx_jac_constant_mask) stay in K.jac after the first full evaluation: later evaluations
    // pass CFX_KEEP_CONSTANT_JAC (CFX_IPM_KEEPJ=0 turns it off, for A/B runs)
    bool keepj = true, jac_filled = false;
    uint32_t jac_flags() const { return CFX_DEVICE | (keepj && jac_filled ? CFX_KEEP_CONSTANT_JAC : 0u); }
    // cfx_ipm_create_ext: the callbacks come from the caller's evaluator (e.g. interval-sharded over several GPUs)
    // instead of a libcfx handle
    bool ext = false;
    cfx_evaluator ev{};
};

#define IPM_HIP(s, call)                                                         \
    do {                                                                         \
        hipError_t e_ = (call);                                                  \
        if (e_ != hipSuccess) {                                                  \
            (s)->err = std::string(#call) + ": " + hipGetErrorString(e_);        \
            return CFX_EHIP;                                                     \
        }                                                                        \
    } while (0)
#define IPM_CFX(s, call)                                                         \
    do {                                                                         \
        int r_ = (call);                                                         \
        if (r_ != CFX_OK) {                                                      \
            (s)->err = std::string(#call) + ": " + cfx_last_error((s)->h);       \
            return r_;                                                           \
        }                                                                        \
    } while (0)
#define IPM_BAND(s, call)                                                        \
    do {                                                                         \
        int r_ = (call);                                                         \
        if (r_ != CFX_OK) {                                                      \
            (s)->err = std::string(#call) + ": " + cfx_last_error(nullptr);      \
            return r_;                                                           \
        }                                                                        \
    } while (0)

// The callbacks at a point (device pointers, AoS): the handle's, or the caller's evaluator (cfx_ipm_create_ext)
static int ipm_eval_all(cfx_ipm* s, const double* v, double* g, double* jac, double* f, double* grad, uint32_t flags) {
    if (s->ext) {
        const int r = s->ev.eval_all(s->ev.ctx, v, g, jac, f, grad);
        if (r != 0) s->err = "cfx_ipm: the evaluator's eval_all returned " + std::to_string(r);
        return r != 0 ? CFX_ECALLBACK : CFX_OK;
    }
    const int r = cfx_eval_all(s->h, v, g, jac, f, grad, flags);
    if (r != CFX_OK) s->err = std::string("cfx_eval_all: ") + cfx_last_error(s->h);
    return r;
}
static int ipm_eval_h(cfx_ipm* s, const double* v, const double* of, const double* lam, double* hess) {
    if (s->ext) {
        const int r = s->ev.eval_h ? s->ev.eval_h(s->ev.ctx, v, of, lam, hess) : -1;
        if (r != 0) s->err = "cfx_ipm: the evaluator's eval_h returned " + std::to_string(r);
        return r != 0 ? CFX_ECALLBACK : CFX_OK;
    }
    const int r = cfx_eval_h(s->h, v, of, lam, hess, CFX_DEVICE);
    if (r != CFX_OK) s->err = std::string("cfx_eval_h: ") + cfx_last_error(s->h);
    return r;
}

template <class T>
static T* dalloc(cfx_ipm* s, size_t n, int* rc) {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) {
        *rc = CFX_ENOMEM;
        s->err = "hipMalloc failed";
        return nullptr;
    }
    s->allocs.push_back(p);
    return static_cast<T*>(p);
}

template <class T>
static const T* dupload(cfx_ipm* s, const std::vector<T>& v, int* rc) {
    T* p = dalloc<T>(s, v.size(), rc);
    if (p && !v.empty() && hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) {
        *rc = CFX_EHIP;
        s->err = "hipMemcpy H2D failed";
        return nullptr;
    }
    return p;
}

extern "C" void cfx_ipm_default_options(cfx_ipm_options* o) {
    if (!o) return;
    o->tol = 1e-6;
    o->max_iter = 200;
    o->acceptable_tol = 1e-6;
    o->acceptable_iter = 15;
    o->mu_init = 0.1;
    o->bound_relax_factor = 0.0;
    o->bound_push = 1e-2;
    o->tau_min = 0.99;
    o->kappa_eps = 10.0;
    o->kappa_mu = 0.2;
    o->theta_mu = 1.5;
    o->s_max = 100.0;
    o->armijo = 1e-4;
    o->max_backtrack = 30;
    o->delta_c = 1e-9;
    o->curv_min = 1e-8;
    o->max_soc = 4;
    o->kappa_soc = 0.99;
    o->watchdog_shortened_iter_trigger = 10;
    o->watchdog_trial_iter_max = 3;
    o->hessian_approximation = CFX_HESSIAN_EXACT;
    o->limited_memory_max_history = 6;
    o->restoration = CFX_RESTORATION_PHASE;
    o->max_resto_iter = 200;
    o->resto_penalty = 1000.0;
    o->required_infeasibility_reduction = 0.9;
    o->filter_reset_trigger = 5;
    o->max_filter_resets = 0;  // Ipopt: 5; off here
    o->max_wall_time = 1e20;   // Ipopt max_wall_time
    o->print_frequency_time = 0.0;
    o->soft_resto_pderror_reduction_factor = 0.0;  // Ipopt: 0.9999
    o->max_soft_resto_iters = 10;
    o->resto_failure_restart = 0;
    o->constr_viol_tol = 1e-4;
    o->dual_inf_tol = 1.0;
    o->compl_inf_tol = 1e-4;
    o->acceptable_constr_viol_tol = 0.01;
    o->acceptable_dual_inf_tol = 1e10;
    o->acceptable_compl_inf_tol = 0.01;
    o->warm_start_bound_push = 1e-3;
    o->warm_start_bound_frac = 1e-3;
    o->warm_start_mult_bound_push = 1e-3;
    o->warm_start_init_point = 0;
    o->honor_original_bounds = 0;  // Ipopt 3.14's default
    o->range_scaling = 1;
    o->bound_mult_init_method = 1;  // mu-based (Ipopt's default is constant, 1)
    o->bound_mult_init_val = 1.0;
    o->inertia_test = 0;
    o->mu_strategy = CFX_MU_MONOTONE;
    o->adaptive_mu_globalization = CFX_MU_GLOBAL_OBJ_CONSTR_FILTER;
    o->mu_max_fact = 1000.0;
    o->mu_max = -1.0;  // mu_max_fact * the first iterate's average complementarity
    o->mu_min = 1e-11;
    o->adaptive_mu_monotone_init_factor = 0.8;
    o->sigma_max = 100.0;
    o->sigma_min = 1e-6;
    o->quality_function_section_sigma_tol = 1e-2;
    o->quality_function_section_qf_tol = 0.0;
    o->quality_function_max_section_steps = 8;
    o->mu_change_resets_filter = 0;  // Ipopt: resets (the adaptive strategy here always does)
    o->filter_margin_fact = 1e-5;
    o->filter_max_margin = 1.0;
    o->monotone_mu_floor = 0;  // tol / 10 (Ipopt: min(tol, compl_inf_tol) / (kappa_eps + 1))
    o->nlp_scaling_method = 1;  // gradient-based
    o->nlp_scaling_max_gradient = 100.0;
    o->nlp_scaling_min_value = 1e-8;
    o->bound_frac = 0.5;  // Ipopt: 0.01
}

// CSR of `key` (values in [0, nkeys)) with the sources of each key in increasing source order
static void csr(const std::vector<int64_t>& key, int64_t nkeys, std::vector<int32_t>& ptr, std::vector<int32_t>& idx) {
    ptr.assign(nkeys + 1, 0);
    for (int64_t k : key) ptr[k + 1]++;
    for (int64_t i = 0; i < nkeys; ++i) ptr[i + 1] += ptr[i];
    idx.assign(key.size(), 0);
    std::vector<int32_t> fill(ptr.begin(), ptr.end() - 1);
    for (size_t s = 0; s < key.size(); ++s) idx[fill[key[s]]++] = (int32_t)s;
}

// Stage-chain grouping of the KKT unknowns (IpmK::chain; cfx_chain.hip).  A node width w over the ORIGINAL variable
// index (node(v) = v / w; for a shooting transcription w = nx + nu puts x_k and u_k in node k) is searched from the
// smallest that can work; a constraint row belongs to the node of its last free column.  Accepted when every Jacobian
// and Hessian entry couples equal or adjacent nodes (block tridiagonal) and the rows of each node match one-to-one to
// variables of that node through Jacobian entries (Kuhn's augmenting paths, rows in index order, so a continuity row
// takes the state its -I falls on): rows left unmatched (a marker row on states already claimed by continuity rows,
// the continuity row of a fixed end state), rows without free columns and the parameters go to the dense border.
// With that matching every contiguous range of nodes has a constraint block of full structural row rank, so the
// pivot blocks of the cyclic reduction are nonsingular KKT matrices.
struct ChainPlan {
    bool ok = false;
    int M = 0, sp = 0, nb = 0, width = 0;
    std::vector<int32_t> pos;  // KKT unknown (free variables, then rows) -> slot (node k: k sp + local; border: M sp + j)
};
static ChainPlan chain_plan(int nf, int m, const std::vector<int32_t>& freev, const std::vector<uint8_t>& par,
                            const std::vector<int32_t>& jrF, const std::vector<int32_t>& jcF,
                            const std::vector<int32_t>& hrF, const std::vector<int32_t>& hcF, int max_border) {
    ChainPlan best;
    const int nj = (int)jrF.size(), nh = (int)hrF.size();
    std::vector<int64_t> rmin(m, INT64_MAX), rmax(m, -1);
    for (int s = 0; s < nj; ++s) {
        const int c = jcF[s];
        if (par[c]) continue;
        rmin[jrF[s]] = std::min<int64_t>(rmin[jrF[s]], freev[c]);
        rmax[jrF[s]] = std::max<int64_t>(rmax[jrF[s]], freev[c]);
    }
    int64_t span = 0, vmax = 0;
    for (int r = 0; r < m; ++r)
        if (rmax[r] >= 0) span = std::max(span, rmax[r] - rmin[r]);
    for (int s = 0; s < nh; ++s)
        if (!par[hrF[s]] && !par[hcF[s]]) span = std::max<int64_t>(span, std::abs((int64_t)freev[hrF[s]] - freev[hcF[s]]));
    for (int i = 0; i < nf; ++i)
        if (!par[i]) vmax = std::max<int64_t>(vmax, freev[i]);
    // Jacobian entries of each row over non-parameter columns (CSR)
    std::vector<int32_t> rptr(m + 1, 0), rcol;
    for (int s = 0; s < nj; ++s)
        if (!par[jcF[s]]) rptr[jrF[s] + 1]++;
    for (int r = 0; r < m; ++r) rptr[r + 1] += rptr[r];
    rcol.resize(rptr[m]);
    {
        std::vector<int32_t> fill(rptr.begin(), rptr.end() - 1);
        for (int s = 0; s < nj; ++s)
            if (!par[jcF[s]]) rcol[fill[jrF[s]]++] = jcF[s];
    }
    for (int64_t w = std::max<int64_t>(1, (span + 2) / 2); w <= span + 1; ++w) {
        const int M = (int)(vmax / w) + 1;
        auto vnode = [&](int i) { return (int)(freev[i] / w); };
        bool tri = true;
        for (int r = 0; r < m && tri; ++r)
            if (rmax[r] >= 0 && rmin[r] / w < rmax[r] / w - 1) tri = false;
        for (int s = 0; s < nh && tri; ++s)
            if (!par[hrF[s]] && !par[hcF[s]] && std::abs(vnode(hrF[s]) - vnode(hcF[s])) > 1) tri = false;
        if (!tri) continue;
        // rows of each node in index order; Kuhn's matching of rows to variables of the same node
        std::vector<int32_t> match_var(nf, -1), match_row(m, -1), rnode(m, -1);
        std::vector<std::vector<int32_t>> nrows(M);
        for (int r = 0; r < m; ++r)
            if (rmax[r] >= 0) {
                rnode[r] = (int)(rmax[r] / w);
                nrows[rnode[r]].push_back(r);
            }
        std::vector<int32_t> seen(nf, -1);
        int stamp = 0;
        std::vector<std::pair<int32_t, int32_t>> stack;  // (row, next entry)
        for (int k = 0; k < M; ++k)
            for (int r0 : nrows[k]) {
                ++stamp;
                // iterative DFS for an augmenting path from row r0
                stack.assign(1, {r0, rptr[r0]});
                std::vector<int32_t> path_var;
                bool found = false;
                while (!stack.empty() && !found) {
                    auto& [r, e] = stack.back();
                    if (e >= rptr[r + 1]) {
                        stack.pop_back();
                        if (!path_var.empty()) path_var.pop_back();
                        continue;
                    }
                    const int v = rcol[e++];
                    if (vnode(v) != k || seen[v] == stamp) continue;
                    seen[v] = stamp;
                    path_var.push_back(v);
                    if (match_var[v] < 0) {
                        found = true;
                    } else {
                        stack.push_back({match_var[v], rptr[match_var[v]]});
                    }
                }
                if (found)  // flip the path: row stack[d] takes path_var[d]
                    for (size_t d = 0; d < stack.size(); ++d) {
                        const int r = stack[d].first, v = path_var[d];
                        match_var[v] = r;
                        match_row[r] = v;
                    }
            }
        std::vector<int32_t> cnt(M, 0);
        int nb = 0;
        for (int i = 0; i < nf; ++i) par[i] ? ++nb : ++cnt[vnode(i)];
        for (int r = 0; r < m; ++r) match_row[r] >= 0 ? ++cnt[rnode[r]] : ++nb;
        int smax = 0;
        for (int k = 0; k < M; ++k) smax = std::max(smax, cnt[k]);
        const int sp = (smax + 15) / 16 * 16;
        if (nb > max_border || !cfx_chain_sp_ok(sp) || M < 2) continue;
        ChainPlan cp;
        cp.ok = true;
        cp.M = M;
        cp.sp = sp;
        cp.nb = nb;
        cp.width = (int)w;
        cp.pos.assign(nf + m, -1);
        std::fill(cnt.begin(), cnt.end(), 0);
        int j = 0;
        for (int i = 0; i < nf; ++i) {
            if (par[i])
                cp.pos[i] = M * sp + j++;
            else {
                const int k = vnode(i);
                cp.pos[i] = k * sp + cnt[k]++;
            }
        }
        for (int r = 0; r < m; ++r) {
            if (match_row[r] >= 0)
                cp.pos[nf + r] = rnode[r] * sp + cnt[rnode[r]]++;
            else
                cp.pos[nf + r] = M * sp + j++;
        }
        return cp;
    }
    return best;
}

// a failed cfx_ipm_create: the message goes to cfx_last_error(NULL), as for cfx_create
static int create_fail(cfx_ipm* s, int code) {
    g_create_error = s->err;
    cfx_ipm_destroy(s);
    return code;
}

static int ipm_fail(cfx_ipm* s, int code, const std::string& msg) {
    s->err = msg;
    return code;
}

static int ipm_create_common(cfx_ipm* s, const cfx_sizes& sz, int layout, const int32_t* jr_in, const int32_t* jc_in,
                             const int32_t* hr_in, const int32_t* hc_in, const double* lb, const double* ub,
                             int32_t n_params, const cfx_ipm_options* opt, cfx_ipm** out);

extern "C" int cfx_ipm_create(cfx_handle* h, const double* lb, const double* ub, int32_t n_params,
                              const cfx_ipm_options* opt, cfx_ipm** out) {
    if (!h || !lb || !ub || !out) return CFX_EINVAL;
    *out = nullptr;
    cfx_ipm* s = new cfx_ipm();
    s->h = h;
    int layout = 0;
    hipStream_t stream = nullptr;
    cfx_sizes sz{};
    if (cfx_internal_info(h, &s->B, &layout, &s->device, &stream) != CFX_OK || cfx_get_sizes(h, &sz) != CFX_OK) {
        s->err = "cfx_ipm_create: bad handle";
        return create_fail(s, CFX_EINVAL);
    }
    std::vector<int32_t> jr(sz.nnz_jac), jc(sz.nnz_jac), hr(sz.nnz_hess), hc(sz.nnz_hess);
    if (cfx_jac_structure(h, jr.data(), jc.data()) != CFX_OK || cfx_hess_structure(h, hr.data(), hc.data()) != CFX_OK) {
        s->err = "cfx_ipm_create: structure query failed";
        return create_fail(s, CFX_EINVAL);
    }
    return ipm_create_common(s, sz, layout, jr.data(), jc.data(), hr.data(), hc.data(), lb, ub, n_params, opt, out);
}

extern "C" int cfx_ipm_create_ext(const cfx_nlp_desc* nlp, const cfx_evaluator* ev, const double* lb, const double* ub,
                                  int32_t n_params, const cfx_ipm_options* opt, cfx_ipm** out) {
    if (!nlp || !ev || !ev->eval_all || !lb || !ub || !out) return CFX_EINVAL;
    *out = nullptr;
    cfx_ipm* s = new cfx_ipm();
    if (nlp->batch < 1 || nlp->nv < 1 || nlp->ng < 0 || nlp->nnz_jac < 0 || nlp->nnz_hess < 0 ||
        (nlp->nnz_jac && (!nlp->jac_row || !nlp->jac_col)) || (nlp->nnz_hess && (!nlp->hess_row || !nlp->hess_col))) {
        s->err = "cfx_ipm_create_ext: invalid NLP description";
        return create_fail(s, CFX_EINVAL);
    }
    for (int64_t e = 0; e < nlp->nnz_jac; ++e)
        if (nlp->jac_row[e] < 0 || nlp->jac_row[e] >= nlp->ng || nlp->jac_col[e] < 0 || nlp->jac_col[e] >= nlp->nv) {
            s->err = "cfx_ipm_create_ext: Jacobian triplet out of range";
            return create_fail(s, CFX_EINVAL);
        }
    for (int64_t e = 0; e < nlp->nnz_hess; ++e)
        if (nlp->hess_row[e] < nlp->hess_col[e] || nlp->hess_col[e] < 0 || nlp->hess_row[e] >= nlp->nv) {
            s->err = "cfx_ipm_create_ext: Hessian triplet out of range or above the diagonal";
            return create_fail(s, CFX_EINVAL);
        }
    s->B = nlp->batch;
    s->device = nlp->device;
    s->stream = (hipStream_t)nlp->hip_stream;
    s->ev = *ev;
    s->ext = true;
    cfx_sizes sz{};
    sz.nv = nlp->nv;
    sz.ng = nlp->ng;
    sz.nnz_jac = nlp->nnz_jac;
    sz.nnz_hess = nlp->nnz_hess;
    return ipm_create_common(s, sz, CFX_LAYOUT_AOS, nlp->jac_row, nlp->jac_col, nlp->hess_row, nlp->hess_col, lb, ub,
                             n_params, opt, out);
}

static int ipm_create_common(cfx_ipm* s, const cfx_sizes& sz, int layout, const int32_t* jr_in, const int32_t* jc_in,
                             const int32_t* hr_in, const int32_t* hc_in, const double* lb, const double* ub,
                             int32_t n_params, const cfx_ipm_options* opt, cfx_ipm** out) {
    int rc = CFX_OK;
    IpmK& K = s->K;
    if (opt)
        K.o = *opt;
    else
        cfx_ipm_default_options(&K.o);
    if (const char* e = std::getenv("CFX_RS_RR_MAX")) {  // experiment override (see rs_rr_max)
        const int v = std::max(1, std::atoi(e));
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_rs_rr_max), &v, sizeof(int)) != hipSuccess) return CFX_EHIP;
    }
    if ((s->B > 1 && layout != CFX_LAYOUT_AOS) || layout == CFX_LAYOUT_TILED64 ||
        n_params < 0 || n_params > sz.nv || K.o.max_iter < 0 || K.o.max_backtrack < 1 || K.o.max_soc < 0 ||
        K.o.watchdog_shortened_iter_trigger < 0 || K.o.watchdog_trial_iter_max < 0 ||
        (K.o.hessian_approximation != CFX_HESSIAN_EXACT && K.o.hessian_approximation != CFX_HESSIAN_LIMITED_MEMORY) ||
        (K.o.hessian_approximation == CFX_HESSIAN_LIMITED_MEMORY &&
         (K.o.limited_memory_max_history < 1 || K.o.limited_memory_max_history > 64)) ||
        (K.o.restoration != CFX_RESTORATION_STEP && K.o.restoration != CFX_RESTORATION_PHASE) ||
        K.o.max_resto_iter < 0 || !(K.o.resto_penalty > 0) || !(K.o.required_infeasibility_reduction > 0) ||
        !(K.o.required_infeasibility_reduction < 1) || K.o.filter_reset_trigger < 1 || K.o.max_filter_resets < 0 ||
        !(K.o.max_wall_time > 0) || !(K.o.print_frequency_time >= 0) ||
        !(K.o.soft_resto_pderror_reduction_factor >= 0) || K.o.max_soft_resto_iters < 0 || s->B > 0x7fffffff ||
        !(K.o.constr_viol_tol > 0) || !(K.o.dual_inf_tol > 0) || !(K.o.compl_inf_tol > 0) ||
        !(K.o.acceptable_constr_viol_tol > 0) || !(K.o.acceptable_dual_inf_tol > 0) ||
        !(K.o.acceptable_compl_inf_tol > 0) || !(K.o.warm_start_bound_push > 0) || !(K.o.warm_start_bound_frac > 0) ||
        !(K.o.warm_start_bound_frac <= 0.5) || !(K.o.warm_start_mult_bound_push > 0) ||
        (K.o.bound_mult_init_method != 0 && K.o.bound_mult_init_method != 1) || !(K.o.bound_mult_init_val > 0) ||
        (K.o.inertia_test != 0 && K.o.inertia_test != 1) ||
        (K.o.mu_strategy != CFX_MU_MONOTONE && K.o.mu_strategy != CFX_MU_ADAPTIVE) ||
        (K.o.adaptive_mu_globalization != CFX_MU_GLOBAL_OBJ_CONSTR_FILTER &&
         K.o.adaptive_mu_globalization != CFX_MU_GLOBAL_NEVER_MONOTONE) ||
        !(K.o.mu_min > 0) || !(K.o.mu_max_fact > 0) || !(K.o.sigma_min > 0) || !(K.o.sigma_min <= 1) ||
        !(K.o.sigma_max >= 1) || !(K.o.adaptive_mu_monotone_init_factor > 0) ||
        K.o.quality_function_max_section_steps < 0 || !(K.o.quality_function_section_sigma_tol > 0) ||
        !(K.o.quality_function_section_sigma_tol < 1) || !(K.o.quality_function_section_qf_tol >= 0) ||
        !(K.o.filter_margin_fact > 0) || !(K.o.filter_max_margin > 0) ||
        (K.o.mu_change_resets_filter != 0 && K.o.mu_change_resets_filter != 1) ||
        (K.o.monotone_mu_floor != 0 && K.o.monotone_mu_floor != 1) ||
        (K.o.nlp_scaling_method != 0 && K.o.nlp_scaling_method != 1) || !(K.o.nlp_scaling_max_gradient > 0) ||
        !(K.o.nlp_scaling_min_value > 0) || !(K.o.bound_frac > 0) || !(K.o.bound_frac <= 0.5)) {
        s->err = "cfx_ipm_create: the handle must use CFX_LAYOUT_AOS (or batch 1) and the options must be valid";
        return create_fail(s, CFX_EINVAL);
    }
    const int n = (int)sz.nv, m = (int)sz.ng;
    K.B = s->B;
    K.n = n;
    K.m = m;
    K.nnzj = (int)sz.nnz_jac;
    K.nnzh = (int)sz.nnz_hess;
    if (hipSetDevice(s->device) != hipSuccess) {
        s->err = "cfx_ipm_create: hipSetDevice failed";
        return create_fail(s, CFX_EHIP);
    }
    // free / fixed variables, scaling d, scaled (and relaxed) bounds: solver.py BatchedIpm.__init__
    std::vector<int32_t> freev, fixedv;
    for (int e = 0; e < n; ++e) (lb[e] == ub[e] ? fixedv : freev).push_back(e);
    const int nf = (int)freev.size();
    if (nf == 0) {
        s->err = "cfx_ipm_create: no free variable";
        return create_fail(s, CFX_EINVAL);
    }
    std::vector<double> d(nf), lbF(nf), ubF(nf), lbF0(nf), ubF0(nf), lbfull(lb, lb + n);
    std::vector<uint8_t> hasL(nf), hasU(nf);
    const double rel = K.o.bound_relax_factor;
    for (int i = 0; i < nf; ++i) {
        const double l = lb[freev[i]], u = ub[freev[i]];
        hasL[i] = std::isfinite(l);
        hasU[i] = std::isfinite(u);
        const double w = u - l;
        d[i] = (K.o.range_scaling && std::isfinite(w) && w < 1.0) ? w : 1.0;
        lbF0[i] = l / d[i];
        ubF0[i] = u / d[i];
        lbF[i] = lbF0[i] - rel * clamp_lo(std::fabs(lbF0[i] * d[i]), 1.0) / d[i];
        ubF[i] = ubF0[i] + rel * clamp_lo(std::fabs(ubF0[i] * d[i]), 1.0) / d[i];
    }
    // triplets over the free variables (solver.py _build_kkt_maps)
    const std::vector<int32_t> jr(jr_in, jr_in + K.nnzj), jc(jc_in, jc_in + K.nnzj), hr(hr_in, hr_in + K.nnzh),
        hc(hc_in, hc_in + K.nnzh);
    std::vector<int64_t> posF(n, -1);
    for (int i = 0; i < nf; ++i) posF[freev[i]] = i;
    std::vector<int32_t> jsel, jrF, jcF, hsel, hrF, hcF;
    std::vector<uint8_t> hoff;
    for (int s2 = 0; s2 < K.nnzj; ++s2)
        if (posF[jc[s2]] >= 0) {
            jsel.push_back(s2);
            jrF.push_back(jr[s2]);
            jcF.push_back((int32_t)posF[jc[s2]]);
        }
    for (int s2 = 0; s2 < K.nnzh; ++s2)
        if (posF[hr[s2]] >= 0 && posF[hc[s2]] >= 0) {
            hsel.push_back(s2);
            hrF.push_back((int32_t)posF[hr[s2]]);
            hcF.push_back((int32_t)posF[hc[s2]]);
            hoff.push_back(hrF.back() != hcF.back());
        }
    const int nj = (int)jsel.size(), nh = (int)hsel.size();
    // stage-wise ordering of the KKT unknowns: variable i -> key i; row -> midpoint of the keys of its free
    // columns; parameters (Hmed) -> mean key of the rows that use them
    std::vector<double> vkey(nf);
    for (int i = 0; i < nf; ++i) vkey[i] = i;
    std::vector<uint8_t> par(nf, 0);
    bool anypar = false;
    if (n_params)
        for (int i = 0; i < nf; ++i) anypar |= (par[i] = freev[i] >= n - n_params) != 0;
    auto row_keys = [&](const std::vector<double>& vk, bool skip_par) {
        std::vector<double> cmin(m, INFINITY), cmax(m, -INFINITY), key(m);
        for (int s2 = 0; s2 < nj; ++s2) {
            if (skip_par && par[jcF[s2]]) continue;
            cmin[jrF[s2]] = std::min(cmin[jrF[s2]], vk[jcF[s2]]);
            cmax[jrF[s2]] = std::max(cmax[jrF[s2]], vk[jcF[s2]]);
        }
        for (int r = 0; r < m; ++r) key[r] = std::isfinite(cmin[r]) ? 0.5 * (cmin[r] + cmax[r]) + 0.25 : nf;
        return key;
    };
    const int nK = nf + m;
    int np_free = 0;
    for (int i = 0; i < nf; ++i) np_free += par[i];
    // KKT entries: H (both triangles), J, J^T, diag_x, diag_y, as (unknown, unknown, source)
    std::vector<int32_t> er, ec, src;
    for (int s2 = 0; s2 < nh; ++s2) er.push_back(hrF[s2]), ec.push_back(hcF[s2]), src.push_back((SRC_W << kSrcShift) | s2);
    for (int s2 = 0; s2 < nh; ++s2)
        if (hoff[s2]) er.push_back(hcF[s2]), ec.push_back(hrF[s2]), src.push_back((SRC_W << kSrcShift) | s2);
    for (int s2 = 0; s2 < nj; ++s2) er.push_back(nf + jrF[s2]), ec.push_back(jcF[s2]), src.push_back((SRC_JV << kSrcShift) | s2);
    for (int s2 = 0; s2 < nj; ++s2) er.push_back(jcF[s2]), ec.push_back(nf + jrF[s2]), src.push_back((SRC_JV << kSrcShift) | s2);
    for (int i = 0; i < nf; ++i) er.push_back(i), ec.push_back(i), src.push_back((SRC_DIAG << kSrcShift) | i);
    for (int j = 0; j < m; ++j) er.push_back(nf + j), ec.push_back(nf + j), src.push_back((SRC_DC << kSrcShift) | j);
    // one ordering: border = true places the free parameters last (keys of the rows computed without them)
    struct Order {
        std::vector<int32_t> pos;
        int64_t kl = 0, ku = 0;
        int nA = 0;
    };
    auto make_order = [&](bool border) {
        std::vector<double> vk(vkey);
        std::vector<double> ck = row_keys(vk, true);
        if (anypar) {
            if (border) {
                for (int i = 0; i < nf; ++i)
                    if (par[i]) vk[i] = INFINITY;
            } else {
                std::vector<double> ssum(nf, 0.0), cnt(nf, 0.0);
                for (int s2 = 0; s2 < nj; ++s2) {
                    ssum[jcF[s2]] += ck[jrF[s2]];
                    cnt[jcF[s2]] += 1.0;
                }
                for (int i = 0; i < nf; ++i)
                    if (par[i] && cnt[i] > 0) vk[i] = ssum[i] / std::max(cnt[i], 1.0) + 0.1;
                ck = row_keys(vk, false);
            }
        }
        std::vector<double> key(vk);
        key.insert(key.end(), ck.begin(), ck.end());
        std::vector<int32_t> order(nK);
        std::iota(order.begin(), order.end(), 0);
        std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t c) { return key[a] < key[c]; });
        Order o;
        o.pos.resize(nK);
        for (int k = 0; k < nK; ++k) o.pos[order[k]] = k;
        o.nA = border ? nK - np_free : nK;
        for (size_t e = 0; e < er.size(); ++e) {
            const int64_t r = o.pos[er[e]], c = o.pos[ec[e]];
            if (r < o.nA && c < o.nA) {
                o.kl = std::max(o.kl, r - c);
                o.ku = std::max(o.ku, c - r);
            }
        }
        return o;
    };
    Order ord = make_order(false);
    // a dense border pays when the parameters widen the band past the one-wavefront factorisation and the rest
    // is narrow enough for it (Hmed windows spanning most of the horizon: NMPC windows with T = N)
    if (np_free >= 1 && np_free <= kMaxBorder && !cfx_band_reg_ok(nK, (int32_t)ord.kl, (int32_t)ord.ku)) {
        Order ob = make_order(true);
        if (cfx_band_reg_ok(ob.nA, (int32_t)ob.kl, (int32_t)ob.ku)) ord = ob;
    }
    // Nested dissection of the band (small batches, where one wavefront per instance leaves the chip idle and
    // the band LU is a chain of nK pivot steps): cut the band order at P - 1 places where few unknowns couple across
    // — the boundary B_c = {v >= c : v has a neighbour < c} separates [0, c) from [c, nA) \ B_c; at a stage
    // boundary it is the next node's states — and move the separators into the dense border.  The P blocks then
    // factor side by side (a batch of B P systems), the border by its Schur complement.
    const int nAb = ord.nA, nparb = nK - ord.nA;  // band unknowns, parameters already in the border
    std::vector<int32_t> minadj(nAb);
    std::vector<std::vector<int32_t>> nbr(nAb);
    for (int v = 0; v < nAb; ++v) minadj[v] = v;
    for (size_t e = 0; e < er.size(); ++e) {
        const int r = ord.pos[er[e]], c = ord.pos[ec[e]];
        if (r < nAb && c < nAb && r != c) minadj[std::max(r, c)] = std::min(minadj[std::max(r, c)], std::min(r, c));
    }
    const int w = (int)std::max(ord.kl, ord.ku);
    auto boundary = [&](int c) {  // B_c
        std::vector<int32_t> bnd;
        for (int v = c; v < std::min(nAb, c + w + 1); ++v)
            if (minadj[v] < c) bnd.push_back(v);
        return bnd;
    };
    struct Cut {
        int P = 1;
        std::vector<int32_t> slot;  // band position -> slot (block q: q nA + local; border: P nA + k), per band unknown
        int nA = 0, nsep = 0;
        int64_t kl = 0, ku = 0;
    };
    auto dissect = [&](int P) {
        Cut d;
        d.P = P;
        std::vector<int32_t> cuts{0};
        std::vector<uint8_t> sep(nAb, 0);
        const double t = (double)nAb / P;
        for (int k = 1; k < P; ++k) {
            int best = -1;
            size_t bsz = SIZE_MAX;
            const int lo = std::max(cuts.back() + w + 2, (int)(k * t - t / 4)), hi = std::min(nAb - w - 2, (int)(k * t + t / 4));
            for (int c = lo; c <= hi; ++c) {
                const size_t z = boundary(c).size();
                if (z < bsz || (z == bsz && std::abs(c - k * t) < std::abs(best - k * t))) {
                    bsz = z;
                    best = c;
                }
            }
            if (best < 0) return Cut{};
            cuts.push_back(best);
            for (int v : boundary(best)) sep[v] = 1;
        }
        cuts.push_back(nAb);
        std::vector<int32_t> part(nAb), local(nAb);
        int nA = 0;
        for (int q = 0; q < P; ++q) {
            int l = 0;
            for (int v = cuts[q]; v < cuts[q + 1]; ++v)
                if (!sep[v]) part[v] = q, local[v] = l++;
            nA = std::max(nA, l);
        }
        d.nA = nA;
        d.slot.assign(nAb, -1);
        int k = 0;
        for (int v = 0; v < nAb; ++v) d.slot[v] = sep[v] ? P * nA + k++ : part[v] * nA + local[v];
        d.nsep = k;
        for (size_t e = 0; e < er.size(); ++e) {
            const int r = ord.pos[er[e]], c = ord.pos[ec[e]];
            if (r >= nAb || c >= nAb || sep[r] || sep[c]) continue;
            if (part[r] != part[c]) return Cut{};  // not a separator (cannot happen for a boundary set)
            d.kl = std::max<int64_t>(d.kl, local[r] - local[c]);
            d.ku = std::max<int64_t>(d.ku, local[c] - local[r]);
        }
        return d;
    };
    // Blocks per instance: up to 8 at batch 1 (cfg 3: 9.6 ms vs 10.3 with 16 / 11.4 with 4), about 128 / B above
    // (cfg 4 NMPC, 64 scenarios: 4.04 / 4.19 / 5.12 ms per horizon with 2 / 4 / 8 blocks, 4.60 undissected;
    // scripts/gpu_nmpc_nd.sh), 2 blocks up to batch 512 (cfg 3, 256 starts: 22.9 vs 27.5 ms; scripts/gpu_cfg3_nd.sh);
    // larger batches fill the chip with one band per instance.
    Cut cut;
    // Stage-chain layout (block cyclic reduction, cfx_chain.hip): by default for bands the register placement cannot
    // hold (the reaching task: n = 119,640, kl = 108, where the band factorisation is one workgroup's 119,640-column
    // chain) at small batches; CFX_IPM_KKT=chain / band forces it on (where a grouping exists) / off.
    ChainPlan cp;
    {
        const char* ke = std::getenv("CFX_IPM_KKT");
        const bool force_chain = ke && std::strcmp(ke, "chain") == 0, no_chain = ke && std::strcmp(ke, "band") == 0;
        const bool wide = !cfx_band_reg_ok(nAb, (int32_t)ord.kl, (int32_t)ord.ku) && s->B <= 64 && nK >= 4096;
        if (force_chain || (wide && !no_chain)) {
            cp = chain_plan(nf, m, freev, par, jrF, jcF, hrF, hcF, kMaxBorder);
        } else if (!no_chain && s->B <= 4) {
            // a few short chains (<= 16 nodes: <= 4 reduction levels) also beat nested dissection at batch 1 once
            // the pivot blocks are fast: cfg 5 (11 nodes of 32) 136 vs 229 ms per solve; cfg 3 (101 nodes of 16,
            // 7 levels) stays with dissection, 13.7 vs 10.1 ms (profiles/round5/b1/b1_layouts_r5end.jsonl)
            cp = chain_plan(nf, m, freev, par, jrF, jcF, hrF, hcF, kMaxBorder);
            if (cp.ok && cp.M > 16) cp = ChainPlan{};
        }
    }
    const bool chain = cp.ok;
    int64_t nd_batch = 512;
    if (const char* e = std::getenv("CFX_IPM_ND_BATCH")) nd_batch = std::atoll(e);  // tuning override
    if (!chain && s->B <= nd_batch && nAb >= 48) {
        int pmax = (int)std::min<int64_t>(std::min(8, nAb / 24), std::max<int64_t>(2, 128 / s->B));
        if (const char* e = std::getenv("CFX_IPM_PARTS")) pmax = std::min(pmax, std::atoi(e));  // tuning override
        for (int P = pmax; P >= 2 && cut.P == 1; --P) {
            Cut d = dissect(P);
            if (d.P > 1 && d.nsep + nparb <= kMaxBorder && (int64_t)s->B * P <= 1024 &&
                cfx_band_reg_ok(d.nA, (int32_t)d.kl, (int32_t)d.ku))
                cut = d;
        }
    }
    const int P = cut.P;
    const int64_t kl = chain ? 0 : (P > 1 ? cut.kl : ord.kl), ku = chain ? 0 : (P > 1 ? cut.ku : ord.ku);
    const int64_t csp = cp.sp, cM = cp.M;
    const int64_t nA = chain ? cM * csp : (P > 1 ? cut.nA : nAb);
    const int64_t npb = chain ? cp.nb : (P > 1 ? cut.nsep : 0) + nparb;
    const int64_t nKp = P * nA + npb;
    // natural unknown -> slot in rb
    std::vector<int32_t> pos(nK);
    for (int i = 0; i < nK; ++i) {
        const int v = ord.pos[i];
        pos[i] = chain ? cp.pos[i]
                       : (v < nAb ? (P > 1 ? cut.slot[v] : v) : (int32_t)(P * nA + (P > 1 ? cut.nsep : 0) + (v - nAb)));
    }
    const int64_t ldab = chain ? 0 : 2 * kl + ku + 1;
    const int64_t PA = P * nA;
    // border structure: active columns of each block, Cc non-zeros by border row
    std::vector<std::vector<uint8_t>> isact(P, std::vector<uint8_t>(npb, 0));
    std::vector<std::vector<int64_t>> ccrow(npb);  // border row k -> (q, a) keys q * nA + a
    for (size_t e = 0; e < er.size(); ++e) {
        const int64_t r = pos[er[e]], c = pos[ec[e]];
        if (r < PA && c >= PA) isact[r / nA][c - PA] = 1;
        if (r >= PA && c < PA) {
            isact[c / nA][r - PA] = 1;
            ccrow[r - PA].push_back(c);
        }
    }
    int na = 0;
    std::vector<int32_t> slv((size_t)P * npb, -1);
    for (int q = 0; q < P; ++q) {
        int cnt = 0;
        for (int k = 0; k < npb; ++k)
            if (isact[q][k]) slv[(size_t)q * npb + k] = cnt++;
        na = std::max(na, cnt);
    }
    std::vector<int32_t> actv((size_t)P * std::max(na, 1), -1);
    for (int q = 0; q < P; ++q)
        for (int k = 0; k < npb; ++k)
            if (slv[(size_t)q * npb + k] >= 0) actv[(size_t)q * na + slv[(size_t)q * npb + k]] = k;
    std::vector<int32_t> ccptr(npb + 1, 0), ccq, cca;
    std::vector<std::vector<int64_t>> ccsorted(npb);
    for (int k = 0; k < npb; ++k) {
        std::vector<int64_t> v = ccrow[k];
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        ccsorted[k] = v;
        ccptr[k + 1] = ccptr[k] + (int32_t)v.size();
        for (int64_t key : v) {
            ccq.push_back((int32_t)(key / nA));
            cca.push_back((int32_t)(key - (key / nA) * nA));
        }
    }
    const int64_t ncc = ccq.size();
    const int64_t NE_A = chain ? 3 * cM * csp * csp : P * nA * ldab, NE = NE_A + P * na * nA + ncc + npb * npb;
    if (nh >= (1 << kSrcShift) || nj >= (1 << kSrcShift) || NE >= INT32_MAX) {
        s->err = "cfx_ipm_create: KKT band too large";
        return create_fail(s, CFX_EUNSUPPORTED);
    }
    // assembled entry -> slot: the blocks' band storage, then (border) Cr active columns per block, the Cc
    // non-zeros, D row-major; padding rows of the blocks get a unit diagonal
    std::vector<int64_t> flat(er.size());
    for (size_t e = 0; e < er.size(); ++e) {
        const int64_t r = pos[er[e]], c = pos[ec[e]];
        if (r < PA && c < PA && chain) {  // [D | L | U] of the stage chain (the grouping makes |kr - kc| <= 1)
            const int64_t kr = r / csp, kc = c / csp, area = kc == kr ? 0 : (kc == kr - 1 ? 1 : 2);
            if (std::abs(kr - kc) > 1) {
                s->err = "cfx_ipm_create: stage-chain grouping is not block tridiagonal";
                return create_fail(s, CFX_EUNSUPPORTED);
            }
            flat[e] = area * cM * csp * csp + kr * csp * csp + (r - kr * csp) * csp + (c - kc * csp);
        } else if (r < PA && c < PA) {  // same block (dissection guarantees it)
            const int64_t q = r / nA, lr = r - q * nA, lc = c - q * nA;
            flat[e] = q * nA * ldab + lc * ldab + kl + ku + lr - lc;
        } else if (r < PA) {
            const int64_t q = r / nA;
            flat[e] = NE_A + (q * na + slv[(size_t)q * npb + (c - PA)]) * nA + (r - q * nA);
        } else if (c < PA) {
            const int64_t k = r - PA;
            const auto& v = ccsorted[k];
            flat[e] = NE_A + P * na * nA + ccptr[k] + (std::lower_bound(v.begin(), v.end(), c) - v.begin());
        } else {
            flat[e] = NE_A + P * na * nA + ncc + (r - PA) * npb + (c - PA);
        }
    }
    std::vector<bool> used(PA, false);
    for (int i = 0; i < nK; ++i)
        if (pos[i] < PA) used[pos[i]] = true;
    for (int64_t sl = 0; sl < PA; ++sl)
        if (!used[sl]) {
            if (chain) {
                const int64_t k = sl / csp, l = sl - k * csp;
                flat.push_back(k * csp * csp + l * csp + l);
            } else {
                const int64_t q = sl / nA, l = sl - q * nA;
                flat.push_back(q * nA * ldab + l * ldab + kl + ku);
            }
            src.push_back((SRC_DC << kSrcShift) | kSrcMask);
        }
    std::vector<int32_t> kptr, kidx, kcode;
    csr(flat, NE, kptr, kidx);
    kcode.resize(kidx.size());
    for (size_t e = 0; e < kidx.size(); ++e) kcode[e] = src[kidx[e]];
    std::vector<int32_t> jtptr, jtidx, jrwptr, jrwidx;
    csr(std::vector<int64_t>(jcF.begin(), jcF.end()), nf, jtptr, jtidx);
    csr(std::vector<int64_t>(jrF.begin(), jrF.end()), m, jrwptr, jrwidx);

    K.nf = nf;
    K.npd = nf + m + (int)std::count(hasL.begin(), hasL.end(), 1) + (int)std::count(hasU.begin(), hasU.end(), 1);
    K.nj = nj;
    K.nh = nh;
    K.nK = nK;
    K.kl = (int)kl;
    K.ku = (int)ku;
    K.ldab = (int)ldab;
    K.P = P;
    K.na = na;
    K.ncc = (int)ncc;
    K.act = dupload(s, actv, &rc);
    K.sl = dupload(s, slv, &rc);
    K.ccr_ptr = dupload(s, ccptr, &rc);
    K.ccr_q = dupload(s, ccq, &rc);
    K.ccr_a = dupload(s, cca, &rc);
    K.nA = (int)nA;
    K.np = (int)npb;
    K.nKp = (int)nKp;
    K.NE_A = NE_A;
    K.NE_tot = NE;
    K.nfix = (int)fixedv.size();
    K.free = dupload(s, freev, &rc);
    K.fixed = dupload(s, fixedv, &rc);
    K.lb_full = dupload(s, lbfull, &rc);
    K.d = dupload(s, d, &rc);
    K.lbF = dupload(s, lbF, &rc);
    K.ubF = dupload(s, ubF, &rc);
    K.lbF0 = dupload(s, lbF0, &rc);
    K.ubF0 = dupload(s, ubF0, &rc);
    K.hasL = dupload(s, hasL, &rc);
    K.hasU = dupload(s, hasU, &rc);
    K.jsel = dupload(s, jsel, &rc);
    K.jr = dupload(s, jrF, &rc);
    K.jc = dupload(s, jcF, &rc);
    K.hsel = dupload(s, hsel, &rc);
    K.hr = dupload(s, hrF, &rc);
    K.hc = dupload(s, hcF, &rc);
    K.hoff = dupload(s, hoff, &rc);
    K.jt_ptr = dupload(s, jtptr, &rc);
    K.jt_idx = dupload(s, jtidx, &rc);
    K.jrw_ptr = dupload(s, jrwptr, &rc);
    K.jrw_idx = dupload(s, jrwidx, &rc);
    K.kkt_ptr = dupload(s, kptr, &rc);
    K.kkt_src = dupload(s, kcode, &rc);
    K.nzpos = nullptr;
    K.nnzA = 0;
    if (chain) {  // the [D | L | U] positions with a source (k_ipm_kkt); the others stay zero after a memset
        std::vector<int32_t> nzp;
        for (int64_t p = 0; p < NE_A; ++p)
            if (kptr[p + 1] > kptr[p]) nzp.push_back((int32_t)p);
        K.nnzA = (int64_t)nzp.size();
        if (!nzp.empty()) K.nzpos = dupload(s, nzp, &rc);
    }
    K.pos = dupload(s, pos, &rc);
    const size_t B = (size_t)s->B;
    double** fbufs[] = {&K.x,   &K.zl,  &K.zu, &K.dx,  &K.dzl, &K.dzu, &K.xt, &K.xacc, &K.xr,
                        &K.dxr, &K.sig, &K.gF, &K.lbI, &K.ubI, &K.wx,  &K.wzl, &K.wzu};
    for (double** p : fbufs) *p = dalloc<double>(s, B * nf, &rc);
    K.rhs = dalloc<double>(s, B * nK, &rc);
    K.rb = dalloc<double>(s, B * nKp, &rc);
    double** mbufs[] = {&K.y, &K.dy, &K.gS, &K.csoc, &K.sg, &K.ysc, &K.graw, &K.gt, &K.wy};
    for (double** p : mbufs) *p = dalloc<double>(s, B * m, &rc);
    K.vx = dalloc<double>(s, B * n, &rc);
    K.vt = dalloc<double>(s, B * n, &rc);
    K.grad = dalloc<double>(s, B * n, &rc);
    K.jac = dalloc<double>(s, B * K.nnzj, &rc);
    K.jv = dalloc<double>(s, B * nj, &rc);
    K.hv = dalloc<double>(s, B * K.nnzh, &rc);
    K.fraw = dalloc<double>(s, B, &rc);
    K.ft = dalloc<double>(s, B, &rc);
    K.of = dalloc<double>(s, B, &rc);
    K.ab = dalloc<double>(s, B * NE_A, &rc);
    K.wide = s->B <= 16 && (int64_t)nj + nh >= 262144;
    K.mu_block = std::getenv("CFX_IPM_MU_ORACLE") && std::string(std::getenv("CFX_IPM_MU_ORACLE")) == "block";
    if (const char* e = std::getenv("CFX_IPM_WIDE")) K.wide = std::atoi(e) != 0;  // tuning / A-B override
    K.gj = dalloc<double>(s, B * nf, &rc);
    K.part = dalloc<double>(s, B * kWideParts * 4, &rc);
    K.wpart = dalloc<double>(s, B * kWideParts * kWP, &rc);
    K.wflag = dalloc<double>(s, B * kWF, &rc);
    K.chain = chain ? 1 : 0;
    K.cM = (int)cM;
    K.csp = (int)csp;
    K.inert = nullptr;
    if (chain) {
        K.cw = dalloc<double>(s, B * 2 * cM * csp * csp, &rc);
        if (K.o.inertia_test) K.inert = dalloc<int32_t>(s, B, &rc);
        K.ct = dalloc<double>(s, B * std::max(na, 1) * nA, &rc);
    }
    K.Xb = dalloc<double>(s, B * P * na * nA, &rc);
    K.Ccb = dalloc<double>(s, B * ncc, &rc);
    K.Db = dalloc<double>(s, B * npb * npb, &rc);
    K.Sf = dalloc<double>(s, B * npb * npb, &rc);
    K.Sp = dalloc<int32_t>(s, B * npb, &rc);
    K.ipiv = dalloc<int32_t>(s, B * nKp, &rc);
    K.info = dalloc<int32_t>(s, B * P, &rc);
    K.filt = dalloc<double>(s, B * kFilt * 2, &rc);
    K.sc = dalloc<Scal>(s, B, &rc);
    K.lbfgs = K.o.hessian_approximation == CFX_HESSIAN_LIMITED_MEMORY;
    K.hmax = K.lbfgs ? K.o.limited_memory_max_history : 0;
    if (K.lbfgs) {
        const size_t H = (size_t)K.hmax, H2 = 2 * H;
        K.Sh = dalloc<double>(s, B * H * nf, &rc);
        K.Yh = dalloc<double>(s, B * H * nf, &rc);
        K.xprev = dalloc<double>(s, B * nf, &rc);
        K.gprev = dalloc<double>(s, B * nf, &rc);
        K.jvprev = dalloc<double>(s, B * nj, &rc);
        K.Mm = dalloc<double>(s, B * H2 * H2, &rc);
        K.Cl = dalloc<double>(s, B * H2 * H2, &rc);
        K.Cp = dalloc<int32_t>(s, B * H2, &rc);
        K.Zb = dalloc<double>(s, H2 * B * nKp, &rc);
    }
    K.rsphase = K.o.restoration == CFX_RESTORATION_PHASE && m > 0;
    if (K.rsphase) {
        double** rbufs[] = {&K.rp, &K.rdp, &K.rn, &K.rdn, &K.rzp, &K.rdzp, &K.rzn, &K.rdzn, &K.rpt, &K.rnt, &K.ry, &K.rdc};
        for (double** p : rbufs) *p = dalloc<double>(s, B * m, &rc);
        K.rzl = dalloc<double>(s, B * nf, &rc);
        K.rzu = dalloc<double>(s, B * nf, &rc);
        K.rfilt = dalloc<double>(s, B * kFilt * 2, &rc);
        if (K.o.soft_resto_pderror_reduction_factor > 0) {
            K.jact = dalloc<double>(s, B * K.nnzj, &rc);
            K.gradt = dalloc<double>(s, B * n, &rc);
        }
    }
    K.rstat = dalloc<unsigned long long>(s, 4, &rc);
    K.adapt = K.o.mu_strategy == CFX_MU_ADAPTIVE;
    K.ncomp = 0;
    for (int i = 0; i < nf; ++i) K.ncomp += (int)hasL[i] + (int)hasU[i];
    K.mfilt = K.rhsmu = K.rbc = K.mgs = nullptr;
    if (K.adapt) {
        K.mgs = dalloc<double>(s, B * kGS, &rc);
        K.mfilt = dalloc<double>(s, B * kFilt * 2, &rc);
        K.rhsmu = dalloc<double>(s, B * nf, &rc);
        K.rbc = dalloc<double>(s, B * nKp, &rc);
    }
    K.cnt = dalloc<int32_t>(s, 4 * kSlots, &rc);
    s->d_fv = dalloc<double>(s, B * K.nfix, &rc);
    s->d_yo = dalloc<double>(s, B * m, &rc);
    s->d_kkt = dalloc<double>(s, B, &rc);
    s->d_zlo = dalloc<double>(s, B * n, &rc);
    s->d_zuo = dalloc<double>(s, B * n, &rc);
    s->d_conv = dalloc<int32_t>(s, B, &rc);
    s->d_its = dalloc<int32_t>(s, B, &rc);
    s->d_status = dalloc<int32_t>(s, B, &rc);
    s->h_status.assign(B, CFX_IPM_MAXIMUM_ITERATIONS_EXCEEDED);
    if (rc == CFX_OK && (hipHostMalloc((void**)&s->h_pub, 16 * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
                         hipHostGetDevicePointer((void**)&s->d_pub, s->h_pub, 0) != hipSuccess)) {
        rc = CFX_ENOMEM;
        s->err = "hipHostMalloc (mapped) failed";
    }
    if (s->h_pub) std::memset(s->h_pub, 0, 16 * sizeof(int32_t));
    if (const char* e = std::getenv("CFX_IPM_SYNC")) s->poll = std::strcmp(e, "stream") != 0;
    if (const char* e = std::getenv("CFX_IPM_KEEPJ")) s->keepj = std::atoi(e) != 0;
    if (const char* e = std::getenv("CFX_IPM_TRACE")) s->trace = std::atoi(e) != 0;
    if (rc == CFX_OK && hipHostMalloc((void**)&s->h_cnt, 4 * sizeof(int32_t), hipHostMallocDefault) != hipSuccess) {
        rc = CFX_ENOMEM;
        s->err = "hipHostMalloc failed";
    }
    if (rc != CFX_OK) return create_fail(s, rc);
    s->st.kkt_n = nK;
    s->st.kkt_kl = kl;
    s->st.kkt_ku = ku;
    s->st.kkt_band_n = nA;
    s->st.kkt_border = npb;
    s->st.kkt_blocks = P;
    s->st.kkt_chain_nodes = chain ? cM : 0;
    s->st.kkt_chain_sp = chain ? csp : 0;
    *out = s;
    return CFX_OK;
}

namespace {

#define IPM_RUN(call)                  \
    do {                               \
        int r2_ = (call);              \
        if (r2_ != CFX_OK) return r2_; \
    } while (0)

struct Run {
    cfx_ipm* s;
    hipStream_t st;
    dim3 g;
    int next_slot() {
        const int k = s->slot;
        s->slot = (s->slot + 1) % kSlots;
        return k;
    }
    int read(int slot, int32_t* c) {
        s->st.host_syncs++;
        if (s->poll) {
            const int32_t seq = ++s->seq;
            hipLaunchKernelGGL(k_ipm_publish, dim3(1), dim3(64), 0, st, (const int32_t*)(s->K.cnt + 4 * slot), s->d_pub,
                               seq);
            IPM_HIP(s, hipGetLastError());
            const auto t0 = std::chrono::steady_clock::now();
            for (long spin = 0;; ++spin) {
                if (__atomic_load_n(s->h_pub, __ATOMIC_ACQUIRE) == seq) {
                    for (int i = 0; i < 4; ++i) c[i] = __atomic_load_n(s->h_pub + 1 + i, __ATOMIC_RELAXED);
                    return CFX_OK;
                }
                // a launch failure never publishes: after a while, let the stream report it
                if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                    IPM_HIP(s, hipStreamSynchronize(st));
                    if (__atomic_load_n(s->h_pub, __ATOMIC_ACQUIRE) == seq) continue;
                    return ipm_fail(s, CFX_EHIP, "cfx_ipm_solve: counter mailbox not written");
                }
            }
        }
        IPM_HIP(s, hipMemcpyAsync(s->h_cnt, s->K.cnt + 4 * slot, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        IPM_HIP(s, hipStreamSynchronize(st));
        std::memcpy(c, s->h_cnt, 4 * sizeof(int32_t));
        return CFX_OK;
    }
    int eval_full(double* v) {
        IPM_RUN(ipm_eval_all(s, v, s->K.graw, s->K.jac, s->K.fraw, s->K.grad, s->jac_flags()));
        s->jac_filled = true;
        s->st.eval_all++;
        return CFX_OK;
    }
    int eval_gf(bool with_f) {
        IPM_RUN(ipm_eval_all(s, s->K.vt, s->K.gt, nullptr, with_f ? s->K.ft : nullptr, nullptr, CFX_DEVICE));
        s->st.eval_g_f++;
        return CFX_OK;
    }
    // Schur complement of the border; wide instances: its back substitution of the blocks as a grid
    int schur(const IpmK& K, int factor) {
        hipLaunchKernelGGL(k_ipm_schur, g, dim3(kIB), 0, st, K, factor, K.wide ? 0 : 1);
        if (K.wide) {
            const int64_t PA = (int64_t)K.P * K.nA;
            hipLaunchKernelGGL(k_wide_border_back, dim3((unsigned)K.B, (unsigned)((PA + kIB - 1) / kIB)), dim3(kIB), 0,
                               st, K);
        }
        IPM_HIP(s, hipGetLastError());
        return CFX_OK;
    }
    // k_ipm_begin, after the wide-instance grids it reads (scaling when mode bit 0; J^T y unless it stops after the
    // scaling, mode bit 1)
    int begin(int mode, int slot) {
        const IpmK& K = s->K;
        if (K.wide) {
            const int64_t n = std::max<int64_t>(std::max<int64_t>(K.nj, K.m), K.nf);
            if (mode & 1)
                hipLaunchKernelGGL(k_wide_scale, dim3((unsigned)K.B, (unsigned)((n + kIB - 1) / kIB)), dim3(kIB), 0,
                                   st, K);
            if (!(mode & 2)) {
                hipLaunchKernelGGL(k_wide_jty, dim3((unsigned)K.B, (unsigned)((K.nf + kIB - 1) / kIB)), dim3(kIB), 0,
                                   st, K);
                hipLaunchKernelGGL(k_wbegin_a, wa(), dim3(kIB), 0, st, K);
            }
        }
        hipLaunchKernelGGL(k_ipm_begin, g, dim3(kIB), 0, st, K, mode, slot);
        if (K.wide && !(mode & 2)) hipLaunchKernelGGL(k_wbegin_c, wc(), dim3(kIB), 0, st, K);
        IPM_HIP(s, hipGetLastError());
        return CFX_OK;
    }
    // wide instances: the partials grid and the elementwise grid of the split kernels
    dim3 wa() const { return dim3((unsigned)s->K.B, kWideParts); }
    dim3 wk() const { return dim3((unsigned)s->K.B, (unsigned)((s->K.nK + kIB - 1) / kIB)); }
    dim3 wc() const {
        const int64_t n = std::max<int64_t>(s->K.nf, s->K.m);
        return dim3((unsigned)s->K.B, (unsigned)((n + kIB - 1) / kIB));
    }
    int curv(int slot) {
        const IpmK& K = s->K;
        if (K.wide) {
            hipLaunchKernelGGL(k_wide_unpack, dim3((unsigned)K.B, kWideParts), dim3(kIB), 0, st, K);
            hipLaunchKernelGGL(k_wide_quad, dim3((unsigned)K.B, kWideParts), dim3(kIB), 0, st, K);
        }
        hipLaunchKernelGGL(k_ipm_curv, g, dim3(kIB), 0, st, K, slot);
        IPM_HIP(s, hipGetLastError());
        return CFX_OK;
    }
    // stage chain (IpmK::chain): the block cyclic reduction of [D | L | U] in ab; solves of nrhs right-hand sides at
    // R + b r_inst + c r_rhs (the chain part, nA entries, of rb-shaped or Xb arrays)
    int chain_factor() {
        const IpmK& K = s->K;
        const int64_t nb = (int64_t)K.cM * K.csp * K.csp;
        return cfx_chain_factor_s(K.B, K.cM, K.csp, K.ab, K.ab + nb, K.ab + 2 * nb, K.NE_A, K.cw, K.cw + nb, 2 * nb,
                                  K.info, st);
    }
    int chain_solve(double* R, int64_t r_inst, int64_t r_rhs, int nrhs) {
        const IpmK& K = s->K;
        const int64_t nb = (int64_t)K.cM * K.csp * K.csp;
        return cfx_chain_solve_s(K.B, K.cM, K.csp, K.ab, K.ab + nb, K.ab + 2 * nb, K.NE_A, K.cw, K.cw + nb, 2 * nb,
                                 nrhs, R, r_inst, r_rhs, K.ct, (int64_t)nrhs * K.nA, K.nA, st);
    }
    int kkt_factor(int mode) {
        const IpmK& K = s->K;
        const int64_t NE = K.nzpos ? K.nnzA + (K.NE_tot - K.NE_A) : K.NE_tot;
        if (K.nzpos) IPM_HIP(s, hipMemsetAsync(K.ab, 0, (size_t)K.B * K.NE_A * sizeof(double), st));
        const int64_t nblk = (std::max<int64_t>(NE, K.nK) + kIB - 1) / kIB;
        hipLaunchKernelGGL(k_ipm_kkt, dim3((unsigned)K.B, (unsigned)std::min<int64_t>(nblk, kMaxY)), dim3(kIB), 0, st,
                           K, mode);
        IPM_HIP(s, hipGetLastError());
        if (K.chain) {  // stage chain: block cyclic reduction, then (border) A^-1 [Cr | r] and the Schur complement
            IPM_BAND(s, chain_factor());
            if (K.inert) {  // the inertia: the chain's pivot blocks here, the border's Schur complement in k_ipm_schur
                IPM_HIP(s, hipMemsetAsync(K.inert, 0, (size_t)K.B * sizeof(int32_t), st));
                IPM_BAND(s, cfx_chain_inertia_s(K.B, K.cM, K.csp, K.ab, K.NE_A, K.inert, st));
            }
            if (K.np) IPM_BAND(s, chain_solve(K.Xb, (int64_t)K.na * K.nA, K.nA, K.na));
            IPM_BAND(s, chain_solve(K.rb, K.nKp, 0, 1));
            if (K.np) IPM_RUN(schur(K, 1));
        } else if (K.np) {  // blocks + border: factor the blocks, A_q^-1 [Cr_q | r_q] (parallel right-hand sides), Schur
            const int64_t BP = K.B * K.P, nb = (int64_t)K.na * K.nA;
            IPM_BAND(s, cfx_band_lu(K.nA, K.kl, K.ku, BP, K.ab, K.ipiv, K.info, 0, nullptr, st));
            IPM_BAND(s, cfx_band_solve_multi(K.nA, K.kl, K.ku, BP, K.P, K.ab, K.ipiv, K.Xb, K.P * nb, nb, K.nA, K.na,
                                             K.rb, K.nKp, K.nA, st));
            IPM_RUN(schur(K, 1));
        } else {
            IPM_BAND(s, cfx_band_lu(K.nK, K.kl, K.ku, K.B, K.ab, K.ipiv, K.info, 1, K.rb, st));
        }
        s->st.kkt_factor++;
        return CFX_OK;
    }
    // another right-hand side (in rb, band order — or in the rb-shaped array `into`) with the factors of the last
    // kkt_factor
    int resolve(double* into = nullptr) {
        IpmK K = s->K;
        if (into) K.rb = into;
        if (K.chain) {
            IPM_BAND(s, chain_solve(K.rb, K.nKp, 0, 1));
            if (K.np) IPM_RUN(schur(K, 0));
        } else if (K.np) {
            IPM_BAND(s, cfx_band_solve_multi(K.nA, K.kl, K.ku, K.B * K.P, K.P, K.ab, K.ipiv, nullptr, 0, 0, 0, 0,
                                             K.rb, K.nKp, K.nA, st));
            IPM_RUN(schur(K, 0));
        } else {
            IPM_BAND(s, cfx_band_lu_solve(K.nK, K.kl, K.ku, K.B, K.ab, K.ipiv, 1, K.rb, st));
        }
        return CFX_OK;
    }
    // adaptive mu: the unit-centering solve with the factors just made, then the quality-function oracle of the
    // free-mode instances, which leaves their combined Newton step in rb (k_mu_oracle)
    int mu_oracle() {
        const IpmK& K = s->K;
        const dim3 gk((unsigned)K.B, (unsigned)((K.nK + kIB - 1) / kIB));
        if (K.wide) hipLaunchKernelGGL(k_wmu_cen_rhs, gk, dim3(kIB), 0, st, K);
        else hipLaunchKernelGGL(k_mu_cen_rhs, g, dim3(kIB), 0, st, K);
        IPM_HIP(s, hipGetLastError());
        IPM_RUN(resolve(K.rbc));
        if (K.lbfgs) {  // the Woodbury correction of the centering solution too
            IpmK K2 = K;
            K2.rb = K.rbc;
            hipLaunchKernelGGL(k_lbfgs_apply, g, dim3(kIB), 0, st, K2);
        }
        if (!K.wide) {
            hipLaunchKernelGGL(k_mu_oracle, g, dim3(kIB), 0, st, K);
            IPM_HIP(s, hipGetLastError());
            return CFX_OK;
        }
        // wide instances: the section's rounds (the pair at sigma = 1, the first pair of section points, one point per
        // section step, the end point), each a no-op once the instance's section has finished
        hipLaunchKernelGGL(k_wmu_init, g, dim3(64), 0, st, K);
        const int rounds = K.o.quality_function_max_section_steps + 3;
        for (int r = 0; r < rounds; ++r) {
            hipLaunchKernelGGL(k_wmu_min, wa(), dim3(kIB), 0, st, K);
            hipLaunchKernelGGL(k_wmu_sum, wa(), dim3(kIB), 0, st, K);
            hipLaunchKernelGGL(k_wmu_ctl, g, dim3(kIB), 0, st, K);
        }
        hipLaunchKernelGGL(k_wmu_apply, gk, dim3(kIB), 0, st, K);
        IPM_HIP(s, hipGetLastError());
        return CFX_OK;
    }
    // L-BFGS: after a Newton factorisation of K0, P = K0^-1 Z column by column, C = M - Z^T P, and the Newton
    // solution corrected (rb += P C^-1 Z^T rb)
    int lbfgs_newton() {
        const IpmK& K = s->K;
        hipLaunchKernelGGL(k_lbfgs_zcols, g, dim3(kIB), 0, st, K);
        IPM_HIP(s, hipGetLastError());
        for (int q = 0; q < 2 * K.hmax; ++q) IPM_RUN(resolve(K.Zb + (size_t)q * K.B * K.nKp));
        hipLaunchKernelGGL(k_lbfgs_factor, g, dim3(kIB), 0, st, K);
        hipLaunchKernelGGL(k_lbfgs_apply, g, dim3(kIB), 0, st, K);
        IPM_HIP(s, hipGetLastError());
        return CFX_OK;
    }
};

}  // namespace


static int ipm_solve(cfx_ipm* s, const double* v0, const double* fixed_values, double* v_out, double* y_out,
                     double* f_out, int32_t* conv_out, int32_t* its_out, double* kkt_out, uint32_t flags) {
    const auto t0 = std::chrono::steady_clock::now();
    int64_t Bq = 0;
    int layout = 0, dev = 0;
    hipStream_t st = nullptr;
    if (s->ext)
        st = s->stream;
    else if (cfx_internal_info(s->h, &Bq, &layout, &dev, &st) != CFX_OK)
        return ipm_fail(s, CFX_EINVAL, "bad handle");
    IPM_HIP(s, hipSetDevice(s->device));
    s->stream = st;
    // MSK handles: eval_h re-uses the stage data of the eval_all just before it at the same point (switched off
    // again on every exit path)
    struct StashGuard {
        cfx_handle* h;
        ~StashGuard() {
            if (h) cfx_internal_msk_stash(h, 0);
        }
    } stash_guard{s->h};
    if (s->h) cfx_internal_msk_stash(s->h, 1);
    IpmK& K = s->K;
    const bool devp = flags & CFX_DEVICE;
    const size_t B = (size_t)K.B;
    const hipMemcpyKind kin = devp ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    const hipMemcpyKind kout = devp ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    Run R{s, st, dim3((unsigned)B)};
    const dim3 blk(kIB);
    s->st.eval_all = s->st.eval_g_f = s->st.eval_h = s->st.kkt_factor = s->st.iterations = s->st.host_syncs = 0;
    s->st.resto_phases = s->st.resto_iterations = s->st.soft_steps = 0;
    IPM_HIP(s, hipMemsetAsync(K.rstat, 0, 4 * sizeof(unsigned long long), st));
    if (K.rsphase)  // the (2,2) block of instances outside the phase
        IPM_HIP(s, hipMemsetAsync(K.rdc, 0, B * K.m * sizeof(double), st));
    s->slot = 0;
    IPM_HIP(s, hipMemsetAsync(K.cnt, 0, 4 * kSlots * sizeof(int32_t), st));
    IPM_HIP(s, hipMemsetAsync(K.rb, 0, B * K.nKp * sizeof(double), st));  // padding rows of the blocks stay 0
    if (K.adapt) IPM_HIP(s, hipMemsetAsync(K.rbc, 0, B * K.nKp * sizeof(double), st));
    if (K.lbfgs) IPM_HIP(s, hipMemsetAsync(K.hv, 0, B * K.nnzh * sizeof(double), st));  // W enters as sigma I
    IPM_HIP(s, hipMemcpyAsync(K.vx, v0, B * K.n * sizeof(double), kin, st));
    if (fixed_values && K.nfix)
        IPM_HIP(s, hipMemcpyAsync(s->d_fv, fixed_values, B * K.nfix * sizeof(double), kin, st));
    hipLaunchKernelGGL(k_ipm_fix, R.g, blk, 0, st, K, (const double*)(fixed_values && K.nfix ? s->d_fv : nullptr));
    IPM_RUN(R.eval_full(K.vx));
    const bool warm = K.o.warm_start_init_point != 0;
    if (warm && !s->warm_set)
        return ipm_fail(s, CFX_EINVAL, "cfx_ipm_solve: warm_start_init_point needs cfx_ipm_set_warm_start first");
    hipLaunchKernelGGL(k_ipm_init, R.g, blk, 0, st, K, warm ? (const double*)s->d_wy : nullptr,
                       warm ? (const double*)s->d_wzl : nullptr, warm ? (const double*)s->d_wzu : nullptr);
    IPM_HIP(s, hipGetLastError());
    IPM_HIP(s, hipMemcpyAsync(K.vt, K.vx, B * K.n * sizeof(double), hipMemcpyDeviceToDevice, st));
    bool reinit = K.m > 0 && !warm, wall_stop = false;
    int32_t c[4];
    int n_active = (int)B, n_resto = 0;
    double last_print = 0.0;
    // some instance may be in the restoration phase: the k_rs_* launches are skipped while none is (the batch-1
    // latency of an iteration is its chain of launches)
    bool rs_live = false;
    // One host iteration advances every instance still iterating by one iteration of its own: a main iteration, or
    // one of the restoration phase (k_rs_*) for the instances in it — the same callback launches, factorisations and
    // line-search loop serve both (section "Ipopt's feasibility-restoration phase" above).  Every instance's
    // iterations (phase ones included) count against its max_iter, so max_iter host iterations bound the loop.
    for (int it = 0; it < K.o.max_iter; ++it) {
        const double elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (elapsed > K.o.max_wall_time) {  // Ipopt max_wall_time: the instances still iterating stop where they are
            wall_stop = true;
            break;
        }
        if (s->trace && it > 0) {  // CFX_IPM_TRACE=1: instance 0's iterate every iteration (diagnostics)
            Scal s0{};
            IPM_HIP(s, hipMemcpyAsync(&s0, K.sc, sizeof(Scal), hipMemcpyDeviceToHost, st));
            IPM_HIP(s, hipStreamSynchronize(st));
            std::fprintf(stderr,
                         "cfx_ipm trace %d: iters %d f %.10e err %.3e mu %.3e theta %.3e alpha %.3e a_z %.3e dw %.2e "
                         "resto %d soft %d wd %d acc %d free %d avgc %.3e\n",
                         it, s0.iters, s0.fS / s0.sf, s0.err0, s0.mu, s0.theta, s0.alpha, s0.a_z, s0.dwl, s0.rs_on,
                         s0.soft_on, s0.wd_on, s0.acc, s0.mfree, s0.avgc);
        }
        if (K.o.print_frequency_time > 0 && it > 0 && elapsed - last_print >= K.o.print_frequency_time) {
            Scal s0{};  // instance 0's optimality error, barrier, infeasibility and last step (one small read)
            IPM_HIP(s, hipMemcpyAsync(&s0, K.sc, sizeof(Scal), hipMemcpyDeviceToHost, st));
            IPM_HIP(s, hipStreamSynchronize(st));
            std::fprintf(stderr,
                         "cfx_ipm: iteration %d, %.1f s: %d of %lld instances iterating, %d in restoration; instance 0: "
                         "error %.3e, mu %.1e, theta %.3e, alpha %.2e\n",
                         it, elapsed, n_active, (long long)B, n_resto, s0.err0, s0.mu, s0.theta, s0.alpha);
            std::fflush(stderr);
            last_print = elapsed;
        }
        // after an ordinary iteration the multipliers of the Hessian are known before k_ipm_begin (k_ipm_update
        // formed them; k_rs_update / k_rs_init for the instances in the restoration phase, objective factor 0): g,
        // J_g, f, grad f and the Hessian of the new iterate from one call
        const bool fused = it > 0 && !reinit && !K.lbfgs && K.m > 0 && !s->ext;
        if (fused) {
            IPM_CFX(s, cfx_eval_all_h(s->h, K.vx, K.of, K.ysc, K.graw, K.jac, K.fraw, K.grad, K.hv, s->jac_flags()));
            s->jac_filled = true;
            s->st.eval_all++;
            s->st.eval_h++;
        } else {
            IPM_RUN(R.eval_full(K.vx));
        }
        if (reinit) {  // least-squares multipliers for the flagged instances (start, after a restoration)
            IPM_RUN(R.begin(3, 0));
            IPM_RUN(R.kkt_factor(KKT_LSMULT));
            hipLaunchKernelGGL(k_ipm_lsmult, R.g, blk, 0, st, K);
            IPM_RUN(R.begin(0, R.next_slot()));
        } else {
            IPM_RUN(R.begin(1, R.next_slot()));
        }
        if (K.rsphase && rs_live) {
            if (K.wide) {
                const int64_t nsc = std::max<int64_t>(K.nj, K.m);
                hipLaunchKernelGGL(k_wrs_scale, dim3((unsigned)K.B, (unsigned)((nsc + kIB - 1) / kIB)), blk, 0, st, K);
                hipLaunchKernelGGL(k_wrs_a, R.wa(), blk, 0, st, K);
            }
            hipLaunchKernelGGL(k_rs_begin, R.g, blk, 0, st, K);
            if (K.wide) hipLaunchKernelGGL(k_wrs_c, R.wc(), blk, 0, st, K);
        }
        reinit = false;
        IPM_HIP(s, hipGetLastError());
        if (K.lbfgs) {  // quasi-Newton pair of the last step, M (no eval_h: hv stays zero)
            hipLaunchKernelGGL(k_lbfgs_update, R.g, blk, 0, st, K);
            IPM_HIP(s, hipGetLastError());
        } else if (!fused) {
            if (s->h) cfx_internal_msk_stash(s->h, 2);  // K.vx is eval_full's point: the MSK stage data may be re-used
            IPM_RUN(ipm_eval_h(s, K.vx, K.of, K.ysc, K.hv));
            s->st.eval_h++;
        }
        // inertia correction by the curvature test: grow dw until dx^T (W + Sigma + dw) dx > 0
        bool all_done = false;
        for (int attempt = 0; attempt < 12; ++attempt) {
            IPM_RUN(R.kkt_factor(KKT_NEWTON));
            if (K.lbfgs) IPM_RUN(R.lbfgs_newton());
            if (K.adapt) IPM_RUN(R.mu_oracle());
            const int sl = R.next_slot();
            IPM_RUN(R.curv(sl));
            IPM_HIP(s, hipGetLastError());
            IPM_RUN(R.read(sl, c));
            if (attempt == 0) {
                n_active = c[0];
                n_resto = c[2];
            }
            if (c[0] == 0) {
                all_done = true;
                break;
            }
            if (c[1] == 0) break;
        }
        if (all_done) break;
        rs_live = n_resto > 0;  // instances iterating in the phase (counted by k_ipm_curv)
        if (K.wide) hipLaunchKernelGGL(k_wdir_a, R.wa(), blk, 0, st, K);
        hipLaunchKernelGGL(k_ipm_dir, R.g, blk, 0, st, K, it);
        if (K.wide) hipLaunchKernelGGL(k_wdir_c, R.wc(), blk, 0, st, K);
        if (K.rsphase && rs_live) hipLaunchKernelGGL(k_rs_dir, R.g, blk, 0, st, K);
        // filter line search with second-order corrections (the phase's own filter line search alongside)
        int notacc = 0, n_soft = 0;
        for (int ls = 0; ls < K.o.max_backtrack; ++ls) {
            IPM_RUN(R.eval_gf(true));
            int sl = R.next_slot();
            if (K.rsphase && rs_live) hipLaunchKernelGGL(k_rs_accept, R.g, blk, 0, st, K);
            if (K.wide) hipLaunchKernelGGL(k_wacc_a, R.wa(), blk, 0, st, K, 0);
            hipLaunchKernelGGL(k_ipm_accept, R.g, blk, 0, st, K, ls, sl);
            if (K.wide) hipLaunchKernelGGL(k_wacc_c, R.wc(), blk, 0, st, K);
            IPM_HIP(s, hipGetLastError());
            IPM_RUN(R.read(sl, c));
            notacc = c[0];
            if (ls == 0) n_soft = c[2];
            if (ls == 0)
                for (int q = 0; q < K.o.max_soc && c[1] > 0; ++q) {
                    if (K.wide) hipLaunchKernelGGL(k_wsoc_rhs, R.wk(), blk, 0, st, K);
                    else hipLaunchKernelGGL(k_ipm_soc_rhs, R.g, blk, 0, st, K);
                    IPM_RUN(R.resolve());
                    if (K.lbfgs) hipLaunchKernelGGL(k_lbfgs_apply, R.g, blk, 0, st, K);
                    if (K.wide) {
                        hipLaunchKernelGGL(k_wsoct_a, R.wa(), blk, 0, st, K);
                        hipLaunchKernelGGL(k_wsoct_c, R.wc(), blk, 0, st, K);
                    } else {
                        hipLaunchKernelGGL(k_ipm_soc_trial, R.g, blk, 0, st, K);
                    }
                    IPM_RUN(R.eval_gf(true));
                    sl = R.next_slot();
                    if (K.wide) hipLaunchKernelGGL(k_wacc_a, R.wa(), blk, 0, st, K, 1);
                    hipLaunchKernelGGL(k_ipm_soc_accept, R.g, blk, 0, st, K, sl);
                    if (K.wide) hipLaunchKernelGGL(k_wsoca_c, R.wc(), blk, 0, st, K);
                    IPM_HIP(s, hipGetLastError());
                    IPM_RUN(R.read(sl, c));
                    notacc = c[0];
                }
            if (notacc == 0) break;
            if (K.wide) {
                hipLaunchKernelGGL(k_wnext_a, R.wc(), blk, 0, st, K);
                hipLaunchKernelGGL(k_wnext_b, dim3((unsigned)((K.B + kIB - 1) / kIB)), blk, 0, st, K);
            } else {
                hipLaunchKernelGGL(k_ipm_next_trial, R.g, blk, 0, st, K);
            }
            if (K.rsphase && rs_live) hipLaunchKernelGGL(k_rs_next_trial, R.g, blk, 0, st, K);
        }
        // Ipopt's soft restoration: the failed searches and the instances taking soft steps try the step at the
        // fraction to the boundary (k_soft_trial counts them; one eval_all at their trial points; k_soft_accept)
        if (K.jact && (notacc > 0 || n_soft > 0)) {
            int sl = R.next_slot();
            hipLaunchKernelGGL(k_soft_trial, R.g, blk, 0, st, K, sl);
            IPM_HIP(s, hipGetLastError());
            IPM_RUN(R.read(sl, c));
            notacc += c[1];  // soft steps exhausted: failed searches from here on
            if (c[0] > 0) {
                IPM_RUN(ipm_eval_all(s, K.vt, K.gt, K.jact, K.ft, K.gradt, CFX_DEVICE));
                s->st.eval_all++;
                sl = R.next_slot();
                hipLaunchKernelGGL(k_soft_accept, R.g, blk, 0, st, K, sl);
                IPM_HIP(s, hipGetLastError());
                IPM_RUN(R.read(sl, c));
                notacc = c[0];
            }
        }
        // failed line searches: the restoration phase (its iterations for the instances in it; the instances whose
        // search failed enter it), or a feasibility-restoration step, a fresh filter and least-squares multipliers
        const bool resto = notacc > 0 && K.m > 0;
        if (K.rsphase) {
            if (rs_live) hipLaunchKernelGGL(k_rs_update, R.g, blk, 0, st, K);
            if (resto) hipLaunchKernelGGL(k_rs_init, R.g, blk, 0, st, K);
            IPM_HIP(s, hipGetLastError());
            rs_live = rs_live || resto;  // entrants (k_rs_init) or instances still in the phase
        } else if (resto) {
            IPM_RUN(R.kkt_factor(KKT_RESTO));
            int sl = R.next_slot();
            hipLaunchKernelGGL(k_ipm_resto_init, R.g, blk, 0, st, K, sl);
            IPM_RUN(R.read(sl, c));
            for (int r = 0; r < 20 && c[0] > 0; ++r) {
                IPM_RUN(R.eval_gf(false));
                sl = R.next_slot();
                hipLaunchKernelGGL(k_ipm_resto_accept, R.g, blk, 0, st, K, sl);
                IPM_HIP(s, hipGetLastError());
                IPM_RUN(R.read(sl, c));
            }
            reinit = true;
        }
        if (K.wide) hipLaunchKernelGGL(k_wupd_a, R.wa(), blk, 0, st, K);
        hipLaunchKernelGGL(k_ipm_update, R.g, blk, 0, st, K, K.rsphase ? 2 : (resto ? 1 : 0));
        if (K.wide) hipLaunchKernelGGL(k_wupd_c, R.wc(), blk, 0, st, K);
        IPM_HIP(s, hipGetLastError());
        s->st.iterations++;
    }
    if (K.rsphase) hipLaunchKernelGGL(k_rs_finish, R.g, blk, 0, st, K);
    hipLaunchKernelGGL(k_ipm_final, R.g, blk, 0, st, K, s->d_zlo, s->d_zuo);
    IPM_RUN(ipm_eval_all(s, K.vx, K.graw, nullptr, K.fraw, nullptr, CFX_DEVICE));
    s->st.eval_g_f++;
    hipLaunchKernelGGL(k_ipm_out, R.g, blk, 0, st, K, devp ? y_out : (y_out ? s->d_yo : nullptr),
                       devp ? conv_out : (conv_out ? s->d_conv : nullptr), devp ? its_out : (its_out ? s->d_its : nullptr),
                       devp ? kkt_out : (kkt_out ? s->d_kkt : nullptr), s->d_status, (int)wall_stop);
    IPM_HIP(s, hipGetLastError());
    unsigned long long rstat[4] = {0, 0, 0, 0};
    IPM_HIP(s, hipMemcpyAsync(rstat, K.rstat, sizeof(rstat), hipMemcpyDeviceToHost, st));
    IPM_HIP(s, hipMemcpyAsync(s->h_status.data(), s->d_status, B * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    IPM_HIP(s, hipStreamSynchronize(st));
    s->st.resto_phases = (int64_t)rstat[0];
    s->st.resto_iterations = (int64_t)rstat[1];
    s->st.soft_steps = (int64_t)rstat[2];
    s->st.mu_mode_switches = (int64_t)rstat[3];
    if (v_out) IPM_HIP(s, hipMemcpyAsync(v_out, K.vx, B * K.n * sizeof(double), kout, st));
    if (f_out) IPM_HIP(s, hipMemcpyAsync(f_out, K.fraw, B * sizeof(double), kout, st));
    if (!devp) {
        if (y_out) IPM_HIP(s, hipMemcpyAsync(y_out, s->d_yo, B * K.m * sizeof(double), kout, st));
        if (conv_out) IPM_HIP(s, hipMemcpyAsync(conv_out, s->d_conv, B * sizeof(int32_t), kout, st));
        if (its_out) IPM_HIP(s, hipMemcpyAsync(its_out, s->d_its, B * sizeof(int32_t), kout, st));
        if (kkt_out) IPM_HIP(s, hipMemcpyAsync(kkt_out, s->d_kkt, B * sizeof(double), kout, st));
        IPM_HIP(s, hipStreamSynchronize(st));
    }
    s->st.wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return CFX_OK;
}

extern "C" int cfx_ipm_solve(cfx_ipm* s, const double* v0, const double* fixed_values, double* v, double* y,
                             double* f, int32_t* converged, int32_t* iterations, double* kkt_error, uint32_t flags) {
    if (!s) return CFX_EINVAL;
    if (!v0) return ipm_fail(s, CFX_EINVAL, "cfx_ipm_solve: v0 is NULL");
    return ipm_solve(s, v0, fixed_values, v, y, f, converged, iterations, kkt_error, flags);
}

extern "C" int cfx_ipm_set_warm_start(cfx_ipm* s, const double* y, const double* z_l, const double* z_u,
                                      uint32_t flags) {
    if (!s) return CFX_EINVAL;
    if ((s->K.m && !y) || !z_l || !z_u) return ipm_fail(s, CFX_EINVAL, "cfx_ipm_set_warm_start: NULL input");
    IPM_HIP(s, hipSetDevice(s->device));
    int rc = CFX_OK;
    const size_t B = (size_t)s->K.B;
    if (!s->d_wy) {
        s->d_wy = dalloc<double>(s, B * s->K.m, &rc);
        s->d_wzl = dalloc<double>(s, B * s->K.n, &rc);
        s->d_wzu = dalloc<double>(s, B * s->K.n, &rc);
        if (rc != CFX_OK) return rc;
    }
    const hipMemcpyKind k = (flags & CFX_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (s->K.m) IPM_HIP(s, hipMemcpy(s->d_wy, y, B * s->K.m * sizeof(double), k));
    IPM_HIP(s, hipMemcpy(s->d_wzl, z_l, B * s->K.n * sizeof(double), k));
    IPM_HIP(s, hipMemcpy(s->d_wzu, z_u, B * s->K.n * sizeof(double), k));
    s->warm_set = true;
    return CFX_OK;
}

extern "C" int cfx_ipm_get_bound_multipliers(cfx_ipm* s, double* z_l, double* z_u, uint32_t flags) {
    if (!s || !z_l || !z_u) return CFX_EINVAL;
    IPM_HIP(s, hipSetDevice(s->device));
    const size_t bytes = (size_t)s->K.B * s->K.n * sizeof(double);
    const hipMemcpyKind k = (flags & CFX_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (s->stream) IPM_HIP(s, hipStreamSynchronize(s->stream));
    IPM_HIP(s, hipMemcpy(z_l, s->d_zlo, bytes, k));
    IPM_HIP(s, hipMemcpy(z_u, s->d_zuo, bytes, k));
    return CFX_OK;
}

extern "C" int cfx_ipm_get_status(const cfx_ipm* s, int32_t* status) {
    if (!s || !status) return CFX_EINVAL;
    std::memcpy(status, s->h_status.data(), s->h_status.size() * sizeof(int32_t));
    return CFX_OK;
}

extern "C" int cfx_ipm_get_stats(const cfx_ipm* s, cfx_ipm_stats* out) {
    if (!s || !out) return CFX_EINVAL;
    *out = s->st;
    return CFX_OK;
}

extern "C" int cfx_ipm_n_fixed(const cfx_ipm* s) { return s ? s->K.nfix : -1; }

extern "C" const char* cfx_ipm_last_error(const cfx_ipm* s) { return s ? s->err.c_str() : ""; }

extern "C" void cfx_ipm_destroy(cfx_ipm* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    for (void* p : s->allocs) (void)hipFree(p);
    if (s->h_cnt) (void)hipHostFree(s->h_cnt);
    if (s->h_pub) (void)hipHostFree(s->h_pub);
    delete s;
}
