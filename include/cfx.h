/*
 * cfx.h — C ABI of libcfx, the MI355X (gfx950) NLP-callback engine for cocofest's FES optimal-control
 * problems (Ding2003 / Ding2007 / Hmed2018 calcium-force models, with or without fatigue).
 *
 * What it replaces (reference: Ipuch/cocofest @ 2025-02-24; transcription/evaluation live in the
 * unvendored bioptim + CasADi + Ipopt stack):
 *   - the bioptim dynamics plugin registered by every model's declare_ding_variables
 *     (cocofest/models/ding2003.py:373-392, ding2007.py:288-308, hmed2018.py:281-301) and called
 *     symbolically through `dynamics(time, states, controls, parameters, algebraic_states,
 *     numerical_timeseries, nlp, ...)` (cocofest/models/fes_model.py:182-202);
 *   - the CasADi-generated NLP callbacks that Ipopt invokes on the OptimalControlProgram built at
 *     cocofest/optimization/fes_ocp.py:171-190 (Ipopt TNLP eval_f / eval_grad_f / eval_g /
 *     eval_jac_g / eval_h: solver-owned contiguous double arrays, COO sparsity fixed up front);
 *   - the single-shooting integration behind IvpFes.integrate (cocofest/integration/ivp_fes.py:282-297).
 *
 * Conventions
 *   - Plain C types only.  Every buffer is caller-owned.  With CFX_DEVICE the pointers are HIP device
 *     pointers and the call is asynchronous on the handle's stream; otherwise they are host pointers
 *     and the call copies in, computes on the GPU and copies out before returning.
 *   - All arithmetic is FP64.  Every evaluation runs on the GPU; there is no CPU fallback: creating a
 *     handle without a usable HIP device fails with CFX_ENODEV.
 *   - Batches: B independent instances of one problem (multi-start, parameter sweeps, NMPC scenarios).
 *     CFX_LAYOUT_AOS: instance-major, element e of instance b at buf[b*len + e] (Ipopt's per-instance
 *     contiguous arrays).  CFX_LAYOUT_SOA: element-major, buf[e*B + b] (coalesced; the native layout).
 *   - Decision vector of one instance (node-major): [x_0, u_0, x_1, u_1, ..., x_{N-1}, u_{N-1}, x_N, p]
 *     with x_k the nx states (Cn, F[, A, Tau1, Km]; state_configure.py:8-319), u_k the nu controls
 *     (Ding2007: last_pulse_width; Hmed2018: the T pulse intensities aligned with the node's stim row),
 *     p the Hmed intensity parameters (fes_ocp.py:350-411).
 *   - Constraints of one instance: per interval k, the nx continuity rows Phi(x_k,u_k) - x_{k+1}
 *     followed (Hmed with parameters) by the T sliding-window rows u_k - window_k(p)
 *     (custom_constraints.py:102-119, fes_ocp.py:413-438).
 *   - Integer error codes; cfx_last_error() gives the message.  A handle is bound to one device and one
 *     stream and is not thread-safe; use one handle per GPU / per thread.
 */
#ifndef CFX_H
#define CFX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CFX_ABI_VERSION 11

/* return codes */
#define CFX_OK 0
#define CFX_EINVAL (-1)
#define CFX_EHIP (-2)
#define CFX_ENOMEM (-3)
#define CFX_EUNSUPPORTED (-4)
#define CFX_ENODEV (-5)
#define CFX_ECALLBACK (-6) /* a caller-supplied evaluator (cfx_ipm_create_ext) returned non-zero */

/* models (cocofest/models/model_maker.py:9-22) */
#define CFX_DING2003 0
#define CFX_DING2003_FATIGUE 1
#define CFX_DING2007 2
#define CFX_DING2007_FATIGUE 3
#define CFX_HMED2018 4
#define CFX_HMED2018_FATIGUE 5

/* transcription (OdeSolver.RK1/RK2/RK4 with n_integration_steps; fes_ocp.py:120,334-338) */
#define CFX_RK1 1
#define CFX_RK2 2
#define CFX_RK4 4
/* direct collocation (OdeSolver.COLLOCATION(polynomial_degree, method)): one Lagrange polynomial per shooting
   interval through the node state and `n_steps` (= the degree d, 1..9) Legendre or Radau IIA points.
   Decision block per interval [x_k^0, x_k^1..x_k^d, u_k]; rows per interval: d defect blocks of nx, the
   continuity block of nx, then the sliding-window rows.  cfx_integrate is not available for it. */
#define CFX_COLLOCATION_LEGENDRE 16
#define CFX_COLLOCATION_RADAU 17

/* layouts and call flags */
#define CFX_LAYOUT_AOS 0
#define CFX_LAYOUT_SOA 1
/* 64-instance tiles: element e of instance b at ((b / 64) * len + e) * 64 + b % 64, len = the per-instance
   length of the buffer (nv, ng, nnz_jac, nv for grad, 1 for f).  batch % 64 == 0.  Keeps each wave's stores
   inside one contiguous tile instead of spreading them over len rows B apart (+6 % on the store-bound
   g + J_g pass).  Shooting and collocation transcriptions: eval_g / eval_jac_g / eval_f / eval_grad_f / eval_all /
   eval_h / eval_all_h (bit-identical to the SoA results). */
#define CFX_LAYOUT_TILED64 2
#define CFX_DEVICE 1u /* pointers are device pointers; call is asynchronous on the handle stream */
/* eval_jac_g / eval_all / eval_all_h: the J_g values cfx_jac_constant_mask lists are not written — the output buffer
   already holds them from an earlier full evaluation (with CFX_DEVICE on a buffer the kernels write directly: the
   caller's buffer; otherwise the handle's staging buffer, filled by the first evaluation).  Ipopt's TNLP contract
   asks for every value on every call: callers bound by it leave this flag off. */
#define CFX_KEEP_CONSTANT_JAC 2u

/* objective terms (fes_ocp.py:531-569) */
#define CFX_OBJ_LAGRANGE 0 /* weight * dt * (z_k - target_k)^2 summed over the node range */
#define CFX_OBJ_MAYER 1    /* weight * (z_k - target_k)^2 summed over the node range */
#define CFX_VAR_STATE 0
#define CFX_VAR_CONTROL 1

typedef struct cfx_constants {
    /* ding2003.py:51-66 */
    double tauc, r0_km_relationship, a_rest, tau1_rest, tau2, km_rest;
    /* ding2007.py:63-79 */
    double a_scale, pd0, pdt;
    /* hmed2018.py:53-63 */
    double ar, bs, Is, cr;
    /* ding2003_with_fatigue.py:50-59 */
    double alpha_a, alpha_tau1, alpha_km, tau_fat;
    /* force-length / force-velocity multipliers and passive force (ding2003.py:274-311) */
    double fl, fv, fp;
} cfx_constants;

typedef struct cfx_objective {
    int32_t kind;       /* CFX_OBJ_LAGRANGE | CFX_OBJ_MAYER */
    int32_t var_kind;   /* CFX_VAR_STATE | CFX_VAR_CONTROL */
    int32_t var_index;  /* state or control component */
    int32_t node_first; /* inclusive node range; controls: 0..N-1, states: 0..N */
    int32_t node_last;
    double weight;
    const double *target; /* per node (indexed by node, length N+1) or NULL -> target_value */
    double target_value;
} cfx_objective;

typedef struct cfx_problem {
    int32_t abi_version; /* CFX_ABI_VERSION */
    int32_t model;       /* CFX_DING2003 ... CFX_HMED2018_FATIGUE */
    int32_t scheme;      /* CFX_RK1 | CFX_RK2 | CFX_RK4 | CFX_COLLOCATION_LEGENDRE | CFX_COLLOCATION_RADAU */
    int32_t n_steps;     /* RK sub-steps per shooting interval (n_integration_steps); collocation degree */
    int32_t n_shooting;  /* N */
    int32_t truncation;  /* sum_stim_truncation T (<= 32) */
    int32_t n_params;    /* Hmed pulse-intensity parameters (0: no sliding-window constraints) */
    int32_t layout;      /* CFX_LAYOUT_AOS | CFX_LAYOUT_SOA | CFX_LAYOUT_TILED64 */
    int64_t batch;       /* B >= 1 */
    double final_time;
    /* stim table, row k = the last T stim times <= k*final_time/N (history placeholders -1e7):
       numerical_data_timeseries of ding2003.py:399-429, row-major [(N+1) * T] */
    const double *stim_rows;
    const int32_t *last_stim_idx; /* [N] index of the last parameter in node k's window (Hmed) */
    double intensity_floor;       /* sliding-window left padding (min_pulse_intensity) */
    cfx_constants constants;
    int32_t n_objectives;
    const cfx_objective *objectives;
    int32_t device; /* HIP device ordinal */
} cfx_problem;

typedef struct cfx_handle cfx_handle;

/* Problem sizes: decision variables, constraints, J_g non-zeros, Hessian (lower triangle) non-zeros,
   per instance. */
typedef struct cfx_sizes {
    int64_t nv, ng, nnz_jac, nnz_hess;
    int32_t nx, nu;
} cfx_sizes;

/* ---- lifetime ------------------------------------------------------------------------------------ */
/* Ipopt: get_nlp_info (sizes fixed at creation) */
int cfx_create(const cfx_problem *problem, cfx_handle **out);
void cfx_destroy(cfx_handle *h);
int cfx_get_sizes(const cfx_handle *h, cfx_sizes *out);
/* Launch stream for CFX_DEVICE calls, used as given (NULL = the HIP null stream).  A new handle uses a
   non-blocking stream of its own until this is called. */
int cfx_set_stream(cfx_handle *h, void *hip_stream);
int cfx_synchronize(cfx_handle *h);
const char *cfx_last_error(const cfx_handle *h); /* h == NULL: last handle-free failure (cfx_create,
                                                     cfx_band_lu*) of this thread */
int cfx_abi_version(void);
int cfx_device_count(void);

/* Launch shape of the handle's g + J_g kernels, fixed at creation from the batch size (tuning; the environment
   variables CFX_KPT, CFX_IFAST, CFX_NI and CFX_MSK_KPB, read by cfx_create / cfx_msk_create, override it).  Every
   shape gives the same bits; the parity tests pin that at the shapes the benchmark times. */
typedef struct cfx_launch_shape {
    int32_t intervals_per_thread;    /* shooting: consecutive intervals one thread integrates, x_{k+1} carried */
    int32_t intervals_fast;          /* shooting: interval chunks on grid.x, instance blocks on grid.y */
    int32_t instances_per_lane;      /* shooting g + J_g: adjacent instances per lane (16-byte accesses) */
    int32_t instances_per_lane_g;    /* shooting g only */
    int32_t msk_intervals_per_block; /* musculoskeletal tangent kernel: intervals per block (LDS double buffer) */
} cfx_launch_shape;
int cfx_get_launch_shape(const cfx_handle *h, cfx_launch_shape *out);

/* ---- sparsity (Ipopt eval_jac_g / eval_h with values == NULL) ---------------------------------- */
int cfx_jac_structure(const cfx_handle *h, int32_t *row, int32_t *col);  /* nnz_jac entries */
int cfx_hess_structure(const cfx_handle *h, int32_t *row, int32_t *col); /* nnz_hess, row >= col */
/* mask[nnz_jac] = 1 for the J_g values that depend on neither the instance nor the point (the -1 on x_{k+1} of every
   continuity row; for the Ding families also dCn+/dCn0, the calcium state being affine in its start value), i.e. the
   values CFX_KEEP_CONSTANT_JAC leaves in place (cfg 2: 60 of 100 per instance).  Collocation: the basis coefficients
   C[i][j] off the point's own state, the whole calcium row (linear in cn), every continuity value D[i] and -1 (cfg 2
   at degree 4: 48 of 56 per interval). */
int cfx_jac_constant_mask(const cfx_handle *h, uint8_t *mask);

/* ---- NLP callbacks over the whole batch -------------------------------------------------------- */
int cfx_eval_g(cfx_handle *h, const double *v, double *g, uint32_t flags);         /* eval_g */
int cfx_eval_jac_g(cfx_handle *h, const double *v, double *jac, uint32_t flags);   /* eval_jac_g values */
int cfx_eval_f(cfx_handle *h, const double *v, double *f, uint32_t flags);         /* eval_f, f[B] */
int cfx_eval_grad_f(cfx_handle *h, const double *v, double *grad, uint32_t flags); /* eval_grad_f */
/* eval_h: values of obj_factor[b]*Hess(f) + sum_i lambda[b,i]*Hess(g_i), lower triangle */
int cfx_eval_h(cfx_handle *h, const double *v, const double *obj_factor, const double *lambda, double *hess,
               uint32_t flags);
/* fused g + J_g (+ f, grad f when non-NULL) in one pass over the decision vectors */
int cfx_eval_all(cfx_handle *h, const double *v, double *g, double *jac, double *f, double *grad,
                 uint32_t flags);
/* g + J_g + eval_h (+ f, grad f when non-NULL) at one point: Ipopt's eval_g / eval_jac_g / eval_h of an
   accepted iterate (IpoptAlgorithm's new point, then the Hessian with the new multipliers).  On the shooting
   transcriptions ONE launch integrates every interval on second-order jets and writes the three outputs; on the
   collocation transcription ONE launch writes every interval's defects, continuity rows, J_g values and Hessian
   blocks (g and J_g bit-identical to eval_all); the musculoskeletal problems run eval_all then eval_h.  g, jac,
   hess must be non-NULL. */
int cfx_eval_all_h(cfx_handle *h, const double *v, const double *obj_factor, const double *lambda, double *g,
                   double *jac, double *f, double *grad, double *hess, uint32_t flags);

/* ---- IvpFes.integrate: single shooting from x0 (NULL: rest state) with per-interval controls
   u [N*nu per instance], writing every sub-step state: traj [(N*n_steps+1)*nx per instance]. ---- */
int cfx_integrate(cfx_handle *h, const double *x0, const double *u, double *traj, uint32_t flags);

/* ---- musculoskeletal problems (FesMskModel + OcpFesMsk) --------------------------------------------
   Replaces the bioptim dynamics plugin FesMskModel registers (cocofest/models/dynamical_model.py:133-203,
   406-451: every muscle's FES ODE scaled by the De Groote force-length / force-velocity / passive-force
   coefficients of hill_coefficients.py:11-126, joint torque -J_L(q)^T F, biorbd forward dynamics) and the NLP
   callbacks of the OCP built by OcpFesMsk.prepare_ocp (cocofest/optimization/fes_ocp_dynamics.py:158-251).
   The skeleton is a serial chain of revolute dofs (the host reduces a bioMod: constant segment transforms
   between dofs are composed, the segments moving with a dof are merged into one composite body).
   Per node the states are [muscle 0 (Cn, F[, A, Tau1, Km]), muscle 1, ..., q (n_dof), qdot (n_dof)]; the
   controls [last_pulse_width of every muscle (Ding2007 families)] then [tau (n_dof)] with
   CFX_MSK_RESIDUAL_TORQUE; the decision vector, constraint rows and layouts are those of cfx_problem's
   shooting transcription (CFX_RK1/2/4, CFX_LAYOUT_AOS or CFX_LAYOUT_SOA).  The handle works with every
   cfx_* call above (sizes, structures, eval_*, eval_h, integrate, destroy). */
#define CFX_MSK_MAX_DOF 4
#define CFX_MSK_MAX_MUSCLES 8
#define CFX_MSK_MAX_POINTS 16
#define CFX_MSK_FORCE_LENGTH 1u   /* hill_coefficients.py:11-63 (the reference gates it with the FV flag) */
#define CFX_MSK_FORCE_VELOCITY 2u /* hill_coefficients.py:66-96 */
#define CFX_MSK_PASSIVE_FORCE 4u  /* hill_coefficients.py:99-126 */
#define CFX_MSK_RESIDUAL_TORQUE 8u
/* Ding2007 muscles: consecutive intervals that follow the same pulse share their pulse widths — rows
   u_k[m] - u_{k-1}[m] = 0 after the marker rows (the decision space of the per-pulse pulse-duration parameters of the
   revision that stored examples/dynamics/reaching_task/result_file pickles, with band-local rows) */
#define CFX_MSK_PULSE_WIDTH_PER_PULSE 16u
/* Ding muscles: that revision's calcium sum — a window's first pulse left out once it holds several, and the fatigue
   models' r0 = Km + r0_km_relationship read from the Km state (today: km_rest + r0_km_relationship, ding2003.py:230-252;
   tests/test_reference_solution.py measures both) */
#define CFX_MSK_LEGACY_CALCIUM 32u
/* objective kind for MSK problems: weight * (target_value / z_k)^2 at the nodes of the range
   (CustomObjective.minimize_overall_muscle_fatigue, cocofest/custom_objectives.py:80-101: a_rest / A) */
#define CFX_OBJ_MAYER_INV 2

typedef struct cfx_msk_muscle {
    int32_t model; /* CFX_DING2003 .. CFX_HMED2018_FATIGUE; all muscles of a problem share the model family */
    cfx_constants constants;
    int32_t n_points;           /* origin, via points, insertion (<= CFX_MSK_MAX_POINTS) */
    const int32_t *point_frame; /* [n_points] dof frame the point is fixed in (moves with q_0..q_j), -1: ground */
    const double *point_pos;    /* [n_points * 3] position in that frame */
    double optimal_length, tendon_slack_length, pennation_angle;
} cfx_msk_muscle;

/* A marker superimposition (bioptim ConstraintFcn.SUPERIMPOSE_MARKERS as OcpFesMsk passes msk_info
   ["custom_constraint"] through, cocofest/optimization/fes_ocp_dynamics.py:424-450; used by
   examples/dynamics/reaching_task/ examples): at node `node`, for each selected world axis, one equality row
   marker(second) - marker(first) = 0 over q_node (bioptim's superimpose_markers penalty).  A marker is a point
   fixed in a dof frame (-1: ground), as the muscle path points. */
typedef struct cfx_msk_marker_pair {
    int32_t node;     /* 0 .. n_shooting */
    int32_t axes;     /* bit a set: a row for world axis a (X = 1, Y = 2, Z = 4), rows in axis order */
    int32_t frame[2]; /* dof frame of the first / second marker (-1: ground) */
    double pos[2][3]; /* their positions in those frames */
} cfx_msk_marker_pair;

typedef struct cfx_msk_problem {
    int32_t abi_version; /* CFX_ABI_VERSION */
    int32_t scheme;      /* CFX_RK1 | CFX_RK2 | CFX_RK4 */
    int32_t n_steps;
    int32_t n_shooting;
    int32_t truncation;
    int32_t layout; /* CFX_LAYOUT_AOS | CFX_LAYOUT_SOA */
    int64_t batch;
    double final_time;
    const double *stim_rows; /* [(N+1) * T], shared by every muscle (fes_ocp_dynamics.py:86-90) */
    int32_t n_dof;
    const int32_t *dof_axis;  /* [n_dof] 0 / 1 / 2: rotation about x / y / z of the dof's joint frame */
    const double *dof_frame;  /* [n_dof * 12] joint frame j relative to frame j-1 (ground for j = 0): row-major
                                 3x3 rotation, then the translation (in frame j-1) */
    double gravity[3];
    const double *body_mass;    /* [n_dof] composite body moving with frame j */
    const double *body_com;     /* [n_dof * 3] its centre of mass, frame j */
    const double *body_inertia; /* [n_dof * 9] its inertia about the com, frame j axes, row-major */
    int32_t n_muscles;
    const cfx_msk_muscle *muscles;
    uint32_t flags; /* CFX_MSK_* */
    int32_t n_objectives;
    const cfx_objective *objectives; /* var_index over the state / control layout above */
    int32_t device;
    /* Hmed2018 muscles (truncation <= 20): the controls of a node are T pulse intensities per muscle (then the
       residual torques), as OcpFesMsk configures them (dynamical_model.py:437-440).  n_params > 0: the pulse
       intensities are trailing parameters of the decision vector and each interval k gets n_muscles * T rows
       u_k[m T + s] - p[param_offset[m] + last_stim_idx[k] - T + 1 + s] (I_min where that index is negative),
       after its continuity rows (CustomConstraint.pulse_intensity_sliding_window_constraint,
       custom_constraints.py:102-119; fes_ocp_dynamics.py:413-438) */
    int32_t n_params;
    const int32_t *last_stim_idx; /* [n_shooting] parameter index of the last pulse <= t_k (muscle-relative) */
    const int32_t *param_offset;  /* [n_muscles] first parameter of each muscle's intensities (equal: shared) */
    /* marker superimpositions: their rows follow every interval's rows (in pair order, axes ascending); J_g
       entries on q_node of the dofs that move either marker; the Hessian gains the (q_node, q_node) pairs */
    int32_t n_marker_pairs;
    const cfx_msk_marker_pair *marker_pairs;
} cfx_msk_problem;

int cfx_msk_create(const cfx_msk_problem *problem, cfx_handle **out);

/* ---- Newton / KKT linear algebra of the batched interior-point driver ----------------------------
   Replaces the sparse symmetric-indefinite factorisation Ipopt runs every iteration on the KKT matrix
   (MUMPS by default; `Solver.IPOPT` as built at cocofest/optimization/fes_ocp.py:171-190 and
   cocofest/examples, bioptim's linear_solver option).  B independent n x n banded systems, LAPACK
   dgbtrf/dgbtrs semantics (partial pivoting), device pointers, instance-major:
     ab   [B][n][2 kl + ku + 1]  column j of instance b at ab + (b n + j)(2 kl + ku + 1); A(i, j) at row
                                 kl + ku + i - j; rows < kl are fill-in (zeroed by cfx_band_lu)
     ipiv [B][n]  0-based pivot rows;   info [B]  0 or j + 1 for the first zero pivot;   rhs [B][nrhs][n]
   cfx_band_lu factors in place and, when nrhs > 0, solves; cfx_band_lu_solve re-uses the factors.
   Launched on `hip_stream` (NULL = the HIP null stream); errors via cfx_last_error(NULL). */
int cfx_band_lu(int64_t n, int32_t kl, int32_t ku, int64_t batch, double *ab, int32_t *ipiv, int32_t *info,
                int32_t nrhs, double *rhs, void *hip_stream);
int cfx_band_lu_solve(int64_t n, int32_t kl, int32_t ku, int64_t batch, const double *ab, const int32_t *ipiv,
                      int32_t nrhs, double *rhs, void *hip_stream);

/* ---- block-tridiagonal (stage chain) systems: block cyclic reduction ----------------------------------------
   The interior point's KKT matrix of ONE large OCP grouped by stage (cfx_ipm: the free variables of node k and the
   constraint rows arriving at it) is block tridiagonal; its sequential band factorisation (above) leaves the chip
   idle, so cfx_ipm factors it by block cyclic reduction instead (MUMPS' role in Ipopt for
   reaching_task_pulse_duration_optimization.py:117 of the reference).  B independent systems of M diagonal blocks,
   sp x sp each (sp a multiple of 16, <= 128), row-major, device pointers:
     D [B][M][sp][sp] diagonal blocks, L [B][M][sp][sp] blocks (k, k-1) (L[.][0] unused), U [B][M][sp][sp] blocks
     (k, k+1) (U[.][M-1] unused), work [2][B][M][sp][sp];  info [B]: 0, or the 1-based unknown of a zero pivot
   cfx_btri_factor overwrites D / L / U and fills work with the factors (no pivoting across blocks: each pivot block is inverted with
   partial pivoting, so the systems must have nonsingular pivot blocks, as the KKT matrices cfx_ipm groups do);
   cfx_btri_solve solves rhs [B][nrhs][M sp] in place (scratch: same shape).  On `hip_stream`. */
int cfx_btri_factor(int64_t batch, int32_t M, int32_t sp, double *D, double *L, double *U, double *work,
                    int32_t *info, void *hip_stream);
int cfx_btri_solve(int64_t batch, int32_t M, int32_t sp, const double *D, const double *L, const double *U,
                   const double *work, int32_t nrhs, double *rhs, double *scratch, void *hip_stream);
/* (ABI 10) the inertia of a SYMMETRIC system factored by cfx_btri_factor: neg [B] receives its number of negative
   eigenvalues (each pivot block counted by a Bunch-Kaufman LDL^T of its inverse; block cyclic reduction is a sequence
   of congruences, so the counts add up to the matrix's), plus 1 << 20 per zero pivot.  The count MUMPS reports to
   Ipopt for its inertia correction (IpPDPerturbationHandler). */
int cfx_btri_inertia(int64_t batch, int32_t M, int32_t sp, const double *D, int32_t *neg, void *hip_stream);

/* ---- batched interior-point solver ---------------------------------------------------------------
   Replaces the solver role of `ocp.solve(Solver.IPOPT(...))` (bioptim's Ipopt interface; called e.g. at
   examples/getting_started/frequency_optimization.py:22 and examples/getting_started/pulse_duration_optimization.py:41
   with `_max_iter` / `_tol`): Ipopt's primal-dual barrier method (monotone Fiacco-McCormick mu update, filter line
   search with second-order corrections, inertia correction by a curvature test, gradient-based problem scaling,
   least-squares multiplier initialisation, a feasibility-restoration step) for the B instances of one handle in
   lockstep.  Every iteration stays on the handle's GPU: the callbacks above, fused vector kernels for the barrier
   algebra, the KKT matrix assembled in band storage (unknowns ordered stage by stage) and factored by the batched
   band LU below; the host only reads a few counters per iteration (all done? wrong inertia? every trial point
   accepted?).  The handle must use CFX_LAYOUT_AOS (or have batch 1).  Fixed variables (lb == ub) are removed. */
typedef struct cfx_ipm_options {
    double tol;                /* Ipopt tol on the scaled KKT error (default 1e-6) */
    int32_t max_iter;          /* default 200 */
    double acceptable_tol;     /* acceptable level (1e-6) held for acceptable_iter (15) iterations */
    int32_t acceptable_iter;
    double mu_init;            /* 0.1 */
    double bound_relax_factor; /* 0 (off) */
    double bound_push;         /* 1e-2 */
    double tau_min;            /* 0.99 */
    double kappa_eps, kappa_mu, theta_mu; /* 10, 0.2, 1.5 */
    double s_max;              /* 100 */
    double armijo;             /* 1e-4 */
    int32_t max_backtrack;     /* 30 */
    double delta_c;            /* 1e-9 */
    double curv_min;           /* 1e-8: dx^T (W + Sigma + dw) dx >= curv_min |dx|^2 */
    int32_t max_soc;           /* 4 */
    double kappa_soc;          /* 0.99 */
    /* Ipopt's watchdog: after this many consecutive shortened line searches (10; 0: off) full steps are taken for
       up to watchdog_trial_iter_max (3) iterations, judged against the iterate where it started; none acceptable:
       back there, backtracking from half the step */
    int32_t watchdog_shortened_iter_trigger;
    int32_t watchdog_trial_iter_max;
    /* Ipopt's hessian_approximation: CFX_HESSIAN_EXACT (the callbacks' eval_h) or CFX_HESSIAN_LIMITED_MEMORY (no
       eval_h: an L-BFGS approximation of the Lagrangian Hessian from the last limited_memory_max_history (6, at
       most 64) steps, compact form sigma I - low rank, sigma = s^T y / s^T s; the low-rank part enters every Newton
       solve through the Sherman-Morrison-Woodbury identity on the band factors) */
    int32_t hessian_approximation;
    int32_t limited_memory_max_history;
    /* What a failed line search starts (for the instances whose search failed):
       CFX_RESTORATION_PHASE (default) — Ipopt's feasibility-restoration phase, an NLP of its own over the constraint
       violation, min rho sum(p + n) + zeta/2 |D_R (x - x_r)|^2 s.t. c(x) - p + n = 0, p, n >= 0 and the bounds,
       solved by the same interior point (own barrier mu_R = max(mu, |c|_inf), filter and line search; p, n and their
       multipliers eliminated, so its KKT matrix has the original band structure) until a point is acceptable to the
       original filter with |c|_1 <= required_infeasibility_reduction times the value where it started (the bound
       multipliers then take a Newton step for complementarity over the phase's dx, the constraint multipliers restart
       from zero, the filter from empty; the phase's iterations count among the instance's max_iter).  A failed line
       search of the phase resets p and n to their closed form at the phase's point (Ipopt's RestoRestorationPhase);
       a second one in a row, max_resto_iter iterations of it, or a point of local infeasibility stop that instance
       (status CFX_IPM_RESTORATION_FAILED / CFX_IPM_INFEASIBLE_PROBLEM_DETECTED), as Ipopt's solve stops.  The phase's
       iterations run inside the same host iterations as the other instances' main iterations (one host iteration
       advances every instance by one iteration of its own).  CFX_RESTORATION_STEP — one minimum-norm step on c = 0
       in the Sigma + I metric, backtracked until |c|_1 decreases, then least-squares multipliers. */
    int32_t restoration;
    int32_t max_resto_iter;                  /* 200 */
    double resto_penalty;                    /* rho, Ipopt resto_penalty_parameter: 1000 */
    double required_infeasibility_reduction; /* 0.9 */
    /* Ipopt's filter reset heuristic (IpFilterLSAcceptor): when in filter_reset_trigger (5) successive iterations the
       line search's last rejected trial point was rejected by the filter (it passed the Armijo / sufficient-decrease
       test), the filter is cleared — at most max_filter_resets times per solve (Ipopt's default 5; default here 0:
       off) */
    int32_t filter_reset_trigger; /* >= 1 */
    int32_t max_filter_resets;    /* >= 0 */
    /* Ipopt's max_wall_time (seconds, default 1e20): the instances still iterating when it is exceeded stop there
       (status CFX_IPM_MAXIMUM_WALLTIME_EXCEEDED) */
    double max_wall_time;
    /* Ipopt's print_frequency_time (seconds, default 0: off): one progress line on stderr at most this often —
       host iteration, elapsed time, instances still iterating, of them in the restoration phase */
    double print_frequency_time;
    /* Ipopt's soft restoration (IpBacktrackingLineSearch::TrySoftRestoStep; restoration phase only): a failed line
       search first tries the step at the smaller of the primal and dual fractions to the boundary, primal and dual
       together; it is taken when the original filter accepts it (sufficient-decrease test) or when it cuts the
       primal-dual system error (mean of |grad L|, |c| and |s z - mu| over the scaled problem) by
       soft_resto_pderror_reduction_factor (Ipopt's default 0.9999; default here 0: off).  A step the filter did not
       accept keeps the instance on such steps, without line search, for up to max_soft_resto_iters (10) iterations
       until one is accepted by the filter; a rejected one starts the restoration phase.  Each try costs one eval_all
       at the trial point. */
    double soft_resto_pderror_reduction_factor; /* >= 0 */
    int32_t max_soft_resto_iters;               /* >= 0 */
    /* extension, not Ipopt (default 0): a failed restoration phase (its line search failed twice in a row, or
       max_resto_iter) restarts the main iteration from the phase's last point — zero constraint multipliers, an
       empty filter — instead of stopping the instance with CFX_IPM_RESTORATION_FAILED */
    int32_t resto_failure_restart;
    /* Ipopt's termination tests on the UNSCALED problem, beside tol on the scaled error (ABI 8): converged needs
       max|g| <= constr_viol_tol (1e-4), max|grad L| <= dual_inf_tol (1), max|s z| <= compl_inf_tol (1e-4); the
       acceptable level (acceptable_tol for acceptable_iter iterations, and a restoration phase called at an acceptable
       point) needs the acceptable_* ones (0.01, 1e10, 0.01) */
    double constr_viol_tol, dual_inf_tol, compl_inf_tol;
    double acceptable_constr_viol_tol, acceptable_dual_inf_tol, acceptable_compl_inf_tol;
    /* Ipopt's warm start (ABI 9): with warm_start_init_point (default 0) the solve starts from the multipliers given
       by cfx_ipm_set_warm_start instead of least-squares multipliers and z = mu / s: x is pushed from its bounds by
       warm_start_bound_push max(1, |bound|) capped at warm_start_bound_frac of the range (1e-3, 1e-3), the bound
       multipliers are raised to at least warm_start_mult_bound_push (1e-3; scaled problem), the barrier starts at
       mu_init */
    double warm_start_bound_push, warm_start_bound_frac, warm_start_mult_bound_push;
    int32_t warm_start_init_point;
    /* Ipopt's honor_original_bounds (ABI 9; default 0, Ipopt 3.14's): 1 moves the returned point into the original
       bounds when bound_relax_factor relaxed them; 0 returns the iterate as it is (within the relaxed bounds) */
    int32_t honor_original_bounds;
    /* variable scaling by the bound range (ABI 9; default 1, an extension): variables whose range ub - lb is below 1
       (pulse widths ~1e-4 s) are iterated as x / (ub - lb).  0: no variable scaling — Ipopt's behaviour (its
       gradient-based nlp scaling scales f and g only), which changes the scaled termination test */
    int32_t range_scaling;
    /* Ipopt's bound_mult_init_method (ABI 9): 0 "constant" (Ipopt's default: z = bound_mult_init_val, 1), 1
       "mu-based" (z = mu_init / slack; this library's default) */
    int32_t bound_mult_init_method;
    double bound_mult_init_val;
    /* inertia correction (ABI 10): 0 (default) the curvature test (dx^T (W + Sigma + dw) dx >= curv_min |dx|^2); 1
       Ipopt's test on the KKT matrix's inertia — the factorisation must have exactly m negative eigenvalues (m
       constraints), else dw grows — counted for the stage-chain layout (cfx_btri_inertia's count on the chain plus a
       Bunch-Kaufman LDL^T of the border's Schur complement; other layouts keep the curvature test) */
    int32_t inertia_test;
    /* Ipopt's barrier-parameter strategy (ABI 11).  mu_strategy CFX_MU_MONOTONE (default): Fiacco-McCormick, mu
       decreased while the barrier problem's scaled error is below kappa_eps mu.  CFX_MU_ADAPTIVE (bioptim's
       Solver.IPOPT setting): Ipopt's free-mu mode — each iteration the KKT matrix is factored once and solved for the
       affine (mu = 0) and unit-centering right-hand sides; mu = sigma * (average complementarity) with sigma minimising
       Ipopt's quality function (predicted 2-norm-squared dual / primal infeasibility and complementarity after the step,
       golden section over log sigma within [sigma_min, sigma_max] and [mu_min, mu_max], at most
       quality_function_max_section_steps sections); the Newton step is the solutions' combination.  Globalisation
       (adaptive_mu_globalization): CFX_MU_GLOBAL_OBJ_CONSTR_FILTER — an iterate not acceptable to a filter of the
       (f, ||c||_1) of accepted iterates (margin filter_margin_fact min(filter_max_margin, ||c||_1)) switches to the
       monotone mode at mu = adaptive_mu_monotone_init_factor * average complementarity, an acceptable one returns to the
       free mode; CFX_MU_GLOBAL_NEVER_MONOTONE — always free.  mu_max <= 0: mu_max_fact times the first iterate's
       average complementarity. */
    int32_t mu_strategy;
    int32_t adaptive_mu_globalization;
    double mu_max_fact, mu_max, mu_min, adaptive_mu_monotone_init_factor;
    double sigma_max, sigma_min, quality_function_section_sigma_tol, quality_function_section_qf_tol;
    int32_t quality_function_max_section_steps;
    /* Ipopt resets the line search's filter whenever mu changes (ABI 11; the adaptive strategy always does, the
       monotone strategy when this is 1; default 0) */
    int32_t mu_change_resets_filter;
    double filter_margin_fact, filter_max_margin;
    /* floor of the monotone mu: 0 (default) tol / 10; 1 Ipopt's min(tol, compl_inf_tol) / (kappa_eps + 1) */
    int32_t monotone_mu_floor;
    /* Ipopt's nlp_scaling_method (ABI 11): 1 gradient-based (default: f and each row of g scaled at the starting point
       by min(1, nlp_scaling_max_gradient / max |gradient|), at least nlp_scaling_min_value), 0 none */
    int32_t nlp_scaling_method;
    double nlp_scaling_max_gradient, nlp_scaling_min_value;
    /* cold-start push from the bounds: min(bound_push max(1, |bound|), bound_frac (ub - lb)); Ipopt's bound_frac is
       0.01, this library's default 0.5 (ABI 11) */
    double bound_frac;
} cfx_ipm_options;
#define CFX_HESSIAN_EXACT 0
#define CFX_HESSIAN_LIMITED_MEMORY 1
#define CFX_RESTORATION_STEP 0
#define CFX_RESTORATION_PHASE 1
#define CFX_MU_MONOTONE 0
#define CFX_MU_ADAPTIVE 1
#define CFX_MU_GLOBAL_OBJ_CONSTR_FILTER 0
#define CFX_MU_GLOBAL_NEVER_MONOTONE 1

/* per-instance outcome of a solve (cfx_ipm_get_status), Ipopt's ApplicationReturnStatus values */
#define CFX_IPM_SOLVE_SUCCEEDED 0
#define CFX_IPM_SOLVED_TO_ACCEPTABLE_LEVEL 1
#define CFX_IPM_INFEASIBLE_PROBLEM_DETECTED 2 /* the restoration phase converged to a point of local infeasibility */
#define CFX_IPM_MAXIMUM_ITERATIONS_EXCEEDED (-1)
#define CFX_IPM_RESTORATION_FAILED (-2)
#define CFX_IPM_MAXIMUM_WALLTIME_EXCEEDED (-5)

typedef struct cfx_ipm_stats {
    int64_t eval_all, eval_g_f, eval_h, kkt_factor, iterations, host_syncs;
    double wall_s; /* last cfx_ipm_solve */
    /* KKT layout: unknowns, the band's half-bandwidths and unknowns, free parameters in a dense border (Schur
       complement; 0: one band) */
    int64_t kkt_n, kkt_kl, kkt_ku, kkt_band_n, kkt_border;
    int64_t kkt_blocks; /* band blocks factored side by side (nested dissection of the stage chain; 1: none) */
    int64_t resto_phases, resto_iterations; /* restoration phases entered / their iterations, summed over the instances */
    int64_t soft_steps;                     /* soft-restoration steps taken, summed over the instances */
    /* stage-chain KKT layout (ABI 9; cfx_btri_*): nodes and their padded size (0: a band layout above) */
    int64_t kkt_chain_nodes, kkt_chain_sp;
    /* (ABI 11) adaptive mu strategy: switches from its free mode to its monotone mode, summed over the instances */
    int64_t mu_mode_switches;
} cfx_ipm_stats;

typedef struct cfx_ipm cfx_ipm;

void cfx_ipm_default_options(cfx_ipm_options *opt);
/* lb, ub: [nv] host arrays (+-inf allowed); n_params: trailing parameters of the decision vector (Hmed) */
int cfx_ipm_create(cfx_handle *h, const double *lb, const double *ub, int32_t n_params, const cfx_ipm_options *opt,
                   cfx_ipm **out);
/* v0 [B][nv] starting points; fixed_values [B][n_fixed] values of the fixed variables in index order (NULL: their
   bound); outputs (any may be NULL): v [B][nv], y [B][ng] multipliers of the unscaled problem, f [B],
   converged [B], iterations [B], kkt_error [B] (scaled).  CFX_DEVICE: every pointer is a device pointer and the
   outputs are written asynchronously on the handle's stream; otherwise host pointers. */
int cfx_ipm_solve(cfx_ipm *s, const double *v0, const double *fixed_values, double *v, double *y, double *f,
                  int32_t *converged, int32_t *iterations, double *kkt_error, uint32_t flags);
/* Ipopt's warm_start_init_point inputs (ABI 9) for the following cfx_ipm_solve calls with the option set: y [B][ng]
   constraint multipliers and z_l, z_u [B][nv] bound multipliers of the UNSCALED problem, Ipopt's sign convention
   (grad f + J^T y - z_l + z_u = 0, z >= 0; entries of fixed variables and of missing bounds are ignored).  Host
   pointers, or device pointers with CFX_DEVICE; copied.  cfx_ipm_get_bound_multipliers returns the last solve's
   z_l, z_u [B][nv] in that form (0 at fixed variables). */
int cfx_ipm_set_warm_start(cfx_ipm *s, const double *y, const double *z_l, const double *z_u, uint32_t flags);
int cfx_ipm_get_bound_multipliers(cfx_ipm *s, double *z_l, double *z_u, uint32_t flags);
/* The same solver over callbacks the caller provides instead of a libcfx handle — e.g. one OCP's intervals sharded
   over several GPUs, each rank evaluating its slice and all-gathering the value slices (cocofest_amd/distributed.py,
   the interval sharding of SURVEY.md section 8(e)).  The NLP is described by its sizes and fixed triplet structures
   (J_g: ng x nv; Hessian: lower triangle, row >= col); the evaluator's functions are called synchronously from
   cfx_ipm_solve's host thread with device pointers (AoS [batch][len]) that the solver's kernels on `hip_stream` wrote
   or read: the evaluator must order its own work after the work queued on that stream, and have finished writing its
   outputs when it returns (a callback on the same stream satisfies both).  Any output pointer may be NULL (not
   wanted).  A non-zero return aborts the solve with CFX_ECALLBACK. */
typedef struct cfx_evaluator {
    void *ctx;
    int (*eval_all)(void *ctx, const double *v, double *g, double *jac, double *f, double *grad);
    int (*eval_h)(void *ctx, const double *v, const double *obj_factor, const double *lambda, double *hess);
} cfx_evaluator;
typedef struct cfx_nlp_desc {
    int64_t batch, nv, ng, nnz_jac, nnz_hess;
    const int32_t *jac_row, *jac_col, *hess_row, *hess_col; /* host arrays, copied */
    int32_t device;
    void *hip_stream;
} cfx_nlp_desc;
int cfx_ipm_create_ext(const cfx_nlp_desc *nlp, const cfx_evaluator *ev, const double *lb, const double *ub,
                       int32_t n_params, const cfx_ipm_options *opt, cfx_ipm **out);
int cfx_ipm_get_stats(const cfx_ipm *s, cfx_ipm_stats *out);
/* status [B] (host): CFX_IPM_* outcome of every instance of the last cfx_ipm_solve */
int cfx_ipm_get_status(const cfx_ipm *s, int32_t *status);
int cfx_ipm_n_fixed(const cfx_ipm *s);
const char *cfx_ipm_last_error(const cfx_ipm *s);
void cfx_ipm_destroy(cfx_ipm *s);

/* ---- placing gathered value slices --------------------------------------------------------------------
   dst[b][i] = sum over s in [ptr[i], ptr[i+1]) of src[b][idx[s]] for the batch-major (AoS) src [batch][src_len] and
   dst [batch][n_dst] on `hip_stream` (device pointers; ptr / idx device int32 arrays): the fixed gather table that
   places every rank's all-gathered value slices of an interval-sharded OCP into the full g / J_g / grad f / Hessian
   arrays, summing the entries several slices contribute (halo nodes, parameters) in a fixed order (no atomics). */
int cfx_gather_sum(int64_t batch, int64_t n_dst, const int32_t *ptr, const int32_t *idx, const double *src,
                   int64_t src_len, double *dst, void *hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* CFX_H */
