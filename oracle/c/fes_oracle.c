/*
 * fes_oracle.c — plain-C restatement of the reference's NLP-callback path, AS WRITTEN.
 *
 * TEST INFRASTRUCTURE ONLY: the CPU baseline of bench.py ("kind": "port") and a second checker for the
 * tests.  Nothing in the product links or loads it.
 *
 * It evaluates, per instance, exactly what the reference's CasADi function does for every RK stage: the
 * calcium sum of cocofest/models/ding2003.py:230-252 with its 2T-1 exponentials (r_i from the
 * stimulation spacing, exp(-(t - t_i)/tauc) decay; lambda_i of hmed2018.py:169-180 for Hmed), then the
 * ODE right-hand side (ding2003.py:254-311, ding2003_with_fatigue.py:197-240, ding2007.py:172-188) and the
 * bioptim RK1/RK2/RK4 sub-stepping, with forward-mode derivatives (dual numbers, nz directions) for the
 * continuity Jacobian block.  Layout and ordering follow include/cfx.h (AoS: v[b*nv + e]).
 * OpenMP over instances.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define NZMAX 40

typedef struct {
    double v;
    double d[NZMAX];
} dual;

typedef struct {
    int nz;
} ctx;

static inline dual dc(const ctx *c, double v) {
    dual r;
    r.v = v;
    memset(r.d, 0, sizeof(double) * c->nz);
    return r;
}
static inline dual dadd(const ctx *c, dual a, dual b) {
    a.v += b.v;
    for (int i = 0; i < c->nz; ++i) a.d[i] += b.d[i];
    return a;
}
static inline dual dsub(const ctx *c, dual a, dual b) {
    a.v -= b.v;
    for (int i = 0; i < c->nz; ++i) a.d[i] -= b.d[i];
    return a;
}
static inline dual dscale(const ctx *c, double s, dual a) {
    a.v *= s;
    for (int i = 0; i < c->nz; ++i) a.d[i] *= s;
    return a;
}
static inline dual dmul(const ctx *c, dual a, dual b) {
    dual r;
    r.v = a.v * b.v;
    for (int i = 0; i < c->nz; ++i) r.d[i] = a.v * b.d[i] + b.v * a.d[i];
    return r;
}
static inline dual ddiv(const ctx *c, dual a, dual b) {
    dual r;
    r.v = a.v / b.v;
    for (int i = 0; i < c->nz; ++i) r.d[i] = (a.d[i] - r.v * b.d[i]) / b.v;
    return r;
}
static inline dual dexp(const ctx *c, dual a) {
    dual r;
    r.v = exp(a.v);
    for (int i = 0; i < c->nz; ++i) r.d[i] = r.v * a.d[i];
    return r;
}
static inline dual dtanh(const ctx *c, dual a) {
    dual r;
    r.v = tanh(a.v);
    for (int i = 0; i < c->nz; ++i) r.d[i] = (1.0 - r.v * r.v) * a.d[i];
    return r;
}

/* constants in cfx_constants order */
enum { TAUC, R0KM, A_REST, TAU1_REST, TAU2, KM_REST, A_SCALE, PD0, PDT, AR, BS, IS, CR, ALPHA_A, ALPHA_TAU1,
       ALPHA_KM, TAU_FAT, FL, FV, FP };

typedef struct {
    int model, nx, nu, T;
    const double *k;    /* constants */
    const double *row;  /* T stim times of the interval's node */
    const dual *lam;    /* Hmed lambda_i (T) */
    dual afac;          /* Ding2007 a_calculation */
} rhs_in;

/* cn_sum_fun as written (ding2003.py:230-252), lambda_i = 1 unless Hmed */
static dual cn_sum(const ctx *c, const rhs_in *in, double t) {
    const double tauc = in->k[TAUC];
    const double r0 = in->k[KM_REST] + in->k[R0KM];
    dual s = dc(c, 0.0);
    for (int i = 0; i < in->T; ++i) {
        const double ri = i == 0 ? 1.0 : 1.0 + (r0 - 1.0) * exp(-(in->row[i] - in->row[i - 1]) / tauc);
        const double term = ri * exp(-(t - in->row[i]) / tauc);
        if (in->lam)
            s = dadd(c, s, dscale(c, term, in->lam[i]));
        else
            s.v += term;
    }
    return s;
}

static void rhs(const ctx *c, const rhs_in *in, double t, const dual *x, dual *dx) {
    const double *k = in->k;
    const int fat = in->model & 1, pw = in->model == 2 || in->model == 3;
    const dual cs = cn_sum(c, in, t);
    dx[0] = dsub(c, dscale(c, 1.0 / k[TAUC], cs), dscale(c, 1.0 / k[TAUC], x[0]));
    dual a, tau1, km;
    if (fat) {
        a = x[2];
        tau1 = x[3];
        km = x[4];
    } else {
        a = dc(c, pw ? k[A_SCALE] : k[A_REST]);
        tau1 = dc(c, k[TAU1_REST]);
        km = dc(c, k[KM_REST]);
    }
    if (pw) a = dmul(c, a, in->afac);
    const dual s = ddiv(c, x[0], dadd(c, km, x[0]));
    const dual den = dadd(c, tau1, dscale(c, k[TAU2], s));
    dx[1] = dscale(c, k[FL] * k[FV] + k[FP], dsub(c, dmul(c, a, s), ddiv(c, x[1], den)));
    if (fat) {
        const double arest = pw ? k[A_SCALE] : k[A_REST];
        dx[2] = dadd(c, dscale(c, -1.0 / k[TAU_FAT], dsub(c, x[2], dc(c, arest))), dscale(c, k[ALPHA_A], x[1]));
        dx[3] = dadd(c, dscale(c, -1.0 / k[TAU_FAT], dsub(c, x[3], dc(c, k[TAU1_REST]))),
                     dscale(c, k[ALPHA_TAU1], x[1]));
        dx[4] = dadd(c, dscale(c, -1.0 / k[TAU_FAT], dsub(c, x[4], dc(c, k[KM_REST]))), dscale(c, k[ALPHA_KM], x[1]));
    }
}

static void interval(const ctx *c, const rhs_in *in, int scheme, int m, double t0, double dt, dual *x) {
    const double h = dt / m;
    dual k1[5], k2[5], k3[5], k4[5], xs[5];
    for (int j = 0; j < m; ++j) {
        const double t = t0 + j * h;
        rhs(c, in, t, x, k1);
        if (scheme == 1) {
            for (int r = 0; r < in->nx; ++r) x[r] = dadd(c, x[r], dscale(c, h, k1[r]));
        } else if (scheme == 2) {
            for (int r = 0; r < in->nx; ++r) xs[r] = dadd(c, x[r], dscale(c, h / 2, k1[r]));
            rhs(c, in, t + h / 2, xs, k2);
            for (int r = 0; r < in->nx; ++r) x[r] = dadd(c, x[r], dscale(c, h, k2[r]));
        } else {
            for (int r = 0; r < in->nx; ++r) xs[r] = dadd(c, x[r], dscale(c, h / 2, k1[r]));
            rhs(c, in, t + h / 2, xs, k2);
            for (int r = 0; r < in->nx; ++r) xs[r] = dadd(c, x[r], dscale(c, h / 2, k2[r]));
            rhs(c, in, t + h / 2, xs, k3);
            for (int r = 0; r < in->nx; ++r) xs[r] = dadd(c, x[r], dscale(c, h, k3[r]));
            rhs(c, in, t + h, xs, k4);
            for (int r = 0; r < in->nx; ++r) {
                dual acc = dadd(c, dadd(c, dadd(c, k1[r], dscale(c, 2.0, k2[r])), dscale(c, 2.0, k3[r])), k4[r]);
                x[r] = dadd(c, x[r], dscale(c, h / 6, acc));
            }
        }
    }
}

/*
 * Continuity residuals + Jacobian values (+ Hmed sliding rows) for B instances, AoS, in the include/cfx.h
 * ordering.  jpos[r*nz + c] / jneg[r]: offsets inside an interval block of the structurally non-zero entries
 * and of the -1 (nnzk per interval).  g / jac may be NULL.  Returns 0, or -1 on unsupported sizes.
 */
int oracle_shooting(int model, int scheme, int m, int N, int T, double tf, const double *rows, const double *consts,
                    int n_params, const int32_t *last_idx, double floor_value, int64_t B, const double *v, double *g,
                    double *jac, const int32_t *jpos, const int32_t *jneg, int nnzk, int nthreads) {
    const int nx = (model & 1) ? 5 : 2;
    const int nu = (model == 2 || model == 3) ? 1 : (model >= 4 ? T : 0);
    const int nz = nx + nu;
    if (nz > NZMAX) return -1;
    const int n_slide = (model >= 4 && n_params > 0) ? T : 0;
    const int ngk = nx + n_slide;
    const int64_t nv = (int64_t)N * nz + nx + n_params;
    const int64_t ng = (int64_t)N * ngk;
    int64_t nnz_slide = 0;
    if (n_slide)
        for (int k = 0; k < N; ++k)
            for (int j = 0; j < T; ++j) {
                const int pi = last_idx[k] + 1 - T + j;
                nnz_slide += 1 + (pi >= 0 && pi <= last_idx[k]);
            }
    const int64_t nnz = (int64_t)N * nnzk + nnz_slide;
    const double dt = tf / N;
    (void)nthreads;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
    for (int64_t b = 0; b < B; ++b) {
        const double *vb = v + b * nv;
        ctx c = {jac ? nz : 0};
        for (int k = 0; k < N; ++k) {
            const double *xk = vb + (int64_t)k * nz;
            dual x[5];
            for (int r = 0; r < nx; ++r) {
                x[r] = dc(&c, xk[r]);
                if (jac) x[r].d[r] = 1.0;
            }
            dual lam[32];
            rhs_in in = {model, nx, nu, T, consts, rows + (int64_t)k * T, NULL, dc(&c, 0.0)};
            if (nu == 1) {
                dual pwd = dc(&c, xk[nx]);
                if (jac) pwd.d[nx] = 1.0;
                const dual e = dexp(&c, dscale(&c, -1.0 / consts[PDT], dsub(&c, pwd, dc(&c, consts[PD0]))));
                in.afac = dsub(&c, dc(&c, 1.0), e);
            } else if (nu > 1) {
                for (int i = 0; i < T; ++i) {
                    dual ui = dc(&c, xk[nx + i]);
                    if (jac) ui.d[nx + i] = 1.0;
                    const dual th = dtanh(&c, dscale(&c, consts[BS], dsub(&c, ui, dc(&c, consts[IS]))));
                    lam[i] = dscale(&c, consts[AR], dadd(&c, th, dc(&c, consts[CR])));
                }
                in.lam = lam;
            }
            interval(&c, &in, scheme, m, k * dt, dt, x);
            const double *xn = vb + (int64_t)(k + 1) * nz;
            if (g)
                for (int r = 0; r < nx; ++r) g[b * ng + (int64_t)k * ngk + r] = x[r].v - xn[r];
            if (jac) {
                double *jb = jac + b * nnz + (int64_t)k * nnzk;
                for (int r = 0; r < nx; ++r) {
                    for (int q = 0; q < nz; ++q)
                        if (jpos[r * nz + q] >= 0) jb[jpos[r * nz + q]] = x[r].d[q];
                    jb[jneg[r]] = -1.0;
                }
            }
        }
        if (n_slide) {
            const double *p = vb + (int64_t)N * nz + nx;
            int64_t jo = (int64_t)N * nnzk;
            for (int k = 0; k < N; ++k)
                for (int j = 0; j < T; ++j) {
                    const int pi = last_idx[k] + 1 - T + j;
                    const int valid = pi >= 0 && pi <= last_idx[k];
                    if (g) g[b * ng + (int64_t)k * ngk + nx + j] = vb[(int64_t)k * nz + nx + j] - (valid ? p[pi] : floor_value);
                    if (jac) {
                        jac[b * nnz + jo] = 1.0;
                        if (valid) jac[b * nnz + jo + 1] = -1.0;
                    }
                    jo += 1 + valid;
                }
        }
    }
    return 0;
}
