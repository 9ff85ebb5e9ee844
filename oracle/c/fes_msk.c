/*
 * fes_msk.c — plain-C port of oracle/fes_msk.py (the CPU restatement of FesMskModel.muscle_dynamic,
 * cocofest/models/dynamical_model.py:133-334, and of the biorbd algorithms behind it).
 *
 * TEST INFRASTRUCTURE ONLY: the CPU baseline of bench.py's musculoskeletal section and a cross-check of the numpy
 * oracle in tests/.  Nothing in the product links or calls it.
 *
 * Same algorithm as the numpy oracle: the full segment tree is walked (frame = parent x RT x R(dofs)), muscle-tendon
 * lengths over origin -> via points -> insertion with the length Jacobian from point Jacobians, De Groote
 * coefficients (hill_coefficients.py:11-126; force-length gated by the force-velocity flag as the reference does,
 * dynamical_model.py:259-269), forward dynamics by Newton-Euler inverse dynamics with unit accelerations, the Ding
 * muscle ODEs with the as-written calcium sum (2T-1 exponentials per RK stage, ding2003.py:230-252), RK-s
 * multiple shooting; derivatives by the complex step (one complex evaluation per Jacobian column), as CasADi's
 * forward mode would sweep the columns.  OpenMP over (instance, interval).
 */
#include <complex.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef double complex cx;

#define MS_SEG 32
#define MS_DOF 8
#define MS_MUS 8
#define MS_PTS 16
#define MS_X 64

typedef struct {
    int32_t nseg, ndof;
    int32_t parent[MS_SEG];      /* -1: root */
    double rt[MS_SEG][16];       /* row-major 4x4 */
    int32_t nrot[MS_SEG];        /* rotation dofs of the segment, applied in order */
    int32_t rot_axis[MS_SEG][3]; /* 0 / 1 / 2 */
    double mass[MS_SEG], com[MS_SEG][3], inertia[MS_SEG][9];
    double grav[3];
    int32_t nmus;
    int32_t model[MS_MUS]; /* 0 ding2003, 1 +fatigue, 2 ding2007, 3 +fatigue */
    /* tauc, r0_km_relationship, a_rest, tau1_rest, tau2, km_rest, a_scale, pd0, pdt, alpha_a, alpha_tau1,
       alpha_km, tau_fat */
    double cst[MS_MUS][13];
    int32_t npts[MS_MUS], pt_seg[MS_MUS][MS_PTS];
    double pt_pos[MS_MUS][MS_PTS][3];
    double lopt[MS_MUS], slack[MS_MUS], penn[MS_MUS];
    int32_t fv_on, fp_on, residual;
    int32_t N, m, scheme, T;
    double tf;
    /* the conventions of the revision that wrote the reference's stored reaching-task solutions (fes_oracle.cn_sum
       legacy_skip_first, fes_oracle.rhs legacy): a window's first pulse left out of the calcium sum once the window
       holds several, r0 from the Km state of the fatigue models */
    int32_t legacy;
} ms_desc;

typedef struct {
    const ms_desc *d;
    const double *rows; /* (N+1) x T stim table */
    int nq, nx, nu, nxm, npw;
    int xoff[MS_MUS], uoff[MS_MUS];
    int dof_seg[MS_DOF];
    int anc[MS_SEG][MS_SEG]; /* anc[s][a]: a is s or an ancestor of s */
    int last_dof[MS_SEG];    /* last dof on the path root -> s, -1 */
    int link_parent[MS_DOF];
} ms_ctx;

static void setup(const ms_desc *d, const double *rows, ms_ctx *c) {
    memset(c, 0, sizeof(*c));
    c->d = d;
    c->rows = rows;
    int k = 0;
    for (int s = 0; s < d->nseg; ++s) {
        for (int a = 0; a < d->nseg; ++a) c->anc[s][a] = 0;
        for (int a = s; a >= 0; a = d->parent[a]) c->anc[s][a] = 1;
        const int p = d->parent[s];
        int prev = p >= 0 ? c->last_dof[p] : -1;
        for (int r = 0; r < d->nrot[s]; ++r) {
            c->dof_seg[k] = s;
            c->link_parent[k] = prev;
            prev = k++;
        }
        c->last_dof[s] = prev;
    }
    c->nq = k;
    for (int mu = 0; mu < d->nmus; ++mu) {
        c->xoff[mu] = c->nxm;
        c->nxm += (d->model[mu] & 1) ? 5 : 2;
        c->uoff[mu] = d->model[mu] >= 2 ? c->npw++ : -1;
    }
    c->nx = c->nxm + 2 * c->nq;
    c->nu = c->npw + (d->residual ? c->nq : 0);
}

static void mat4mul(const cx *a, const cx *b, cx *r) {
    cx t[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            cx s = 0;
            for (int k = 0; k < 4; ++k) s += a[i * 4 + k] * b[k * 4 + j];
            t[i * 4 + j] = s;
        }
    memcpy(r, t, sizeof(t));
}

static void cross(const cx *a, const cx *b, cx *r) {
    cx t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
    r[0] = t0, r[1] = t1, r[2] = t2;
}

/* frames of every segment; per dof its world axis and origin */
static void fk(const ms_ctx *c, const cx *q, cx (*T)[16], cx (*ax)[3], cx (*org)[3]) {
    const ms_desc *d = c->d;
    int k = 0;
    for (int s = 0; s < d->nseg; ++s) {
        cx M[16], R[16];
        for (int e = 0; e < 16; ++e) R[e] = d->rt[s][e];
        if (d->parent[s] >= 0) {
            mat4mul(T[d->parent[s]], R, M);
        } else {
            memcpy(M, R, sizeof(M));
        }
        for (int r = 0; r < d->nrot[s]; ++r, ++k) {
            const int a = d->rot_axis[s][r];
            for (int e = 0; e < 3; ++e) ax[k][e] = M[e * 4 + a], org[k][e] = M[e * 4 + 3];
            const int i = a == 0 ? 1 : (a == 1 ? 2 : 0), j = a == 0 ? 2 : (a == 1 ? 0 : 1);
            cx Rot[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
            const cx co = ccos(q[k]), si = csin(q[k]);
            Rot[i * 4 + i] = co, Rot[i * 4 + j] = -si, Rot[j * 4 + i] = si, Rot[j * 4 + j] = co;
            mat4mul(M, Rot, M);
        }
        memcpy(T[s], M, sizeof(M));
    }
}

static cx hill_fl(cx nl) {
    const double b1[3] = {0.815, 0.433, 0.100}, b2[3] = {1.055, 0.717, 1.000}, b3[3] = {0.162, -0.030, 0.354},
                 b4[3] = {0.063, 0.200, 0.0};
    cx r = 0;
    for (int i = 0; i < 3; ++i) {
        const cx w = b3[i] + b4[i] * nl;
        r += b1[i] * cexp((-0.5 * ((nl - b2[i]) * (nl - b2[i]))) / (w * w));
    }
    return r;
}
static cx hill_fv(cx vel) {
    const cx w = -8.149 * (vel / 10) + -0.374;
    return -0.318 * clog(w + csqrt(w * w + 1)) + 0.886;
}
static cx hill_fp(cx nl) {
    const cx fp = (cexp(4 * (nl - 1) / 0.6) - 1) / (exp(4.0) - 1);
    return creal(fp) > 0 ? fp : 0;
}

/* Newton-Euler inverse dynamics in world coordinates (gravity as a base acceleration) */
static void inverse_dynamics(const ms_ctx *c, cx (*T)[16], cx (*ax)[3], cx (*org)[3], const cx *qd, const cx *qdd,
                             int gravity, cx *tau) {
    const ms_desc *d = c->d;
    const int nq = c->nq;
    cx w[MS_DOF][3], al[MS_DOF][3], acc[MS_DOF][3];
    for (int k = 0; k < nq; ++k) {
        const int p = c->link_parent[k];
        cx wp[3] = {0, 0, 0}, alp[3] = {0, 0, 0}, ap[3], op[3] = {0, 0, 0};
        for (int e = 0; e < 3; ++e) ap[e] = gravity ? -d->grav[e] : 0;
        if (p >= 0)
            for (int e = 0; e < 3; ++e) wp[e] = w[p][e], alp[e] = al[p][e], ap[e] = acc[p][e], op[e] = org[p][e];
        cx r[3], zq[3], t1[3], t2[3], t3[3], t4[3];
        for (int e = 0; e < 3; ++e) r[e] = org[k][e] - op[e], zq[e] = ax[k][e] * qd[k];
        cross(wp, zq, t4);
        cross(alp, r, t1);
        cross(wp, r, t2);
        cross(wp, t2, t3);
        for (int e = 0; e < 3; ++e) {
            w[k][e] = wp[e] + zq[e];
            al[k][e] = alp[e] + ax[k][e] * qdd[k] + t4[e];
            acc[k][e] = ap[e] + t1[e] + t3[e];
        }
    }
    for (int k = 0; k < nq; ++k) tau[k] = 0;
    for (int s = 0; s < d->nseg; ++s) {
        int zero = d->mass[s] == 0;
        for (int e = 0; e < 9; ++e) zero &= d->inertia[s][e] == 0;
        const int k = c->last_dof[s];
        if (zero || k < 0) continue;
        cx cw[3], rc[3], Iw[9], RI[9];
        for (int e = 0; e < 3; ++e)
            cw[e] = T[s][e * 4] * d->com[s][0] + T[s][e * 4 + 1] * d->com[s][1] + T[s][e * 4 + 2] * d->com[s][2] +
                    T[s][e * 4 + 3];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                cx v = 0;
                for (int l = 0; l < 3; ++l) v += T[s][i * 4 + l] * d->inertia[s][l * 3 + j];
                RI[i * 3 + j] = v;
            }
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                cx v = 0;
                for (int l = 0; l < 3; ++l) v += RI[i * 3 + l] * T[s][j * 4 + l];
                Iw[i * 3 + j] = v;
            }
        for (int e = 0; e < 3; ++e) rc[e] = cw[e] - org[k][e];
        cx t1[3], t2[3], t3[3], F[3], Ia[3], Iww[3], t5[3], N[3];
        cross(al[k], rc, t1);
        cross(w[k], rc, t2);
        cross(w[k], t2, t3);
        for (int e = 0; e < 3; ++e) F[e] = d->mass[s] * (acc[k][e] + t1[e] + t3[e]);
        for (int e = 0; e < 3; ++e) {
            Ia[e] = Iw[e * 3] * al[k][0] + Iw[e * 3 + 1] * al[k][1] + Iw[e * 3 + 2] * al[k][2];
            Iww[e] = Iw[e * 3] * w[k][0] + Iw[e * 3 + 1] * w[k][1] + Iw[e * 3 + 2] * w[k][2];
        }
        cross(w[k], Iww, t5);
        for (int e = 0; e < 3; ++e) N[e] = Ia[e] + t5[e];
        for (int j = k; j >= 0; j = c->link_parent[j]) {
            cx r[3], m1[3];
            for (int e = 0; e < 3; ++e) r[e] = cw[e] - org[j][e];
            cross(r, F, m1);
            tau[j] += ax[j][0] * (m1[0] + N[0]) + ax[j][1] * (m1[1] + N[1]) + ax[j][2] * (m1[2] + N[2]);
        }
    }
}

/* FesMskModel.muscle_dynamic at time t: x (nx), u (nu), stim row (T) */
static void msk_rhs(const ms_ctx *c, double t, const double *row, const cx *x, const cx *u, cx *f) {
    const ms_desc *d = c->d;
    const int nq = c->nq, XQ = c->nxm;
    const cx *q = x + XQ, *qd = x + XQ + nq;
    cx T[MS_SEG][16], ax[MS_DOF][3], org[MS_DOF][3];
    fk(c, q, T, ax, org);
    cx tau[MS_DOF];
    for (int k = 0; k < nq; ++k) tau[k] = d->residual ? u[c->npw + k] : 0;
    for (int mu = 0; mu < d->nmus; ++mu) {
        const double *cs = d->cst[mu];
        /* geometry */
        cx P[MS_PTS][3], JP[MS_PTS][MS_DOF][3];
        const int np = d->npts[mu];
        for (int i = 0; i < np; ++i) {
            const int s = d->pt_seg[mu][i];
            for (int e = 0; e < 3; ++e)
                P[i][e] = T[s][e * 4] * d->pt_pos[mu][i][0] + T[s][e * 4 + 1] * d->pt_pos[mu][i][1] +
                          T[s][e * 4 + 2] * d->pt_pos[mu][i][2] + T[s][e * 4 + 3];
            for (int k = 0; k < nq; ++k) {
                if (c->anc[s][c->dof_seg[k]]) {
                    cx r[3];
                    for (int e = 0; e < 3; ++e) r[e] = P[i][e] - org[k][e];
                    cross(ax[k], r, JP[i][k]);
                } else {
                    JP[i][k][0] = JP[i][k][1] = JP[i][k][2] = 0;
                }
            }
        }
        cx L = 0, JL[MS_DOF];
        for (int k = 0; k < nq; ++k) JL[k] = 0;
        for (int i = 0; i + 1 < np; ++i) {
            cx dd[3];
            for (int e = 0; e < 3; ++e) dd[e] = P[i + 1][e] - P[i][e];
            const cx n = csqrt(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
            L += n;
            for (int k = 0; k < nq; ++k)
                JL[k] += (dd[0] * (JP[i + 1][k][0] - JP[i][k][0]) + dd[1] * (JP[i + 1][k][1] - JP[i][k][1]) +
                          dd[2] * (JP[i + 1][k][2] - JP[i][k][2])) / n;
        }
        const cx nl = (L - d->slack[mu]) / cos(d->penn[mu]) / d->lopt[mu];
        cx vel = 0;
        for (int k = 0; k < nq; ++k) vel += JL[k] * qd[k];
        const cx fl = d->fv_on ? hill_fl(nl) : 1, fv = d->fv_on ? hill_fv(vel) : 1, fp = d->fp_on ? hill_fp(nl) : 0;
        /* muscle ODE (ding2003.py:230-311, ding2003_with_fatigue.py:197-240, ding2007.py:172-188) */
        const cx *xm = x + c->xoff[mu];
        cx *fm = f + c->xoff[mu];
        const int fat = d->model[mu] & 1, pw = d->model[mu] >= 2;
        const double tauc = cs[0];
        const cx r0 = (d->legacy && fat) ? xm[4] + cs[1] : cs[5] + cs[1];
        int skip = -1;
        if (d->legacy) {
            int nreal = 0;
            for (int i = 0; i < d->T; ++i) nreal += row[i] > -1e6;
            if (nreal > 1) skip = d->T - nreal;
        }
        cx sum = 0;
        for (int i = 0; i < d->T; ++i) {
            if (i == skip) continue;
            const cx ri = i == 0 ? 1.0 : 1.0 + (r0 - 1.0) * exp(-(row[i] - row[i - 1]) / tauc);
            sum += ri * exp(-(t - row[i]) / tauc);
        }
        fm[0] = (1 / tauc) * sum - xm[0] / tauc;
        cx A = fat ? xm[2] : (pw ? cs[6] : cs[2]);
        const cx tau1 = fat ? xm[3] : cs[3], km = fat ? xm[4] : cs[5];
        if (pw) A = A * (1 - cexp(-(u[c->uoff[mu]] - cs[7]) / cs[8]));
        const cx s = xm[0] / (km + xm[0]);
        fm[1] = (A * s - xm[1] / (tau1 + cs[4] * s)) * (fl * fv + fp);
        if (fat) {
            const double arest = pw ? cs[6] : cs[2];
            fm[2] = -(xm[2] - arest) / cs[12] + cs[9] * xm[1];
            fm[3] = -(tau1 - cs[3]) / cs[12] + cs[10] * xm[1];
            fm[4] = -(km - cs[5]) / cs[12] + cs[11] * xm[1];
        }
        for (int k = 0; k < nq; ++k) tau[k] -= JL[k] * xm[1];
    }
    /* qddot = M^-1 (tau - h) */
    cx zero[MS_DOF], h[MS_DOF], M[MS_DOF][MS_DOF + 1], g0[MS_DOF], e[MS_DOF];
    for (int k = 0; k < nq; ++k) zero[k] = 0;
    inverse_dynamics(c, T, ax, org, qd, zero, 1, h);
    inverse_dynamics(c, T, ax, org, zero, zero, 0, g0);
    for (int j = 0; j < nq; ++j) {
        cx col[MS_DOF];
        for (int k = 0; k < nq; ++k) e[k] = k == j ? 1 : 0;
        inverse_dynamics(c, T, ax, org, zero, e, 0, col);
        for (int k = 0; k < nq; ++k) M[k][j] = col[k] - g0[k];
    }
    for (int k = 0; k < nq; ++k) M[k][nq] = tau[k] - h[k];
    for (int p = 0; p < nq; ++p) { /* Gauss-Jordan, SPD */
        const cx ip = 1 / M[p][p];
        for (int j = p; j <= nq; ++j) M[p][j] *= ip;
        for (int i = 0; i < nq; ++i)
            if (i != p) {
                const cx fi = M[i][p];
                for (int j = p; j <= nq; ++j) M[i][j] -= fi * M[p][j];
            }
    }
    for (int k = 0; k < nq; ++k) {
        f[XQ + k] = qd[k];
        f[XQ + nq + k] = M[k][nq];
    }
}

static void interval(const ms_ctx *c, int k, cx *x, const cx *u) {
    const ms_desc *d = c->d;
    const int nx = c->nx;
    const double dt = d->tf / d->N, h = dt / d->m;
    const double *rw = c->rows + (int64_t)k * d->T;
    for (int j = 0; j < d->m; ++j) {
        const double t = k * dt + j * h;
        cx k1[MS_X], k2[MS_X], k3[MS_X], k4[MS_X], xs[MS_X];
        msk_rhs(c, t, rw, x, u, k1);
        if (d->scheme == 1) {
            for (int r = 0; r < nx; ++r) x[r] += h * k1[r];
        } else if (d->scheme == 2) {
            for (int r = 0; r < nx; ++r) xs[r] = x[r] + h / 2 * k1[r];
            msk_rhs(c, t + h / 2, rw, xs, u, k2);
            for (int r = 0; r < nx; ++r) x[r] += h * k2[r];
        } else {
            for (int r = 0; r < nx; ++r) xs[r] = x[r] + h / 2 * k1[r];
            msk_rhs(c, t + h / 2, rw, xs, u, k2);
            for (int r = 0; r < nx; ++r) xs[r] = x[r] + h / 2 * k2[r];
            msk_rhs(c, t + h / 2, rw, xs, u, k3);
            for (int r = 0; r < nx; ++r) xs[r] = x[r] + h * k3[r];
            msk_rhs(c, t + h, rw, xs, u, k4);
            for (int r = 0; r < nx; ++r) x[r] += h / 6 * (k1[r] + 2 * k2[r] + 2 * k3[r] + k4[r]);
        }
    }
}

/* g (B x ng) and the dense interval Jacobian blocks dPhi_k / d(x_k, u_k) (B x N x nx x nz, may be NULL) for
   decision vectors v (B x nv, node-major [x_0, u_0, ..., x_N]). */
int ms_shooting(const ms_desc *d, const double *rows, int64_t B, const double *v, double *g, double *jac, int threads) {
    ms_ctx c;
    setup(d, rows, &c);
    const int N = d->N, nx = c.nx, nz = c.nx + c.nu;
    const int64_t nv = (int64_t)N * nz + nx;
    if (nx > MS_X || c.nq > MS_DOF) return -1;
#pragma omp parallel for num_threads(threads) schedule(static) collapse(2)
    for (int64_t b = 0; b < B; ++b)
        for (int k = 0; k < N; ++k) {
            const double *z = v + b * nv + (int64_t)k * nz;
            const double *xn = z + nz;
            const int ncol = jac ? nz : 0;
            for (int col = -1; col < ncol; ++col) {
                cx x[MS_X], u[MS_X];
                for (int r = 0; r < nx; ++r) x[r] = z[r];
                for (int i = 0; i < c.nu; ++i) u[i] = z[nx + i];
                if (col >= 0) {
                    if (col < nx) x[col] += 1e-30 * I;
                    else u[col - nx] += 1e-30 * I;
                }
                interval(&c, k, x, u);
                if (col < 0) {
                    if (g)
                        for (int r = 0; r < nx; ++r) g[b * (int64_t)N * nx + (int64_t)k * nx + r] = creal(x[r]) - xn[r];
                } else {
                    double *J = jac + ((b * N + k) * (int64_t)nx) * nz;
                    for (int r = 0; r < nx; ++r) J[(int64_t)r * nz + col] = cimag(x[r]) / 1e-30;
                }
            }
        }
    return 0;
}
