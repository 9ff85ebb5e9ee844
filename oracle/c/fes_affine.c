/*
 * fes_affine.c — CPU baseline in the SAME formulation as the GPU headline kernel (test infrastructure only).
 *
 * bench.py times it beside the as-written port (fes_oracle.c) so that the GPU / CPU ratio separates hardware from
 * algorithm: the two-state Ding families (Ding2003, Ding2007 pulse width; OcpFes's default
 * RK1 x m transcription) with the calcium state affine in the interval's start value — cn(slot) = cna[slot] cn0 +
 * cnb[k][slot], tables built on the host from the reference's calcium sums (cn_sum_fun,
 * cocofest/models/ding2003.py:230-252) — and the fused explicit-Euler force step with its tangents (F+ = F (1 - u)
 * + h mult A s, ding2003.py:274-311; cfx_kernels.h:euler_force), over 64-instance tiles (CFX_LAYOUT_TILED64, the
 * layout the GPU bench streams).  Every inner loop runs over the 64 instances of a tile, so the compiler vectorises
 * it (AVX-512 where the host has it: target_clones below); OpenMP spreads the tiles over the threads.
 * Outputs: g (continuity rows) and the J_g values at the positions given by jpos / jneg (the callbacks' structure).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define TILE 64

typedef struct {
    int32_t pw;      /* Ding2007: one pulse-width control per interval */
    int32_t N, m, nz;
    double km, tau12, tau1km, hm, hmkm, hmkmt2, a_force, pd0, pdt;
} affine_params;

__attribute__((target_clones("arch=skylake-avx512", "arch=haswell", "default")))
static void tile_run(const affine_params *P, const double *cna, const double *cnb, const double *v, double *g,
                     double *jac, int64_t nv, int64_t ng, int64_t nnz, int nnzk, const int32_t *jpos,
                     const int32_t *jneg) {
    const int N = P->N, m = P->m, nz = P->nz;
    double cn0[TILE], F[TILE], dFc[TILE], dFF[TILE], dFp[TILE], A[TILE], dA[TILE];
    for (int k = 0; k < N; ++k) {
        const double *xk = v + (int64_t)k * nz * TILE, *xn = v + (int64_t)(k + 1) * nz * TILE;
        const double *bk = cnb + (int64_t)k * (m + 1);
#pragma omp simd
        for (int i = 0; i < TILE; ++i) {
            cn0[i] = xk[i];
            F[i] = xk[TILE + i];
            dFc[i] = 0.0;
            dFF[i] = 1.0;
            dFp[i] = 0.0;
            A[i] = P->a_force;
            dA[i] = 0.0;
        }
        if (P->pw) {
            for (int i = 0; i < TILE; ++i) {  /* ding2007.py:172-188 */
                const double ex = exp(-(xk[2 * TILE + i] - P->pd0) / P->pdt);
                A[i] = P->a_force * (1.0 - ex);
                dA[i] = P->a_force * ex / P->pdt;
            }
        }
        for (int j = 0; j < m; ++j) {
            const double a = cna[j], b = bk[j];
#pragma omp simd
            for (int i = 0; i < TILE; ++i) {
                const double cn = a * cn0[i] + b;
                const double d1 = cn + P->km;
                const double d2 = P->tau12 * cn + P->tau1km;
                const double R = 1.0 / (d1 * d2);
                const double q1 = d2 * R, q2 = d1 * R;
                const double u = P->hm * d1 * q2, s = cn * q1, om = 1.0 - u;
                const double w = P->hmkm * A[i] * q1 * q1 + F[i] * P->hmkmt2 * q2 * q2;
                dFc[i] = om * dFc[i] + w * a;
                dFF[i] = om * dFF[i];
                dFp[i] = om * dFp[i] + P->hm * dA[i] * s;
                F[i] = P->hm * A[i] * s + om * F[i];
            }
        }
        const double ae = cna[m], be = bk[m];
        double *gk = g + (int64_t)k * 2 * TILE;
        double *jk = jac + (int64_t)k * nnzk * TILE;
        const int p00 = jpos[0 * nz + 0], p10 = jpos[1 * nz + 0], p11 = jpos[1 * nz + 1];
        const int p12 = P->pw ? jpos[1 * nz + 2] : -1, n0 = jneg[0], n1 = jneg[1];
#pragma omp simd
        for (int i = 0; i < TILE; ++i) {
            gk[i] = ae * cn0[i] + be - xn[i];
            gk[TILE + i] = F[i] - xn[TILE + i];
            jk[p00 * TILE + i] = ae;
            jk[n0 * TILE + i] = -1.0;
            jk[p10 * TILE + i] = dFc[i];
            jk[p11 * TILE + i] = dFF[i];
            jk[n1 * TILE + i] = -1.0;
        }
        if (p12 >= 0) {
#pragma omp simd
            for (int i = 0; i < TILE; ++i) jk[p12 * TILE + i] = dFp[i];
        }
    }
    (void)nv, (void)ng, (void)nnz;
}

/* v: (B / 64, nv, 64) tiles; g: (B / 64, ng, 64); jac: (B / 64, nnz, 64).  jpos: [2][nz] (-1: structural zero),
   jneg: [2].  Returns 0, or -1 for an unsupported problem. */
int affine_shooting(const affine_params *P, const double *cna, const double *cnb, int64_t B, const double *v,
                    double *g, double *jac, const int32_t *jpos, const int32_t *jneg, int32_t nnzk, int threads) {
    if (B % TILE || P->nz != 2 + (P->pw ? 1 : 0) || P->m < 1) return -1;
    const int64_t nt = B / TILE, nv = (int64_t)P->N * P->nz + 2, ng = (int64_t)P->N * 2,
                  nnz = (int64_t)P->N * nnzk;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
#endif
    for (int64_t t = 0; t < nt; ++t)
        tile_run(P, cna, cnb, v + t * nv * TILE, g + t * ng * TILE, jac + t * nnz * TILE, nv, ng, nnz, nnzk, jpos,
                 jneg);
    (void)threads;
    return 0;
}
