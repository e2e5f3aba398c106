/*
 * bsls_cpu_bb.c -- the z-space projected BB loop as a C port for the CPU
 * baseline leg of bench.py (all host cores, OpenMP).
 *
 * TEST INFRASTRUCTURE ONLY (like the rest of oracle/): timed by bench.py's
 * cpu_baseline leg, never part of the product.  It does the reference's work
 * per iteration -- python/BB.py:17-41 over the closures of python/main.py:53-65:
 * nabla_f(z) = N'A'(A N z + target), f(z) = 0.5 ||A N z + target||^2 (its own
 * residual, as the reference recomputes it), the BB2 step, PAVA v1 + clip on
 * every z-block (isotonic_regression.h:13-58, orc_iso_v1) -- with the
 * SpMVs split over rows, the projection over blocks and the dot products
 * reduced over threads.  Sums run in a different order than NumPy/SciPy, so
 * iterates agree with the 1-thread restatement to rounding, not bit for bit
 * (tests/test_oracle_pinning.py checks 1e-9).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void orc_iso_v1(double *y, int64_t lo, int64_t hi, int32_t *w, int expand);

/* y = A x (+ add), rows split over threads; each row summed in CSR order */
static void spmv(int64_t rows, const int64_t *ip, const int32_t *ix, const double *v,
                 const double *x, const double *add, double *y) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < rows; ++i) {
        double s = 0.0;
        for (int64_t k = ip[i]; k < ip[i + 1]; ++k) s += v[k] * x[ix[k]];
        y[i] = add ? s + add[i] : s;
    }
}

/* x = N z: per block x_0 = z_0, x_j = z_j - z_{j-1}, x_{k-1} = -z_{k-2} */
static void n_apply(int64_t nb, const int64_t *xs, int64_t n, const double *z, double *x) {
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t x0 = xs[b], x1 = (b + 1 < nb) ? xs[b + 1] : n, z0 = x0 - b;
        const int64_t k = x1 - x0;
        if (k == 1) {
            x[x0] = 0.0;
            continue;
        }
        x[x0] = z[z0];
        for (int64_t j = 1; j < k - 1; ++j) x[x0 + j] = z[z0 + j] - z[z0 + j - 1];
        x[x1 - 1] = 0.0 - z[z0 + k - 2];
    }
}

/* g = N' w: g_j = w_j - w_{j+1} within a block */
static void nt_apply(int64_t nb, const int64_t *xs, int64_t n, const double *w, double *g) {
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t x0 = xs[b], x1 = (b + 1 < nb) ? xs[b + 1] : n, z0 = x0 - b;
        for (int64_t j = 0; j < x1 - x0 - 1; ++j) g[z0 + j] = w[x0 + j] - w[x0 + j + 1];
    }
}

static double dot(int64_t n, const double *a, const double *b) {
    double s = 0.0;
#pragma omp parallel for reduction(+ : s) schedule(static)
    for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
    return s;
}

typedef struct {
    int64_t m, n, nb;
    const int64_t *ip, *ipt, *xs;
    const int32_t *ix, *ixt;
    const double *v, *vt, *target;
    double *x, *r, *w;
} cpubb;

static double f_of(cpubb *P, const double *z) {
    n_apply(P->nb, P->xs, P->n, z, P->x);
    spmv(P->m, P->ip, P->ix, P->v, P->x, P->target, P->r);
    const double nr = sqrt(dot(P->m, P->r, P->r));
    return 0.5 * nr * nr;
}

static void grad_of(cpubb *P, const double *z, double *g) {
    n_apply(P->nb, P->xs, P->n, z, P->x);
    spmv(P->m, P->ip, P->ix, P->v, P->x, P->target, P->r);
    spmv(P->n, P->ipt, P->ixt, P->vt, P->r, NULL, P->w);
    nt_apply(P->nb, P->xs, P->n, P->w, g);
}

/* `iters` BB iterations from z (in place; z_prev = z + 1 as BB.py:14), early
 * exits disabled (bench.py times a fixed count).  Returns the last f. */
double cpubb_run(int64_t m, int64_t n, int64_t nb, const int64_t *xs, const int64_t *ip,
                 const int32_t *ix, const double *v, const int64_t *ipt, const int32_t *ixt,
                 const double *vt, const double *target, double *z, int64_t iters, int threads) {
    if (threads > 0) omp_set_num_threads(threads);
    const int64_t nz = n - nb;
    cpubb P = {m, n, nb, ip, ipt, xs, ix, ixt, v, vt, target, NULL, NULL, NULL};
    P.x = malloc(sizeof(double) * n);
    P.r = malloc(sizeof(double) * m);
    P.w = malloc(sizeof(double) * n);
    double *zp = malloc(sizeof(double) * nz), *g = malloc(sizeof(double) * nz);
    double *gp = malloc(sizeof(double) * nz), *dg = malloc(sizeof(double) * nz);
    double *dx = malloc(sizeof(double) * nz);
    int32_t *wt = malloc(sizeof(int32_t) * nz);
    for (int64_t i = 0; i < nz; ++i) zp[i] = z[i] + 1;
    grad_of(&P, zp, gp);
    double fx = 0.0;
    for (int64_t it = 0; it < iters; ++it) {
        grad_of(&P, z, g);
        double sdg = 0.0;
#pragma omp parallel for reduction(+ : sdg) schedule(static)
        for (int64_t i = 0; i < nz; ++i) {
            dg[i] = g[i] - gp[i];
            dx[i] = z[i] - zp[i];
            sdg += dg[i];
        }
        (void)sdg;   /* BB.py:22's exit is disabled for timing */
        const double t = dot(nz, dx, dg) / dot(nz, dg, dg);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < nz; ++i) {
            zp[i] = z[i];
            z[i] = z[i] - t * g[i];
            gp[i] = g[i];
        }
#pragma omp parallel for schedule(dynamic, 256)
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t z0 = xs[b] - b, z1 = ((b + 1 < nb) ? xs[b + 1] : n) - (b + 1);
            if (z1 <= z0) continue;
            for (int64_t j = z0; j < z1; ++j) wt[j] = 1;
            orc_iso_v1(z, z0, z1, wt, 1);
            for (int64_t j = z0; j < z1; ++j) {
                const double a = z[j] < 1.0 ? z[j] : 1.0;
                z[j] = a > 0.0 ? a : 0.0;
            }
        }
        fx = f_of(&P, z);
    }
    free(P.x); free(P.r); free(P.w); free(zp); free(g); free(gp); free(dg); free(dx); free(wt);
    return fx;
}
