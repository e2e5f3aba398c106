/*
 * bsls_oracle.c -- CPU restatement of the reference's hot-path kernels.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline.
 *
 * Every function restates the reference's arithmetic in the same operation
 * order so that results are bit-identical to the reference C++ built with
 * g++ (x86-64, no FMA contraction).  Build with -ffp-contract=off.
 *
 * Parity is pinned two ways (see tests/test_oracle_pinning.py):
 *   - against oracle/_ref/libbsls_ref.so, compiled from the reference's own
 *     headers under /root/reference (recipe: oracle/Makefile), and
 *   - against the golden fixtures in tests/golden/ (reference KATs + vectors
 *     captured from the reference itself by tests/golden/make_golden.py).
 *
 * Reference anchors (paths relative to /root/reference):
 *   orc_proj_simplex         python/c_extensions/proj_simplex.h:17-34
 *   orc_proj_multi_simplex   python/c_extensions/proj_simplex.h:37-47
 *   orc_proj_multi_ball      python/c_extensions/proj_simplex.h:50-74
 *   orc_iso_v1               python/c_extensions/isotonic_regression.h:13-58
 *   orc_iso_v2               python/c_extensions/isotonic_regression.h:61-82
 *   orc_iso_v3               python/c_extensions/isotonic_regression.h:105-155
 *   orc_iso_multi_*          python/c_extensions/isotonic_regression.h:85-102,157-164
 *   orc_quad_obj             python/c_extensions/quadratic_objective.h:15-26
 *   orc_line_search          python/c_extensions/quadratic_objective.h:29-61
 *   orc_x2z / orc_z2x        python/c_extensions/c_extensions.pyx:195-248
 *   orc_csr_matvec           scipy.sparse._sparsetools csr_matvec (called via
 *                            A.dot at python/main.py:53-54)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- simplex */

static int cmp_desc(const void *a, const void *b) {
    double x = *(const double *)a, y = *(const double *)b;
    return (x < y) - (x > y);
}

/* Projection of y[lo:hi) onto {x >= 0, sum x = 1}.  The threshold is the
 * value (1 - S_i)/(i+1) at the LAST i whose test u_i + tmp_i > 0 passes,
 * S_i being the left-to-right running sum of the descending-sorted block;
 * i = 0 always qualifies (it seeds lambda = 1 - u_0). */
void orc_proj_simplex(double *y, int64_t lo, int64_t hi) {
    int64_t k = hi - lo;
    if (k <= 0) return;
    double *u = (double *)malloc((size_t)k * sizeof(double));
    memcpy(u, y + lo, (size_t)k * sizeof(double));
    qsort(u, (size_t)k, sizeof(double), cmp_desc);
    double run = u[0];
    double lam = 1. - run;
    for (int64_t i = 1; i < k; ++i) {
        run += u[i];
        double cand = (1. - run) / ((double)i + 1.);
        if (u[i] + cand > 0) lam = cand;
    }
    free(u);
    for (int64_t i = lo; i < hi; ++i) {
        double v = lam + y[i];
        y[i] = (v < 0.) ? 0. : v;           /* std::max(v, 0.) */
    }
}

static int64_t block_end(const int64_t *starts, int64_t nb, int64_t b, int64_t n) {
    return (b + 1 < nb) ? starts[b + 1] : n;
}

void orc_proj_multi_simplex(double *y, const int64_t *starts, int64_t nb, int64_t n) {
    for (int64_t b = 0; b < nb; ++b)
        orc_proj_simplex(y, starts[b], block_end(starts, nb, b, n));
}

/* l1-ball {x >= 0, sum x <= 1}: clamp negatives, project only if the
 * clamped block still sums above one. */
void orc_proj_multi_ball(double *y, const int64_t *starts, int64_t nb, int64_t n) {
    for (int64_t b = 0; b < nb; ++b) {
        int64_t lo = starts[b], hi = block_end(starts, nb, b, n);
        double acc = 0.0;
        for (int64_t j = lo; j < hi; ++j) {
            if (y[j] < 0.0) y[j] = 0.0;
            else acc += y[j];
        }
        if (acc > 1.0) orc_proj_simplex(y, lo, hi);
    }
}

/* ---------------------------------------------------------------- PAVA */

/* v1 ("PAVA+"): sweep the run heads left to right, pooling every maximal
 * non-increasing chain of runs into its weighted mean, until a sweep pools
 * nothing.  w[h] is the run length stored at run head h. */
void orc_iso_v1(double *y, int64_t lo, int64_t hi, int32_t *w, int expand) {
    for (;;) {
        int changed = 0;
        int64_t h = lo;
        while (h < hi) {
            int64_t last = h, nxt = h + w[h];
            while (nxt < hi && y[nxt] <= y[last]) {
                last = nxt;
                nxt += w[nxt];
            }
            if (y[h] != y[last]) {
                double num = 0.0;
                int32_t den = 0;
                for (int64_t r = h; r < nxt; r += w[r]) {
                    num += y[r] * w[r];
                    den += w[r];
                }
                y[h] = num / den;
                w[h] = den;
                changed = 1;
            }
            h = nxt;
        }
        if (!changed) break;
    }
    if (expand) {
        for (int64_t h = lo; h < hi; h += w[h])
            for (int64_t r = h + 1; r < h + w[h]; ++r) y[r] = y[h];
    }
}

/* v2: unweighted repeated sweeps; every non-increasing stretch is replaced
 * by its plain mean, in place. */
void orc_iso_v2(double *y, int64_t lo, int64_t hi) {
    int64_t last = hi - 1;
    for (;;) {
        int changed = 0;
        int64_t a = lo;
        while (a < last) {
            int64_t b = a;
            while (b < last && y[b] >= y[b + 1]) ++b;
            if (y[a] != y[b]) {
                double s = 0.0;
                for (int64_t r = a; r <= b; ++r) s += y[r];
                double mean = s / (b + 1 - a);
                for (int64_t r = a; r <= b; ++r) y[r] = mean;
                changed = 1;
            }
            a = b + 1;
        }
        if (!changed) break;
    }
}

/* v3: single sweep with backtracking.  w[head] and w[tail] both carry the
 * run length so the previous run's head is reachable from the left. */
void orc_iso_v3(double *y, int64_t lo, int64_t hi, int32_t *w, int expand) {
    int64_t h = lo;
    while (h < hi) {
        int64_t last = h, nxt = h + w[h];
        while (nxt < hi && y[nxt] <= y[last]) {
            last = nxt;
            nxt += w[nxt];
        }
        if (y[h] != y[last]) {
            double num = 0.0;
            int32_t den = 0;
            for (int64_t r = h; r < nxt; r += w[r]) {
                num += y[r] * w[r];
                den += w[r];
            }
            y[h] = num / den;
            w[h] = den;
            w[nxt - 1] = den;
            if (h > lo) {
                int64_t p = h - w[h - 1];
                while (p >= lo && y[p] >= y[h]) {
                    y[p] = (w[h] * y[h] + w[p] * y[p]) / (w[h] + w[p]);
                    w[p] = w[h] + w[p];
                    h = p;
                    if (p == lo) break;
                    p -= w[p - 1];
                }
                w[nxt - 1] = w[h];
            }
        } else {
            h = nxt;
        }
    }
    if (expand) {
        for (int64_t a = lo; a < hi; a += w[a])
            for (int64_t r = a + 1; r < a + w[a]; ++r) y[r] = y[a];
    }
}

void orc_iso_multi_v1(double *y, const int64_t *starts, int64_t nb, int64_t n,
                      int32_t *w, int expand) {
    for (int64_t b = 0; b < nb; ++b)
        orc_iso_v1(y, starts[b], block_end(starts, nb, b, n), w, expand);
}

void orc_iso_multi_v2(double *y, const int64_t *starts, int64_t nb, int64_t n) {
    for (int64_t b = 0; b < nb; ++b)
        orc_iso_v2(y, starts[b], block_end(starts, nb, b, n));
}

void orc_iso_multi_v3(double *y, const int64_t *starts, int64_t nb, int64_t n,
                      int32_t *w, int expand) {
    for (int64_t b = 0; b < nb; ++b)
        orc_iso_v3(y, starts[b], block_end(starts, nb, b, n), w, expand);
}

/* ---------------------------------------------------------------- dense QP */

double orc_quad_obj(const double *x, const double *Q, const double *c, double *g,
                    int64_t n) {
    double f = 0;
    for (int64_t i = 0; i < n; ++i) {
        g[i] = c[i];
        const double *row = Q + i * n;
        for (int64_t j = 0; j < n; ++j) g[i] += row[j] * x[j];
        f += 0.5 * (g[i] + c[i]) * x[i];
    }
    return f;
}

/* Backtracking line search between x and x_new (halving).  The reference's
 * "step too small" branch copies x into x_new and, through an unbraced for,
 * writes g_new[n] out of bounds instead of copying g: the observable effect
 * on valid memory is that g_new keeps its last value.  We keep that
 * observable behaviour and drop the out-of-bounds store. */
double orc_line_search(const double *x, double f, const double *g, double *x_new,
                       double f_new, double *g_new, const double *Q,
                       const double *c, int64_t n) {
    const double suff = 1e-4, prog = 1e-8;
    double t = 1, upper = f;
    for (int64_t i = 0; i < n; ++i) upper += suff * g[i] * (x_new[i] - x[i]);
    while (f_new > upper) {
        t *= .5;
        double span = 0.0;
        for (int64_t i = 0; i < n; ++i) {
            if (x_new[i] - x[i] > span) span = x_new[i] - x[i];
            if (x[i] - x_new[i] > span) span = x[i] - x_new[i];
        }
        if (t * span < prog) {
            for (int64_t i = 0; i < n; ++i) x_new[i] = x[i];
            f_new = f;
            break;
        }
        for (int64_t i = 0; i < n; ++i) x_new[i] = x[i] + t * (x_new[i] - x[i]);
        f_new = orc_quad_obj(x_new, Q, c, g_new, n);
        for (int64_t i = 0; i < n; ++i) upper += suff * g[i] * (x_new[i] - x[i]);
    }
    return f_new;
}

/* ---------------------------------------------------------------- x <-> z */

void orc_x2z(const double *x, double *z, const int64_t *starts, int64_t nb, int64_t n) {
    int64_t j = 0;
    for (int64_t b = 0; b < nb; ++b) {
        int64_t lo = starts[b], hi = block_end(starts, nb, b, n);
        double acc = 0.0;
        for (int64_t i = lo; i < hi - 1; ++i) {
            acc += x[i];
            z[j++] = acc;
        }
    }
}

void orc_z2x(double *x, const double *z, const int64_t *starts, int64_t nb, int64_t n) {
    int64_t j = 0;
    for (int64_t b = 0; b < nb; ++b) {
        int64_t lo = starts[b], hi = block_end(starts, nb, b, n);
        double prev = 0.0;
        for (int64_t i = lo; i < hi - 1; ++i) {
            x[i] = z[j] - prev;
            prev = z[j++];
        }
        x[hi - 1] = 1.0 - prev;
    }
}

/* ---------------------------------------------------------------- CSR */

/* out[r] = sum over the row's entries in storage order, starting from 0
 * (scipy csr_matvec accumulates into a zeroed result). */
void orc_csr_matvec(int64_t m, const int32_t *indptr, const int32_t *indices,
                    const double *data, const double *x, double *out) {
    for (int64_t r = 0; r < m; ++r) {
        double acc = 0.0;
        for (int32_t e = indptr[r]; e < indptr[r + 1]; ++e) acc += data[e] * x[indices[e]];
        out[r] = acc;
    }
}
