// bsls_cpu.cpp -- the host path of the c_extensions drop-in (include/bsls_cpu.h).
//
// What the reference's Cython module does on the CPU (python/c_extensions/
// c_extensions.pyx:22-248 over proj_simplex.h, isotonic_regression.h and
// quadratic_objective.h), for callers that select the CPU explicitly
// (BSLS_DEVICE=cpu / main.py --device cpu: BASELINE configs[0]).  Each kernel
// keeps the reference's operation order, so results are bit-identical to it;
// what differs is the engineering around them:
//   * a block's sort buffer is thread-local heap memory sized once to the
//     largest block, not a stack VLA (the reference's `double u[end-start]`
//     overflows the stack for blocks of ~1M elements);
//   * independent blocks are spread over OpenMP threads (dynamic schedule:
//     block sizes are ragged); each block only touches its own range of y and
//     of the weight array, so the result does not depend on the thread count;
//   * 64-bit indices and block starts (the reference narrows to int).
// Built with -ffp-contract=off: the reference's x86-64 build has no FMAs.
#include "../../include/bsls_cpu.h"

#include <algorithm>
#include <cstring>
#include <functional>
#include <vector>

namespace {

inline int64_t block_end(const int64_t *starts, int64_t nb, int64_t b, int64_t n) {
    return (b + 1 < nb) ? starts[b + 1] : n;
}

bool starts_ok(const int64_t *starts, int64_t nb, int64_t n) {
    if (!starts || nb < 1 || starts[0] < 0 || starts[nb - 1] >= n) return false;
    for (int64_t b = 1; b < nb; ++b)
        if (starts[b] <= starts[b - 1]) return false;
    return true;
}

int64_t max_block(const int64_t *starts, int64_t nb, int64_t n) {
    int64_t m = 0;
    for (int64_t b = 0; b < nb; ++b) m = std::max(m, block_end(starts, nb, b, n) - starts[b]);
    return m;
}

// proj_simplex.h:17-34: sort a copy descending, sequential running sum, the
// LAST index whose test passes sets lambda, then y = std::max(lambda + y, 0).
void simplex_block(double *y, int64_t start, int64_t end, double *u) {
    const int64_t k = end - start;
    if (k <= 0) return;
    std::memcpy(u, y + start, (size_t)k * sizeof(double));
    std::sort(u, u + k, std::greater<double>());
    double sum = u[0];
    double lambda = 1. - sum;
    for (int64_t i = 1; i < k; ++i) {
        sum += u[i];
        const double tmp = (1. - sum) / ((double)i + 1.);
        if (u[i] + tmp > 0) lambda = tmp;
    }
    for (int64_t i = start; i < end; ++i) y[i] = std::max(lambda + y[i], 0.);
}

// proj_simplex.h:50-74 for one block: clamp negatives, sum the rest in order,
// project only when the sum exceeds 1
void ball_block(double *y, int64_t start, int64_t end, double *u) {
    double sum = 0.0;
    for (int64_t j = start; j < end; ++j) {
        if (y[j] < 0.0) y[j] = 0.0;
        else sum += y[j];
    }
    if (sum > 1.0) simplex_block(y, start, end, u);
}

// isotonic_regression.h:13-58 ("PAVA+"): forward passes over run heads until
// a pass pools nothing; a non-increasing chain with distinct ends is replaced
// by its weighted mean (numerator in run order, integer denominator)
void iso_v1(double *y, int64_t start, int64_t end, int32_t *w, int update) {
    for (;;) {
        bool pooled = false;
        int64_t i = start;
        while (i < end) {
            int64_t k = i + w[i], j = i;
            while (k < end && y[k] <= y[j]) {
                j = k;
                k += w[k];
            }
            if (y[i] != y[j]) {
                double num = 0.0;
                int den = 0;
                for (j = i; j < k; j += w[j]) {
                    num += y[j] * w[j];
                    den += w[j];
                }
                y[i] = num / den;
                w[i] = den;
                pooled = true;
            }
            i = k;
        }
        if (!pooled) break;
    }
    if (update)
        for (int64_t i = start; i < end; i += w[i])
            for (int64_t j = i + 1; j < i + w[i]; ++j) y[j] = y[i];
}

// isotonic_regression.h:61-82: unweighted passes, each violating run averaged
void iso_v2(double *y, int64_t start, int64_t end) {
    end -= 1;
    for (;;) {
        bool pooled = false;
        int64_t i = start;
        while (i < end) {
            int64_t k = i;
            while (k < end && y[k] >= y[k + 1]) k += 1;
            if (y[i] != y[k]) {
                double num = 0.0;
                for (int64_t j = i; j < k + 1; ++j) num += y[j];
                const double avg = num / (double)(int)(k + 1 - i);
                for (int64_t j = i; j < k + 1; ++j) y[j] = avg;
                pooled = true;
            }
            i = k + 1;
        }
        if (!pooled) break;
    }
}

// isotonic_regression.h:105-155: one forward pass with backtracking; w mirrors
// the run length at run heads and tails
void iso_v3(double *y, int64_t start, int64_t end, int32_t *w, int update) {
    int64_t i = start;
    while (i < end) {
        int64_t k = i + w[i], j = i;
        while (k < end && y[k] <= y[j]) {
            j = k;
            k += w[k];
        }
        if (y[i] != y[j]) {
            double num = 0.0;
            int den = 0;
            for (j = i; j < k; j += w[j]) {
                num += y[j] * w[j];
                den += w[j];
            }
            y[i] = num / den;
            w[i] = den;
            w[k - 1] = den;
            if (i > start) {
                j = i - w[i - 1];
                while (j >= start && y[j] >= y[i]) {
                    y[j] = (w[i] * y[i] + w[j] * y[j]) / (w[i] + w[j]);
                    w[j] = w[i] + w[j];
                    i = j;
                    if (j == start) break;
                    j -= w[j - 1];
                }
                w[k - 1] = w[i];
            }
        } else {
            i = k;
        }
    }
    if (update)
        for (int64_t a = start; a < end; a += w[a])
            for (int64_t b = a + 1; b < a + w[a]; ++b) y[b] = y[a];
}

int nthreads(int threads) { return threads > 0 ? threads : 1; }

}  // namespace

extern "C" {

int bsls_cpu_proj_simplex(double *y, int64_t start, int64_t end) {
    if (!y || start < 0 || end < start) return -1;
    std::vector<double> u((size_t)(end - start) + 1);
    simplex_block(y, start, end, u.data());
    return 0;
}

static int proj_multi(bool ball, double *y, const int64_t *starts, int64_t nb, int64_t n,
                      int threads) {
    if (!y || !starts_ok(starts, nb, n)) return -1;
    const int64_t mb = max_block(starts, nb, n);
#pragma omp parallel num_threads(nthreads(threads))
    {
        std::vector<double> u((size_t)mb + 1);
#pragma omp for schedule(dynamic, 256)
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t s = starts[b], e = block_end(starts, nb, b, n);
            if (ball) ball_block(y, s, e, u.data());
            else simplex_block(y, s, e, u.data());
        }
    }
    return 0;
}

int bsls_cpu_proj_multi_simplex(double *y, const int64_t *starts, int64_t nb, int64_t n,
                                int threads) {
    return proj_multi(false, y, starts, nb, n, threads);
}

int bsls_cpu_proj_multi_ball(double *y, const int64_t *starts, int64_t nb, int64_t n,
                             int threads) {
    return proj_multi(true, y, starts, nb, n, threads);
}

int bsls_cpu_isotonic_multi(int variant, double *y, const int64_t *starts, int64_t nb, int64_t n,
                            int32_t *weight, int update, int threads) {
    if (!y || !starts_ok(starts, nb, n) || variant < 1 || variant > 3) return -1;
    if (variant != 2 && !weight) return -1;
#pragma omp parallel for num_threads(nthreads(threads)) schedule(dynamic, 256)
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t s = starts[b], e = block_end(starts, nb, b, n);
        if (variant == 1) iso_v1(y, s, e, weight, update);
        else if (variant == 2) iso_v2(y, s, e);
        else iso_v3(y, s, e, weight, update);
    }
    return 0;
}

double bsls_cpu_quad_obj(const double *x, const double *Q, const double *c, double *g,
                         int64_t n) {
    double f = 0;
    for (int64_t i = 0; i < n; ++i) {
        g[i] = c[i];
        const int64_t k = i * n;
        for (int64_t j = 0; j < n; ++j) g[i] += Q[k + j] * x[j];
        f += 0.5 * (g[i] + c[i]) * x[i];
    }
    return f;
}

double bsls_cpu_line_search(const double *x, double f, const double *g, double *x_new,
                            double f_new, double *g_new, const double *Q, const double *c,
                            int64_t n) {
    // quadratic_objective.h:29-61; upper_line keeps accumulating across the
    // backtracking steps, as the reference's does
    double t = 1, suffDec = 1e-4, upper_line = f, progTol = 1e-8;
    for (int64_t i = 0; i < n; ++i) upper_line += suffDec * g[i] * (x_new[i] - x[i]);
    while (f_new > upper_line) {
        t *= .5;
        double mx = 0.0;
        for (int64_t i = 0; i < n; ++i) {
            if (x_new[i] - x[i] > mx) mx = x_new[i] - x[i];
            if (x[i] - x_new[i] > mx) mx = x[i] - x_new[i];
        }
        if (t * mx < progTol) {
            for (int64_t i = 0; i < n; ++i) x_new[i] = x[i];
            f_new = f;
            break;
        }
        for (int64_t i = 0; i < n; ++i) x_new[i] = x[i] + t * (x_new[i] - x[i]);
        f_new = bsls_cpu_quad_obj(x_new, Q, c, g_new, n);
        for (int64_t i = 0; i < n; ++i) upper_line += suffDec * g[i] * (x_new[i] - x[i]);
    }
    return f_new;
}

int bsls_cpu_x2z(const double *x, double *z, const int64_t *starts, int64_t nb, int64_t n) {
    if (!x || !z || !starts_ok(starts, nb, n) || starts[0] != 0) return -1;
    int64_t j = 0;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t e = block_end(starts, nb, b, n);
        double tmp = 0.0;
        for (int64_t i = starts[b]; i < e - 1; ++i) {
            tmp += x[i];
            z[j++] = tmp;
        }
    }
    return 0;
}

int bsls_cpu_z2x(double *x, const double *z, const int64_t *starts, int64_t nb, int64_t n) {
    if (!x || !z || !starts_ok(starts, nb, n) || starts[0] != 0) return -1;
    int64_t j = 0;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t e = block_end(starts, nb, b, n);
        double tmp = 0.0;
        for (int64_t i = starts[b]; i < e - 1; ++i) {
            x[i] = z[j] - tmp;
            tmp = z[j];
            ++j;
        }
        x[e - 1] = 1.0 - tmp;
    }
    return 0;
}

const char *bsls_cpu_version(void) { return "bsls-cpu 1 (c_extensions host path, OpenMP)"; }

}  // extern "C"
